"""Transposed bf16 weight shadow (hip_ops.TransposedShadow, ea_transpose_bf16_grouped): the
Linear input-gradient GEMMs of narrow outputs read W^T K-major from copies the optimizer
refreshes.  Checks the grouped transpose, the refresh after an Adam step and after
load_state_dict, and that an AMP training step gives the same gradients with and without it."""
import numpy as np
import pytest
import torch

from goldens import load, section
from test_model_build import build

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_grouped_transpose_and_refresh():
    from espnet_amd import hip_ops as ops
    g = torch.Generator().manual_seed(0)
    shadow = torch.randn(3 * 4096 + 5000 * 512 + 1536 * 512, generator=g).to(torch.bfloat16).to(DEV)
    ts = ops.TransposedShadow(shadow)
    views = [shadow[64:64 + 64 * 64].view(64, 64), shadow[8192:8192 + 5000 * 512].view(5000, 512),
             shadow[8192 + 5000 * 512:8192 + 5000 * 512 + 1536 * 512].view(1536, 512)]
    wts = [ts.get(v) for v in views]
    torch.cuda.synchronize()
    for v, wt in zip(views, wts):
        assert wt.shape == (v.shape[1], v.shape[0]) and torch.equal(wt, v.t().contiguous())
    shadow.mul_(-2.0)
    ts.refresh()
    torch.cuda.synchronize()
    for v, wt in zip(views, wts):
        assert torch.equal(wt, v.t().contiguous())
    assert ts.get(views[1]) is wts[1]  # registered once
    # a captured refresh freezes the table: a weight first seen afterwards is not registered
    # (the graph would never refresh its copy, and rebuilding would free the captured table)
    tiles_ptr = ts.tiles.data_ptr()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ts.refresh()
    late = shadow[:64 * 64].view(64, 64)
    assert ts.frozen and ts.get(late) is None and ts.tiles.data_ptr() == tiles_ptr
    shadow.mul_(3.0)
    g.replay()
    torch.cuda.synchronize()
    for v, wt in zip(views, wts):
        assert torch.equal(wt, v.t().contiguous())


def _amp_grads(wt_on):
    from espnet_amd import hip_ops as ops
    cfg, d = load("medium_hybrid")
    old = ops.WT_SHADOW
    ops.WT_SHADOW = wt_on
    try:
        torch.manual_seed(0)
        m = build(cfg)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
        m.prepare("cuda", amp=True)
    finally:
        ops.WT_SHADOW = old
    assert (m.arena.tshadow is not None) == wt_on
    m.train()
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    loss, _, _ = m(**inp)
    loss.backward()
    torch.cuda.synchronize()
    return m, loss.item(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}


def test_amp_step_same_with_transposed_shadow():
    m1, l1, g1 = _amp_grads(True)
    assert m1.arena.tshadow.items, "no input-gradient GEMM used the transposed shadow"
    _, l0, g0 = _amp_grads(False)
    assert l1 == l0
    for k in g0:
        e = float((g1[k].double() - g0[k].double()).norm() / g0[k].double().norm().clamp_min(1e-30))
        assert e < 1e-5, (k, e)


def test_transposed_shadow_follows_optimizer_and_loads():
    from espnet_amd.optim.adam import ArenaAdam
    m, _, _ = _amp_grads(True)
    ts = m.arena.tshadow
    opt = ArenaAdam(m, lr=1e-3)
    opt.step()
    torch.cuda.synchronize()
    for (off, R, C), wt in ts.items.items():
        w = m.arena.shadow[off:off + R * C].view(R, C)
        assert torch.equal(wt, w.t().contiguous())
    sd = {k: v.clone() * 0.5 for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    torch.cuda.synchronize()
    for (off, R, C), wt in ts.items.items():
        w = m.arena.shadow[off:off + R * C].view(R, C)
        assert torch.equal(wt, w.t().contiguous())
