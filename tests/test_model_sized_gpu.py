"""Whole-model parity at BASELINE.json sizes on the MI355X.

Goldens `c3_b2` (configs[2]: Conformer-L 12x512 + 6-layer decoder, V=5000, T=1000, L=40),
`c2_b2` (configs[1]: Conformer-S 6x256, CTC only, T=500, L=20) and `amp_hybrid` (d_k=64,
2+2 blocks, T'=99) were captured from the reference itself at B=2 with one ragged
utterance (oracle/make_goldens.py capture_sized: weights regenerated from the seed and
checked against stored per-tensor sums).  Every parameter gradient is also compared in
full against the oracle run in float64 on the host cores (oracle/asr_oracle.py, pinned to
the same goldens in fp32 by tests/test_oracle_goldens.py::test_oracle_sized_goldens).

fp32: loss/stats atol 1e-4 + rtol 2e-6; encoder output atol/rtol 1e-4; CTC argmax
bit-exact (frames whose reference top-2 logit gap is below the 1e-4 logit tolerance are
reported, and may differ only there).  Gradients: against the float64 oracle (exact
arithmetic) every parameter's relative L2 error must be <= 2e-5 — measured 0.6-3.9e-6 on
the MI355X, while ATen fp32 (what the reference computes) sits at 0.4-5.3e-4 of the same
yardstick (scripts/sized_diag.py, profiles/r3_sized_diag.txt); against the reference's
own fp32 gradients (norm + 256-element head per tensor) the bound is the reference's fp32
noise: norm rtol 1e-3, head relative L2 <= 3e-3.

`c5_b2` (configs[4]: Conformer-L + decoder with SpecAug conformer8, a bucketed pair of
T = 2000 and 1317 frames, T' = 499, L = 80 / 53; the TimeWarp / mask / layer-drop draws
from torch.manual_seed(spec_seed) before the forward, identical in the reference, the
oracle and the HIP model) is checked in bf16 only: the HIP bicubic warp differs from
ATen's by up to 5e-5 (tests/test_specaug.py), above the fp32 gradient bound.

bf16 (AMP, the benchmarked code path: fused rel-pos attention, ping-pong 256x256 GEMMs,
grouped weight gradients, LayerNorm-backward dropout fusion): per-tensor relative L2
distance from the float64 gradient, bounded by the reference's OWN bf16 distance (the
same step under torch.autocast("cpu", bfloat16), stored per tensor as `ampdev`) times 2,
with a floor of 2e-2 (bf16 keeps 8 significant bits: 2^-9 = 2e-3 per rounding,
accumulated over ~10 roundings along a layer's forward and backward).
"""
import numpy as np
import pytest
import torch

from goldens import is_null_grad, regenerate_sized, section, sibling_weight
from test_model_build import build

pytestmark = pytest.mark.gpu


_EXACT = {}


def _exact(name, cfg, d, m_cpu):
    """The float64 oracle's loss and gradients for this golden (cached per module)."""
    if name not in _EXACT:
        from oracle.asr_oracle import OracleASR
        torch.set_num_threads(16)
        ora = OracleASR(cfg, {k: v.detach() for k, v in m_cpu.state_dict().items()}, dtype=torch.float64)
        inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
        _reseed(cfg)
        loss, _, _ = ora(**inp)
        loss.backward()
        _EXACT[name] = (loss.item(), {k: p.grad.detach() for k, p in ora.params.items()})
    return _EXACT[name]


def _rel_l2(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    den = b.norm().item()
    return (a - b).norm().item() / den if den > 0 else (a - b).norm().item()


def _reseed(cfg):
    """c5_b2: the step's host draws (SpecAug's TimeWarp / masks, then repeat.py:27's layer-drop
    uniforms) come from torch.manual_seed(spec_seed), as in the capture."""
    if cfg.get("spec_seed") is not None:
        torch.manual_seed(cfg["spec_seed"])


def _hip(cfg, d, m, amp):
    if cfg.get("specaug_conf"):
        from espnet_amd.asr.specaug import SpecAug
        m.specaug = SpecAug(**cfg["specaug_conf"])
    m.prepare("cuda:0", amp=amp)
    m.train()
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    _reseed(cfg)
    loss, stats, weight = m(**inp)
    loss.backward()
    torch.cuda.synchronize()
    return loss, stats, weight


def _ctc_argmax_check(am, d, tol_gap=1e-4):
    ref = d["out.ctc_argmax"]
    gap = d["out.ctc_top2_gap"]
    olens = d["out.encoder_out_lens"]
    valid = np.arange(ref.shape[1])[None, :] < olens[:, None]
    diff = am != ref
    # a flip is only admissible where the reference's own top-2 gap is inside the logit tolerance
    assert not (diff & (gap >= tol_gap)).any(), np.argwhere(diff & (gap >= tol_gap))[:10]
    assert int((diff & valid).sum()) <= max(1, int((gap < tol_gap).sum())), int(diff.sum())
    return int(diff.sum()), int((gap < tol_gap).sum())


@pytest.mark.parametrize("name", ["amp_hybrid", "c2_b2", "c3_b2"])
def test_sized_fp32_parity(name):
    cfg, d, m = regenerate_sized(name, build)
    x_loss, x_grads = _exact(name, cfg, d, m)
    loss, stats, weight = _hip(cfg, d, m, amp=False)
    np.testing.assert_allclose(loss.item(), d["out.loss"], rtol=2e-6, atol=1e-4)
    np.testing.assert_allclose(loss.item(), x_loss, rtol=2e-6, atol=1e-4)
    assert weight.item() == d["out.weight"]
    for k, v in section(d, "stat").items():
        np.testing.assert_allclose(stats[k].item(), v, rtol=2e-6, atol=1e-4, err_msg=k)
    enc, olens = m._last_encoder_out
    np.testing.assert_array_equal(olens.cpu().numpy(), d["out.encoder_out_lens"])
    np.testing.assert_allclose(enc.detach().cpu().numpy(), d["out.encoder_out"], atol=1e-4, rtol=1e-4)
    flips, near = _ctc_argmax_check(m.ctc.argmax(enc.detach()).cpu().numpy(), d)
    print(f"{name}: CTC argmax flips {flips} (frames with top-2 gap < 1e-4: {near})")
    params = dict(m.named_parameters())
    gn = section(d, "gn")
    worst = []
    for k, p in params.items():
        mine = p.grad.detach().cpu()
        if is_null_grad(k):
            assert mine.double().norm().item() <= 1e-3 * gn[sibling_weight(k)], k
            continue
        np.testing.assert_allclose(mine.double().norm().item(), gn[k], rtol=1e-3, err_msg=k)
        e_head = _rel_l2(mine.reshape(-1)[:256], torch.from_numpy(d["gh." + k]))
        assert e_head <= 3e-3, (k, e_head)
        e = _rel_l2(mine, x_grads[k])
        worst.append((e, k))
        assert e <= 2e-5, (k, e)
    worst.sort(reverse=True)
    print(f"{name}: fp32 gradient relative L2 vs float64, worst: {worst[:3]}")
    sd = m.state_dict()
    for k, v in section(d, "buf_after").items():
        np.testing.assert_allclose(sd[k].cpu().numpy(), v, atol=1e-5, rtol=1e-5, err_msg=k)


AMP_FLOOR = 2e-2


@pytest.mark.parametrize("name", ["amp_hybrid", "c2_b2", "c3_b2", "c5_b2"])
def test_sized_bf16_amp_per_tensor(name):
    cfg, d, m = regenerate_sized(name, build)
    x_loss, x_grads = _exact(name, cfg, d, m)
    loss, stats, _ = _hip(cfg, d, m, amp=True)
    ref_loss_dev = abs(float(d["amp.loss"]) - float(d["out.loss"])) / abs(float(d["out.loss"]))
    loss_dev = abs(loss.item() - x_loss) / abs(x_loss)
    assert loss_dev <= max(2 * ref_loss_dev, 2e-3), (loss_dev, ref_loss_dev)
    ampdev = section(d, "ampdev")
    gn = section(d, "gn")
    worst = []
    for k, p in dict(m.named_parameters()).items():
        mine = p.grad.detach().cpu()
        if is_null_grad(k):
            assert mine.double().norm().item() <= 1e-2 * gn[sibling_weight(k)], k
            continue
        e = _rel_l2(mine, x_grads[k])
        bound = max(2.0 * float(ampdev[k]), AMP_FLOOR)
        worst.append((e / bound, e, float(ampdev[k]), k))
    worst.sort(reverse=True)
    print(f"{name}: loss dev {loss_dev:.2e} (reference bf16 {ref_loss_dev:.2e}); worst e/bound:",
          "; ".join(f"{k} {e:.2e} (ref {r:.2e})" for _, e, r, k in worst[:5]))
    bad = [w for w in worst if w[0] > 1.0]
    assert not bad, bad[:10]
