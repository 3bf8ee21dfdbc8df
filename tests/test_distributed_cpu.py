"""World-size-2 gloo tests (CPU) of the data-parallel layer over the parameter arena:
bucketed gradient all-reduce driven by grad-ready hooks, the packed recursive_average,
rank-0 parameter / BatchNorm-buffer broadcast (trainer.py:229-244, :604-619)."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.enc = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.BatchNorm1d(64))
        self.dec = torch.nn.Linear(64, 128)
        self.head = torch.nn.Linear(128, 8)


def _worker(rank, world, init, q):
    from espnet_amd import hip_ops
    from espnet_amd.arena import ParamArena
    from espnet_amd.layers.common import Bound
    from espnet_amd.train.distributed import ArenaDataParallel

    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank: broadcast must unify
    m = Toy()
    with torch.no_grad():
        m.enc[1].running_mean.fill_(float(rank + 1))
    m.arena = ParamArena(m, "cpu", [])
    for name in ("enc", "dec", "head"):
        getattr(m, name)._b = Bound(m.arena, name + ".", torch.float32)
    dp = ArenaDataParallel(m, bucket_mb=0.02)  # tiny buckets -> several
    out = {}
    out["w0"] = m.enc[0].weight.detach().clone()
    out["rm"] = m.enc[1].running_mean.clone()
    out["nb"] = len(dp.buckets)
    # gradients: rank-dependent; hooks fire in backward order head -> dec -> enc
    m.arena.grad.copy_(torch.arange(m.arena.numel, dtype=torch.float32) * (rank + 1))
    dp.begin_backward()
    for pre in ("head.", "dec.", "enc."):
        if hip_ops.GRAD_READY:
            hip_ops.GRAD_READY(pre)
    dp.allreduce_grads()
    out["g"] = m.arena.grad.clone()
    loss = torch.tensor(2.0 + rank, requires_grad=True)
    stats = {"loss": torch.tensor(10.0 * (rank + 1)), "acc": torch.tensor(0.5 + 0.25 * rank)}
    weight = torch.tensor([3 + rank])
    l2, s2, w2 = dp.weighted_average(loss, stats, weight)
    out["loss"] = float(l2.detach())
    out["stats"] = {k: float(v) for k, v in s2.items()}
    out["w"] = int(w2)
    out = {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
    q.put((rank, out))
    dist.destroy_process_group()


def test_arena_ddp_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = tempfile.mktemp(prefix="ea_dp_")
    ps = [ctx.Process(target=_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
    a, b = res[0], res[1]
    for d in (a, b):
        for k in ("w0", "rm", "g"):
            d[k] = torch.from_numpy(d[k])
    assert a["nb"] > 2
    torch.testing.assert_close(a["w0"], b["w0"])           # K3: rank-0 params everywhere
    torch.testing.assert_close(b["rm"], torch.full((64,), 1.0))  # K2: rank-0 BN buffers
    n = a["g"].numel()
    torch.testing.assert_close(a["g"], torch.arange(n, dtype=torch.float32) * 3)  # K1: SUM
    torch.testing.assert_close(a["g"], b["g"])
    # trainer.py:604-619: loss_r * w_r / sum(w); stats weighted by w
    assert abs(a["loss"] - 2.0 * 3 / 7) < 1e-6 and abs(b["loss"] - 3.0 * 4 / 7) < 1e-6
    assert a["w"] == 7 and b["w"] == 7
    assert abs(a["stats"]["loss"] - (10 * 3 + 20 * 4) / 7) < 1e-5
    assert abs(a["stats"]["acc"] - (0.5 * 3 + 0.75 * 4) / 7) < 1e-6
