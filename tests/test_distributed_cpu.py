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


class ToyLoss(Toy):
    """Toy with the model interface Trainer.train_one_step drives: forward(**batch) ->
    (loss, stats, weight), the batch size as the weight (espnet_model.py:326-337)."""

    def forward(self, x, y):
        h = self.head(torch.relu(self.dec(self.enc[0](x))))
        loss = ((h - y) ** 2).mean()
        return loss, {"loss": loss.detach()}, torch.tensor([x.shape[0]])


def _micro_batches(rank, k):
    g = torch.Generator().manual_seed(1000 * k + rank)
    n = 3 + rank  # unequal shard sizes: the loss weights w_r / sum(w) differ
    return dict(x=torch.randn(n, 64, generator=g), y=torch.randn(n, 8, generator=g))


class _NoStepOpt:
    """compute_grad_norm only: the reduced gradient stays in the arena."""

    def __init__(self, arena):
        self.arena = arena

    def compute_grad_norm(self):
        return self.arena.grad.norm()

    def step(self, **kw):
        pass

    def zero_grad(self):
        pass


def _accum_worker(rank, world, init, q):
    from espnet_amd.arena import ParamArena
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.trainer import Trainer

    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    torch.manual_seed(7)
    m = ToyLoss()
    m.eval()  # (BatchNorm unused by the loss)
    m.arena = ParamArena(m, "cpu", [])
    from espnet_amd.layers.common import Bound
    for name in ("enc", "dec", "head"):
        getattr(m, name)._b = Bound(m.arena, name + ".", torch.float32)
    dp = ArenaDataParallel(m, bucket_mb=0.02)
    opt = _NoStepOpt(m.arena)
    for k in (1, 2):
        Trainer.train_one_step(m, _micro_batches(rank, k), opt, None, grad_clip=5.0, dp=dp, accum_grad=2, iiter=k)
    got = m.arena.grad.clone()
    # DDP's accumulated gradient (trainer.py:229-244 + 604-619): every rank's micro-step loss
    # weighted by w_r / sum_r w_r and divided by accum_grad, summed over ranks and micro-steps
    m.arena.grad.zero_()
    for k in (1, 2):
        shards = [_micro_batches(r, k) for r in range(world)]
        wsum = sum(s["x"].shape[0] for s in shards)
        for s in shards:
            loss, _, w = m(**s)
            (loss * float(w) / wsum / 2).backward()
    q.put((rank, got.numpy(), m.arena.grad.clone().numpy()))
    dist.destroy_process_group()


def test_dp_accum_grad_reduces_on_the_updating_micro_step():
    """accum_grad = 2 over two micro-steps on two gloo ranks: the arena holds the SUM over ranks
    and micro-steps of the weighted micro-step gradients (DDP's result), not the first
    micro-step counted world_size times (round-5 advisor finding)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = tempfile.mktemp(prefix="ea_acc_cpu_")
    ps = [ctx.Process(target=_accum_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (g, e)) for r, g, e in (q.get(timeout=120) for _ in range(2)))
    for p in ps:
        p.join(60)
    for r in (0, 1):
        got, exp = (torch.from_numpy(a) for a in res[r])
        assert float(exp.abs().sum()) > 0
        torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(torch.from_numpy(res[0][0]), torch.from_numpy(res[1][0]))
