"""Trainer.validate_one_epoch host logic (espnet2/train/trainer.py:735-783 and the
WeightedAverage epoch summary of espnet2/train/reporter.py:aggregate) on CPU with a stub
model: eval/train mode handling, per-batch weighted averages skipping None and non-finite
values, and the iterator_stop protocol over world-size-2 gloo with unequal iterators."""
import math
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class StubModel:
    """Returns the stats of a batch as given: (loss, stats, weight) like ESPnetASRModel."""

    def __init__(self, bn_mean=0.0):
        self.training = True
        self.calls = 0
        # stands in for a BatchNorm running mean (the arena's flat f32 buffer): the eval
        # forward adds it to the loss, so a rank that skipped the rank-0 broadcast shows
        self.buf_f32 = torch.tensor([bn_mean])
        self.buf_i64 = torch.zeros(1, dtype=torch.long)

    def eval(self):
        self.training = False

    def train(self):
        self.training = True

    def __call__(self, stats, weight):
        assert not self.training
        self.calls += 1
        st = {k: (None if v is None else torch.tensor(v) + (self.buf_f32[0] if k == "loss" else 0.0))
              for k, v in stats.items()}
        return torch.tensor(0.0), st, torch.tensor([weight])


def test_validate_weighted_average_single_process():
    from espnet_amd.train.trainer import Trainer
    m = StubModel()
    batches = [dict(stats={"loss": 2.0, "cer": 0.5, "cer_ctc": None}, weight=2),
               dict(stats={"loss": 4.0, "cer": float("nan"), "cer_ctc": None}, weight=6),
               dict(stats={"loss": 1.0, "cer": 0.1, "cer_ctc": 0.3}, weight=2)]
    out = Trainer.validate_one_epoch(m, iter(batches), device="cpu")
    assert m.training and m.calls == 3
    assert out["loss"] == pytest.approx((2 * 2 + 4 * 6 + 1 * 2) / 10)
    assert out["cer"] == pytest.approx((0.5 * 2 + 0.1 * 2) / 4)  # nan batch skipped
    assert out["cer_ctc"] == pytest.approx(0.3)                  # None batches skipped


class _DP:
    def __init__(self, model):
        self.world_size = dist.get_world_size()
        self.active = self.world_size > 1
        self.group = None
        self.arena = model  # buf_f32 / buf_i64

    def broadcast_buffers(self):
        from espnet_amd.train.distributed import ArenaDataParallel
        return ArenaDataParallel.broadcast_buffers(self)

    def weighted_average(self, loss, stats, weight):
        from espnet_amd.train.distributed import ArenaDataParallel
        return ArenaDataParallel.weighted_average(self, loss, stats, weight)


def _worker(rank, world, init, q):
    from espnet_amd.train.trainer import Trainer
    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    m = StubModel(bn_mean=100.0 if rank == 0 else -7.0)  # per-replica BN stats differ
    n = 3 if rank == 0 else 2  # rank 0 holds one batch more: it must stop with rank 1
    # cer_ctc is None on rank 0 and present on rank 1 (e.g. every reference empty after
    # blank/space removal on one rank): the one packed all-reduce must still line up
    batches = [dict(stats={"loss": float(10 * rank + i), "cer_ctc": (None if rank == 0 else 0.25 + i)},
                    weight=1 + rank) for i in range(n)]
    out = Trainer.validate_one_epoch(m, iter(batches), dp=_DP(m), device="cpu")
    q.put((rank, out, m.calls))
    dist.destroy_process_group()


def test_validate_gloo_world2_unequal_iterators():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = tempfile.mktemp(prefix="ea_val_")
    ps = [ctx.Process(target=_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (o, c) for r, o, c in (q.get(timeout=120) for _ in range(2))}
    for p in ps:
        p.join(60)
    if os.path.exists(init):
        os.remove(init)
    # batch i: rank0 loss i (w 1), rank1 loss 10+i (w 2), both evaluated with rank 0's
    # broadcast BN buffer (+100) -> (i + 2(10+i)) / 3 + 100, weight 3
    want = sum(((i + 2 * (10 + i)) / 3 + 100.0) * 3 for i in range(2)) / 6
    want_cer = sum((0.25 + i) * 3 for i in range(2)) / 6  # rank 1's values only
    for r in (0, 1):
        out, calls = res[r]
        assert calls == 2
        assert math.isclose(out["loss"], want, rel_tol=1e-6)
        assert math.isclose(out["cer_ctc"], want_cer, rel_tol=1e-6)
