"""Cross-stream ordering of the training step, made deterministic.

The step overlaps work on three HIP streams (hip_ops: the main stream, the weight-gradient
side stream, the auxiliary stream of the CTC head) and, under data parallelism, starts bucket
all-reduces from the side stream while the backward goes on (espnet2/train/trainer.py:229-244
wraps the model in DDP, which overlaps the same way).  A missing dependency between streams
shows up only now and then in an ordinary run; these tests make it show up every time:

1. every side / auxiliary stream segment is held 300 us before its first launch
   (hip_ops.DEBUG_DELAY_NS -> ea_debug_spin): a consumer that does not wait for its producer
   reads stale data in every run.  The delayed step must be bit-identical to the serialised
   step (hip_ops.DEBUG_SERIAL: the main stream joins every segment) and to the default one.
2. data parallel, world-1 gloo group with the production (side-stream) issue order: every
   bucket is compared between its all-reduce issue point and the end of the backward
   (ArenaDataParallel.check_issue); a gradient written into a bucket after its all-reduce was
   issued fails the step, naming the parameter.
3. two gloo ranks, accum_grad=2 over two micro-steps: the reduced gradient equals the sum of
   the four shards' weighted gradients (DDP's mean of the accumulated .grad), not the earlier
   micro-step counted world_size times.
"""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _paths():
    import sys
    for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "espnet-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _steps(dp=None, n=4, mode="default"):
    """n training steps of the tiny Conformer (dropout 0.1, bf16) on the ragged batches; ->
    (per-step gradient arenas, final weights)."""
    _paths()
    import test_dp_capture_gpu as C
    import test_dp_ragged_gpu as R
    from espnet_amd import hip_ops
    from espnet_amd.train.trainer import Trainer
    _, m, opt, sched = C._setup(amp=True, dropout=0.1)
    if dp is not None:
        dp = dp(m)
    grads = []
    orig = opt.compute_grad_norm

    def snap(*a, **k):
        grads.append(m.arena.grad.detach().cpu().clone())
        return orig(*a, **k)

    opt.compute_grad_norm = snap
    prev = hip_ops.DEBUG_DELAY_NS, hip_ops.DEBUG_SERIAL
    hip_ops.DEBUG_DELAY_NS = 300_000 if mode == "delay" else 0
    hip_ops.DEBUG_SERIAL = mode == "serial"
    try:
        for b in R._global_batches(n):
            Trainer.train_one_step(m, {k: v.to("cuda:0") for k, v in b.items()}, opt, sched, grad_clip=5.0, dp=dp)
        torch.cuda.synchronize()
    finally:
        hip_ops.DEBUG_DELAY_NS, hip_ops.DEBUG_SERIAL = prev
    return grads, m.arena.data.cpu().clone(), m


def _first_diff(a, b, m):
    for s, (x, y) in enumerate(zip(a, b)):
        if not torch.equal(x, y):
            names = [n for n in m.arena.names
                     if not torch.equal(x[m.arena.offsets[n]:m.arena.offsets[n] + m.arena._params[n].numel()],
                                        y[m.arena.offsets[n]:m.arena.offsets[n] + m.arena._params[n].numel()])]
            return f"step {s}: {names[:8]}"
    return None


def test_delayed_side_streams_bit_identical_to_serial():
    torch.cuda.set_device(0)
    gs, ws, m = _steps(mode="serial")
    gd, wd, _ = _steps(mode="delay")
    g0, w0, _ = _steps(mode="default")
    assert _first_diff(gd, gs, m) is None, _first_diff(gd, gs, m)
    assert _first_diff(g0, gs, m) is None, _first_diff(g0, gs, m)
    assert torch.equal(wd, ws) and torch.equal(w0, ws)
    assert all(float(g.abs().sum()) > 0 for g in gs)


def _dp_worker(init, q):
    _paths()
    import torch.distributed as dist
    from espnet_amd.train.distributed import ArenaDataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init}", rank=0, world_size=1)
    try:
        def mk(m):
            dp = ArenaDataParallel(m, bucket_mb=0.25, force_collectives=True, check_issue=True)
            assert dp.active and len(dp.buckets) > 2
            return dp
        res = {}
        # numpy (pickled by value): a queued tensor is shared by file descriptor and lost if
        # this process exits before the parent has read it
        np_ = lambda g, w: ([x.numpy() for x in g], w.numpy())  # noqa: E731
        res["serial"] = np_(*_steps(mode="serial")[:2])
        for mode in ("delay", "default"):
            res[mode] = np_(*_steps(dp=mk, mode=mode)[:2])
        q.put(res)
    except Exception:
        import traceback
        q.put({"error": traceback.format_exc()})
        raise
    finally:
        dist.destroy_process_group()


def test_dp_buckets_unchanged_after_issue_and_equal_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_dp_worker, args=(tempfile.mktemp(prefix="ea_dps_"), q))
    p.start()
    res = q.get(timeout=170)
    p.join(60)
    assert "error" not in res, res["error"]
    import numpy as np
    gs, ws = res["serial"]
    for mode in ("delay", "default"):
        g, w = res[mode]
        bad = [s for s, (x, y) in enumerate(zip(g, gs)) if not np.array_equal(x, y)]
        assert not bad, f"{mode}: gradients differ from the single-process serial step at steps {bad}"
        assert np.array_equal(w, ws), mode


def _accum_worker(rank, world, init, q):
    _paths()
    import torch.distributed as dist
    import test_dp_capture_gpu as C
    from espnet_amd import hip_ops as ops
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.trainer import Trainer
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    try:
        d, m, opt, sched = C._setup(amp=True, dropout=0.0)
        glob = C._batches(d, 2)
        dp = ArenaDataParallel(m, bucket_mb=0.25)
        opt.step = lambda *a, **k: None  # keep the reduced gradient in the arena
        opt.zero_grad = lambda *a, **k: None
        for k, b in enumerate(glob, 1):
            Trainer.train_one_step(m, {n: v[rank::world].to("cuda:0") for n, v in b.items()}, opt, sched,
                                   grad_clip=5.0, dp=dp, accum_grad=2, iiter=k)
        torch.cuda.synchronize()
        out = dict(dp=m.arena.grad.cpu().numpy())
        if rank == 0:
            # DDP's accumulated gradient: every shard's loss weighted by w_r / sum_r w_r
            # (trainer.py:604-619) and / accum_grad, summed over ranks and micro-steps
            _, m1, _, _ = C._setup(amp=True, dropout=0.0)
            for b in glob:
                shards = [{n: v[r::world].to("cuda:0") for n, v in b.items()} for r in range(world)]
                wsum = sum(float(s["speech"].shape[0]) for s in shards)
                for s in shards:
                    loss, _, w = m1(**s)
                    with ops.deferred_wgrad():
                        (loss * (float(w) / wsum) / 2).backward()
            torch.cuda.synchronize()
            out["ref"] = m1.arena.grad.cpu().numpy()
            q.put(out)
        dist.barrier()
    except Exception:
        import traceback
        q.put({"error": traceback.format_exc()})
        raise
    finally:
        dist.destroy_process_group()


def test_dp_accum_grad_two_micro_steps_matches_ddp():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = tempfile.mktemp(prefix="ea_acc_")
    ps = [ctx.Process(target=_accum_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=170)
    for p in ps:
        p.join(60)
    assert "error" not in out, out["error"]
    g, ref = torch.from_numpy(out["dp"]), torch.from_numpy(out["ref"])
    assert float(ref.abs().sum()) > 0
    # the same shard gradients, summed in another order (fp32): ~1e-7 relative per element
    rel = float((g - ref).norm() / ref.norm())
    assert rel < 1e-5, rel
    torch.testing.assert_close(g, ref, rtol=1e-4, atol=1e-6 * float(ref.abs().max()))
