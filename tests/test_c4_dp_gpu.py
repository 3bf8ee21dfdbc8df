"""C4 at its per-rank workload: Conformer-L data parallel, 32 utterances x 1000 frames per rank.

BASELINE.json configs[3] / SURVEY.md section 8(e): the C3 model (12x512 Conformer encoder, 6-layer
Transformer decoder, V=5000, dropout 0.1, bf16 AMP, Adam + WarmupLR + clip 5) trained data
parallel, each rank holding its own B=32 shard, the weight gradients all-reduced in 64 MiB
buckets from the side stream while the backward runs (espnet2/train/trainer.py:229-244 wraps
the model in DDP; the shard per rank is espnet2/tasks/abs_task.py:1566-1575).  Two gloo ranks
share cuda:0 (RCCL needs one GPU per rank); since round 6 gloo issues its bucket all-reduces
from the same side-stream points as RCCL (train/distributed.py), so this is the production
ordering at the production bucket size and tensor sizes.

Checks, each bit-exact:
1. the reduced gradient of the DP step equals the sum over ranks of each rank's own shard
   gradient computed by a second, non-DP copy of the model (same weights, same dropout seeds,
   the same loss weighting w_r / sum_r w_r: trainer.py:604-619) and summed after its backward
   (two ranks: a + b, the same fp32 addition the bucket all-reduce does);
2. after two full steps (clip + Adam) both ranks hold identical weights.
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


def _worker(rank, world, init, q):
    _paths()
    import numpy as np
    import torch.distributed as dist
    import bench
    from espnet_amd import hip_ops as ops
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.trainer import Trainer
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    try:
        cfg = bench.c3_config()

        def model():
            m = bench.build(cfg)
            m.prepare(dev, amp=True, seed=1234)
            m.train()
            return m

        m, ref = model(), model()
        assert torch.equal(m.arena.data, ref.arena.data)
        opt = ArenaAdam(m, lr=cfg["optim"]["lr"], weight_decay=cfg["optim"]["weight_decay"])
        sched = WarmupLR(opt, warmup_steps=cfg["warmup_steps"])
        dp = ArenaDataParallel(m)  # production bucket size (64 MiB)
        nb = len(dp.buckets)
        batches = [{k: v.to(dev) for k, v in bench.synthetic_batch(cfg, s + rank).items()} for s in (1, 11)]

        # 1. each rank's own shard gradient, non-DP model, DDP's loss weighting; summed after
        loss, _, w = ref(**batches[0])
        w = w.to(torch.float32).view(1)
        wsum = w.clone()
        dist.all_reduce(wsum)
        with ops.deferred_wgrad():
            ((loss * w).sum() / wsum).backward()
        torch.cuda.synchronize()
        expect = ref.arena.grad.clone()
        dist.all_reduce(expect)
        del ref

        grads = []
        orig = opt.compute_grad_norm

        def snap(*a, **k):
            grads.append(m.arena.grad.clone())
            return orig(*a, **k)
        opt.compute_grad_norm = snap
        for b in batches:
            Trainer.train_one_step(m, b, opt, sched, grad_clip=5.0, dp=dp)
        torch.cuda.synchronize()
        bad = [n for n in m.arena.names
               if not torch.equal(*(g[m.arena.offsets[n]:m.arena.offsets[n] + m.arena._params[n].numel()]
                                    for g in (grads[0], expect)))]
        # 2. both ranks' weights after two full steps
        w0 = m.arena.data.clone()
        dist.broadcast(w0, src=0)
        res = dict(rank=rank, buckets=nb, grad_mismatch=bad, weights_equal=bool(torch.equal(w0, m.arena.data)),
                   grad_abs=float(expect.abs().sum()), finite=bool(torch.isfinite(m.arena.data).all()),
                   loss=np.float64(float(loss)))
        q.put(res)
        dist.barrier()
    except Exception:
        import traceback
        q.put(dict(rank=rank, error=traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def test_c4_per_rank_workload_dp_step_bit_exact():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = tempfile.mktemp(prefix="ea_c4_")
    ps = [ctx.Process(target=_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=280) for _ in range(2)), key=lambda r: r["rank"])
    for p in ps:
        p.join(60)
    for r in res:
        assert "error" not in r, r["error"]
    for r in res:
        assert r["buckets"] > 4, r["buckets"]  # ~465 MB of f32 gradients in 64 MiB buckets
        assert r["grad_abs"] > 0 and r["finite"]
        assert not r["grad_mismatch"], f"rank {r['rank']}: {r['grad_mismatch'][:8]}"
        assert r["weights_equal"], r["rank"]
