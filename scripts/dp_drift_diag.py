"""Locate the two-process DP drift (tests/test_dp_ragged_gpu.py): two gloo ranks on one GPU
run the ragged test's eager DP steps R times each, in the same two processes, every run from
the same weights; every run is compared with run 0 per step: the local loss, the bucket
contents handed to each all-reduce (a stream-ordered copy at the issue point, --snap) and the
reduced gradient arena.  The first step and tensor that differ name the segment.

    dp_drift_diag.py [--runs R] [--steps S] [--side] [--no-overlap] [--snap] [--fresh]

--fresh: every run is a new pair of processes (as every run of the test is), running the
ragged test's own protocol (Trainer.train_one_epoch, two epochs, rank 0 one step short in the
second); each run's records go to a file and the parent compares them with run 0's.
"""
import argparse
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "espnet-1_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, init, args):
    for p in (HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "espnet-1_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import test_dp_capture_gpu as C
    import test_dp_ragged_gpu as R
    from espnet_amd import hip_ops
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.trainer import Trainer
    import espnet_amd.train.distributed as dmod
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    if args.no_overlap:
        hip_ops.OVERLAP_WGRAD = False
    glob = R._global_batches(6)
    shards = [R._shard(glob[0], 0, world)] * 6 if rank == 0 else [R._shard(glob[i % 2], 1, world) for i in range(6)]
    real_ar = dist.all_reduce
    snaps = []

    def ar(t, *a, **k):
        if args.snap and k.get("async_op"):
            snaps[-1].append(t.detach().clone())
        return real_ar(t, *a, **k)

    dmod.dist.all_reduce = ar
    ref = None
    bad = 0
    for run in range(args.runs):
        _, m, opt, sched = C._setup(amp=True, dropout=0.1)
        dp = ArenaDataParallel(m, bucket_mb=0.25)
        if args.side:
            dp.ar_main = False
        rec = dict(loss=[], grad=[], snap=[])
        orig = opt.compute_grad_norm

        def cg(*a, **k):
            rec["grad"].append(m.arena.grad.detach().cpu().clone())
            return orig(*a, **k)

        opt.compute_grad_norm = cg
        for s in range(args.steps):
            snaps.append([])
            loss, _, _, _ = Trainer.train_one_step(m, {k: v.to("cuda:0") for k, v in shards[s].items()}, opt, sched,
                                                   grad_clip=5.0, dp=dp)
            torch.cuda.synchronize()
            rec["loss"].append(float(loss))
            rec["snap"].append([x.cpu() for x in snaps.pop()])
        if ref is None:
            ref = rec
            continue
        msgs = []
        for s in range(args.steps):
            if rec["loss"][s] != ref["loss"][s]:
                msgs.append(f"step {s} loss {rec['loss'][s]!r} vs {ref['loss'][s]!r}")
            for i, (x, y) in enumerate(zip(rec["snap"][s], ref["snap"][s])):
                if not torch.equal(x, y):
                    msgs.append(f"step {s} all-reduce #{i} input ({x.numel()} el) differs: "
                                f"{int((x != y).sum())} el, max {float((x - y).abs().max()):.3g}")
            if not torch.equal(rec["grad"][s], ref["grad"][s]):
                g, h = rec["grad"][s], ref["grad"][s]
                names = []
                for n in m.arena.names:
                    o, k = m.arena.offsets[n], m.arena._params[n].numel()
                    if not torch.equal(g[o:o + k], h[o:o + k]):
                        names.append(f"{n}({int((g[o:o+k] != h[o:o+k]).sum())}/{k}, {float((g[o:o+k]-h[o:o+k]).abs().max()):.2g})")
                msgs.append(f"step {s} reduced grads differ: {'; '.join(names[:10])}"
                            + (f" ... {len(names)} params" if len(names) > 10 else ""))
            if msgs:
                break
        if msgs:
            bad += 1
            print(f"rank {rank} run {run}: " + " | ".join(msgs[:6]), flush=True)
    print(f"rank {rank}: {bad} of {args.runs - 1} runs differ from run 0 ({vars(args)})", flush=True)
    dist.barrier()
    dist.destroy_process_group()


def fresh_worker(rank, world, init, args, out):
    for p in (HERE, os.path.join(HERE, "..", "tests"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "espnet-1_amd")):
        sys.path.insert(0, p)
    import numpy as np
    import torch.distributed as dist
    if args.poison:
        import drift_diag
        drift_diag.poison()
    if args.guard:  # before the first device allocation of the process
        from espnet_amd._lib import LIB_PATH
        torch.cuda.memory.change_current_allocator(
            torch.cuda.memory.CUDAPluggableAllocator(LIB_PATH, "ea_guard_malloc", "ea_guard_free"))
        torch.cuda.max_memory_reserved = lambda *a, **k: 0  # (no statistics from a pluggable allocator)
    import test_dp_capture_gpu as C
    import test_dp_ragged_gpu as R
    from espnet_amd import hip_ops
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.distributed_utils import DistributedOption
    from espnet_amd.train.reporter import Reporter
    from espnet_amd.train.trainer import Trainer
    import espnet_amd.train.distributed as dmod
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    if args.no_overlap:
        hip_ops.OVERLAP_WGRAD = False
    if args.no_aux:
        hip_ops.OVERLAP_AUX = False
    real_ar = dist.all_reduce
    snaps = []

    def ar(t, *a, **k):
        if k.get("async_op"):
            base = dp.arena.grad.data_ptr()
            snaps.append(((t.data_ptr() - base) // 4, t.detach().clone()))
        return real_ar(t, *a, **k)

    dmod.dist.all_reduce = ar
    _, m, opt, sched = C._setup(amp=True, dropout=0.1)
    dp = ArenaDataParallel(m, bucket_mb=0.25)
    if args.side:
        dp.ar_main = False
    n = m.arena.numel
    recs = []
    orig = opt.compute_grad_norm

    def cg(*a, **k):
        local = np.full(n, np.nan, dtype=np.float32)
        for off, x in snaps:
            local[off:off + x.numel()] = x.cpu().numpy()
        snaps.clear()
        recs.append((m.arena.data.detach().cpu().numpy().copy(), local, m.arena.grad.detach().cpu().numpy().copy()))
        return orig(*a, **k)

    opt.compute_grad_norm = cg
    dopt = DistributedOption(distributed=True, dist_backend="gloo", dist_rank=rank, dist_world_size=world)
    glob = R._global_batches(6)
    shards = [R._shard(glob[0], 0, world)] * 6 if rank == 0 else [R._shard(glob[i % 2], 1, world) for i in range(6)]
    rep = Reporter()
    runner = None
    if args.capture:
        from espnet_amd.train.graph import CapturedTrainStep
        runner = CapturedTrainStep(m, opt, sched, grad_clip=5.0, dp=dp, warmup=1, pseudo_capture=True)
        if args.warmup_main:
            runner._side = torch.cuda.current_stream()
    for ep in (1, 2):
        rep.set_epoch(ep)
        items = [(["u"], b) for b in shards[: (5 if (ep == 2 and rank == 0) else 6)]]
        with rep.observe("train") as sub:
            Trainer.train_one_epoch(m, iter(items), [opt], [sched], reporter=sub, options=R._opts(),
                                    distributed_option=dopt, dp=dp, step_runner=runner)
    torch.cuda.synchronize()
    flat = {}
    for i, (w, lg, g) in enumerate(recs):
        flat[f"w{i}"], flat[f"l{i}"], flat[f"g{i}"] = w, lg, g
    flat["w"] = m.arena.data.cpu().numpy()
    np.savez(f"{out}_r{rank}.npz", **flat)
    if rank == 0:
        import json
        json.dump([(nm, m.arena.offsets[nm], m.arena._params[nm].numel()) for nm in m.arena.names],
                  open(f"{out}_spans.json", "w"))
    dist.barrier()
    dist.destroy_process_group()


def _where(a, b, spans):
    out = []
    for nm, o, k in spans:
        x, y = a[o:o + k], b[o:o + k]
        ne = ~((x == y) | (np.isnan(x) & np.isnan(y)))
        if ne.any():
            out.append(f"{nm}({int(ne.sum())}/{k}, {float(np.nanmax(np.abs(x - y))):.2g})")
    return out


def fresh(args):
    import json
    import numpy as np
    import test_dp_capture_gpu as C  # noqa: F401 (paths)
    base = tempfile.mkdtemp(prefix="ea_fresh_")
    refs = {}
    bad = 0
    for run in range(args.runs):
        out = os.path.join(base, f"run{run}")
        mp.start_processes(fresh_worker, args=(2, tempfile.mktemp(prefix="ea_dpf_"), args, out), nprocs=2,
                           start_method="spawn")
        recs = {r: dict(np.load(f"{out}_r{r}.npz")) for r in (0, 1)}
        spans = json.load(open(f"{out}_spans.json"))
        if run == 0:
            refs = recs
            for r in (0, 1):
                nans = [s for s in range(99) if f"l{s}" in recs[r] and (np.isnan(recs[r][f"g{s}"]).any()
                                                                       or np.isnan(recs[r][f"w{s}"]).any())]
                if nans:
                    print(f"run 0 rank {r}: NaN reduced gradients at steps {nans}: "
                          + "; ".join(_where(recs[r][f"g{nans[0]}"], np.zeros_like(recs[r]["w"]), spans)[:12]))
            continue
        msgs = []
        for r in (0, 1):
            a, b = recs[r], refs[r]
            s = 0
            while f"g{s}" in a:
                if not np.array_equal(a[f"w{s}"], b[f"w{s}"]):
                    msgs.append(f"rank {r} step {s}: weights at step start differ")
                    break
                if not np.array_equal(a[f"l{s}"], b[f"l{s}"], equal_nan=True):
                    msgs.append(f"rank {r} step {s}: LOCAL grads differ in " + "; ".join(_where(a[f"l{s}"], b[f"l{s}"], spans)[:12]))
                    break
                if not np.array_equal(a[f"g{s}"], b[f"g{s}"]):
                    msgs.append(f"rank {r} step {s}: reduced grads differ (local equal) in "
                                + "; ".join(_where(a[f"g{s}"], b[f"g{s}"], spans)[:6]))
                    break
                s += 1
        if msgs:
            bad += 1
            print(f"run {run}: " + " | ".join(msgs), flush=True)
        else:
            print(f"run {run}: equal", flush=True)
    print(f"fresh: {bad} of {args.runs - 1} runs differ from run 0 ({vars(args)})", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=24)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--side", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--snap", action="store_true")
    ap.add_argument("--fresh", action="store_true")
    ap.add_argument("--capture", action="store_true", help="--fresh: the test's pseudo-capture runner")
    ap.add_argument("--warmup-main", action="store_true", help="--capture: warm-up steps on the main stream")
    ap.add_argument("--no-aux", action="store_true")
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--guard", action="store_true", help="guarded allocator (csrc/debug_alloc.hip): NaN past every "
                    "buffer's end")
    args = ap.parse_args()
    if args.fresh:
        return fresh(args)
    init = tempfile.mktemp(prefix="ea_dpdiag_")
    mp.start_processes(worker, args=(2, init, args), nprocs=2, start_method="spawn")


if __name__ == "__main__":
    main()
