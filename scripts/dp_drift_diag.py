"""Locate the two-process DP drift (tests/test_dp_ragged_gpu.py): two gloo ranks on one GPU
run the ragged test's eager DP steps R times each, in the same two processes, every run from
the same weights; every run is compared with run 0 per step: the local loss, the bucket
contents handed to each all-reduce (a stream-ordered copy at the issue point, --snap) and the
reduced gradient arena.  The first step and tensor that differ name the segment.

    dp_drift_diag.py [--runs R] [--steps S] [--no-overlap] [--snap] [--fresh]

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
    # the step's inputs (as the forward receives them), encoder output and local loss: stream-
    # ordered device copies, read back at the next compute_grad_norm
    fwd_rec, fwd_pending = [], []
    real_fwd = m.forward

    # every encoder block's output (subsampling, conformer layers), the bf16 weight shadow and
    # the dropout salt as the forward starts
    from espnet_amd.layers import conformer as lconf, subsampling as lsub
    blk = []
    for cls in (lsub.SubsampleFn, lconf.ConformerBlockFn):
        f0 = cls.forward

        def wrapped(ctx, *a, _f0=f0, _n=cls.__name__):
            out = _f0(ctx, *a)
            if _n == "SubsampleFn" and getattr(ctx, "implicit", False) and dup:
                s0, s2, pre, post, _ = dup.pop()
                x1 = ctx.save[1].view(-1)[:s0.numel()]
                md = lambda a_, b_: (a_.float() - b_.float()).abs().max().view(1)  # noqa: E731
                for nm_, u, v in (("01", s0, x1), ("12", x1, s2)):
                    u16, v16 = u.view(torch.int16), v.view(torch.int16)
                    idx = torch.nonzero(u16 != v16).view(-1)
                    if idx.numel():
                        dumps.append((len(fwd_rec) + len(fwd_pending), nm_, idx.cpu().numpy(), u16[idx].cpu().numpy(),
                                      v16[idx].cpu().numpy(), v.data_ptr() if nm_ == "12" else u.data_ptr()))
                blk.append(("sub_dupdiff", torch.cat([md(s0, x1), md(x1, s2), md(s0, s2),
                                                      md(pre[0], post[0]), md(pre[1], post[1]), md(pre[2], post[2]),
                                                      md(pre[0], ctx.save[0])])))
                dup.clear()
            if _n == "SubsampleFn" and getattr(ctx, "implicit", False):
                for nm, t in zip(("feats", "x1p", "w2", "x2", "wl", "pos1"), ctx.save):
                    if t is not None:
                        blk.append((f"sub_{nm}", t.detach().clone()))
            blk.append((_n, out.detach().clone()))
            return out
        cls.forward = staticmethod(wrapped)

    # conv1 run twice: into x1p, then into a scratch copy right behind it on the same stream; the
    # subsampling wrapper compares the two (different -> conv1's inputs changed while it ran, or
    # something wrote into x1p after conv1)
    from espnet_amd._lib import lib as _lib
    real_c1 = _lib.ea_conv1_fwd2
    dup = []

    ctx_holder = {}
    dumps = []

    def c1(B, T, F, C, x, w, bias, y, dt, pos, st):
        T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
        n = B * T1 * F1 * C
        s0 = torch.empty(n, dtype=torch.bfloat16, device="cuda:0")
        s2 = torch.empty(n, dtype=torch.bfloat16, device="cuda:0")
        # stream-ordered copies of the inputs just before / after (via the known views)
        feats, wv, bv = ctx_holder["x"], ctx_holder["w"], ctx_holder["b"]
        assert feats.data_ptr() == x and wv.data_ptr() == w and bv.data_ptr() == bias
        pre = (feats.clone(), wv.clone(), bv.clone())
        real_c1(B, T, F, C, x, w, bias, s0.data_ptr(), dt, 0, st)
        real_c1(B, T, F, C, x, w, bias, y, dt, pos, st)
        real_c1(B, T, F, C, x, w, bias, s2.data_ptr(), dt, 0, st)
        post = (feats.clone(), wv.clone(), bv.clone())
        dup.append((s0, s2, pre, post, y))

    _lib.ea_conv1_fwd2 = c1
    real_fi = lsub.SubsampleFn._forward_implicit

    def fi(ctx, feats, mm, seed, training, *a):
        ctx_holder.update(x=feats, w=mm._b.f("conv.0.weight"), b=mm._b.f("conv.0.bias"))
        return real_fi(ctx, feats, mm, seed, training, *a)

    lsub.SubsampleFn._forward_implicit = staticmethod(fi)

    _lib.ea_conv1_fwd2 = c1

    def fwd(**kw):
        ins = {k: kw[k].detach().clone() for k in ("speech", "speech_lengths", "text", "text_lengths")}
        ins["shadow"] = m.arena.shadow.detach().clone()
        ins["salt"] = m._rng_salt.detach().clone()
        blk.clear()
        loss, stats, weight = real_fwd(**kw)
        for i, (nm, t) in enumerate(blk):
            ins[f"blk{i}" if not nm.startswith("sub_") else f"s{nm}"] = t
        blk.clear()
        eo = m._last_encoder_out[0].detach().clone()
        fwd_pending.append((ins, eo, loss.detach().clone(), {k: v.detach().clone() for k, v in stats.items()
                                                              if v is not None}))
        return loss, stats, weight

    m.forward = fwd
    real_cg = opt.compute_grad_norm

    def cg2(*a, **k):
        for ins, eo, loss, st in fwd_pending:
            fwd_rec.append(({k: v.cpu().float().numpy() for k, v in ins.items()}, eo.cpu().numpy(), float(loss),
                            {k: float(v) for k, v in st.items()}))
        fwd_pending.clear()
        return real_cg(*a, **k)

    opt.compute_grad_norm = cg2
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
    for i, (ins, eo, loss, st) in enumerate(fwd_rec):
        for k, v in ins.items():
            flat[f"in{i}_{k}"] = v
        flat[f"eo{i}"] = eo
        flat[f"loss{i}"] = np.array([loss] + [st[k] for k in sorted(st)])
    flat["w"] = m.arena.data.cpu().numpy()
    for i, (st_, nm_, idx, a_, b_, ptr) in enumerate(dumps):
        print(f"DUMP rank {rank} step {st_} pair #{nm_[0]}/#{nm_[1]} victim ptr {ptr:#x}: {idx.size} elements; "
              f"flat idx {idx[:24].tolist()}; good {[f'{int(v) & 0xffff:04x}' for v in a_[:24]]}; "
              f"bad {[f'{int(v) & 0xffff:04x}' for v in b_[:24]]}", flush=True)
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
        for r in (0, 1):
            for k in sorted(recs[r]):
                if k.endswith("_ssub_dupdiff") and float(recs[r][k].max()) != 0.0:
                    v = recs[r][k].tolist()
                    print(f"run {run} rank {r} {k.split('_')[0]}: conv1 runs differ: |#0-#1| {v[0]:.3g} |#1-#2| {v[1]:.3g} "
                          f"|#0-#2| {v[2]:.3g}; inputs pre vs post: x {v[3]:.3g} w {v[4]:.3g} b {v[5]:.3g}; "
                          f"pre-x vs saved feats {v[6]:.3g}", flush=True)
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
                bad_in = [k for k in a if k.startswith(f"in{s}_") and "blk" not in k and "_ssub_" not in k
                          and not np.array_equal(a[k], b[k])]
                bad_sub = [k.split("_ssub_")[1] for k in a if k.startswith(f"in{s}_ssub_") and "dupdiff" not in k
                           and not np.array_equal(a[k], b[k])]
                if bad_sub:
                    msgs.append(f"rank {r} step {s}: subsampling tensors differ: {bad_sub}")
                    for k in ("x1p", "x2"):
                        kk = f"in{s}_ssub_{k}"
                        if kk in a and not np.array_equal(a[kk], b[kk]):
                            d = np.abs(a[kk] - b[kk])
                            rows = sorted(set(np.nonzero(d)[0].tolist()))
                            msgs.append(f"{k} {a[kk].shape}: {int((d > 0).sum())} el differ, rows {rows[:16]} "
                                        f"cols [{np.nonzero(d)[1].min()},{np.nonzero(d)[1].max()}] max {d.max():.3g}")
                if bad_in:
                    msgs.append(f"rank {r} step {s}: forward INPUTS differ: {bad_in}")
                    break
                bad_blk = sorted((int(k.split("blk")[1]), k) for k in a if k.startswith(f"in{s}_blk")
                                 and not np.array_equal(a[k], b[k]))
                if bad_blk:
                    k = bad_blk[0][1]
                    d = np.abs(a[k] - b[k])
                    nz = np.nonzero(d)
                    msgs.append(f"rank {r} step {s}: first differing encoder block {k} ({int((d > 0).sum())}/{d.size}, "
                                f"max {d.max():.3g}; index ranges " + ", ".join(f"[{v.min()},{v.max()}]" for v in nz) +
                                f"; shape {a[k].shape}); differing blocks {[x[0] for x in bad_blk]}")
                    break
                if f"eo{s}" in a and not np.array_equal(a[f"eo{s}"], b[f"eo{s}"]):
                    d = np.abs(a[f"eo{s}"] - b[f"eo{s}"])
                    msgs.append(f"rank {r} step {s}: ENCODER OUTPUT differs ({int((d > 0).sum())}/{d.size}, max {d.max():.3g}"
                                f", rows {sorted(set(np.nonzero(d)[0].tolist()))[:8]} frames {sorted(set(np.nonzero(d)[1].tolist()))[:8]})")
                    break
                if f"loss{s}" in a and not np.array_equal(a[f"loss{s}"], b[f"loss{s}"]):
                    msgs.append(f"rank {r} step {s}: LOSS/stats differ {a[f'loss{s}'].tolist()} vs {b[f'loss{s}'].tolist()}")
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
