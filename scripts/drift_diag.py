"""Locate run-to-run nondeterminism of the training step (the round-5 DP drift).

Single process, the DP tests' tiny Conformer (tests/test_dp_capture_gpu.py:_setup, dropout 0.1,
bf16), the ragged-shard test's 6 global batches; every run starts from the same weights and
records the gradient arena of every step just before the optimizer reads it.  Each run is
compared with run 0: the first step whose gradients differ, and the parameters that differ
there, name the backward segment that produced the difference.

    drift_diag.py [--runs N] [--poison] [--delay-ns NS] [--serial] [--hog MB] [--dp]

--poison    every torch.empty / empty_like / new_empty float buffer starts as NaN (set before the
            package is imported): a kernel that reads an element nobody wrote turns NaN
--delay-ns  hold every side / auxiliary stream segment that long (hip_ops.DEBUG_DELAY_NS)
--serial    the main stream joins every side / auxiliary segment at its end
--hog MB    a second stream copies MB-sized buffers back to back during every step (HBM and
            CU contention, as a second process on the card gives)
--dp        world-1 gloo group, ArenaDataParallel(force_collectives=True, check_issue=True):
            the bucket hooks run and every bucket is checked unchanged between its all-reduce
            issue point and the end of the backward
"""
import argparse
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(HERE, "..", "tests"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "espnet-1_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def poison():
    e, el, ne = torch.empty, torch.empty_like, torch.Tensor.new_empty

    def fill(t):
        if t.is_cuda and t.is_floating_point():
            t.fill_(float("nan"))
        return t

    torch.empty = lambda *a, **k: fill(e(*a, **k))
    torch.empty_like = lambda *a, **k: fill(el(*a, **k))
    torch.Tensor.new_empty = lambda self, *a, **k: fill(ne(self, *a, **k))


def one_run(args, hog, runner=False):
    import test_dp_capture_gpu as C
    import test_dp_ragged_gpu as R
    from espnet_amd.train.trainer import Trainer
    _, m, opt, sched = C._setup(amp=True, dropout=0.1)
    dp = None
    if args.dp:
        from espnet_amd.train.distributed import ArenaDataParallel
        dp = ArenaDataParallel(m, bucket_mb=0.25, force_collectives=True, check_issue=True)
    grads = []
    orig = opt.compute_grad_norm

    def snap(*a, **k):
        grads.append(m.arena.grad.detach().cpu().clone())
        return orig(*a, **k)

    opt.compute_grad_norm = snap
    run = None
    if runner:
        from espnet_amd.train.graph import CapturedTrainStep
        run = CapturedTrainStep(m, opt, sched, grad_clip=5.0, dp=dp, warmup=1, pseudo_capture=True)
    for i, b in enumerate(R._global_batches(args.steps)):
        if hog is not None:
            src, dst, n, st = hog
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                for _ in range(n):
                    dst.copy_(src)
        b = {k: v.to("cuda:0") for k, v in b.items()}
        if run is not None:
            run(b, iiter=i + 1)
        else:
            Trainer.train_one_step(m, b, opt, sched, grad_clip=5.0, dp=dp)
    torch.cuda.synchronize()
    spans = [(n, m.arena.offsets[n], m.arena._params[n].numel()) for n in m.arena.names]
    return grads, m.arena.data.cpu().clone(), spans


def diff(ga, gb, spans):
    out = []
    for n, o, k in spans:
        x, y = ga[o:o + k], gb[o:o + k]
        if not torch.equal(x, y):
            nan = int(torch.isnan(x).sum())
            out.append(f"{n}: {int((x != y).sum())}/{k} differ, max |d| {float((x - y).abs().nan_to_num(9e9).max()):.3g}"
                       + (f", {nan} NaN" if nan else ""))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--delay-ns", type=int, default=0)
    ap.add_argument("--serial", action="store_true")
    ap.add_argument("--hog", type=int, default=0)
    ap.add_argument("--dp", action="store_true")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--modes", default="", help="comma list of serial / delay / runner / runner-delay / "
                    "runner-serial: one run each, compared with the first (overrides --runs)")
    args = ap.parse_args()
    if args.poison:
        poison()
    from espnet_amd import hip_ops
    hip_ops.DEBUG_DELAY_NS = args.delay_ns
    hip_ops.DEBUG_SERIAL = args.serial
    torch.cuda.set_device(0)
    if args.dp:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"file://{tempfile.mktemp(prefix='ea_diag_')}", rank=0,
                                world_size=1)
    hog = None
    if args.hog:
        n = args.hog * 2 ** 20 // 4
        hog = (torch.ones(n, device="cuda:0"), torch.empty(n, device="cuda:0"), 64, torch.cuda.Stream())
    tag = " ".join(f"{k}={v}" for k, v in vars(args).items())
    if args.modes:
        res = []
        for mode in args.modes.split(","):
            hip_ops.DEBUG_DELAY_NS = 300_000 if "delay" in mode else args.delay_ns
            hip_ops.DEBUG_SERIAL = "serial" in mode
            g, w, spans = one_run(args, hog, runner=mode.startswith("runner"))
            res.append((mode, g, w))
        m0, g0, w0 = res[0]
        for mode, g, w in res[1:]:
            first = next((i for i, (a, b) in enumerate(zip(g, g0)) if not torch.equal(a, b)), None)
            if first is None:
                print(f"[{tag}] {mode} == {m0}" + ("" if torch.equal(w, w0) else " (grads; weights differ)"), flush=True)
            else:
                print(f"[{tag}] {mode} != {m0}: first differing step {first}: "
                      + "; ".join(diff(g[first], g0[first], spans)[:12]), flush=True)
        return
    ref_g, ref_w, spans = one_run(args, hog)
    nan_steps = [i for i, g in enumerate(ref_g) if torch.isnan(g).any()]
    if nan_steps:
        print(f"[{tag}] run 0: NaN gradients at steps {nan_steps}: "
              + "; ".join(diff(ref_g[nan_steps[0]], torch.zeros_like(ref_g[0]), spans)[:20]), flush=True)
    bad = 0
    for r in range(1, args.runs):
        g, w, _ = one_run(args, hog)
        first = next((i for i, (a, b) in enumerate(zip(g, ref_g)) if not torch.equal(a, b)), None)
        if first is None and torch.equal(w, ref_w):
            continue
        bad += 1
        if first is None:
            print(f"[{tag}] run {r}: gradients equal, weights differ", flush=True)
        else:
            print(f"[{tag}] run {r}: first differing step {first}: " + "; ".join(diff(g[first], ref_g[first], spans)),
                  flush=True)
    print(f"[{tag}] {bad} of {args.runs - 1} runs differ from run 0", flush=True)


if __name__ == "__main__":
    main()
