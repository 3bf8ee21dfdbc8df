"""How latency-bound is the C3 decoder?  Captured DecoderFn forward + backward (weight
gradients queued and dropped: the end-of-pass grouped GEMM is the same work either way) at
B = 32, at B = 16, and as two B = 16 halves on two streams (the halves' gradient outputs
race: timing only).  usage: dec_split_probe.py [replays [fwd,bwd]]"""
import os
import sys
import types

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "espnet-1_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd.layers.decoder import DecoderFn  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
modes = (False, True) if len(sys.argv) < 3 else tuple(m == "bwd" for m in sys.argv[2].split(","))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cfg = bench.c3_config()
model = bench.build(cfg)
model.prepare(dev, amp=True, seed=1234)
model.train()
dec = model.decoder
B, Tm, d, L, V = 32, 249, 512, 41, cfg["vocab_size"]
g = torch.Generator(device=dev).manual_seed(0)
mem = torch.randn(B, Tm, d, device=dev, generator=g)
hlens = torch.full((B,), Tm, dtype=torch.long, device=dev)
ys = torch.randint(2, V - 1, (B, L), device=dev, generator=g)
ylens = torch.full((B,), L, dtype=torch.long, device=dev)
dlog = torch.randn(B, L, V, device=dev, generator=g) * 1e-3


# queue overlapping outputs without flushing (the halves share gradient buffers; timing only)
ops.REDUCE_Q._claim = lambda out, n: None


def _add(dy, x, dw, **k):
    ops.WGRAD_Q.items.append((k["K"], dy, x, dw, k["M"], k["N"], k["lda"], k["ldb"], k["ldc"], k["beta"], 0, 0))
    return True


ops.WGRAD_Q.add = _add


def run(parts, streams, bwd=True):
    ops.WGRAD_Q.active = ops.REDUCE_Q.active = True
    cur = torch.cuda.current_stream()
    ctxs = []
    for (b0, b1), s in zip(parts, streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            ctx = types.SimpleNamespace()
            DecoderFn.forward(ctx, mem[b0:b1], hlens[b0:b1], ys[b0:b1], ylens[b0:b1], dec, 7, True)
            ctxs.append(ctx)
    if bwd:
        for ctx, (b0, b1), s in zip(ctxs, parts, streams):
            with torch.cuda.stream(s):
                DecoderFn.backward(ctx, dlog[b0:b1])
    for s in streams:
        cur.wait_stream(s)
    ops.WGRAD_Q.items, ops.WGRAD_Q.posts, ops.WGRAD_Q.pending = [], [], 0
    ops.REDUCE_Q.colsums, ops.REDUCE_Q.reduces, ops.REDUCE_Q.spans, ops.REDUCE_Q.pending = [], [], [], 0
    ops.WGRAD_Q.active = ops.REDUCE_Q.active = False


def timed(parts, streams, bwd=True):
    run(parts, streams, bwd)
    torch.cuda.synchronize()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cs):
        run(parts, streams, bwd)
    torch.cuda.synchronize()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


s1, s2, s3, s4 = (torch.cuda.Stream() for _ in range(4))
for bwd in modes:
    tag = "fwd+bwd" if bwd else "fwd"
    print(f"{tag:8s} B=32 one stream      {timed([(0, 32)], [s1], bwd):8.1f} us", flush=True)
    print(f"{tag:8s} B=16 one stream      {timed([(0, 16)], [s1], bwd):8.1f} us", flush=True)
    print(f"{tag:8s} 2 x B=16 two streams {timed([(0, 16), (16, 32)], [s1, s2], bwd):8.1f} us", flush=True)
    print(f"{tag:8s} B=8 one stream       {timed([(0, 8)], [s1], bwd):8.1f} us", flush=True)
    print(f"{tag:8s} 4 x B=8 four streams {timed([(0, 8), (8, 16), (16, 24), (24, 32)], [s1, s2, s3, s4], bwd):8.1f} us",
          flush=True)
