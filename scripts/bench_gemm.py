"""Microbench of ea_gemm on the C3 (Conformer-L) shapes; prints TFLOP/s per shape."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops

def bench(name, dtype, M, N, K, a_k, b_k, iters=20):
    A = torch.randn((M, K) if a_k else (K, M), device="cuda").to(dtype)
    B = torch.randn((N, K) if b_k else (K, N), device="cuda").to(dtype)
    C = torch.empty(M, N, device="cuda")
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0), ldc=N)
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(f"{name:28s} {str(dtype):15s} M={M:6d} N={N:5d} K={K:5d} ak={a_k} bk={b_k}: {ms*1e3:8.1f} us  {2*M*N*K/ms/1e9:7.1f} TF/s", flush=True)

from espnet_amd._lib import lib
import sys as _s
pipes = [int(x) for x in (_s.argv[1].split(",") if len(_s.argv) > 1 else ["2"])]
for pipe in pipes:
  lib.ea_gemm_set_pipeline(pipe)
  print("pipeline", pipe)
  for dt in (torch.bfloat16,):
    bench("ffn_w1 fwd", dt, 7968, 2048, 512, 1, 1)
    bench("ffn_w2 fwd", dt, 7968, 512, 2048, 1, 1)
    bench("qkv fwd", dt, 7968, 1536, 512, 1, 1)
    bench("ffn_w1 dX", dt, 7968, 512, 2048, 1, 0)
    bench("ffn_w1 dW", dt, 2048, 512, 7968, 0, 0)
    bench("ctc_lo fwd", dt, 7968, 5000, 512, 1, 1)
    bench("conv2 fwd", dt, 151392, 512, 4608, 1, 1, iters=5)
    bench("conv2 dcol", dt, 151392, 4608, 512, 1, 0, iters=5)
    bench("conv2 dW", dt, 512, 4608, 151392, 0, 0, iters=5)
    bench("square 4096", dt, 4096, 4096, 4096, 1, 1, iters=5)
    bench("square 8192", dt, 8192, 8192, 8192, 1, 1, iters=3)
