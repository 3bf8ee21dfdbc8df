"""Time vs K at fixed M,N to split a GEMM launch into fixed cost + per-K-tile cost."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib


def t(M, N, K, ak, bk, iters=30):
    A = torch.randn((M, K) if ak else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if bk else (K, N), device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0), ldb=B.stride(0), ldc=N, splitk=False)
    for _ in range(3): f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(iters): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for pipe in [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["2"])]:
    lib.ea_gemm_set_pipeline(pipe)
    for (M, N, ak, bk) in [(7968, 512, 1, 1), (7968, 2048, 1, 1), (7968, 512, 1, 0), (4096, 4096, 1, 1)]:
        row = []
        for K in (256, 512, 1024, 2048, 4096):
            us = t(M, N, K, ak, bk)
            row.append(f"K={K}:{us:7.1f}us/{2*M*N*K/us/1e6:6.0f}TF")
        print(f"pipe {pipe} M={M} N={N} ak={ak} bk={bk} | " + "  ".join(row), flush=True)
