"""Split-K on/off for the small (decoder / rel-pos / dW) GEMM shapes of a C3 step."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops

SHAPES = [  # name, M, N, K, a_k, b_k, out dtype
    ("dec dX 1312x512x512", 1312, 512, 512, 1, 0, torch.bfloat16),
    ("dec dW 512x512x1312", 512, 512, 1312, 0, 0, torch.float32),
    ("dec dW 2048x512x1312", 2048, 512, 1312, 0, 0, torch.float32),
    ("dec fwd 1312x512x2048", 1312, 512, 2048, 1, 1, torch.float32),
    ("dec dX 1312x512x2048", 1312, 512, 2048, 1, 0, torch.bfloat16),
    ("dec fwd 1312x2048x512", 1312, 2048, 512, 1, 1, torch.bfloat16),
    ("relpos dW 512x512x497", 512, 512, 497, 0, 0, torch.float32),
    ("enc dW 512x512x7968", 512, 512, 7968, 0, 0, torch.float32),
    ("enc dW 2048x512x7968", 2048, 512, 7968, 0, 0, torch.float32),
    ("enc dW 1536x512x7968", 1536, 512, 7968, 0, 0, torch.float32),
]


def bench(M, N, K, a_k, b_k, cdt, splitk, iters=20):
    A = torch.randn((M, K) if a_k else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if b_k else (K, N), device="cuda").to(torch.bfloat16)
    C = torch.zeros(M, N, device="cuda", dtype=cdt)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0),
                         ldc=N, splitk=splitk)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for name, M, N, K, ak, bk, cdt in SHAPES:
    on = bench(M, N, K, ak, bk, cdt, True)
    off = bench(M, N, K, ak, bk, cdt, False)
    print(f"{name:26s} splitK {on:7.1f} us   none {off:7.1f} us", flush=True)
