"""Fixed-cost probe: small K, output dtype f32 vs bf16, several grid sizes."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib


def t(M, N, K, cdt, iters=50):
    A = torch.randn((M, K), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K), device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=cdt)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=K, ldb=K, ldc=N, splitk=False)
    for _ in range(3): f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(iters): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3

lib.ea_gemm_set_pipeline(12)
for M, N in [(1024, 1024), (2048, 2048), (4096, 4096), (8192, 4096)]:
    for K in (64, 128, 256):
        a = t(M, N, K, torch.float32); b = t(M, N, K, torch.bfloat16)
        print(f"M={M} N={N} K={K}: f32out {a:7.1f}us ({M*N*4/a/1e3:6.0f} GB/s)  bf16out {b:7.1f}us ({M*N*2/b/1e3:6.0f} GB/s)", flush=True)
x = torch.empty(4096 * 4096, device="cuda"); y = torch.empty_like(x)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); e0.record()
for _ in range(50): y.copy_(x)
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 50 * 1e3
print(f"torch copy 64MB: {us:.1f}us  {2*x.numel()*4/us/1e3:.0f} GB/s")
