"""Epilogue cost split: FFN-shape GEMMs with and without the dropout mask in the epilogue."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, lib

lib.ea_set_rng_salt(None)


def bench(M, N, K, a_k, b_k, kind, p, cdt, iters=30):
    A = torch.randn((M, K) if a_k else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if b_k else (K, N), device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=cdt)
    bias = torch.randn(N, device="cuda")
    if kind == "act":
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        e = ops.make_epi(EPI_ACT, bias=bias, act=ACT_SWISH, aux=aux, drop_p=p, seed=7)
    elif kind == "dact":
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        e = ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=aux, drop_p=p, seed=7)
    elif kind == "resid":
        resid = torch.randn(M, N, device="cuda")
        e = ops.make_epi(EPI_RESID, bias=bias, resid=resid, rscale=0.5, drop_p=p, seed=7)
    else:
        e = ops.make_epi(drop_p=p, seed=7)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0),
                         ldc=N, epi=e)
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


for name, M, N, K, ak, bk, kind, cdt in [("ffn w1 ACT", 7968, 2048, 512, 1, 1, "act", torch.bfloat16),
                                         ("ffn w2 dX DACT", 7968, 2048, 512, 1, 0, "dact", torch.bfloat16),
                                         ("ffn w2 RESID", 7968, 512, 2048, 1, 1, "resid", torch.float32),
                                         ("plain bf16", 7968, 2048, 512, 1, 1, "store", torch.bfloat16),
                                         ("plain bf16 bk0", 7968, 2048, 512, 1, 0, "store", torch.bfloat16)]:
    t1 = bench(M, N, K, ak, bk, kind, 0.1, cdt)
    t0 = bench(M, N, K, ak, bk, kind, 0.0, cdt)
    print(f"{name:16s} drop 0.1: {t1:6.1f} us   no drop: {t0:6.1f} us", flush=True)
