"""Epilogue cost on the 256x256 pipe kernel: the same GEMM with STORE (bf16 / f32 out) and DACT
(aux read + bf16 out) epilogues, several K (fixed M x N), random operands."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import ACT_RELU, EPI_DACT, lib  # noqa: E402

lib.ea_gemm_set_tile(256, 256)
M, N = 160000, 512
for K in (512, 1024, 2048):
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    B = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Cf = torch.empty(M, N, device="cuda", dtype=torch.float32)
    cases = {
        "store bf16": (Cb, None),
        "store f32": (Cf, None),
        "dact bf16": (Cb, ops.make_epi(EPI_DACT, act=ACT_RELU, aux=aux)),
    }
    res = {}
    for r in range(3):
        for name, (C, e) in cases.items():
            f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=0, lda=K, ldb=N, ldc=N, epi=e,  # noqa
                                 splitk=False)
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(e0.elapsed_time(e1) / 10 * 1e3)
    line = f"M={M} N={N} K={K:5d} (1,0):"
    for name, v in res.items():
        v = sorted(v)
        line += f"  {name} {v[1]:7.1f} us ({2 * M * N * K / v[1] / 1e6:6.0f} TF/s)"
    print(line, flush=True)
lib.ea_gemm_set_tile(0, 0)
