"""Tile A/B on the C3 step's small-M GEMMs (decoder M = 32 x 41 = 1312 tokens, positional rows
M = 497) with their step epilogues and the step's split-K rule: forced 32x128 / 64x128 tiles
vs the automatic choice, HIP-event timed (50 launches after warm-up), hipBLASLt (no epilogue)
beside.

    python scripts/gemm_dec.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import EPI_ACT, EPI_RESID, ACT_SWISH, lib  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [  # (M, N, K, b_kmajor, epilogue, out dtype)
    (1312, 512, 512, 1, "resid", torch.float32),
    (1312, 512, 512, 0, "store", torch.bfloat16),
    (1312, 512, 2048, 1, "resid", torch.float32),
    (1312, 512, 2048, 0, "store", torch.bfloat16),
    (1312, 2048, 512, 1, "act", torch.bfloat16),
    (1312, 1536, 512, 1, "store", torch.bfloat16),
    (1312, 512, 1536, 0, "store", torch.bfloat16),
    (497, 512, 512, 1, "store", torch.bfloat16),
    (7968, 512, 512, 1, "resid", torch.float32),
]


def timed(f, iters=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    for M, N, K, bk, kind, odt in SHAPES:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        B = (torch.randn((N, K) if bk else (K, N), device=dev) * 0.05).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=odt)
        bias = torch.randn(N, device=dev)
        resid = torch.randn(M, N, device=dev)
        aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        epi = (ops.make_epi(EPI_RESID, bias=bias, resid=resid, drop_p=0.1, seed=3) if kind == "resid" else
               ops.make_epi(EPI_ACT, bias=bias, act=ACT_SWISH, aux=aux, drop_p=0.1, seed=3) if kind == "act" else
               ops.make_epi())
        out = []
        for label, tile in (("auto", (0, 0)), ("32x128", (32, 128)), ("64x128", (64, 128))):
            lib.ea_gemm_set_tile(*tile)
            us = timed(lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=bk, lda=K,
                                        ldb=B.stride(0), ldc=N, epi=epi))
            out.append(f"{label}={us:6.1f}us")
        lib.ea_gemm_set_tile(0, 0)
        b = B.t() if bk else B
        us = timed(lambda: torch.matmul(A, b))
        out.append(f"hipblaslt={us:6.1f}us")
        print(f"{M}x{N}x{K} bk={bk} {kind:5s} " + "  ".join(out), flush=True)


if __name__ == "__main__":
    main()
