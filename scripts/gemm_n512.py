"""Tile A/B on the C3 step's N = 512 / N = 2048 Linear GEMM shapes (M = 7,968 tokens), with the
epilogues they run in the step (RESID f32 for forward projections, STORE bf16 for input
gradients, ACT Swish + aux for FFN w_1).  Event-timed, 50 launches each, after warm-up.

    python scripts/gemm_n512.py            -> one line per (shape, config): us/call, TF/s
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import EPI_ACT, EPI_RESID, ACT_SWISH, lib  # noqa: E402

M = 7968
dev = torch.device("cuda", 0)
SHAPES = [  # (name, N, K, a_kmajor, b_kmajor, epilogue, out dtype)
    ("fwd_resid N512 K512", 512, 512, 1, 1, "resid", torch.float32),
    ("fwd_resid N512 K2048", 512, 2048, 1, 1, "resid", torch.float32),
    ("dx N512 K512", 512, 512, 1, 0, "store", torch.bfloat16),
    ("dx N512 K1536", 512, 1536, 1, 0, "store", torch.bfloat16),
    ("dx N512 K2048", 512, 2048, 1, 0, "store", torch.bfloat16),
    ("dxT N512 K1536 (W^T shadow)", 512, 1536, 1, 1, "store", torch.bfloat16),
    ("dxT N512 K2048 (W^T shadow)", 512, 2048, 1, 1, "store", torch.bfloat16),
    ("fwd_swish N2048 K512", 2048, 512, 1, 1, "act", torch.bfloat16),
    ("qkv N1536 K512", 1536, 512, 1, 1, "store", torch.bfloat16),
]
CONFIGS = [  # (label, pipe bits, forced tile (bm, bn) or None, 128x128 ring slots)
    ("auto", 1, None, 4),
    ("lds64x128", 1, (64, 128), 4),
    ("lds128", 1, (128, 128), 4),
    ("pipe128", 3, (128, 128), 4),
    ("pipe256", 1, (256, 256), 4),
    ("k128s3", 1, "k128:3", 4),
    ("k128s4", 1, "k128:4", 4),
]


def run(name, N, K, ak, bk, kind, odt, iters=50):
    A = torch.randn((M, K) if ak else (K, M), device=dev).to(torch.bfloat16)
    B = (torch.randn((N, K) if bk else (K, N), device=dev) * 0.05).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=odt)
    bias = torch.randn(N, device=dev)
    resid = torch.randn(M, N, device=dev)
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if kind == "resid":
        epi = ops.make_epi(EPI_RESID, bias=bias, resid=resid, drop_p=0.1, seed=3)
    elif kind == "act":
        epi = ops.make_epi(EPI_ACT, bias=bias, act=ACT_SWISH, aux=aux, drop_p=0.1, seed=3)
    else:
        epi = ops.make_epi()
    out = []
    for label, pipe, tile, slots in CONFIGS:
        lib.ea_gemm_set_pipe(pipe)
        if isinstance(tile, str):  # gemm_k128 with a ring depth (K-major A and B only)
            if not (ak and bk):
                continue
            lib.ea_gemm_set_tile(0, 0)
            lib.ea_gemm_set_k128(3, int(tile.split(":")[1]))
        else:
            lib.ea_gemm_set_k128(0, 4)
            lib.ea_gemm_set_tile(*(tile or (0, 0)))
        f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0),  # noqa: E731
                             ldb=B.stride(0), ldc=N, epi=epi, splitk=False)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / iters * 1e3
        out.append((label, us, 2.0 * M * N * K / us * 1e-6))
    lib.ea_gemm_set_tile(0, 0)
    lib.ea_gemm_set_pipe(1)
    lib.ea_gemm_set_k128(0, 4)
    # hipBLASLt reference (plain bf16 GEMM, no epilogue)
    a = A if ak else A.t()
    b = B.t() if bk else B
    for _ in range(5):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    out.append(("hipblaslt(no epi)", us, 2.0 * M * N * K / us * 1e-6))
    print(f"{name:24s} " + "  ".join(f"{lab}={us:6.1f}us/{tf:5.0f}TF" for lab, us, tf in out), flush=True)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    lib.load() if hasattr(lib, "load") else None
    for s in SHAPES:
        run(*s)
