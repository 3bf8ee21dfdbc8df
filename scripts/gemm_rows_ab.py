"""Event timing of the training decoder's GEMM shapes (M = 1,312) on the tile kernels vs the
K-split 32 x 32 blocks (ea_gemm_set_rows32) vs hipBLASLt (plain products)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import _lib as L  # noqa: E402
from espnet_amd import hip_ops as ops  # noqa: E402

SHAPES = [(1312, 512, 512, "resid"), (1312, 1536, 512, "bias"), (1312, 2048, 512, "act"), (1312, 512, 2048, "resid"),
          (1312, 5000, 512, "bias"), (1312, 512, 512, "plain"), (1312, 512, 2048, "plain")]


def run(M, N, K, kind, reps=50):
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = torch.randn(N, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda")
    if kind == "resid":
        C = torch.randn(M, N, device="cuda")
        epi = ops.make_epi(L.EPI_RESID, bias=b, resid=C)
    elif kind == "act":
        C = torch.empty(M, N, device="cuda").bfloat16()
        aux = torch.empty(M, N, device="cuda").bfloat16()
        epi = ops.make_epi(L.EPI_ACT, bias=b, act=L.ACT_RELU, aux=aux)
    elif kind == "bias":
        C = torch.empty(M, N, device="cuda").bfloat16()
        epi = ops.make_epi(bias=b)
    else:
        C = torch.empty(M, N, device="cuda").bfloat16()
        epi = ops.make_epi()
    f = lambda: ops.gemm(A, W, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=K, ldb=K, ldc=N, epi=epi)  # noqa: E731
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for M, N, K, kind in SHAPES:
    out = []
    for name, rows, blt in (("tile", 0, 0), ("rows32", 4096, 0), ("blaslt", 0, 1)):
        L.lib.ea_gemm_set_rows32(rows)
        L.lib.ea_gemm_set_blaslt(3 if blt else 0)
        out.append(f"{name} {run(M, N, K, kind):6.1f}")
    L.lib.ea_gemm_set_rows32(0)
    L.lib.ea_gemm_set_blaslt(1)
    print(f"{M}x{N}x{K} {kind:6s}: " + "  ".join(out) + " us", flush=True)
