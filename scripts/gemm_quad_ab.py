"""Event timing: 256x256 tiles on gemm_pipe (8 waves of 128x64) vs gemm_quad (4 waves of
128x128, ea_gemm_set_quad) for the step's K-major 256-tile GEMMs and a square reference."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import _lib as L  # noqa: E402
from espnet_amd import hip_ops as ops  # noqa: E402

SHAPES = [(4096, 4096, 4096, "store", 1), (7968, 2048, 512, "act_drop", 1), (7968, 1536, 512, "bias", 1),
          (7968, 2048, 512, "store", 1), (151392, 512, 4608, "store", 1), (7968, 6144, 512, "bias", 1),
          (7968, 2048, 512, "store", 0), (4096, 4096, 4096, "store", 0)]


def run(M, N, K, kind, bk, reps=20):
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = torch.randn(N, K, device="cuda").bfloat16() if bk else torch.randn(K, N, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda").bfloat16()
    if kind == "act_drop":
        aux = torch.empty(M, N, device="cuda").bfloat16()
        epi = ops.make_epi(L.EPI_ACT, bias=b, act=L.ACT_SWISH, aux=aux, drop_p=0.1, seed=3)
    elif kind == "bias":
        epi = ops.make_epi(bias=b)
    else:
        epi = ops.make_epi()
    f = lambda: ops.gemm(A, W, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=bk, lda=K, ldb=K if bk else N, ldc=N,  # noqa: E731
                         epi=epi)
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    return us, 2.0 * M * N * K / us * 1e-6


L.lib.ea_gemm_set_tile(256, 256)
for M, N, K, kind, bk in SHAPES:
    out = []
    for name, q, s in (("pipe", 0, 5), ("quad5", 3, 5), ("quad4", 3, 4)):
        L.lib.ea_gemm_set_quad(q, s)
        us, tf = run(M, N, K, kind, bk)
        out.append(f"{name} {us:7.1f} us {tf:6.0f} TF/s")
    L.lib.ea_gemm_set_quad(0, 5)
    print(f"{M}x{N}x{K} {kind:8s} bk={bk}: " + " | ".join(out), flush=True)
L.lib.ea_gemm_set_tile(0, 0)
