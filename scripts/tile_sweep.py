"""Forced-tile sweep over the C3 step's fwd / input-gradient GEMM shapes (bf16, with their
epilogues): each tile config timed in interleaved rounds in one process, plus the chooser's
own pick ("auto").  Prints us per launch per config and the winner.

    python scripts/tile_sweep.py [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import GEMM_PIPE, ACT_RELU, ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, lib  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
# M, N, K, a_k, b_k, epi, out dtype, calls per C3 step
SHAPES = [
    (7968, 2048, 512, 1, 0, "dact", torch.bfloat16, 24),
    (7968, 2048, 512, 1, 1, "act", torch.bfloat16, 24),
    (7968, 512, 2048, 1, 1, "resid", torch.float32, 24),
    (7968, 512, 2048, 1, 0, None, torch.bfloat16, 24),
    (7968, 512, 512, 1, 1, "resid", torch.float32, 24),
    (7968, 512, 512, 1, 0, None, torch.bfloat16, 24),
    (7968, 512, 1536, 1, 0, None, torch.bfloat16, 12),
    (7968, 1536, 512, 1, 1, None, torch.bfloat16, 12),
    (7968, 512, 1024, 1, 0, None, torch.bfloat16, 12),
    (7968, 1024, 512, 1, 1, None, torch.bfloat16, 12),
    (1312, 512, 512, 1, 0, None, torch.bfloat16, 18),
    (1312, 2048, 512, 1, 0, "dact", torch.bfloat16, 6),
    (1312, 512, 2048, 1, 0, None, torch.bfloat16, 6),
    (7968, 9728, 512, 1, 0, "dactrelu", torch.bfloat16, 1),
    (7968, 512, 9728, 1, 1, "resid", torch.float32, 1),
    (1312, 512, 512, 1, 1, "resid", torch.float32, 12),
    (1312, 2048, 512, 1, 1, "act", torch.bfloat16, 6),
    (1312, 512, 2048, 1, 1, "resid", torch.float32, 6),
    (497, 512, 512, 1, 1, None, torch.bfloat16, 12),
]
# (bm, bn, ea_gemm_set_pipe bits): 1 = 256x256 on gemm_pipe, 3 = 128x128 on gemm_pipe too
TILES = [(64, 128, 1), (128, 128, 1), (128, 128, 3), (256, 256, 1), (0, 0, 1), (0, 0, 3)]


def setup(M, N, K, a_k, b_k, epi, cdt):
    A = torch.randn((M, K) if a_k else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if b_k else (K, N), device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=cdt)
    keep = [A, B, C]
    e = None
    if epi == "act":
        keep += [torch.empty(M, N, device="cuda", dtype=torch.bfloat16), torch.randn(N, device="cuda")]
        e = ops.make_epi(EPI_ACT, bias=keep[-1], act=ACT_SWISH, aux=keep[-2], drop_p=0.1, seed=7)
    elif epi in ("dact", "dactrelu"):
        keep.append(torch.randn(M, N, device="cuda").to(torch.bfloat16))
        e = ops.make_epi(EPI_DACT, act=ACT_SWISH if epi == "dact" else ACT_RELU, aux=keep[-1],
                         drop_p=0.1 if epi == "dact" else 0.0, seed=7)
    elif epi == "resid":
        keep += [torch.randn(N, device="cuda"), torch.randn(M, N, device="cuda")]
        e = ops.make_epi(EPI_RESID, bias=keep[-2], resid=keep[-1], rscale=0.5, drop_p=0.1, seed=7)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0),  # noqa: E731
                         ldb=B.stride(0), ldc=N, epi=e)
    f.keep = keep
    return f


def timed(f, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


tot = {t: 0.0 for t in TILES}
best_tot = 0.0
for M, N, K, a_k, b_k, epi, cdt, calls in SHAPES:
    f = setup(M, N, K, a_k, b_k, epi, cdt)
    res = {t: [] for t in TILES}
    for r in range(ROUNDS):
        for t in TILES:
            bm, bn, pipe = t
            if bm == 64 and not a_k:
                continue
            lib.ea_gemm_set_tile(bm, bn)
            lib.ea_gemm_set_pipe(pipe)
            f()
            res[t].append(timed(f))
    lib.ea_gemm_set_tile(0, 0)
    lib.ea_gemm_set_pipe(GEMM_PIPE)
    med = {t: sorted(v)[len(v) // 2] for t, v in res.items() if v}
    best = min(med, key=med.get)
    for t in med:
        tot[t] += med[t] * calls
    best_tot += med[best] * calls
    line = f"{M:6d} {N:5d} {K:5d} ({a_k},{b_k}) {str(epi):8s} x{calls:2d}:"
    for t in TILES:
        if t in med:
            name = ("auto" if t[0] == 0 else f"{t[0]}x{t[1]}") + ("P" if t[2] == 3 else "")
            line += f"  {name} {med[t]:7.1f}"
    print(line + f"   best {best}", flush=True)
print("per-step totals (ms):", {(("auto" if t[0] == 0 else f"{t[0]}x{t[1]}") + ("P" if t[2] == 3 else "")): round(v / 1e3, 3)
                                for t, v in tot.items()}, "best-of:", round(best_tot / 1e3, 3))
