"""A/B of the 256x256 GEMM kernels: gemm_bf16_lds (2-stage BK=64 ring) vs gemm_pipe (4-slot
ring of 32-deep slices), interleaved rounds in one process, random operands.

    python scripts/gemm_pipe_ab.py [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, lib  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
SHAPES = [  # name, M, N, K, a_k, b_k, epi, out dtype, forced tile (0 = model's choice)
    ("sq4096", 4096, 4096, 4096, 1, 1, None, torch.float32, 256),
    ("conv2-like dense", 151392, 512, 4608, 1, 1, None, torch.bfloat16, 256),
    ("ffn_w1 fwd ACT", 7968, 2048, 512, 1, 1, "act", torch.bfloat16, 256),
    ("ffn_w2 fwd RESID", 7968, 512, 2048, 1, 1, "resid", torch.float32, 256),
    ("ffn_w2 dX DACT", 7968, 2048, 512, 1, 0, "dact", torch.bfloat16, 256),
    ("ffn_w1 dX", 7968, 512, 2048, 1, 0, None, torch.bfloat16, 256),
    ("ffn_w1 dW", 2048, 512, 7968, 0, 0, None, torch.float32, 256),
    ("ffn_w2 dW", 512, 2048, 7968, 0, 0, None, torch.float32, 256),
    ("qkv fwd", 7968, 1536, 512, 1, 1, None, torch.bfloat16, 256),
]


def setup(M, N, K, a_k, b_k, epi, cdt):
    A = torch.randn((M, K) if a_k else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if b_k else (K, N), device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=cdt)
    e = None
    keep = []  # make_epi stores raw pointers: the tensors must outlive the launches
    if epi == "act":
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        keep += [aux, torch.randn(N, device="cuda")]
        e = ops.make_epi(EPI_ACT, bias=keep[-1], act=ACT_SWISH, aux=aux, drop_p=0.1, seed=7)
    elif epi == "dact":
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        keep.append(aux)
        e = ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=aux, drop_p=0.1, seed=7)
    elif epi == "resid":
        keep += [torch.randn(N, device="cuda"), torch.randn(M, N, device="cuda")]
        e = ops.make_epi(EPI_RESID, bias=keep[0], resid=keep[1], rscale=0.5, drop_p=0.1, seed=7)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0),  # noqa: E731
                         ldb=B.stride(0), ldc=N, epi=e)
    f.keep = keep
    return f, C


def timed(f, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for name, M, N, K, a_k, b_k, epi, cdt, tile in SHAPES:
    f, C = setup(M, N, K, a_k, b_k, epi, cdt)
    lib.ea_gemm_set_tile(tile, tile) if tile else lib.ea_gemm_set_tile(0, 0)
    flop = 2.0 * M * N * K
    iters = max(3, min(50, int(2e12 / flop)))
    res = {0: [], 1: []}
    outs = {}
    for r in range(ROUNDS):
        for pipe in (0, 1):
            lib.ea_gemm_set_pipe(pipe)
            f()
            torch.cuda.synchronize()
            if r == 0:
                outs[pipe] = C.float().clone()
            res[pipe].append(timed(f, iters))
    lib.ea_gemm_set_pipe(0)
    diff = (outs[0] - outs[1]).abs().max().item()
    line = f"{name:18s} M={M:6d} N={N:5d} K={K:5d} ak={a_k} bk={b_k}:"
    for pipe in (0, 1):
        v = sorted(res[pipe])
        med = v[len(v) // 2]
        line += f"  {'pipe' if pipe else 'lds '} {med * 1e3:8.1f} us {flop / med / 1e9:7.1f} TF/s (min {v[0]*1e3:7.1f})"
    print(line + f"  maxdiff {diff:.3g}", flush=True)
lib.ea_gemm_set_tile(0, 0)
