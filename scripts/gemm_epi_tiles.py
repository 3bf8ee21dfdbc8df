"""Forced-tile timing of the C3 GEMMs WITH their real epilogues (ACT/DACT/RESID, dropout),
as the model issues them — to see how the epilogue changes the best tile."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, EPI_STORE, lib  # noqa: E402

TILES = [(0, 0), (64, 128), (128, 128), (256, 128), (256, 256)]
bf, f32 = torch.bfloat16, torch.float32


def case(name, M, N, K, ak, bk, cdt, epi):
    A = torch.randn((M, K) if ak else (K, M), device="cuda").to(bf)
    B = torch.randn((N, K) if bk else (K, N), device="cuda").to(bf)
    C = torch.randn(M, N, device="cuda").to(cdt)
    e = ops.make_epi()
    if epi == "act":
        e = ops.make_epi(EPI_ACT, bias=torch.randn(N, device="cuda"), act=ACT_SWISH,
                         aux=torch.empty(M, N, device="cuda", dtype=bf), drop_p=0.1, seed=7)
    elif epi == "dact":
        e = ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=torch.randn(M, N, device="cuda").to(bf), drop_p=0.1, seed=7)
    elif epi == "resid":
        e = ops.make_epi(EPI_RESID, bias=torch.randn(N, device="cuda"), resid=torch.randn(M, N, device="cuda"),
                         rscale=0.5, drop_p=0.1, seed=7)
    elif epi == "bias":
        e = ops.make_epi(EPI_STORE, bias=torch.randn(N, device="cuda"))
    elif epi == "acc":
        e = ops.make_epi(EPI_STORE, beta=1.0)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0), ldb=B.stride(0),  # noqa
                         ldc=N, epi=e)
    iters = 5 if M * N > 1e8 else 40
    res = []
    for bm, bn in TILES:
        if bm == 64 and not ak:
            res.append(float("nan"))
            continue
        lib.ea_gemm_set_tile(bm, bn)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters * 1e3)
    lib.ea_gemm_set_tile(0, 0)
    best = min(r for r in res[1:] if r == r)
    print(f"{name:22s}", " ".join(f"{v:8.1f}" for v in res), f"  best {2 * M * N * K / best / 1e6:6.0f} TF/s",
          flush=True)


print(f"{'shape':22s}", " ".join(f"{'auto' if bm == 0 else f'{bm}x{bn}':>8s}" for bm, bn in TILES))
for stages in (2, 3):
    lib.ea_gemm_set_pipeline(stages)
    print("stages", stages)
    case("ffn_w1 fwd ACT", 7968, 2048, 512, 1, 1, bf, "act")
    case("ffn_w1 fwd plain", 7968, 2048, 512, 1, 1, bf, "none")
    case("ffn_w2 dX DACT", 7968, 2048, 512, 1, 0, bf, "dact")
    case("ffn_w2 dX plain", 7968, 2048, 512, 1, 0, bf, "none")
    case("ffn_w2 fwd RESID", 7968, 512, 2048, 1, 1, f32, "resid")
    case("ffn_w1 dX", 7968, 512, 2048, 1, 0, bf, "none")
    case("ffn dW acc", 2048, 512, 7968, 0, 0, f32, "acc")
    case("proj fwd RESID", 7968, 512, 512, 1, 1, f32, "resid")
    case("qkv fwd bias", 7968, 1536, 512, 1, 1, bf, "bias")
    case("conv2 dcol", 151392, 4608, 512, 1, 0, bf, "none")
    case("conv2 fwd ACT", 151392, 512, 4608, 1, 1, bf, "act")
