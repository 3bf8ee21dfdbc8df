"""Time every forced LDS-DMA tile shape on the C3 model's GEMM shapes (tile-chooser calibration)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib

SHAPES = [  # name, M, N, K, a_k, b_k, out dtype
    ("ffn_w1 fwd", 7968, 2048, 512, 1, 1, torch.bfloat16),
    ("ffn_w2 fwd", 7968, 512, 2048, 1, 1, torch.float32),
    ("qkv fwd", 7968, 1536, 512, 1, 1, torch.bfloat16),
    ("pw1 fwd", 7968, 1024, 512, 1, 1, torch.bfloat16),
    ("proj fwd", 7968, 512, 512, 1, 1, torch.float32),
    ("ffn_w2 dX", 7968, 2048, 512, 1, 0, torch.bfloat16),
    ("ffn_w1 dX", 7968, 512, 2048, 1, 0, torch.bfloat16),
    ("qkv dX", 7968, 512, 1536, 1, 0, torch.bfloat16),
    ("ctc_lo fwd", 7968, 5000, 512, 1, 1, torch.float32),
    ("ctc_lo dX", 7968, 512, 5000, 1, 0, torch.bfloat16),
    ("conv2 fwd", 151392, 512, 4608, 1, 1, torch.bfloat16),
    ("conv2 dcol", 151392, 4608, 512, 1, 0, torch.bfloat16),
    ("dec ffn fwd", 1280, 2048, 512, 1, 1, torch.bfloat16),
]
TILES = [(0, 0), (64, 128), (128, 128), (256, 256)]


def t(M, N, K, ak, bk, cdt, iters):
    A = torch.randn((M, K) if ak else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if bk else (K, N), device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=cdt)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0), ldb=B.stride(0),
                         ldc=N, splitk=False)
    res = []
    for bm, bn in TILES:
        lib.ea_gemm_set_tile(bm, bn)
        for _ in range(3): f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(iters): f()
        e1.record(); torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters * 1e3)
    lib.ea_gemm_set_tile(0, 0)
    return res


print("shape".ljust(14), " ".join(f"{'auto' if bm == 0 else f'{bm}x{bn}':>9s}" for bm, bn in TILES))
for name, M, N, K, ak, bk, cdt in SHAPES:
    it = 5 if M > 100000 else 30
    r = t(M, N, K, ak, bk, cdt, it)
    print(name.ljust(14), " ".join(f"{v:9.1f}" for v in r), f"  best TF/s {2 * M * N * K / min(r[1:]) / 1e6:7.0f}", flush=True)
