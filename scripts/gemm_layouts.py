"""Operand-layout cost of the bf16 GEMM kernels: event-timed C = A.B at 4096^3 and at the
weight-gradient shape (dW[N_out, K_in] = dY^T X over 7,968 tokens: both operands MN-major) for
the four (a_kmajor, b_kmajor) layouts, plus the grouped weight-gradient launch on the C3 step's
problem list (one encoder layer's Linears x 12).

    python scripts/gemm_layouts.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(f, iters=20):
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


def layouts(M, N, K, tile=(256, 256)):
    lib.ea_gemm_set_tile(*tile)
    out = []
    for ak, bk in ((1, 1), (1, 0), (0, 1), (0, 0)):
        A = torch.randn((M, K) if ak else (K, M), device=dev).to(torch.bfloat16)
        B = torch.randn((N, K) if bk else (K, N), device=dev).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev)
        us = timeit(lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0),
                                     ldb=B.stride(0), ldc=N, splitk=False))
        out.append(f"ak{ak}bk{bk}={us:7.1f}us/{2.0 * M * N * K / us * 1e-6:6.0f}TF")
    lib.ea_gemm_set_tile(0, 0)
    print(f"{M}x{N}x{K} tile {tile}: " + "  ".join(out), flush=True)


def grouped():
    T = 7968
    shapes = [(2048, 512), (512, 2048), (2048, 512), (512, 2048), (1536, 512), (512, 512), (1024, 512), (512, 512)]
    probs = []
    for l in range(12):
        for (n, k) in shapes:
            dy = torch.randn(T, n, device=dev).to(torch.bfloat16)
            x = torch.randn(T, k, device=dev).to(torch.bfloat16)
            dw = torch.zeros(n, k, device=dev)
            probs.append((dy, x, dw))
    flops = sum(2.0 * T * dy.shape[1] * x.shape[1] for dy, x, _ in probs)

    def run():
        with ops.deferred_wgrad():
            for dy, x, dw in probs:
                ops.linear_dw(dy, x, dw, accumulate=True)
    us = timeit(run, 5)
    print(f"grouped wgrad ({len(probs)} problems, {flops * 1e-12:.2f} TFLOP): {us:8.1f}us  "
          f"{flops / us * 1e-6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    layouts(4096, 4096, 4096)
    layouts(512, 2048, 7968)
    layouts(2048, 512, 7968)
    grouped()
