"""torch.matmul (hipBLASLt) bf16 vs our ea_gemm on the step's N = 512 / short-K GEMM shapes
(plain bf16 output, no epilogue: the main-loop comparison).

    python scripts/blaslt_fwd_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402

dev = "cuda"
# (M, N, K, a_kmajor, b_kmajor): C[M,N] = A B; a_k: A rows M x K; b_k: B stored [N][K]
SHAPES = [(7968, 512, 2048, 1, 1), (7968, 512, 2048, 1, 0), (7968, 512, 512, 1, 1), (7968, 512, 512, 1, 0),
          (7968, 2048, 512, 1, 1), (7968, 2048, 512, 1, 0), (7968, 512, 1536, 1, 0), (1312, 512, 2048, 1, 1),
          (4096, 4096, 4096, 1, 1), (4096, 4096, 4096, 0, 0)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for M, N, K, ak, bk in SHAPES:
    A = torch.randn((M, K) if ak else (K, M), device=dev).to(torch.bfloat16)
    B = torch.randn((N, K) if bk else (K, N), device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    At = A if ak else A.t()
    Bt = B.t() if bk else B

    def ours():
        ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0), ldb=B.stride(0), ldc=N)

    def lt():
        return torch.mm(At, Bt)
    t0, t1 = timeit(ours), timeit(lt)
    f = 2.0 * M * N * K
    print(f"{M:5d}x{N:5d}x{K:5d} ({ak},{bk}): ours {t0:7.1f} us {f / t0 / 1e6:5.0f} TF | hipBLASLt {t1:7.1f} us "
          f"{f / t1 / 1e6:5.0f} TF", flush=True)
