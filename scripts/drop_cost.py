"""Cost of regenerating dropout masks in the backward: the FF DACT epilogue GEMM and the
residual-branch scale_dropout, each with p = 0.1 vs p = 0 (same shapes as the C3 step)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


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


M, N, K = 7968, 2048, 512
A = torch.randn(M, K, device=dev).to(bf)
W = torch.randn(K, N, device=dev).to(bf)   # (1,0): B [K][N]
Wk = torch.randn(N, K, device=dev).to(bf)  # (1,1)
aux = torch.randn(M, N, device=dev).to(bf)
C = torch.empty(M, N, device=dev, dtype=bf)
bias = torch.randn(N, device=dev)
for p in (0.0, 0.1):
    e = ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=aux, drop_p=p, seed=7)
    t = timeit(lambda: ops.gemm(A, W, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=0, lda=K, ldb=N, ldc=N, epi=e))
    e2 = ops.make_epi(EPI_ACT, bias=bias, act=ACT_SWISH, aux=aux, drop_p=p, seed=7)
    t2 = timeit(lambda: ops.gemm(A, Wk, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=K, ldb=K, ldc=N, epi=e2))
    print(f"FF1 fwd ACT p={p}: {t2:6.1f} us   FF2-bwd DACT p={p}: {t:6.1f} us", flush=True)
x = torch.randn(M, 512, device=dev)
y = torch.empty(M, 512, device=dev, dtype=bf)
cs = torch.zeros(512, device=dev)
for p in (0.0, 0.1):
    t = timeit(lambda: ops.scale_dropout(x, y, 1.0, p, 7))
    t2 = timeit(lambda: ops.scale_dropout_colsum(x, y, cs, p=p, seed=7))
    print(f"scale_dropout 7968x512 p={p}: {t:6.1f} us   scale_dropout_colsum: {t2:6.1f} us", flush=True)
