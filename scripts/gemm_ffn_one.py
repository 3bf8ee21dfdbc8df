"""The C3 step's FFN GEMMs with their step epilogues, repeated (rocprofv3 counter passes and
kernel traces): w_1 forward (7968 x 2048 x 512, bias + Swish, pre-activation kept as bf16 aux,
dropout 0.1) and the w_2 input gradient (7968 x 2048 x 512, W_2 read MN-major, dropout + Swish
derivative from the bf16 pre-activation).  Also a square 4096^3 plain product (the main loop
alone).  usage: gemm_ffn_one.py [iters]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import ACT_SWISH, EPI_ACT, EPI_DACT  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
M, N, K = 7968, 2048, 512
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
w1 = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
b1 = torch.randn(N, device=dev, generator=g)
h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
a = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
dy = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
w2 = (torch.randn(K, N, device=dev, generator=g) * 0.05).to(torch.bfloat16)  # (512, 2048): row-major
dh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
S = 4096
sa = torch.randn(S, S, device=dev, generator=g).to(torch.bfloat16)
sb = torch.randn(S, S, device=dev, generator=g).to(torch.bfloat16)
sc = torch.empty(S, S, device=dev, dtype=torch.bfloat16)
for _ in range(iters):
    ops.gemm(x, w1, a, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=K, ldb=K, ldc=N,
             epi=ops.make_epi(EPI_ACT, bias=b1, act=ACT_SWISH, aux=h, drop_p=0.1, seed=3))
    ops.gemm(dy, w2, dh, M=M, N=N, K=K, a_kmajor=1, b_kmajor=0, lda=K, ldb=N, ldc=N,
             epi=ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=h, drop_p=0.1, seed=4))
    ops.gemm(sa, sb, sc, M=S, N=S, K=S, a_kmajor=1, b_kmajor=1, lda=S, ldb=S, ldc=S)
torch.cuda.synchronize()
print("done")
