"""Small-launch latency probe: ours vs torch (hipBLASLt) on tiny shapes (run under rocprofv3)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib

lib.ea_gemm_set_pipeline(int(sys.argv[1]) if len(sys.argv) > 1 else 12)
for M, N, K in [(1024, 1024, 64), (128, 128, 64), (4096, 4096, 256)]:
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(20):
        ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=K, ldb=K, ldc=N, splitk=False)
    torch.cuda.synchronize()
    for _ in range(20):
        torch.matmul(A, B.t())
    torch.cuda.synchronize()
