"""Run one ea_gemm shape repeatedly (for rocprofv3 counter passes).
usage: gemm_one.py M N K a_kmajor b_kmajor [iters] [pipeline]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib

M, N, K, ak, bk = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
if len(sys.argv) > 7:
    lib.ea_gemm_set_pipeline(int(sys.argv[7]))
if os.environ.get("EA_TILE"):  # force an output tile, e.g. EA_TILE=256
    t = int(os.environ["EA_TILE"])
    lib.ea_gemm_set_tile(t if t != 64 else 64, t if t != 64 else 128)
if os.environ.get("EA_PIPE"):
    lib.ea_gemm_set_pipe(int(os.environ["EA_PIPE"]))
A = torch.randn((M, K) if ak else (K, M), device="cuda").to(torch.bfloat16)
B = torch.randn((N, K) if bk else (K, N), device="cuda").to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0), ldb=B.stride(0), ldc=N)
torch.cuda.synchronize()
print("done")
