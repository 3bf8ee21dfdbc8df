"""torch.matmul (hipBLASLt) bf16 C = A B^T at one shape, repeated (for rocprofv3 counter passes).
usage: blaslt_one.py M N K [iters]"""
import sys
import torch
M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
for _ in range(iters):
    C = A @ B.t()
torch.cuda.synchronize()
print("done")
