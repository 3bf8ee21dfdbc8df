"""Probe: torch (hipBLASLt) bf16 GEMM time at the C3 weight-gradient shapes vs our kernel."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
dev = "cuda"
for (N, K, R) in [(2048, 512, 7968), (512, 2048, 7968), (512, 512, 7968), (1536, 512, 7968)]:
    dy = torch.randn(R, N, device=dev).to(torch.bfloat16)
    x = torch.randn(R, K, device=dev).to(torch.bfloat16)
    dw = torch.zeros(N, K, device=dev)
    def ours():
        ops.linear_dw(dy, x, dw, accumulate=True)
    def lt():
        return torch.mm(dy.t(), x)
    def lt32():
        return torch.mm(dy.t().float(), x.float())
    for name, fn in (("ours", ours), ("torch_bf16", lt)):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"dW {N}x{K} K={R} {name}: {us:.1f} us  {2*N*K*R/us/1e6:.0f} TFLOP/s", flush=True)
