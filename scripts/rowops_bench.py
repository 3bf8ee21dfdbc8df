"""Input-end kernels alone at the C3 shape (B=32, T=1000, F=80, C=512): conv1 forward
(phase-split bf16 + ReLU support bytes) and utterance MVN, timed with HIP events on the
launch stream; prints mean us per call and the effective bytes/s.
EA_CONV1_FWD_PIX=1 selects the per-pixel conv1 kernel for A/B."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib, BF16 as EA_BF16

B, T, F, C = 32, 1000, 80, 512
dev = torch.device("cuda", 0)
x = torch.randn(B, T, F, device=dev)
lens = torch.full((B,), T, dtype=torch.long, device=dev)
T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
y1 = torch.empty(B * T1 * F1 * C, dtype=torch.bfloat16, device=dev)
pos = torch.empty(B * T1 * F1 * C // 8, dtype=torch.uint8, device=dev)
w = torch.randn(C, 9, device=dev)
bias = torch.randn(C, device=dev)
ym = torch.empty_like(x)
n = ctypes.c_long(0)
lib.ea_utterance_mvn_ws_bytes(B, T, F, ctypes.addressof(n))
ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
st = ops.stream()
hs = torch.cuda.current_stream()


def conv1():
    lib.ea_conv1_fwd2(B, T, F, C, x.data_ptr(), w.data_ptr(), bias.data_ptr(), y1.data_ptr(), EA_BF16,
                      pos.data_ptr(), st)


def mvn():
    lib.ea_utterance_mvn2(B, T, F, x.data_ptr(), lens.data_ptr(), ym.data_ptr(), ws.data_ptr(), ws.numel(), st)


for name, fn, nbytes in (("conv1_fwd", conv1, y1.numel() * 2 + pos.numel() + x.numel() * 4),
                         ("utterance_mvn", mvn, 2 * x.numel() * 4)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    k = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(hs)
    for _ in range(k):
        fn()
    e1.record(hs)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / k * 1e3
    print(f"{name}: {us:.1f} us  ({nbytes / us / 1e6:.2f} TB/s algorithmic)", flush=True)
