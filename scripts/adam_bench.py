"""ea_adam_step alone at the C3 model's parameter count (f32 master + m + v + bf16 shadow),
HIP events on the launch stream."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib

n = int(os.environ.get("ADAM_N", "115000000"))
p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4))
v.abs_()
p16 = torch.empty(n, dtype=torch.bfloat16, device="cuda")
st = ops.stream()
f = lambda: lib.ea_adam_step(n, p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p16.data_ptr(),  # noqa
                             1e-3, 0.9, 0.98, 1e-9, 0.0, 5, 0, 0.0, st)
for _ in range(3):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    f()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
print(f"adam: {us:.1f} us  ({30 * n / us / 1e6:.2f} TB/s)", flush=True)
