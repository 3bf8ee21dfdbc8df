"""The LayerNorm backward with the fused residual-dropout output (ea_layernorm_bwd_partials_drop,
the step's 54 ln_bwd_vec launches) alone at the C3 encoder shape, HIP events on the launch
stream.  Buffer sets rotate so the 64 MB per call comes from HBM, not the 256 MB MALL.
    python scripts/ln_bwd_bench.py [rows d]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import lib  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 7968
d = int(sys.argv[2]) if len(sys.argv) > 2 else 512
NSET = 8
dev = torch.device("cuda")
sets = []
for s in range(NSET):
    x = torch.randn(rows, d, device=dev)
    dy = torch.randn(rows, d, device=dev).to(torch.bfloat16)
    dx = torch.randn(rows, d, device=dev)
    y = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
    mean = x.mean(-1)
    rstd = (x.var(-1, unbiased=False) + 1e-12).rsqrt()
    sets.append((x, dy, dx, y, mean, rstd))
gamma = torch.randn(d, device=dev)
nparts = (rows + 15) // 16
part = torch.empty(nparts * 3 * d, device=dev)
ycol = torch.zeros(d, device=dev)
np_, yp = ctypes.c_int(0), ctypes.c_int(0)
st = ops.stream()


def f(i, drop=True):
    x, dy, dx, y, mean, rstd = sets[i % NSET]
    if drop:
        rc = lib.ea_layernorm_bwd_partials_drop(rows, d, dy.data_ptr(), ops.dt(dy), d, x.data_ptr(), d,
                                                gamma.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), d,
                                                1, part.data_ptr(), part.numel(), ctypes.addressof(np_), y.data_ptr(),
                                                ops.dt(y), d, ctypes.c_float(0.5), ctypes.c_float(0.1), 7,
                                                ycol.data_ptr(), ctypes.addressof(yp), st)
    else:
        rc = lib.ea_layernorm_bwd_partials(rows, d, dy.data_ptr(), ops.dt(dy), d, x.data_ptr(), d, gamma.data_ptr(),
                                           mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), d, 1, part.data_ptr(),
                                           part.numel(), ctypes.addressof(np_), st)
    assert rc == 0, rc


for drop in (True, False):
    for i in range(NSET):
        f(i, drop)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 8 * NSET
    e0.record()
    for i in range(n):
        f(i, drop)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    # x f32, dy bf16, dx f32 read + write, y bf16 write (drop), partials
    byts = rows * d * (4 + 2 + 4 + 4 + (2 if drop else 0)) + np_.value * (3 if drop else 2) * d * 4
    print(f"ln_bwd{'_drop' if drop else ''} {rows}x{d}: {us:.1f} us  {byts / us / 1e6:.2f} TB/s  ({np_.value} blocks)",
          flush=True)
