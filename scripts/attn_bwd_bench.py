"""Fused rel-pos attention fwd/bwd alone at the C3 encoder shape (B=32, H=8, T'=249, d=512),
timed with HIP events on the launch stream: prints the mean kernel time per call."""
import math
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops
from espnet_amd._lib import lib
from espnet_amd.layers.common import attn_fused_bwd

dev = torch.device("cuda", 0)
bf = torch.bfloat16
B, H, T = 32, 8, 249
d = H * 64
g = torch.Generator().manual_seed(0)
r = lambda *s: (torch.randn(*s, generator=g) * 0.5).to(bf).to(dev)  # noqa: E731
q, k, v, dO = r(B, T, d), r(B, T, d), r(B, T, d), r(B, T, d)
pp = r(2 * T - 1, d)
u = (torch.randn(d, generator=g) * 0.1).to(dev)
vb = (torch.randn(d, generator=g) * 0.1).to(dev)
klen = torch.full((B,), T, dtype=torch.long, device=dev)
O = torch.empty(B, T, d, dtype=bf, device=dev)
lse = torch.empty(B * H * T, device=dev)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
V1 = os.environ.get("ATTN_V1", "0") == "1"  # the original dQ pass (unshifted dbd) for A/B
if V1:
    ldbd = (2 * T - 1 + 7) // 8 * 8
else:
    from espnet_amd.layers.common import dbd_layout
    _, ldbd = dbd_layout(T)
dbd = torch.empty(H * B * T * ldbd, dtype=bf, device=dev)  # written in full by the kernel
ldm = 2 * ((T + 63) // 64)
dmask = torch.empty(B * H * T * ldm, dtype=torch.int32, device=dev)
nqb = (T + 63) // 64
part = torch.empty(2 * B * nqb * d, device=dev)
qv_out = torch.empty(B, T, d, dtype=bf, device=dev)
scale, p, seed = 1.0 / math.sqrt(64), float(os.environ.get("ATTN_P", "0.1")), 7
st = ops.stream()
hs = torch.cuda.current_stream()  # ops.stream() launches on it


def fwd():
    lib.ea_attn_fused_fwd2(B, H, T, T, 64, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, u.data_ptr(),
                           vb.data_ptr(), pp.data_ptr(), d, klen.data_ptr(), 0, scale, p, seed, O.data_ptr(), d,
                           lse.data_ptr(), dmask.data_ptr() if p > 0 else 0, ldm, st)


def bwd():
    # as the conformer layer calls it: dq with the rel-pos term, bias partials, q+v, keep bits
    attn_fused_bwd(B=B, H=H, T1=T, T2=T, q=q, ldq=d, k=k, ldk=d, v=v, ldv=d, bu=u, bv=vb, pp=pp, ldp=d, klen=klen,
                   causal=False, scale=scale, p=p, seed=seed, O=O, ldo=d, lse=lse, dO=dO, lddo=d, dq=dq, lddq=d,
                   dk=dk, lddk=d, dv=dv, lddv=d, dbd=dbd, ldbd=ldbd, part=part, ldpart=d, qv_out=qv_out, ldqv=d,
                   dmask=dmask if p > 0 else None, ldm=ldm, flags=1 | (4 if V1 else 2))

for name, fn in (("fwd", fwd), ("bwd", bwd)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    n = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(hs)
    for _ in range(n):
        fn()
    e1.record(hs)
    torch.cuda.synchronize()
    print(f"attn_{name}_rel C3 (B={B}, H={H}, T={T}): {e0.elapsed_time(e1) / n * 1e3:.1f} us", flush=True)
print("checksum dq/dk/dv", float(dq.float().abs().sum()), float(dk.float().abs().sum()),
      float(dv.float().abs().sum()), float(dbd.float().abs().sum()))
