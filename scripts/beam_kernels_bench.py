"""Event timing of the device beam-step kernels at the C3 decode shapes (T'=249, V=5000,
10 hypotheses, pre-beam 15): back-to-back (GPU busy) and one launch after an idle gap."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import lib  # noqa: E402

T, V, n, P = 249, 5000, 10, 15
Pc = P + 1
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
logits = torch.randn(T, V, generator=g).to(dev)
logp_ctc = torch.log_softmax(logits, -1).contiguous()
r_prev = torch.log_softmax(torch.randn(n, T, 2, generator=g), -1).to(dev).contiguous()
rptr = torch.tensor([r_prev[h].data_ptr() for h in range(n)], dtype=torch.int64, device=dev)
last = torch.randint(0, V, (n,), dtype=torch.int32).to(dev)
dec_logp = torch.log_softmax(torch.randn(n, V, generator=g), -1).to(dev).contiguous()
cand = torch.empty(n * Pc, dtype=torch.int32, device=dev)
psi = torch.empty(n * Pc, device=dev)
r_new = torch.empty(n * Pc, T, 2, device=dev)
rec = torch.empty(8 * n, dtype=torch.int32, device=dev)
st = {k: torch.zeros(n, dtype=d, device=dev) for k, d in (("last", torch.int32), ("prefix", torch.float32),
                                                          ("score", torch.float32))}
rptr_n = torch.zeros(n, dtype=torch.int64, device=dev)
s = ops.stream()
K = 10


def prebeam():
    lib.ea_beam_prebeam(n, V, dec_logp.data_ptr(), V, 0.7, 0.0, 0, P, V - 1, cand.data_ptr(), s)


def prefix():
    lib.ea_ctc_prefix_score_dev(T, V, 0, V - 1, n, Pc, logp_ctc.data_ptr(), rptr.data_ptr(), 5, last.data_ptr(),
                                cand.data_ptr(), psi.data_ptr(), r_new.data_ptr(), s)


def select():
    lib.ea_beam_select(n, V, P, K, T, dec_logp.data_ptr(), V, cand.data_ptr(), psi.data_ptr(), st["prefix"].data_ptr(),
                       st["score"].data_ptr(), 0.7, 0.0, 0, 0.3, r_new.data_ptr(), rec.data_ptr(),
                       rec.data_ptr() + 16 * K, st["last"].data_ptr(), rptr_n.data_ptr(), st["prefix"].data_ptr(),
                       st["score"].data_ptr(), s)


for name, fn in (("prebeam", prebeam), ("prefix", prefix), ("select", select)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        fn()
    e1.record()
    torch.cuda.synchronize()
    busy = e0.elapsed_time(e1) / 100 * 1e3
    idle = []
    for _ in range(5):
        time.sleep(0.002)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        idle.append(e0.elapsed_time(e1) * 1e3)
    print(f"{name:8s}: back-to-back {busy:7.1f} us; after 2 ms idle {min(idle):7.1f}-{max(idle):7.1f} us", flush=True)
