"""Event timing of ea_beam_prebeam vs the pre-beam size P and the vocabulary V (10 rows)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import lib  # noqa: E402

n = 10
for V in (5000, 1000):
    logp = torch.log_softmax(torch.randn(n, V), -1).cuda().contiguous()
    for P in (1, 4, 15, 30):
        cand = torch.empty(n * (P + 1), dtype=torch.int32, device="cuda")
        f = lambda: lib.ea_beam_prebeam(n, V, logp.data_ptr(), V, 0.7, 0.0, 0, P, V - 1, cand.data_ptr(), ops.stream())  # noqa: E731
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"V={V} P={P}: {e0.elapsed_time(e1) / 100 * 1e3:.1f} us", flush=True)
