"""Conv2dSubsampling (C3 shapes: B=32, T=1000, d=512) forward + backward in isolation, bf16
implicit-GEMM route, serial weight-gradient stream (EA_OVERLAP_WGRAD=0 unless set), for
rocprofv3 --kernel-trace: each conv2 GEMM launch timed alone.

    EA_OVERLAP_WGRAD=0 python scripts/sub_bench.py [iters]
"""
import os
import sys

os.environ.setdefault("EA_OVERLAP_WGRAD", "0")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd.arena import ParamArena  # noqa: E402
from espnet_amd.layers import subsampling as S  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B, T, C = 32, 1000, 512
dev = torch.device("cuda", 0)
torch.manual_seed(0)
sub = S.Conv2dSubsampling(80, C, 0.1)
arena = ParamArena(sub, dev, [], shadow_dtype=torch.bfloat16)
sub.bind(arena, "", torch.bfloat16)
sub._anchor = torch.zeros(1, device=dev, requires_grad=True)
sub.train()
feats = torch.randn(B, T, 80, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(iters + 1):
    if it == 1:
        torch.cuda.synchronize()
        e0.record()
    y = sub(feats, 0)
    y.backward(torch.ones_like(y))
e1.record()
torch.cuda.synchronize()
print(f"subsampling fwd+bwd: {e0.elapsed_time(e1) / iters:.3f} ms/iter", flush=True)
