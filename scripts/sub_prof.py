"""Conv2dSubsampling fwd+bwd alone at C3 shapes (B=32, T=1000, 80 -> 512), serial (run with
EA_OVERLAP_WGRAD=0 under rocprofv3 --kernel-trace to time every conv GEMM on its own)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd.arena import ParamArena
from espnet_amd.layers import subsampling as S

dev = torch.device("cuda", 0)
torch.manual_seed(0)
sub = S.Conv2dSubsampling(80, 512, 0.1)
arena = ParamArena(sub, dev, [], shadow_dtype=torch.bfloat16)
sub.bind(arena, "", torch.bfloat16)
sub._anchor = torch.zeros(1, device=dev, requires_grad=True)
sub.train()
feats = torch.randn(32, 1000, 80, device=dev)
if os.environ.get("SUB_TILE"):
    from espnet_amd._lib import lib
    bm = int(os.environ["SUB_TILE"])
    lib.ea_gemm_set_tile(bm, bm)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    y = sub(feats, 0)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
print("ok", y.shape)
