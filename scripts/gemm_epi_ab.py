"""A/B of GEMM epilogue cost by output tile and split-K combine mode on the C3 FFN shapes."""
import os
import sys
sys.argv = sys.argv[:1]
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
os.environ["EA_BENCH_TORCH"] = "0"
import bench_gemm as bg  # runs its default list first (pipeline 2)
import torch
from espnet_amd._lib import lib

dt = torch.bfloat16
for tile in [(0, 0), (64, 128), (128, 128), (256, 256)]:
    lib.ea_gemm_set_tile(*tile)
    print("tile", tile)
    bg.bench("ffn_w1 fwd ACT", dt, 7968, 2048, 512, 1, 1, epi="act", cdt=torch.bfloat16)
    if tile != (64, 128):
        bg.bench("ffn_w2 dX DACT", dt, 7968, 2048, 512, 1, 0, epi="dact", cdt=torch.bfloat16)
    bg.bench("ffn_w2 fwd RESID", dt, 7968, 512, 2048, 1, 1, epi="resid")
    bg.bench("ffn_w1 fwd bf16", dt, 7968, 2048, 512, 1, 1, cdt=torch.bfloat16)
lib.ea_gemm_set_tile(0, 0)
