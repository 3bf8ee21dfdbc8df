"""In-kernel timeline of one gemm_pipe launch (ea_gemm_set_diag): per block the shader-clock
cycles of its main loop and its epilogue, and its start offset (100 MHz clock) from the
first block, for a given shape / epilogue.

    python scripts/gemm_timeline.py M N K a_k b_k [store|store_drop|dact|act|resid[_nodrop]] [out: bf16|f32]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import ACT_RELU, ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, lib  # noqa: E402

M, N, K, ak, bk = (int(v) for v in sys.argv[1:6])
kind = sys.argv[6] if len(sys.argv) > 6 else "store"
drop = 0.0 if kind.endswith("_nodrop") else 0.1  # act_nodrop / dact_nodrop / store_drop
kind = kind.replace("_nodrop", "")
if kind == "store_drop":
    kind = "store"
elif kind == "store":
    drop = 0.0
odt = torch.float32 if (len(sys.argv) > 7 and sys.argv[7] == "f32") else torch.bfloat16
lib.ea_gemm_set_tile(256, 256)
A = torch.randn((M, K) if ak else (K, M), device="cuda").to(torch.bfloat16)
B = torch.randn((N, K) if bk else (K, N), device="cuda").to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=odt)
keep = []
e = None
if kind == "dact":
    keep.append(torch.randn(M, N, device="cuda").to(torch.bfloat16))
    e = ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=keep[0], drop_p=drop, seed=3)
elif kind == "act":
    keep += [torch.empty(M, N, device="cuda", dtype=torch.bfloat16), torch.randn(N, device="cuda")]
    e = ops.make_epi(EPI_ACT, bias=keep[1], act=ACT_SWISH, aux=keep[0], drop_p=drop, seed=3)
elif kind == "store" and drop > 0:
    e = ops.make_epi(drop_p=drop, seed=3)
elif kind == "resid":
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    keep += [torch.randn(M, N, device="cuda"), torch.randn(N, device="cuda")]
    e = ops.make_epi(EPI_RESID, bias=keep[1], resid=keep[0], rscale=0.5, drop_p=drop, seed=3)
nblk = ((M + 255) // 256) * ((N + 255) // 256)
diag = torch.zeros(4 * nblk, dtype=torch.int64, device="cuda")
f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=ak, b_kmajor=bk, lda=A.stride(0), ldb=B.stride(0),  # noqa
                     ldc=N, epi=e, splitk=False)
for _ in range(5):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    f()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 10 * 1e3
lib.ea_gemm_set_diag(diag.data_ptr())
f()
torch.cuda.synchronize()
lib.ea_gemm_set_diag(None)
lib.ea_gemm_set_tile(0, 0)
d = diag.view(nblk, 4).cpu().double()
main = d[:, 1] - d[:, 0]
epi = d[:, 2] - d[:, 1]
start = (d[:, 3] - d[:, 3].min()) * 10.0  # ns (100 MHz)
q = lambda x: f"med {x.median().item():9.0f} p10 {x.quantile(0.1).item():9.0f} p90 {x.quantile(0.9).item():9.0f}"  # noqa
print(f"{M}x{N}x{K} ({ak},{bk}) {kind} drop {drop} {str(odt)[6:]}: {us:.1f} us/launch, {nblk} blocks, "
      f"{2.0 * M * N * K / us / 1e6:.0f} TF/s")
print("  main loop cycles ", q(main))
print("  epilogue cycles  ", q(epi))
print("  start offset ns  ", q(start), f"max {start.max().item():.0f}")
