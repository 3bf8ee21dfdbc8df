"""Microbench of ea_gemm on the C3 (Conformer-L) shapes; prints TFLOP/s per shape."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd"))
import torch
from espnet_amd import hip_ops as ops

def bench(name, dtype, M, N, K, a_k, b_k, iters=20, epi=None, cdt=torch.float32):
    A = torch.randn((M, K) if a_k else (K, M), device="cuda").to(dtype)
    B = torch.randn((N, K) if b_k else (K, N), device="cuda").to(dtype)
    C = torch.empty(M, N, device="cuda", dtype=cdt)
    e = None
    if epi == "act":      # FFN w_1: bias + swish + dropout, pre-activation kept (bf16)
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        e = ops.make_epi(EPI_ACT, bias=bias, act=ACT_SWISH, aux=aux, drop_p=0.1, seed=7)
    elif epi == "dact":   # FFN w_2 dX: dropout mask + swish' (aux read)
        aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        e = ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=aux, drop_p=0.1, seed=7)
    elif epi == "resid":  # FFN w_2: bias + dropout + scaled residual add into f32
        resid = torch.randn(M, N, device="cuda")
        bias = torch.randn(N, device="cuda")
        e = ops.make_epi(EPI_RESID, bias=bias, resid=resid, rscale=0.5, drop_p=0.1, seed=7)
    f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0), ldc=N, epi=e)
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tl = ""
    if TORCH:
        Ao = A if a_k else A.t()
        Bo = B.t() if b_k else B
        g = lambda: torch.matmul(Ao, Bo)
        for _ in range(3): g()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters): g()
        e1.record(); torch.cuda.synchronize()
        tms = e0.elapsed_time(e1) / iters
        tl = f"   | torch/hipBLASLt {tms*1e3:8.1f} us {2*M*N*K/tms/1e9:7.1f} TF/s"
    print(f"{name:28s} {str(dtype):15s} M={M:6d} N={N:5d} K={K:5d} ak={a_k} bk={b_k}: {ms*1e3:8.1f} us  {2*M*N*K/ms/1e9:7.1f} TF/s{tl}", flush=True)

TORCH = os.environ.get("EA_BENCH_TORCH", "0") == "1"

from espnet_amd._lib import lib, EPI_ACT, EPI_DACT, EPI_RESID, ACT_SWISH
import sys as _s
pipes = [int(x) for x in (_s.argv[1].split(",") if len(_s.argv) > 1 else ["2"])]
for pipe in pipes:
  lib.ea_gemm_set_pipeline(pipe)
  print("pipeline", pipe)
  for dt in (torch.bfloat16,):
    bench("ffn_w1 fwd", dt, 7968, 2048, 512, 1, 1)
    bench("ffn_w1 fwd bf16 out", dt, 7968, 2048, 512, 1, 1, cdt=torch.bfloat16)
    bench("ffn_w1 fwd ACT", dt, 7968, 2048, 512, 1, 1, epi="act", cdt=torch.bfloat16)
    bench("ffn_w2 dX DACT", dt, 7968, 2048, 512, 1, 0, epi="dact", cdt=torch.bfloat16)
    bench("ffn_w2 fwd RESID", dt, 7968, 512, 2048, 1, 1, epi="resid")
    bench("ffn_w2 fwd", dt, 7968, 512, 2048, 1, 1)
    bench("qkv fwd", dt, 7968, 1536, 512, 1, 1)
    bench("ffn_w1 dX", dt, 7968, 512, 2048, 1, 0)
    bench("ffn_w1 dW", dt, 2048, 512, 7968, 0, 0)
    bench("ctc_lo fwd", dt, 7968, 5000, 512, 1, 1)
    bench("conv2 fwd", dt, 151392, 512, 4608, 1, 1, iters=5)
    bench("conv2 dcol", dt, 151392, 4608, 512, 1, 0, iters=5)
    bench("conv2 dW", dt, 512, 4608, 151392, 0, 0, iters=5)
    bench("square 4096", dt, 4096, 4096, 4096, 1, 1, iters=5)
    bench("square 8192", dt, 8192, 8192, 8192, 1, 1, iters=3)
