"""Feasibility probe: does the HBM-bound Adam update (116 M parameters, ~3.5 GB moved) overlap
with an MFMA-bound GEMM of the conv2 forward's size (151392 x 512 x 4608 bf16) when the two run
on separate HIP streams?  Prints serial and concurrent wall times (HIP events, median of 7).

    python scripts/overlap_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "espnet-1_amd")]
import torch  # noqa: E402

from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd._lib import lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = 116_146_960
    p = torch.randn(n, device=dev) * 0.02
    g = torch.randn(n, device=dev) * 1e-3
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    norm = torch.tensor([1.0], device=dev)
    M, N, K = 151392, 512, 4608
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream(device=dev)

    def gemm():
        ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=K, ldb=K, ldc=N)

    def adam(st):
        lib.ea_adam_step(n, p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), pb.data_ptr(), 1e-4, 0.9,
                         0.98, 1e-9, 0.0, 10, norm.data_ptr(), 5.0, st.cuda_stream)

    def timed(fn):
        ts = []
        for _ in range(7):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1)
            fn()
            e1.record(s1)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[3]

    def conc():
        s2.wait_stream(s1)
        with torch.cuda.stream(s2):
            adam(s2)
        gemm()
        s1.wait_stream(s2)

    for _ in range(3):
        gemm()
        adam(s1)
    tg = timed(gemm)
    ta = timed(lambda: adam(s1))
    ts = timed(lambda: (gemm(), adam(s1)))
    tc = timed(conc)
    print(f"gemm {tg:.3f} ms, adam {ta:.3f} ms, serial {ts:.3f} ms, concurrent {tc:.3f} ms "
          f"(saved {ts - tc:.3f} ms = {100 * (ts - tc) / ta:.0f}% of adam)", flush=True)


if __name__ == "__main__":
    main()
