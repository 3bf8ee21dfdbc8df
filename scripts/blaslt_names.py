"""hipBLASLt kernel selection on the C3 step's Linear shapes (run under rocprofv3 --kernel-trace:
the Cijk_... kernel names carry the macro tile MT<M>x<N>x<K>, the wave tiling and stream-K
flags), timed with HIP events for reference."""
import torch

dev = torch.device("cuda", 0)
shapes = [(7968, 512, 2048), (7968, 2048, 512), (7968, 512, 512), (7968, 1536, 512), (1312, 512, 2048)]
for M, N, K in shapes:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(5):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        torch.matmul(a, b.t())
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{M}x{N}x{K}: {us:.1f} us  {2 * M * N * K / us * 1e-6:.0f} TF/s", flush=True)
