// Dense GEMM launches on the ping-pong kernel (gemm_kern.h: gemm_pipe), 256x256 and 128x128 tiles.
#include "gemm_kern.h"

namespace eag {
int launch_pipe(GemmP& p, int a_k, int b_k, dim3 grid, hipStream_t st) {
  if (p.bm == 256) {
    if (a_k && b_k) hipLaunchKernelGGL((gemm_pipe<true, true, 0, 256>), grid, dim3(512), 0, st, p);
    else if (a_k) hipLaunchKernelGGL((gemm_pipe<true, false, 0, 256>), grid, dim3(512), 0, st, p);
    else if (b_k) hipLaunchKernelGGL((gemm_pipe<false, true, 0, 256>), grid, dim3(512), 0, st, p);
    else hipLaunchKernelGGL((gemm_pipe<false, false, 0, 256>), grid, dim3(512), 0, st, p);
  } else {
    if (a_k && b_k) hipLaunchKernelGGL((gemm_pipe<true, true, 0, 128>), grid, dim3(512), 0, st, p);
    else if (a_k) hipLaunchKernelGGL((gemm_pipe<true, false, 0, 128>), grid, dim3(512), 0, st, p);
    else if (b_k) hipLaunchKernelGGL((gemm_pipe<false, true, 0, 128>), grid, dim3(512), 0, st, p);
    else hipLaunchKernelGGL((gemm_pipe<false, false, 0, 128>), grid, dim3(512), 0, st, p);
  }
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
