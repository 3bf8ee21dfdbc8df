// Conv2dSubsampling conv2 implicit-GEMM launches on the ping-pong kernel (gemm_kern.h).
#include "gemm_kern.h"

namespace eag {
int launch_pipe_conv(GemmP& p, dim3 grid, hipStream_t st) {
  if (p.g.mode == EA_CONV_FWD) hipLaunchKernelGGL((gemm_pipe<true, true, EA_CONV_FWD>), grid, dim3(512), 0, st, p);
  // DGRAD: B = W2t [9][co][ci] (ldb = C, MN-major) or W2k [ci][9][co] (ldb = 9C, K-major)
  else if (p.g.mode == EA_CONV_DGRAD && p.ldb == 9L * p.g.C)
    hipLaunchKernelGGL((gemm_pipe<true, true, EA_CONV_DGRAD>), grid, dim3(512), 0, st, p);
  else if (p.g.mode == EA_CONV_DGRAD) hipLaunchKernelGGL((gemm_pipe<true, false, EA_CONV_DGRAD>), grid, dim3(512), 0, st, p);
  else hipLaunchKernelGGL((gemm_pipe<false, false, EA_CONV_WGRAD>), grid, dim3(512), 0, st, p);
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
