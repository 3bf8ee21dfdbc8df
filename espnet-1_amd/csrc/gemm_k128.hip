// Launches of gemm_k128 (gemm_kern.h): 128x128 tiles, K-major A and B, 8 waves in two K groups.
#include "gemm_kern.h"

namespace eag {
int g_k128_slots = 4;
int launch_k128(GemmP& p, dim3 grid, hipStream_t st) {
  if (g_k128_slots == 3) hipLaunchKernelGGL((gemm_k128<3>), grid, dim3(512), 0, st, p);
  else hipLaunchKernelGGL((gemm_k128<4>), grid, dim3(512), 0, st, p);
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
