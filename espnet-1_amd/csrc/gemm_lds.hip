// Dense GEMM launches on the LDS-DMA kernel (gemm_kern.h: gemm_bf16_lds): 2-stage ring, except
// the 64x128 tile, whose 3-deep ring (two blocks per CU instead of three) measured 0.9-1.2%
// faster on the C3 step (round 2, scripts/gpu_lds64_ab.sh).
#include "gemm_kern.h"

#include <cstdlib>

namespace eag {
int launch_lds_dense(GemmP& p, int a_k, int b_k, dim3 grid, hipStream_t st) {
#define EA_GL(BMV, BNV, AKV, BKV, S) \
  hipLaunchKernelGGL((gemm_bf16_lds<BMV, BNV, (BNV == 256 ? 4 : 2), AKV, BKV, S>), grid, dim3(BNV == 256 ? 512 : 256), 0, st, p)
#define EA_GL4(BMV, BNV, S)                            \
  if (a_k && b_k) EA_GL(BMV, BNV, true, true, S);      \
  else if (a_k) EA_GL(BMV, BNV, true, false, S);       \
  else if (b_k) EA_GL(BMV, BNV, false, true, S);       \
  else EA_GL(BMV, BNV, false, false, S);
  if (p.bm == 32) {  // small-M GEMMs (decoder tokens, positional rows): twice the blocks of 64x128
    if (b_k) EA_GL(32, 128, true, true, 3);
    else EA_GL(32, 128, true, false, 3);
  } else if (p.bm == 64) {
    if (b_k) EA_GL(64, 128, true, true, 3);
    else EA_GL(64, 128, true, false, 3);
  } else if (p.bm == 256 && p.bn == 256) {
    EA_GL4(256, 256, 2)
  } else {
    EA_GL4(128, 128, 2)
  }
#undef EA_GL4
#undef EA_GL
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
