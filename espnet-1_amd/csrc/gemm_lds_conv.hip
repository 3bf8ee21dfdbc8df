// Conv2dSubsampling conv2 implicit-GEMM launches on the 2-stage LDS-DMA kernel (gemm_kern.h).
#include "gemm_kern.h"

namespace eag {
int launch_lds_conv(GemmP& p, dim3 grid, hipStream_t st) {
#define EA_GC(BMV, BNV, AKV, BKV, MD) \
  hipLaunchKernelGGL((gemm_bf16_lds<BMV, BNV, (BNV == 256 ? 4 : 2), AKV, BKV, 2, MD>), grid, dim3(BNV == 256 ? 512 : 256), 0, st, p)
  const bool big = p.bm == 256;
  if (p.g.mode == EA_CONV_FWD) {
    if (big) EA_GC(256, 256, true, true, EA_CONV_FWD); else EA_GC(128, 128, true, true, EA_CONV_FWD);
  } else if (p.g.mode == EA_CONV_DGRAD) {
    if (big) EA_GC(256, 256, true, false, EA_CONV_DGRAD); else EA_GC(128, 128, true, false, EA_CONV_DGRAD);
  } else {
    if (big) EA_GC(256, 256, false, false, EA_CONV_WGRAD); else EA_GC(128, 128, false, false, EA_CONV_WGRAD);
  }
#undef EA_GC
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
