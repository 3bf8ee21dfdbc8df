// Guarded device allocator for torch's CUDAPluggableAllocator (diagnostic, not on the product
// path; scripts/dp_drift_diag.py --guard).  Every allocation is a fresh hipMalloc of the
// requested size plus a 64 KiB tail guard: the body starts zeroed, the guard is filled with
// 0xFF bytes (NaN in f32 / bf16), so a kernel that reads past the end of its buffer turns its
// result NaN in every run, instead of reading whatever the caching allocator placed next to
// it (which depends on when blocks held by record_stream() come back: run to run).  Frees
// synchronise the device first, so no block is ever reused under a pending kernel.
#include "common.h"

namespace {
constexpr size_t kGuard = 64 << 10;
}

extern "C" void* ea_guard_malloc(size_t size, int device, void* stream) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (prev != device) (void)hipSetDevice(device);
  void* p = nullptr;
  if (hipMalloc(&p, size + kGuard) != hipSuccess) p = nullptr;
  if (p) {
    (void)hipMemsetAsync(p, 0, size, (hipStream_t)stream);
    (void)hipMemsetAsync((char*)p + size, 0xFF, kGuard, (hipStream_t)stream);
    (void)hipStreamSynchronize((hipStream_t)stream);
  }
  if (prev != device) (void)hipSetDevice(prev);
  return p;
}

extern "C" void ea_guard_free(void* p, size_t size, int device, void* stream) {
  (void)size;
  (void)device;
  (void)stream;
  (void)hipDeviceSynchronize();
  (void)hipFree(p);
}
