// Stream-ordering diagnostics (include/espnet_amd.h: ea_debug_spin).
//
// ea_debug_spin holds a stream for a fixed time: one single-lane workgroup that polls the
// GPU's constant 100 MHz clock (s_memrealtime, a read) and sleeps between polls.  Launched at
// the head of every side / auxiliary stream segment (hip_ops.DEBUG_DELAY_NS), it makes a
// missing cross-stream edge deterministic: a consumer on the main stream that does not wait
// for a side-stream producer reads its buffer before the producer ran, every time.
#include "common.h"

namespace {
__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
}  // namespace

extern "C" int ea_debug_spin(long ns, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(ns >= 0 && ns <= 100000000L);  // at most 100 ms
  if (ns == 0) return 0;
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, (unsigned long long)(ns + 9) / 10);
  EA_LAUNCH_CHECK();
  return 0;
}
