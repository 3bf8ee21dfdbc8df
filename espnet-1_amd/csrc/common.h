// Shared device helpers for the espnet-amd HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/espnet_amd.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define EA_DEV __device__ __forceinline__

#define EA_LAUNCH_CHECK()                                  \
  do {                                                     \
    hipError_t _e = hipGetLastError();                     \
    if (_e != hipSuccess) return (int)_e;                  \
  } while (0)

// Clear a stale thread-local HIP error left by another library (e.g. the host framework's
// device probing) so EA_LAUNCH_CHECK reports only this entry point's own launches.
#define EA_ENTRY() ((void)hipGetLastError())

#define EA_CHECK_ARG(cond)                                 \
  do {                                                     \
    if (!(cond)) return EA_ERR_BAD_ARG;                    \
  } while (0)

// ------------------------------------------------------------------ conversions
EA_DEV float to_f(float x) { return x; }
EA_DEV float to_f(bf16 x) { return (float)x; }
template <typename T> EA_DEV T from_f(float x);
template <> EA_DEV float from_f<float>(float x) { return x; }
template <> EA_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

EA_DEV float load_as_f(const void* p, long i, int dtype) {
  return dtype == EA_BF16 ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
EA_DEV void store_from_f(void* p, long i, int dtype, float v) {
  if (dtype == EA_BF16)
    ((bf16*)p)[i] = (bf16)v;
  else
    ((float*)p)[i] = v;
}

// ------------------------------------------------------------------ dropout RNG
// Counter-based: the keep decision of element `idx` under stream `seed` is a pure
// function, so backward regenerates the forward mask with no mask tensor.
EA_DEV uint32_t ea_hash(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}
// returns scale (1/(1-p)) if kept, 0 if dropped; p<=0 -> 1
EA_DEV float drop_scale(uint64_t seed, uint64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
  return ea_hash(seed, idx) >= thr ? 1.f / (1.f - p) : 0.f;
}

// ------------------------------------------------------------------ activations
EA_DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
EA_DEV float act_fwd(int act, float h) {
  if (act == EA_ACT_SWISH) return h * sigmoidf_(h);
  if (act == EA_ACT_RELU) return h > 0.f ? h : 0.f;
  return h;
}
EA_DEV float act_bwd(int act, float h) {  // derivative wrt pre-activation h
  if (act == EA_ACT_SWISH) {
    float s = sigmoidf_(h);
    return s * (1.f + h * (1.f - s));
  }
  if (act == EA_ACT_RELU) return h > 0.f ? 1.f : 0.f;
  return 1.f;
}

// ------------------------------------------------------------------ reductions (wave64)
EA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
EA_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
EA_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// block-wide sum for blockDim.x a multiple of 64 (<=1024); `red` has >=16 floats.
EA_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
EA_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}
EA_DEV double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__host__ __device__ static inline int ea_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
static inline int ea_grid_cap(long blocks, int cap = 4096) { return (int)(blocks < cap ? (blocks > 0 ? blocks : 1) : cap); }
