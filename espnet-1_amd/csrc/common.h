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

// 4-wide vector load/store (16-B f32, 8-B bf16; caller guarantees alignment)
EA_DEV void vld4(const float* p, float (&v)[4]) {
  const float4 f = *(const float4*)p;
  v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
}
EA_DEV void vld4(const bf16* p, float (&v)[4]) {
  const uint2 u = *(const uint2*)p;
  const bf16* b = (const bf16*)&u;
  v[0] = (float)b[0]; v[1] = (float)b[1]; v[2] = (float)b[2]; v[3] = (float)b[3];
}
EA_DEV void vst4(float* p, const float (&v)[4]) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
EA_DEV void vst4(bf16* p, const float (&v)[4]) {
  union { uint2 u; bf16 b[4]; } t;
  t.b[0] = (bf16)v[0]; t.b[1] = (bf16)v[1]; t.b[2] = (bf16)v[2]; t.b[3] = (bf16)v[3];
  *(uint2*)p = t.u;
}
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
// function, so backward regenerates the forward mask with no mask tensor.  One 32-bit
// hash serves the element pair idx>>1, each element using 16 of its bits; the 64-bit seed is
// folded into a 32-bit stream key that is uniform across the launch (scalar unit, hoisted
// out of the loops).  The per-pair mixer is Bob Jenkins' 6-shift integer hash (adds, shifts
// and xors only): full-rate VALU on CDNA, where a 32-bit multiply is quarter rate — the
// multiply-based mixer it replaces was half of a dropout-fused GEMM epilogue's cost.
__host__ __device__ inline uint32_t ea_mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__host__ __device__ inline uint32_t ea_seed_key(uint64_t seed) {
  return ea_mix32((uint32_t)seed ^ ea_mix32((uint32_t)(seed >> 32) ^ 0x5bd1e995U));
}
// the six mixing rounds on a = low word of the pair + key (+ the high word's term)
EA_DEV uint32_t ea_pair_mix(uint32_t a) {
  a = (a + 0x7ed55d16u) + (a << 12);
  a = (a ^ 0xc761c23cu) ^ (a >> 19);
  a = (a + 0x165667b1u) + (a << 5);
  a = (a + 0xd3a2646cu) ^ (a << 9);
  a = (a + 0xfd7046c5u) + (a << 3);
  a = (a ^ 0xb55a4f09u) ^ (a >> 16);
  return a;
}
EA_DEV uint32_t ea_pair_hash(uint32_t key, uint64_t pair) {
  return ea_pair_mix((uint32_t)pair + key + __umul24((uint32_t)(pair >> 32), 0x9e3779u));
}
// Per-step salt of every dropout stream (ea_set_rng_salt): launchers pass the process-wide
// device pointer ea_g_rng_salt to their kernels, which mix *salt into the site seed.  The
// salt lives in device memory so a captured hipGraph draws fresh masks on every replay
// (ea_rng_advance is part of the graph); salt 0 leaves the seed unchanged.
extern const unsigned long long* ea_g_rng_salt;
EA_DEV uint64_t ea_salted(uint64_t seed, const unsigned long long* salt) {
  return salt ? seed ^ (*salt * 0x9E3779B97F4A7C15ull) : seed;
}
EA_DEV uint32_t ea_drop_thr(float p) { return (uint32_t)fminf(p * 65536.f + 0.5f, 65536.f); }
// returns scale (1/(1-p)) if kept, 0 if dropped; p<=0 -> 1
EA_DEV float drop_scale(uint64_t seed, uint64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  const uint32_t h = ea_pair_hash(ea_seed_key(seed), idx >> 1);
  const uint32_t bits = (idx & 1) ? h >> 16 : h & 0xffffu;
  return bits >= ea_drop_thr(p) ? 1.f / (1.f - p) : 0.f;
}
// Attention-score dropout stream: element (row, j) of a (rows x T2) score matrix, rows
// z*T1 + i.  Keys 2m and 2m+1 of a row share one pair hash (its low / high 16 bits), so two
// adjacent lanes draw a single hash for both; every path (fused kernels, unfused softmax,
// forward and backward) uses this law.
EA_DEV uint64_t attn_pair(uint64_t row, int T2, int j) { return row * (uint64_t)((T2 + 1) >> 1) + (uint64_t)(j >> 1); }
EA_DEV bool attn_keep(uint32_t key, uint32_t thr, uint64_t row, int T2, int j) {
  const uint32_t h = ea_pair_hash(key, attn_pair(row, T2, j));
  return ((j & 1) ? h >> 16 : h & 0xffffu) >= thr;
}
EA_DEV float attn_drop_scale(uint64_t seed, uint64_t row, int T2, int j, float p) {
  if (p <= 0.f) return 1.f;
  return attn_keep(ea_seed_key(seed), ea_drop_thr(p), row, T2, j) ? 1.f / (1.f - p) : 0.f;
}
// four consecutive elements idx .. idx+3, idx even (two hashes); s[k] *= scale
EA_DEV void drop_scale4(uint64_t seed, uint64_t idx, float p, float (&v)[4]) {
  if (p <= 0.f) return;
  const uint32_t key = ea_seed_key(seed), thr = ea_drop_thr(p);
  const float sc = 1.f / (1.f - p);
  const uint32_t h0 = ea_pair_hash(key, idx >> 1), h1 = ea_pair_hash(key, (idx >> 1) + 1);
  v[0] *= (h0 & 0xffffu) >= thr ? sc : 0.f;
  v[1] *= (h0 >> 16) >= thr ? sc : 0.f;
  v[2] *= (h1 & 0xffffu) >= thr ? sc : 0.f;
  v[3] *= (h1 >> 16) >= thr ? sc : 0.f;
}

// ------------------------------------------------------------------ activations
EA_DEV float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
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

// N elements at once: the activation branch (uniform) taken once outside the element loop, so
// the N independent exp -> rcp chains share one basic block and interleave (a branch per
// element serialises each chain's latency)
template <int N>
EA_DEV void act_fwd_n(int act, float (&v)[N]) {
  if (act == EA_ACT_SWISH) {
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = v[c] * sigmoidf_(v[c]);
  } else if (act == EA_ACT_RELU) {
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = v[c] > 0.f ? v[c] : 0.f;
  }
}
template <int N>
EA_DEV void act_bwd_mul_n(int act, float (&v)[N], const float (&h)[N]) {  // v *= act'(h)
  if (act == EA_ACT_SWISH) {
#pragma unroll
    for (int c = 0; c < N; ++c) {
      const float s = sigmoidf_(h[c]);
      v[c] *= s * (1.f + h[c] * (1.f - s));
    }
  } else if (act == EA_ACT_RELU) {
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] *= h[c] > 0.f ? 1.f : 0.f;
  }
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

// internal cross-file helper (norm.hip): reduce_partials with a transposed output
int ea_reduce_partials_tr(int nparts, int n, const float* part, long stride, float* out, int accumulate,
                          int tr_rows, int tr_cols, void* stream);
