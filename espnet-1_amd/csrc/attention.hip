// Masked softmax + dropout of multi-head attention (transformer/attention.py:63-93), with
// the relative-position term of RelPositionMultiHeadedAttention (attention.py:262-305):
//   score[i,j] = (AC[i,j] + BD_raw[i, T1-1-i+j]) / sqrt(d_k)
// rel_shift (attention.py:237-260) is the index law above (bit-exact), so
// the shifted (T1,T1) matrix is never materialised: the softmax row kernel gathers the
// band, and the backward scatters dS straight into dBD_raw.
// Masks: key j valid iff j < klen[b] (and j <= i when causal) — the padding mask of
// make_pad_mask + subsequent_mask; a fully-masked row gives P = 0 like the reference's
// masked_fill(min) -> softmax -> masked_fill(0).
#include "common.h"

namespace {

struct SmP {
  int B, H, T1, T2;
  float scale;
  const float* S; long ldS;        // [z][i][ldS], z = b*H + h
  const float* BD; long ldBD;      // [h][b][i][ldBD] or null
  const long long* klen;           // [B] or null
  int causal;
  float p; uint64_t seed; const unsigned long long* salt;
  float* P; long ldP;              // f32 softmax [z][i][ldP] (may alias S)
  void* Pd; int pd_dtype; long ldPd;  // dropout(P) in compute dtype
};

template <int MAXE>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(SmP a) {
  const int lane = threadIdx.x & 63;
  const long rows = (long)a.B * a.H * a.T1;
  const long nw = (long)gridDim.x * 4;
  for (long r = blockIdx.x * 4L + (threadIdx.x >> 6); r < rows; r += nw) {
    const int i = (int)(r % a.T1);
    const long z = r / a.T1;
    const int b = (int)(z / a.H), h = (int)(z % a.H);
    const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
    const int lim = a.causal ? min(kl, i + 1) : kl;
    const float* srow = a.S + r * a.ldS;
    const float* brow = a.BD ? a.BD + (((long)h * a.B + b) * a.T1 + i) * a.ldBD + (a.T1 - 1 - i) : nullptr;
    float v[MAXE];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int j = e * 64 + lane;
      float s = -INFINITY;
      if (j < lim) {
        s = srow[j];
        if (brow) s += brow[j];
        s *= a.scale;
      }
      v[e] = s;
      mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int j = e * 64 + lane;
      const float t = j < lim ? __expf(v[e] - mx) : 0.f;
      v[e] = t;
      sum += t;
    }
    sum = wave_sum(sum);
    const float inv = lim > 0 ? 1.f / sum : 0.f;
    float* prow = a.P + r * a.ldP;
    const uint64_t base = (uint64_t)r * a.T2;
    const uint64_t seed = ea_salted(a.seed, a.salt);
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int j = e * 64 + lane;
      if (j < a.T2) {
        const float pj = v[e] * inv;
        prow[j] = pj;
        const float pd = a.p > 0.f ? pj * attn_drop_scale(seed, r, a.T2, j, a.p) : pj;
        store_from_f(a.Pd, r * a.ldPd + j, a.pd_dtype, pd);
      }
    }
  }
}

struct SmBP {
  int B, H, T1, T2;
  float scale;
  const float* dPd; long ldd;      // d(dropout(P)) [z][i][ldd] f32
  const float* P; long ldP;
  float p; uint64_t seed; const unsigned long long* salt;
  void* dS; int ds_dtype; long ldS;    // scale * dS [z][i][ldS]
  void* dBD; long ldBD; int nbd;       // [h][b][i][ldBD], rows of nbd = 2*T1-1 entries, or null
};

template <int MAXE>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(SmBP a) {
  __shared__ float stash[4][64 * MAXE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long rows = (long)a.B * a.H * a.T1;
  const long nw = (long)gridDim.x * 4;
  for (long r = blockIdx.x * 4L + w; r < rows; r += nw) {
    const int i = (int)(r % a.T1);
    const long z = r / a.T1;
    const int b = (int)(z / a.H), h = (int)(z % a.H);
    const float* drow = a.dPd + r * a.ldd;
    const float* prow = a.P + r * a.ldP;
    const uint64_t base = (uint64_t)r * a.T2;
    const uint64_t seed = ea_salted(a.seed, a.salt);
    float pv[MAXE], dv[MAXE];
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int j = e * 64 + lane;
      if (j < a.T2) {
        pv[e] = prow[j];
        float d = drow[j];
        if (a.p > 0.f) d *= attn_drop_scale(seed, r, a.T2, j, a.p);
        dv[e] = d;
        dot += pv[e] * d;
      } else {
        pv[e] = dv[e] = 0.f;
      }
    }
    dot = wave_sum(dot);
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int j = e * 64 + lane;
      if (j < a.T2) {
        const float g = pv[e] * (dv[e] - dot) * a.scale;
        store_from_f(a.dS, r * a.ldS + j, a.ds_dtype, g);
        stash[w][j] = g;
      }
    }
    if (a.dBD) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const long orow = (((long)h * a.B + b) * a.T1 + i) * a.ldBD;
      const int off = a.T1 - 1 - i;
      for (int q = lane; q < a.nbd; q += 64) {
        const int j = q - off;
        const float g = (j >= 0 && j < a.T2) ? stash[w][j] : 0.f;
        store_from_f(a.dBD, orow + q, a.ds_dtype, g);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

}  // namespace

#define EA_SM_DISPATCH(KER, T2, ARG)                                                          \
  do {                                                                                        \
    dim3 grid(ea_grid_cap(ea_cdiv((long)B * H * T1, 4), 4096)), blk(256);                     \
    hipStream_t st = (hipStream_t)stream;                                                     \
    if (T2 <= 64) hipLaunchKernelGGL(KER<1>, grid, blk, 0, st, ARG);                          \
    else if (T2 <= 128) hipLaunchKernelGGL(KER<2>, grid, blk, 0, st, ARG);                    \
    else if (T2 <= 256) hipLaunchKernelGGL(KER<4>, grid, blk, 0, st, ARG);                    \
    else if (T2 <= 512) hipLaunchKernelGGL(KER<8>, grid, blk, 0, st, ARG);                    \
    else if (T2 <= 1024) hipLaunchKernelGGL(KER<16>, grid, blk, 0, st, ARG);                  \
    else if (T2 <= 2048) hipLaunchKernelGGL(KER<32>, grid, blk, 0, st, ARG);                  \
    else return EA_ERR_BAD_ARG;                                                               \
  } while (0)

extern "C" int ea_attn_softmax_fwd(int B, int H, int T1, int T2, float scale, const float* S, long ldS,
                                   const float* BD, long ldBD, const long long* klen, int causal, float p,
                                   unsigned long long seed, float* P, long ldP, void* Pd, int pd_dtype,
                                   long ldPd, void* stream) {
  EA_ENTRY();
  if ((long)B * H * T1 == 0) return 0;
  if (BD) EA_CHECK_ARG(T1 == T2);
  SmP a{B, H, T1, T2, scale, S, ldS, BD, ldBD, klen, causal, p, (uint64_t)seed, ea_g_rng_salt, P, ldP, Pd, pd_dtype, ldPd};
  EA_SM_DISPATCH(softmax_fwd_kernel, T2, a);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_attn_softmax_bwd(int B, int H, int T1, int T2, float scale, const float* dPd, long ldd,
                                   const float* P, long ldP, float p, unsigned long long seed, void* dS,
                                   int ds_dtype, long ldS, void* dBD, long ldBD, void* stream) {
  EA_ENTRY();
  if ((long)B * H * T1 == 0) return 0;
  if (dBD) EA_CHECK_ARG(T1 == T2);
  SmBP a{B, H, T1, T2, scale, dPd, ldd, P, ldP, p, (uint64_t)seed, ea_g_rng_salt, dS, ds_dtype, ldS, dBD, ldBD, 2 * T1 - 1};
  EA_SM_DISPATCH(softmax_bwd_kernel, T2, a);
  EA_LAUNCH_CHECK();
  return 0;
}
