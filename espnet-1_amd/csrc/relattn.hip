// Fused multi-head attention with the relative-position term of
// RelPositionMultiHeadedAttention (transformer/attention.py:209-305, rel_shift :237-260)
// and plain MultiHeadedAttention (attention.py:15-111), head dim 64, bf16 operands,
// f32 softmax / accumulation.  See include/espnet_amd.h: ea_attn_fused_fwd / _bwd.
//
//   score[i,j] = ((q_i + u)·k_j + (q_i + v)·p[T-1-i+j]) * scale      (rel-pos; T1 == T2)
//   score[i,j] = q_i·k_j * scale                                     (plain)
//   masked (j >= klen[b], causal j > i), P = softmax, Pd = dropout(P), O = Pd·V.
//
// rel_shift is never materialised: a query block times the band of 64+63 positional rows
// its keys need is ONE MFMA product (BDfull), and BD[i,j] = BDfull[i, 63-i+j] is a
// diagonal gather through LDS.  Forward: one workgroup per (b, h, 64 queries), 4 wave64s
// of 16 query rows, keys streamed in chunks of 64 with an online softmax; only O and the
// row log-sum-exp are written.  Backward: one workgroup per (b, h), wave w owns keys
// [64w, 64w+64) (so dK, dV stay in its registers, no atomics), query tiles of 32 rows;
// the cross-wave dQ sum goes through LDS in fixed order (bit-reproducible); the rel-pos
// gradient is emitted as the band dBD_raw[h][b][i][T-1-i+j] for the linear_pos / q_v
// GEMMs.  Dropout masks use the same counter hash as the unfused path (index
// (z*T1 + i)*T2 + j), regenerated in backward.
#include "common.h"

namespace {

constexpr int DK = 64;     // head dim
constexpr int QB = 64;     // forward: query rows per workgroup
constexpr int KC = 64;     // forward: keys per chunk
constexpr int BQ = 32;     // backward: query rows per tile
constexpr int NWAVE = 4;

// [rows][64] bf16 image, 128-B rows, 16-B chunk c stored at c ^ swz_k(row) (conflict-free
// ds_read_b128 over 16 consecutive rows; 2-way on the transposed reads)
EA_DEV int km_swz(int row) { return (row >> 1) & 7; }
EA_DEV int km_off(int row, int chunk) { return row * 128 + ((chunk ^ km_swz(row)) << 4); }

// A/B fragment (16 rows from r0, k-step ks of 32): row r0 + lane&15, k = 32ks + 8(lane>>4) ..+7
EA_DEV bf16x8 km_frag(const char* img, int r0, int ks, int lane) {
  return *(const bf16x8*)(img + km_off(r0 + (lane & 15), ks * 4 + (lane >> 4)));
}
// Transposed fragment from a [k][n] image: lane holds n = n0 + lane&15 at k = kb + 8(lane>>4) ..+7
// (two ds_read_b64_tr_b16: rows kb+8g+4h+q supplied by lane 4q+p, columns n0+4p..+3)
EA_DEV bf16x8 km_frag_tr(const char* img, int kb, int n0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  const int col = n0 + 4 * p;
  union { bf16x8 v; s16x4 h[2]; } out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = kb + 8 * g + 4 * h + q;
    const char* a = img + km_off(row, col >> 3) + (col & 7) * 2;
    out.h[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(uintptr_t)a);
  }
  return out.v;
}
// Same, with the k rows of the two halves chosen freely: rows k0 + q (half 0), k1 + q (half 1)
EA_DEV bf16x8 km_frag_tr2(const char* img, int k0, int k1, int n0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = n0 + 4 * p;
  union { bf16x8 v; s16x4 h[2]; } out;
  const char* a0 = img + km_off(k0 + q, col >> 3) + (col & 7) * 2;
  const char* a1 = img + km_off(k1 + q, col >> 3) + (col & 7) * 2;
  out.h[0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(uintptr_t)a0);
  out.h[1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(uintptr_t)a1);
  return out.v;
}

// stage rows [r0, r0+nrows) of a row-major bf16 matrix (64 columns at col0) into a km image;
// rows outside [0, rlim) are zero.  `tid`/`nthr` split the 8 chunks x nrows pieces.
EA_DEV void km_stage(char* img, const bf16* __restrict__ src, long ld, int r0, int nrows, int rlim, int tid,
                     int nthr) {
  for (int c = tid; c < nrows * 8; c += nthr) {
    const int row = c >> 3, ch = c & 7;
    const int r = r0 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r >= 0 && r < rlim) v = *(const uint4*)(src + (long)r * ld + ch * 8);
    *(uint4*)(img + km_off(row, ch)) = v;
  }
}
// same with a per-column f32 bias added before rounding to bf16 (q + pos_bias)
EA_DEV void km_stage_bias(char* img, const bf16* __restrict__ src, long ld, int r0, int nrows, int rlim,
                          const float* __restrict__ bias, int tid, int nthr) {
  for (int c = tid; c < nrows * 8; c += nthr) {
    const int row = c >> 3, ch = c & 7;
    const int r = r0 + row;
    union { uint4 u; bf16 e[8]; } t;
    t.u = make_uint4(0u, 0u, 0u, 0u);
    if (r >= 0 && r < rlim) {
      t.u = *(const uint4*)(src + (long)r * ld + ch * 8);
      if (bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) t.e[e] = (bf16)((float)t.e[e] + bias[ch * 8 + e]);
      }
    }
    *(uint4*)(img + km_off(row, ch)) = t.u;
  }
}

EA_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
EA_DEV float max16(float v) {  // max over the 16 lanes of a lane group (same lane>>4)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
EA_DEV float sum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}
EA_DEV void lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct AttnP {
  int B, H, T1, T2;
  const bf16* q; long ldq;   // rows b*T1 + i, head h at column h*64
  const bf16* k; long ldk;   // rows b*T2 + j
  const bf16* v; long ldv;
  const float* bu;           // pos_bias_u [H*64] or null
  const float* bv;           // pos_bias_v [H*64] (rel-pos)
  const bf16* pp; long ldp;  // linear_pos(pos_emb) rows r < 2*T1-1, head h at column h*64, or null
  const long long* klen;     // [B] or null
  int causal;
  float scale, p;
  uint64_t seed;
  const unsigned long long* salt;
  bf16* o; long ldo;         // forward output (bwd: input O)
  float* lse;                // [B*H*T1]
  // backward
  const bf16* dO; long lddo;
  bf16* dq; long lddq;
  bf16* dk; long lddk;
  bf16* dv; long lddv;
  bf16* dbd; long lddbd;     // [h][b][i][lddbd] band gradient (rel-pos), pre-zeroed
};

// ------------------------------------------------------------------------------ forward
constexpr int F_K = 0, F_V = F_K + KC * 128, F_P = F_V + KC * 128;  // K, V chunk, P band (128 rows)
constexpr int F_WS = F_P + 128 * 128;                               // per-wave scratch
constexpr int F_BDLD = 81;                                          // BDfull row stride (floats)
constexpr int F_WSZ = 16 * F_BDLD * 4 + 16 * 128;                   // BD gather + Pd image
constexpr int F_LDS = F_WS + NWAVE * F_WSZ;

template <bool REL>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnP a) {
  __shared__ __attribute__((aligned(16))) char sm[F_LDS];
  const int nqb = (a.T1 + QB - 1) / QB;
  const int z = blockIdx.x / nqb, qb = blockIdx.x % nqb;
  const int b = z / a.H, h = z % a.H;
  const int i0 = qb * QB;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = a.p > 0.f ? ea_salted(a.seed, a.salt) : 0;
  char* ws = sm + F_WS + w * F_WSZ;
  float* bds = (float*)ws;
  char* pimg = ws + 16 * F_BDLD * 4;

  // this wave's 16 query rows as A fragments (q + u, q + v), from a staged image
  bf16x8 qa[2], qv[2];
  {
    char* qimg = sm + F_K;  // borrow the K/V chunk space before the key loop
    const bf16* qsrc = a.q + (long)b * a.T1 * a.ldq + h * DK;
    km_stage_bias(qimg, qsrc, a.ldq, i0, QB, a.T1, a.bu ? a.bu + h * DK : nullptr, tid, 256);
    if (REL) km_stage_bias(qimg + QB * 128, qsrc, a.ldq, i0, QB, a.T1, a.bv + h * DK, tid, 256);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qa[ks] = km_frag(qimg, 16 * w, ks, lane);
      if (REL) qv[ks] = km_frag(qimg + QB * 128, 16 * w, ks, lane);
    }
    __syncthreads();
  }
  f32x4 oacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) oacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float mrun[4], lrun[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrun[r] = -INFINITY; lrun[r] = 0.f; }
  const int ibase = i0 + 16 * w + 4 * g;  // query row of register rr: ibase + rr
  const int kend = a.causal ? min(kl, i0 + QB) : kl;

  for (int j0 = 0; j0 < kend; j0 += KC) {
    km_stage(sm + F_K, a.k + (long)b * a.T2 * a.ldk + h * DK, a.ldk, j0, KC, a.T2, tid, 256);
    km_stage(sm + F_V, a.v + (long)b * a.T2 * a.ldv + h * DK, a.ldv, j0, KC, a.T2, tid, 256);
    const int rb = a.T1 - 1 - (i0 + QB - 1) + j0;  // first positional row of the block's band
    if (REL) km_stage(sm + F_P, a.pp + h * DK, a.ldp, rb, 128, 2 * a.T1 - 1, tid, 256);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) s[t] = mfma(qa[ks], km_frag(sm + F_K, 16 * t, ks, lane), s[t]);
    }
    if (REL) {
      // BDfull (16 x 80) for this wave's rows: band rows 48 - 16w + [0, 80)
      const int pb = 48 - 16 * w;
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        f32x4 bd = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bd = mfma(qv[ks], km_frag(sm + F_P, pb + 16 * t, ks, lane), bd);
#pragma unroll
        for (int r = 0; r < 4; ++r) bds[(4 * g + r) * F_BDLD + 16 * t + lc] = bd[r];
      }
      lds_fence();
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = 4 * g + r, jl = 16 * t + lc;
          s[t][r] += bds[il * F_BDLD + 15 - il + jl];
        }
    }
    // mask, online softmax
    float pv[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ibase + r;
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = j0 + 16 * t + lc;
        const bool ok = j < kl && (!a.causal || j <= i);
        const float x = ok ? s[t][r] * a.scale : -INFINITY;
        pv[t][r] = x;
        mx = fmaxf(mx, x);
      }
      mx = max16(mx);
      const float mnew = fmaxf(mrun[r], mx);
      const float alpha = mnew == -INFINITY ? 1.f : __expf(mrun[r] - mnew);
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float e = pv[t][r] == -INFINITY ? 0.f : __expf(pv[t][r] - mnew);
        pv[t][r] = e;
        sum += e;
      }
      sum = sum16(sum);
      lrun[r] = lrun[r] * alpha + sum;
      mrun[r] = mnew;
#pragma unroll
      for (int t = 0; t < 4; ++t) oacc[t][r] *= alpha;
    }
    // dropout, Pd -> bf16 image (16 rows x 64 keys) -> A fragments
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float e = pv[t][r];
        if (a.p > 0.f) {
          const int i = ibase + r, j = j0 + 16 * t + lc;
          e *= drop_scale(seed, ((uint64_t)z * a.T1 + i) * a.T2 + j, a.p);
        }
        const int il = 4 * g + r, jl = 16 * t + lc;
        *(bf16*)(pimg + km_off(il, jl >> 3) + (jl & 7) * 2) = (bf16)e;
      }
    lds_fence();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = km_frag(pimg, 0, ks, lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) oacc[t] = mfma(pa, km_frag_tr(sm + F_V, 32 * ks, 16 * t, lane), oacc[t]);
    }
    __syncthreads();  // K/V/P images are restaged next chunk
  }
  // normalise, store O (bf16) and the row log-sum-exp
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ibase + r;
    if (i >= a.T1) continue;
    const float inv = lrun[r] > 0.f ? 1.f / lrun[r] : 0.f;
    bf16* orow = a.o + ((long)b * a.T1 + i) * a.ldo + h * DK;
#pragma unroll
    for (int t = 0; t < 4; ++t) orow[16 * t + lc] = (bf16)(oacc[t][r] * inv);
    if (lc == 0) a.lse[(long)z * a.T1 + i] = lrun[r] > 0.f ? mrun[r] + __logf(lrun[r]) : INFINITY;
  }
}

// ------------------------------------------------------------------------------ backward
constexpr int B_KV = 0;                                   // per wave: K_w, V_w images (8 KB each)
constexpr int B_Q = B_KV + NWAVE * 2 * 64 * 128;          // Qu, Qv, dO tile images (32 rows)
constexpr int B_D = B_Q + 3 * BQ * 128;                   // D_i, lse_i (32 each)
constexpr int B_WS = B_D + 2 * BQ * 4;                    // per-wave scratch
constexpr int B_BDLD = 97;                                // BDfull row stride (floats)
constexpr int B_XSZ = BQ * B_BDLD * 4 > BQ * 64 * 4 ? BQ * B_BDLD * 4 : BQ * 64 * 4;  // BD gather | dQ partial
constexpr int B_WSZ = ((B_XSZ + 15) / 16) * 16 + BQ * 128; // + dS image
constexpr int B_BIAS = B_WS + NWAVE * B_WSZ;              // pos_bias_u, pos_bias_v of head h (f32)
constexpr int B_LDS = B_BIAS + 2 * DK * 4;

template <bool REL>
__global__ __launch_bounds__(256, 1) void attn_bwd_kernel(AttnP a) {
  __shared__ __attribute__((aligned(16))) char sm[B_LDS];
  const int z = blockIdx.x;
  const int b = z / a.H, h = z % a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = a.p > 0.f ? ea_salted(a.seed, a.salt) : 0;
  char* kimg = sm + B_KV + w * 2 * 64 * 128;
  char* vimg = kimg + 64 * 128;
  char* quimg = sm + B_Q;
  char* qvimg = quimg + BQ * 128;
  char* doimg = qvimg + BQ * 128;
  float* Dv = (float*)(sm + B_D);
  float* Lv = Dv + BQ;
  char* ws = sm + B_WS + w * B_WSZ;
  float* xs = (float*)ws;
  char* dsimg = ws + ((B_XSZ + 15) / 16) * 16;
  const int jw = 64 * w;  // this wave's keys [jw, jw+64)
  const bool active = jw < kl;

  km_stage(kimg, a.k + (long)b * a.T2 * a.ldk + h * DK, a.ldk, jw, 64, kl, lane, 64);
  km_stage(vimg, a.v + (long)b * a.T2 * a.ldv + h * DK, a.ldv, jw, 64, kl, lane, 64);
  f32x4 dka[4][4], dva[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) dka[m][n] = dva[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // The next query tile's inputs are fetched into registers while the current tile's MFMA
  // work runs (one workgroup per CU, so global latency is otherwise exposed): thread tid
  // owns row tid>>3, 16-B chunk tid&7 of the Q / dO / O tiles (BQ * 8 == 256 pieces).
  static_assert(BQ * 8 == 256, "one 16-B piece per thread");
  const bf16* qsrc = a.q + (long)b * a.T1 * a.ldq + h * DK;
  const bf16* dosrc = a.dO + (long)b * a.T1 * a.lddo + h * DK;
  const bf16* osrc = a.o + (long)b * a.T1 * a.ldo + h * DK;
  const bf16* pbase = REL ? a.pp + h * DK : nullptr;
  const int nqt = (a.T1 + BQ - 1) / BQ;
  const int prow = tid >> 3, pch = tid & 7;
  float* bias_s = (float*)(sm + B_BIAS);  // [u | v], read at each tile's staging
  if (tid < DK) {
    bias_s[tid] = a.bu ? a.bu[h * DK + tid] : 0.f;
    bias_s[DK + tid] = REL ? a.bv[h * DK + tid] : 0.f;
  }  // ordered before the first read by the loop's first __syncthreads
  struct Pre { uint4 q, dO, o; float lse; };
  auto fetch = [&](int i0n, Pre& pr) {
    const int i = i0n + prow;
    pr.q = pr.dO = pr.o = make_uint4(0u, 0u, 0u, 0u);
    pr.lse = INFINITY;
    if (i < a.T1) {
      pr.q = *(const uint4*)(qsrc + (long)i * a.ldq + pch * 8);
      pr.dO = *(const uint4*)(dosrc + (long)i * a.lddo + pch * 8);
      pr.o = *(const uint4*)(osrc + (long)i * a.ldo + pch * 8);
      pr.lse = a.lse[(long)z * a.T1 + i];
    }
  };
  auto tile_on = [&](int i0n) { return active && !(a.causal && jw > i0n + BQ - 1); };
  // BDfull B fragments: band rows rs + 16t + lc, rs = T-1-(i0+31)+jw (clamped rows only
  // feed BDfull entries the diagonal gather never reads)
  auto fetch_band = [&](int i0n, bf16x8 (&pf)[6][2]) {
    const int rs = a.T1 - 1 - (i0n + BQ - 1) + jw;
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const int r = min(max(rs + 16 * t + lc, 0), 2 * a.T1 - 2);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) pf[t][ks] = *(const bf16x8*)(pbase + (long)r * a.ldp + ks * 32 + g * 8);
    }
  };
  Pre pre;
  fetch(0, pre);
  for (int qt = 0; qt < nqt; ++qt) {
    const int i0 = qt * BQ;
    __syncthreads();  // previous tile's readers of the shared images / exchange are done
    {  // stage the Q + u, Q + v, dO images; D_i = dO_i . O_i (8 threads per row), lse_i
      const bool ok = i0 + prow < a.T1;
      union { uint4 u; bf16 e[8]; } x, y, qu, qv;
      x.u = pre.q;
      qu.u = qv.u = make_uint4(0u, 0u, 0u, 0u);
      if (ok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          qu.e[e] = a.bu ? (bf16)((float)x.e[e] + bias_s[pch * 8 + e]) : x.e[e];
          if (REL) qv.e[e] = (bf16)((float)x.e[e] + bias_s[DK + pch * 8 + e]);
        }
      }
      *(uint4*)(quimg + km_off(prow, pch)) = qu.u;
      if (REL) *(uint4*)(qvimg + km_off(prow, pch)) = qv.u;
      *(uint4*)(doimg + km_off(prow, pch)) = pre.dO;
      x.u = pre.dO;
      y.u = pre.o;
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d += (float)x.e[e] * (float)y.e[e];
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) d += __shfl_xor(d, o, 64);
      if (pch == 0) {
        Dv[prow] = d;
        Lv[prow] = pre.lse;
      }
    }
    __syncthreads();
    if (qt + 1 < nqt) fetch(i0 + BQ, pre);
    if (tile_on(i0)) {
      // band fragments issued before the AC MFMAs so their latency hides under them
      bf16x8 pfc[6][2];
      if (REL) fetch_band(i0, pfc);
      // scores (32 queries x 64 keys): s[mi][t], lane = key column 16t + lc, rows 16mi + 4g + r
      f32x4 s[2][4];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s[mi][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            s[mi][t] = mfma(km_frag(quimg, 16 * mi, ks, lane), km_frag(kimg, 16 * t, ks, lane), s[mi][t]);
        }
      if (REL) {
        // BDfull (32 x 96): band rows rs + [0, 96), B fragments prefetched into pfc
        bf16x8 bq[2][2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) bq[mi][ks] = km_frag(qvimg, 16 * mi, ks, lane);
#pragma unroll
        for (int t = 0; t < 6; ++t) {
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            f32x4 bd = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) bd = mfma(bq[mi][ks], pfc[t][ks], bd);
#pragma unroll
            for (int r2 = 0; r2 < 4; ++r2) xs[(16 * mi + 4 * g + r2) * B_BDLD + 16 * t + lc] = bd[r2];
          }
        }
        lds_fence();
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r2 = 0; r2 < 4; ++r2) {
              const int il = 16 * mi + 4 * g + r2, jl = 16 * t + lc;
              s[mi][t][r2] += xs[il * B_BDLD + (BQ - 1 - il) + jl];
            }
        lds_fence();
      }
      // dPd = dO . V_w^T
      f32x4 dp[2][4];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          dp[mi][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            dp[mi][t] = mfma(km_frag(doimg, 16 * mi, ks, lane), km_frag(vimg, 16 * t, ks, lane), dp[mi][t]);
        }
      // P, Pd, dS (scaled): in place of s (-> dS) and dp (-> Pd)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2) {
          const int il = 16 * mi + 4 * g + r2, i = i0 + il;
          const float L = Lv[il], D = Dv[il];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int j = jw + 16 * t + lc;
            const bool ok = i < a.T1 && j < kl && (!a.causal || j <= i);
            const float P = ok ? __expf(s[mi][t][r2] * a.scale - L) : 0.f;
            float keep = 1.f;
            if (a.p > 0.f) keep = drop_scale(seed, ((uint64_t)z * a.T1 + i) * a.T2 + j, a.p);
            const float dP = dp[mi][t][r2] * keep;
            s[mi][t][r2] = P * (dP - D) * a.scale;  // d(raw score AC+BD)
            dp[mi][t][r2] = P * keep;               // Pd
          }
        }
      // dV_w += Pd^T dO, dK_w += dS^T Qu: A = the C-layout tile read as (key, 8 queries
      // {4g..4g+3, 16+4g..16+4g+3}); B = dO / Qu rows in the same order (transposed reads)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        union { bf16x8 v; bf16 e[8]; } ap, as;
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2) {
          ap.e[r2] = (bf16)dp[0][t][r2];
          ap.e[4 + r2] = (bf16)dp[1][t][r2];
          as.e[r2] = (bf16)s[0][t][r2];
          as.e[4 + r2] = (bf16)s[1][t][r2];
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          dva[t][n] = mfma(ap.v, km_frag_tr2(doimg, 4 * g, 16 + 4 * g, 16 * n, lane), dva[t][n]);
          dka[t][n] = mfma(as.v, km_frag_tr2(quimg, 4 * g, 16 + 4 * g, 16 * n, lane), dka[t][n]);
        }
      }
      // dS (bf16) image [32 queries][64 keys] -> dQ partial = dS . K_w
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) {
            const int il = 16 * mi + 4 * g + r2, jl = 16 * t + lc;
            *(bf16*)(dsimg + km_off(il, jl >> 3) + (jl & 7) * 2) = (bf16)s[mi][t][r2];
          }
      lds_fence();
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 kb0 = km_frag_tr(kimg, 0, 16 * n, lane), kb1 = km_frag_tr(kimg, 32, 16 * n, lane);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          f32x4 dq = (f32x4){0.f, 0.f, 0.f, 0.f};
          dq = mfma(km_frag(dsimg, 16 * mi, 0, lane), kb0, dq);
          dq = mfma(km_frag(dsimg, 16 * mi, 1, lane), kb1, dq);
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) xs[(16 * mi + 4 * g + r2) * 64 + 16 * n + lc] = dq[r2];
        }
      }
      // rel-pos band gradient dBD_raw[h][b][i][T-1-i+j] = dS
      if (REL) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) {
            const int i = i0 + 16 * mi + 4 * g + r2;
            if (i >= a.T1) continue;
            bf16* drow = a.dbd + (((long)h * a.B + b) * a.T1 + i) * a.lddbd + (a.T1 - 1 - i);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int j = jw + 16 * t + lc;
              if (j < kl) drow[j] = (bf16)s[mi][t][r2];
            }
          }
      }
    } else {
      for (int e = lane; e < BQ * 64; e += 64) xs[e] = 0.f;
    }
    __syncthreads();
    // dQ = sum over the waves' partials in fixed order
    for (int e = tid; e < BQ * 64; e += 256) {
      const int il = e >> 6, c = e & 63;
      const int i = i0 + il;
      float acc = 0.f;
#pragma unroll
      for (int v = 0; v < NWAVE; ++v) acc += ((const float*)(sm + B_WS + v * B_WSZ))[e];
      if (i < a.T1) a.dq[((long)b * a.T1 + i) * a.lddq + h * DK + c] = (bf16)acc;
    }
  }
  // dK_w, dV_w: rows = keys jw + 16t + 4g + r, columns 16n + lc
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jw + 16 * t + 4 * g + r;
      if (j >= a.T2) continue;
      bf16* dkr = a.dk + ((long)b * a.T2 + j) * a.lddk + h * DK;
      bf16* dvr = a.dv + ((long)b * a.T2 + j) * a.lddv + h * DK;
      const bool ok = j < kl;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        dkr[16 * n + lc] = (bf16)(ok ? dka[t][n][r] : 0.f);
        dvr[16 * n + lc] = (bf16)(ok ? dva[t][n][r] : 0.f);
      }
    }
}

AttnP make_p(int B, int H, int T1, int T2, const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
             const float* bu, const float* bv, const void* pp, long ldp, const long long* klen, int causal, float scale,
             float p, unsigned long long seed) {
  AttnP a{};
  a.B = B; a.H = H; a.T1 = T1; a.T2 = T2;
  a.q = (const bf16*)q; a.ldq = ldq; a.k = (const bf16*)k; a.ldk = ldk; a.v = (const bf16*)v; a.ldv = ldv;
  a.bu = bu; a.bv = bv; a.pp = (const bf16*)pp; a.ldp = ldp; a.klen = klen; a.causal = causal;
  a.scale = scale; a.p = p; a.seed = seed; a.salt = ea_g_rng_salt;
  return a;
}

}  // namespace

extern "C" int ea_attn_fused_fwd(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                                 long ldk, const void* v, long ldv, const float* bu, const float* bv,
                                 const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                                 unsigned long long seed, void* o, long ldo, float* lse, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(dk == DK && B >= 1 && H >= 1 && T1 >= 1 && T2 >= 1);
  EA_CHECK_ARG(!pp || (T1 == T2 && bv != nullptr));
  EA_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && (!pp || ldp % 8 == 0));
  AttnP a = make_p(B, H, T1, T2, q, ldq, k, ldk, v, ldv, bu, bv, pp, ldp, klen, causal, scale, p, seed);
  a.o = (bf16*)o; a.ldo = ldo; a.lse = lse;
  dim3 grid(B * H * ((T1 + QB - 1) / QB));
  if (pp) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_attn_fused_bwd(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                                 long ldk, const void* v, long ldv, const float* bu, const float* bv,
                                 const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                                 unsigned long long seed, const void* o, long ldo, const float* lse, const void* dO,
                                 long lddo, void* dq, long lddq, void* dkout, long lddk, void* dvout, long lddv,
                                 void* dbd, long lddbd, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(dk == DK && B >= 1 && H >= 1 && T1 >= 1 && T2 >= 1 && T2 <= NWAVE * 64);
  EA_CHECK_ARG(!pp || (T1 == T2 && bv != nullptr && dbd != nullptr && lddbd >= 2 * T1 - 1));
  EA_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 8 == 0 && lddo % 8 == 0);
  AttnP a = make_p(B, H, T1, T2, q, ldq, k, ldk, v, ldv, bu, bv, pp, ldp, klen, causal, scale, p, seed);
  a.o = (bf16*)o; a.ldo = ldo; a.lse = (float*)lse;
  a.dO = (const bf16*)dO; a.lddo = lddo;
  a.dq = (bf16*)dq; a.lddq = lddq; a.dk = (bf16*)dkout; a.lddk = lddk; a.dv = (bf16*)dvout; a.lddv = lddv;
  a.dbd = (bf16*)dbd; a.lddbd = lddbd;
  dim3 grid(B * H);
  if (pp) hipLaunchKernelGGL(attn_bwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(attn_bwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  EA_LAUNCH_CHECK();
  return 0;
}
