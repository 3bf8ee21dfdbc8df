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
#include <stdlib.h>

// timing experiments only (scripts/build_def.py): bit 1 no dBD stores, 2 no d(q+v) term, 4 K/V/band
// staged for the first chunk only, 8 no BD gather in attn_bwdq
#ifndef ATTN_EXP
#define ATTN_EXP 0
#endif

namespace {

constexpr int DK = 64;     // head dim
constexpr int QB = 64;     // forward: query rows per workgroup
constexpr int KC = 64;     // forward: keys per chunk
constexpr int NWAVE = 4;

// [rows][64] bf16 image, 128-B rows, 16-B chunk c stored at c ^ km_swz(row): conflict-free for
// every access kind the kernels make — ds_read_b128 fragments over 16 consecutive rows (lane
// row r0 + (L & 15), chunk 4ks + (L >> 4)) and the ds_read_b64_tr_b16 fragments, whose 32-lane
// halves read chunk pair n0/8 + {0, 1} of rows {r, r+2, r+8, r+10} (km_tr_rows, km_frag_tr)
// or {r, r+2, r+4, r+6} (km_tr2_asm): each such row set gets four different chunk pairs (found
// by exhaustive search over 16-row swizzles; round 4's (row >> 1) & 7 was 2-way on both)
EA_DEV int km_swz(int row) { return (row & 6) ^ (((row >> 3) & 1) * 5); }
// a lane's LDS-DMA slot swizzle within an 8-row group (km_dma8u): rows ir + (L >> 3), ir % 8 == 0
EA_DEV int km_chx(int lane) { return (lane & 7) ^ ((lane >> 3) & 6); }
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

// Stage rows [r0, r0+NR) of a row-major bf16 matrix (64 columns) into a km image: thread tid
// owns 16-B chunk tid&7 of rows (tid>>3) + 32u (a 256-thread block); rows outside [0, rlim)
// are zero.  gsrc = this thread's element (row tid>>3, chunk tid&7) of the matrix at row 0, so
// each piece costs one uniform row offset; km_off(row + 32u, c) = km_off(row, c) + 4096u.
// KmRows splits it into the global loads (into registers) and the LDS stores, so a loop can
// fetch the next chunk while it computes on the current one.
template <int NR>
struct KmRows {
  static constexpr int NU = (NR + 31) / 32;
  uint4 v[NU];
  EA_DEV void load(const bf16* gsrc, long ld, int r0, int rlim, int tid) {
    const int row = tid >> 3;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int r = r0 + row + 32 * u;
      v[u] = make_uint4(0u, 0u, 0u, 0u);
      if ((NR % 32 == 0 || row + 32 * u < NR) && r >= 0 && r < rlim) v[u] = *(const uint4*)(gsrc + (long)(r0 + 32 * u) * ld);
    }
  }
  EA_DEV void store(char* img, int tid) const {
    const int lofs = km_off(tid >> 3, tid & 7);
#pragma unroll
    for (int u = 0; u < NU; ++u)
      if (NR % 32 == 0 || (tid >> 3) + 32 * u < NR) *(uint4*)(img + lofs + 4096 * u) = v[u];
  }
};
template <int NR>
EA_DEV void stage_km(char* img, const bf16* gsrc, long ld, int r0, int rlim, int tid) {
  KmRows<NR> t;
  t.load(gsrc, ld, r0, rlim, tid);
  t.store(img, tid);
}

EA_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
// 16-lane (lane >> 4 group) reductions with DPP: swap within pairs, within quads, then the
// half-row and row mirrors; every lane ends with the same value (each step is a commutative
// pairing)
template <int CTRL>
EA_DEV float dppf(float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false)); }
EA_DEV float max16(float v) {
  v = fmaxf(v, dppf<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dppf<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dppf<0x141>(v));  // row_half_mirror
  return fmaxf(v, dppf<0x140>(v));  // row_mirror
}
EA_DEV float sum16(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  return v + dppf<0x140>(v);
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
  bf16* dbd; long lddbd;     // [h][b][i][lddbd] band gradient (rel-pos), written in full
  float* bias_part; long ldpart;  // [2][B*ceil(T1/64)][ldpart] column sums of dQ_u, dQ_v
  bf16* qv_out; long ldqv;   // q + pos_bias_v (rel-pos), rows b*T1 + i, or null
  int flags;                 // bit 0: dq includes the rel-pos term dBD.p
  float* wsD;                // backward workspace: D_i = dO_i.O_i [z*T1 + i]
  bf16* wsQu; long ldqu;     //   q + u rows (b*T1 + i, head columns), written by attn_bwdq
  bf16* wsQv; long ldqvw;    //   q + v rows (rel-pos: qv_out when given, else workspace)
  uint32_t* dmask; int ldm;  // dropout keep bits [z*T1 + i][ldm words], bit j&31 of word j>>5:
                             // written by the forward, read by the backward (else rehashed)
  char* wsDummy;             // 1 KiB sink for the pipelined dQ pass's out-of-range dbd stores
};
// ldm >= 2 * ceil(T2 / 64): a 64-key chunk is the word pair (j0 >> 5, +1)

// Shifted dbd layout of the pipelined dQ pass (flags bit 1): logical column r of every row at
// physical column r + shift, shift >= 15 with (T1 + shift) % 8 == 0, so that the band window of
// any 16-row wave starts on a 16-B boundary; row stride ea_attn_dbd_ld(T1) (multiple of 8).
__host__ __device__ inline int ea_attn_dbd_shift_dev(int T1) { return 15 + ((8 - (T1 + 15) % 8) % 8); }
__host__ __device__ inline long ea_attn_dbd_ld(int T1) { return (2L * T1 - 1 + ea_attn_dbd_shift_dev(T1) + 7) / 8 * 8; }

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
  // dropout pair index of (row, key 0) for the two rows this lane hashes: the even lane of a
  // pair hashes rows 0 and 2 of its group, the odd lane rows 1 and 3 (see attn_pair)
  const int odd = lc & 1;
  const uint64_t npair = (uint64_t)((a.T2 + 1) >> 1);
  const uint64_t prA = ((uint64_t)z * a.T1 + ibase + odd) * npair, prB = prA + 2 * npair;
  const long pofs = (long)(tid >> 3), cofs = h * DK + (tid & 7) * 8;  // stage_km thread bases
  const bf16* gK = a.k + ((long)b * a.T2 + pofs) * a.ldk + cofs;
  const bf16* gV = a.v + ((long)b * a.T2 + pofs) * a.ldv + cofs;
  const bf16* gP = REL ? a.pp + pofs * a.ldp + cofs : nullptr;

  // K / V / band rows of chunk j0 + KC are fetched into registers while chunk j0 computes
  KmRows<KC> pk, pv_;
  KmRows<128> pp;
  auto fetch = [&](int jn) {
    pk.load(gK, a.ldk, jn, a.T2, tid);
    pv_.load(gV, a.ldv, jn, a.T2, tid);
    if (REL) pp.load(gP, a.ldp, a.T1 - 1 - (i0 + QB - 1) + jn, 2 * a.T1 - 1, tid);  // the block's band
  };
  if (kend > 0) fetch(0);
  for (int j0 = 0; j0 < kend; j0 += KC) {
    pk.store(sm + F_K, tid);
    pv_.store(sm + F_V, tid);
    if (REL) pp.store(sm + F_P, tid);
    __syncthreads();
    if (j0 + KC < kend) fetch(j0 + KC);
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
    // dropout (keep bits -> dmask for the backward), Pd -> bf16 image (16 rows x 64 keys)
    if (a.p > 0.f) {
      const uint32_t key = ea_seed_key(seed), thr = ea_drop_thr(a.p);
      const float sc = 1.f / (1.f - a.p);
      uint64_t bal[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint64_t jp = (uint64_t)((j0 + 16 * t + lc) >> 1);  // shared by the lane pair
        const uint32_t hA = ea_pair_hash(key, prA + jp), hB = ea_pair_hash(key, prB + jp);
        const uint32_t pA = (uint32_t)__builtin_amdgcn_mov_dpp((int)hA, 0xB1, 0xF, 0xF, false);
        const uint32_t pB = (uint32_t)__builtin_amdgcn_mov_dpp((int)hB, 0xB1, 0xF, 0xF, false);
        const uint32_t h[4] = {odd ? pA : hA, odd ? hA : pA, odd ? pB : hB, odd ? hB : pB};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool kept = (odd ? h[r] >> 16 : h[r] & 0xffffu) >= thr;  // key parity = lane parity
          pv[t][r] *= kept ? sc : 0.f;
          bal[t][r] = __ballot(kept);
        }
      }
      if (a.dmask && lc < 2) {  // lane lc = u writes word u of each of its group's 4 rows
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = ibase + r;
          const uint64_t lo = lc ? bal[2][r] : bal[0][r], hi = lc ? bal[3][r] : bal[1][r];
          const uint32_t word = (uint32_t)((lo >> (16 * g)) & 0xffffu) | ((uint32_t)((hi >> (16 * g)) & 0xffffu) << 16);
          if (i < a.T1) a.dmask[((long)z * a.T1 + i) * a.ldm + (j0 >> 5) + lc] = word;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 4 * g + r, jl = 16 * t + lc;
        *(bf16*)(pimg + km_off(il, jl >> 3) + (jl & 7) * 2) = (bf16)pv[t][r];
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
// Two launches of many workgroups each; no cross-workgroup sums, so results are
// bit-reproducible.  Both recompute S (+ the rel-pos band), P = exp(S*scale - lse) from the
// forward's row log-sum-exp, dP = dO.V^T and dS = P (dP keep - D) scale with D_i = dO_i.O_i;
// dropout keep factors come from the forward's bit mask (or the counter hash without one).
//  * attn_bwdq: one workgroup per (b, h, 64 queries), the forward kernel's layout (wave w owns
//    16 query rows, keys in chunks of 64).  dQ = dS.K, plus (rel-pos) dS laid onto its band
//    times the positional rows: d(q+v) = dBD.p, so the caller's band GEMM and add disappear.
//    Emits the band gradient dBD rows in full (zeros off the band: no memset) for the
//    linear_pos weight gradient, and per-workgroup column sums of both dQ terms
//    (pos_bias_u / pos_bias_v gradients, reduced by the caller in fixed order).
//  * attn_bwdkv: one workgroup per (b, h, 64 keys), wave w owns 16 keys; 32-query tiles are
//    staged once per workgroup (next tile prefetched into registers during the MFMA work) and
//    dV = Pd^T.dO, dK = dS^T.(Q+u) stay in registers.
// Masked rows / keys give P = 0 and so dS = 0.
constexpr int BQ = 32;  // attn_bwdkv query tile
constexpr float LOG2E = 1.4426950408889634f;

// dS^T image [64 keys][16 queries] bf16 (32-B rows), written 4 queries (8 B) at a time from
// the C layout; read back as A fragments (16 queries x 32 keys) with transposed reads
EA_DEV bf16x8 dst_frag(const char* img, int kb, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  union { bf16x8 v; s16x4 h[2]; } out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const char* a = img + (kb + 8 * g + 4 * h + q) * 32 + p * 8;
    out.h[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(uintptr_t)a);
  }
  return out.v;
}
// dS band image [16 queries][96 band columns] bf16, 192-B rows, 16-B chunk c of row r at
// c ^ ((r >> 2) & 3) (conflict-free b128 A-fragment reads)
EA_DEV int band_off(int r, int c) { return r * 192 + ((((c >> 3) ^ ((r >> 2) & 3))) << 4) + (c & 7) * 2; }
EA_DEV bf16x8 band_frag(const char* img, int ks, int lane) {
  const int r = lane & 15, c = ks * 4 + (lane >> 4);
  return *(const bf16x8*)(img + r * 192 + ((c ^ ((r >> 2) & 3)) << 4));
}
EA_DEV uint32_t pack_bf16x2(float lo, float hi) {
  union { bf16 h[2]; uint32_t u; } x;
  x.h[0] = (bf16)lo;
  x.h[1] = (bf16)hi;
  return x.u;
}

// attn_bwdq shared memory
constexpr int Q_K = 0, Q_V = Q_K + KC * 128, Q_P = Q_V + KC * 128;  // K, V chunk, band (144 rows)
constexpr int Q_D = Q_P + 144 * 128;                                // D_i, lse_i (64 each)
constexpr int Q_WS = Q_D + 2 * QB * 4;                              // per-wave scratch
constexpr int Q_XSZ = 16 * F_BDLD * 4;                              // BD gather | dS band image
constexpr int Q_WSZ = Q_XSZ + 64 * 32;                              // + dS^T image
constexpr int Q_RED = Q_WS + NWAVE * Q_WSZ;                         // column-sum exchange
constexpr int Q_LDS = Q_RED + 2 * NWAVE * DK * 4;
static_assert(Q_XSZ >= 16 * 192 && Q_XSZ % 16 == 0, "band image fits the gather scratch");
static_assert(3 * QB * 128 <= Q_D, "setup images fit the chunk space");

// rows [r0, r0+nrows) of (src [+ bias]) into a km image, also written to out (if non-null)
EA_DEV void km_stage_out(char* img, const bf16* __restrict__ src, long ld, int r0, int nrows, int rlim,
                         const float* __restrict__ bias, bf16* out, long ldout, int tid, int nthr) {
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
      if (out) *(uint4*)(out + (long)r * ldout + ch * 8) = t.u;
    }
    *(uint4*)(img + km_off(row, ch)) = t.u;
  }
}

template <bool REL>
__global__ __launch_bounds__(256, 2) void attn_bwdq_kernel(AttnP a) {
  __shared__ __attribute__((aligned(16))) char sm[Q_LDS];
  const int nqb = (a.T1 + QB - 1) / QB;
  const int z = blockIdx.x / nqb, qb = blockIdx.x % nqb;
  const int b = z / a.H, h = z % a.H;
  const int i0 = qb * QB;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = a.p > 0.f ? ea_salted(a.seed, a.salt) : 0;
  const bool with_dqv = REL && (a.flags & 1) && !(ATTN_EXP & 2);
  char* ws = sm + Q_WS + w * Q_WSZ;
  float* bds = (float*)ws;
  char* band = ws;                // dS on its band (after the gather has read bds)
  char* dst = ws + Q_XSZ;
  float* Dv = (float*)(sm + Q_D);
  float* Lv = Dv + QB;

  // this wave's 16 rows of Q + u, Q + v and dO as A fragments; D_i and lse_i
  bf16x8 qa[2], qv[2], doa[2];
  {
    // q + u, q + v also to the workspace / qv_out for attn_bwdkv (and the linear_pos gradient)
    const bf16* qsrc = a.q + (long)b * a.T1 * a.ldq + h * DK;
    km_stage_out(sm, qsrc, a.ldq, i0, QB, a.T1, a.bu ? a.bu + h * DK : nullptr,
                 a.wsQu + (long)b * a.T1 * a.ldqu + h * DK, a.ldqu, tid, 256);
    if (REL)
      km_stage_out(sm + QB * 128, qsrc, a.ldq, i0, QB, a.T1, a.bv + h * DK,
                   a.wsQv + (long)b * a.T1 * a.ldqvw + h * DK, a.ldqvw, tid, 256);
    km_stage(sm + 2 * QB * 128, a.dO + (long)b * a.T1 * a.lddo + h * DK, a.lddo, i0, QB, a.T1, tid, 256);
    {  // D_i = dO_i . O_i: 4 threads per row, 16 columns each
      const int row = tid >> 2, qd = tid & 3, i = i0 + row;
      float d = 0.f;
      if (i < a.T1) {
        const bf16* dr = a.dO + ((long)b * a.T1 + i) * a.lddo + h * DK + qd * 16;
        const bf16* orow = a.o + ((long)b * a.T1 + i) * a.ldo + h * DK + qd * 16;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          union { uint4 u; bf16 e[8]; } x, y;
          x.u = *(const uint4*)(dr + hf * 8);
          y.u = *(const uint4*)(orow + hf * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) d += (float)x.e[e] * (float)y.e[e];
        }
      }
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      if (qd == 0) {
        Dv[row] = d;
        Lv[row] = i < a.T1 ? a.lse[(long)z * a.T1 + i] * LOG2E : INFINITY;
        if (i < a.T1) a.wsD[(long)z * a.T1 + i] = d;
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qa[ks] = km_frag(sm, 16 * w, ks, lane);
      if (REL) qv[ks] = km_frag(sm + QB * 128, 16 * w, ks, lane);
      doa[ks] = km_frag(sm + 2 * QB * 128, 16 * w, ks, lane);
    }
  }
  const int ibase = i0 + 16 * w + 4 * g;  // query row of register r: ibase + r
  float Dr[4], Lr[4];
  int lim[4];  // key j of row r is valid iff j < lim[r]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ibase + r;
    Dr[r] = Dv[16 * w + 4 * g + r];
    Lr[r] = Lv[16 * w + 4 * g + r];
    lim[r] = i < a.T1 ? (a.causal ? min(kl, i + 1) : kl) : 0;
  }
  const float sl2 = a.scale * LOG2E;
  const int kend = a.causal ? min(kl, i0 + QB) : kl;
  const int nch = (kend + KC - 1) / KC;
  bf16* dbd_h = REL && a.dbd && !(ATTN_EXP & 1) ? a.dbd + ((long)h * a.B + b) * a.T1 * a.lddbd : nullptr;
  if (dbd_h) {
    // zeros off the part of each row the chunk loop writes (r < T-1-i, r >= T-1-i+jcov), in
    // whole 8-column segments (lddbd % 8 == 0, 16-B aligned rows): a segment straddling the
    // band edge is zeroed in full and its band columns are rewritten by this same wave's chunk
    // stores, which the loop's first __syncthreads (vmcnt(0)) orders after these
    const int jcov = min(a.T2, nch * KC);
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (int il = 0; il < 16; ++il) {
      const int i = i0 + 16 * w + il;
      if (i >= a.T1) break;
      bf16* drow = dbd_h + (long)i * a.lddbd;
      const int lo = a.T1 - 1 - i, hi = lo + jcov;
      for (int c0 = 8 * lane; c0 < a.lddbd; c0 += 512)
        if (c0 < lo || c0 + 8 > hi) *(uint4*)(drow + c0) = zero;
    }
  }
  const bool use_mask = a.p > 0.f && a.dmask != nullptr;
  const uint32_t* mrow = a.dmask + ((long)z * a.T1 + ibase) * a.ldm;  // rows ibase + r (< T1)
  const float dsc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;

  const long pofs = (long)(tid >> 3), cofs = h * DK + (tid & 7) * 8;  // stage_km thread bases
  const bf16* gK = a.k + ((long)b * a.T2 + pofs) * a.ldk + cofs;
  const bf16* gV = a.v + ((long)b * a.T2 + pofs) * a.ldv + cofs;
  const bf16* gP = REL ? a.pp + pofs * a.ldp + cofs : nullptr;
  f32x4 dqu[4], dqv[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) dqu[n] = dqv[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int pb = 48 - 16 * w;  // this wave's first band row in the chunk's band image
  for (int j0 = 0; j0 < kend; j0 += KC) {
    // keep words of rows ibase + r for keys j0 .. j0+63 (bit 16(t&1) + lc of word t>>1): the
    // forward's mask, else rebuilt from the counter hash (this lane's bits only), else all kept
    uint2 mw[4];
    if (use_mask) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        mw[r] = ibase + r < a.T1 ? *(const uint2*)(mrow + (long)r * a.ldm + (j0 >> 5)) : make_uint2(0u, 0u);
    } else if (a.p > 0.f) {
      const uint32_t key = ea_seed_key(seed), thr = ea_drop_thr(a.p);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint64_t row = (uint64_t)z * a.T1 + ibase + r;
        uint32_t x = 0u, y = 0u;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t bit = (uint32_t)attn_keep(key, thr, row, a.T2, j0 + 16 * t + lc) << (16 * (t & 1) + lc);
          if (t < 2) x |= bit; else y |= bit;
        }
        mw[r] = make_uint2(x, y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) mw[r] = make_uint2(~0u, ~0u);
    }
    __syncthreads();  // the setup images / previous chunk's images are no longer read
    if (!(ATTN_EXP & 4) || j0 == 0) {
    stage_km<KC>(sm + Q_K, gK, a.ldk, j0, a.T2, tid);
    stage_km<KC>(sm + Q_V, gV, a.ldv, j0, a.T2, tid);
    const int rb = a.T1 - 1 - (i0 + QB - 1) + j0;  // first positional row of the block's band
    if (REL) stage_km<144>(sm + Q_P, gP, a.ldp, rb, 2 * a.T1 - 1, tid);
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) s[t] = mfma(qa[ks], km_frag(sm + Q_K, 16 * t, ks, lane), s[t]);
    }
    if (REL && !(ATTN_EXP & 8)) {
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        f32x4 bd = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bd = mfma(qv[ks], km_frag(sm + Q_P, pb + 16 * t, ks, lane), bd);
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
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) dp[t] = mfma(doa[ks], km_frag(sm + Q_V, 16 * t, ks, lane), dp[t]);
    }
    // dS (scaled), in place of s
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = j0 + 16 * t + lc;
        const float e = __builtin_amdgcn_exp2f(fmaf(s[t][r], sl2, -Lr[r]));
        const float P = j < lim[r] ? e : 0.f;
        const float kp = (((t < 2 ? mw[r].x : mw[r].y) >> (16 * (t & 1) + lc)) & 1u) ? dsc : 0.f;
        s[t][r] = (P * a.scale) * fmaf(dp[t][r], kp, -Dr[r]);
      }
    // dS^T image (4 queries per 8-B write) and (rel-pos) the band image, column 15-il+jl
    if (with_dqv) {
      lds_fence();  // the gather above has read bds
      const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int c = 0; c < 3; ++c) *(uint4*)(band + (c * 64 + lane) * 16) = zero;
      lds_fence();
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint2 v = make_uint2(pack_bf16x2(s[t][0], s[t][1]), pack_bf16x2(s[t][2], s[t][3]));
      *(uint2*)(dst + (16 * t + lc) * 32 + g * 8) = v;
      if (with_dqv) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = 4 * g + r;
          *(bf16*)(band + band_off(il, 15 - il + 16 * t + lc)) = (bf16)s[t][r];
        }
      }
    }
    lds_fence();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 af = dst_frag(dst, 32 * ks, lane);
#pragma unroll
      for (int n = 0; n < 4; ++n) dqu[n] = mfma(af, km_frag_tr(sm + Q_K, 32 * ks, 16 * n, lane), dqu[n]);
    }
    if (with_dqv) {
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x8 af = band_frag(band, ks, lane);
#pragma unroll
        for (int n = 0; n < 4; ++n) dqv[n] = mfma(af, km_frag_tr(sm + Q_P, pb + 32 * ks, 16 * n, lane), dqv[n]);
      }
    }
    if (dbd_h) {  // dBD_raw[h][b][i][T-1-i+j] = dS
      const bool full = j0 + KC <= a.T2;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ibase + r;
        if (i >= a.T1) continue;
        bf16* drow = dbd_h + (long)i * a.lddbd + (a.T1 - 1 - i) + j0 + lc;
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (full || j0 + 16 * t + lc < a.T2) drow[16 * t] = (bf16)s[t][r];
      }
    }
  }
  // dQ (bf16) = dS.K (+ dBD.p); column sums of both terms over this block's rows
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ibase + r;
    if (i >= a.T1) continue;
    bf16* qrow = a.dq + ((long)b * a.T1 + i) * a.lddq + h * DK;
#pragma unroll
    for (int n = 0; n < 4; ++n) qrow[16 * n + lc] = (bf16)(dqu[n][r] + (with_dqv ? dqv[n][r] : 0.f));
  }
  if (a.bias_part) {
    float* red = (float*)(sm + Q_RED);  // [2][NWAVE][64]
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      float su = (dqu[n][0] + dqu[n][1]) + (dqu[n][2] + dqu[n][3]);
      float sv = (dqv[n][0] + dqv[n][1]) + (dqv[n][2] + dqv[n][3]);
      su += __shfl_xor(su, 16, 64);
      sv += __shfl_xor(sv, 16, 64);
      su += __shfl_xor(su, 32, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (g == 0) {
        red[w * DK + 16 * n + lc] = su;
        red[(NWAVE + w) * DK + 16 * n + lc] = sv;
      }
    }
    __syncthreads();
    if (tid < 2 * DK) {
      const int which = tid / DK, c = tid % DK;
      const float* rr = red + which * NWAVE * DK;
      const float v = (rr[c] + rr[DK + c]) + (rr[2 * DK + c] + rr[3 * DK + c]);
      const long prow = (long)which * a.B * nqb + (long)b * nqb + qb;
      if (which == 0 || REL) a.bias_part[prow * a.ldpart + h * DK + c] = v;
    }
  }
}

// ------------------------------------------------------------- attn_bwdq, pipelined (v2)
// The dQ pass of attn_bwdq_kernel restructured around the latency it paid per key chunk:
//  * K and V chunks are double-buffered and the positional rows live in a 208-row ring (a
//    chunk's band is 144 rows, the next chunk adds 64); every image is filled by LDS-DMA one
//    chunk ahead, so a chunk costs one barrier and no staging registers;
//  * the BD diagonal gather is a ds_bpermute per (band tile, register) instead of an LDS
//    image written and re-read;
//  * dS is laid onto a per-wave band window whose column c is positional row Rw + c for all
//    16 rows of the wave, so d(q+v) = window . p needs K = 64 per chunk (the window's last 16
//    columns carry into the next window) and the first 64 columns are final: they leave as
//    16-B stores into dbd rows shifted by ea_attn_dbd_shift(T1) columns (flags bit 1), with
//    the shift chosen so that every window starts on a 16-B boundary.
// Dropout keep words come from the forward's bit mask (prefetched a chunk ahead), else from
// the counter hash.  Summation order differs from attn_bwdq_kernel only in d(q+v) (64-column
// windows instead of 96), so dq / bias partials agree to f32 rounding, dbd bit for bit.
constexpr int RING = 208;  // band ring rows (13 x 16)
template <bool REL>
struct Q2 {
  static constexpr int K = 0, V = K + 2 * KC * 128;                 // [2][64 rows] each
  static constexpr int P = V + 2 * KC * 128;                        // ring [208 rows]
  static constexpr int WS = P + (REL ? RING * 128 : 0);             // per wave: window + dS^T
  static constexpr int WIN = REL ? 16 * 192 : 0;                    // [16][96] bf16 window
  static constexpr int WSZ = WIN + 64 * 32;
  static constexpr int D = WS + NWAVE * WSZ;                        // D_i, lse_i (64 each)
  static constexpr int LDS = D + 2 * QB * 4;
};
static_assert(Q2<true>::LDS <= 80 * 1024 + 512, "two workgroups per CU");

// ds_read_b64_tr_b16 as inline asm (the builtin makes hipcc drain vmcnt while an LDS-DMA is in
// flight); the caller waits lgkmcnt(0) before using the result
EA_DEV s16x4 tr_asm(const char* p) {
  s16x4 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// LDS reads as inline asm too: hipcc cannot tell an image being read from the one an LDS-DMA is
// filling and would drain vmcnt in front of every compiler-visible LDS read
EA_DEV bf16x8 ld128_asm(const char* p) {
  bf16x8 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int OFF>  // LDS byte address + immediate offset
EA_DEV bf16x8 ld128_at(uint32_t a) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}
// max of two scores that are never NaN (no canonicalisation of the operands)
EA_DEV float fmax_nn(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
EA_DEV uint2 ld64_asm(const char* p) {
  __attribute__((ext_vector_type(2))) unsigned v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return make_uint2(v.x, v.y);
}
EA_DEV uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p; }
EA_DEV void st16_asm(char* p, bf16 x) {
  const uint32_t v = (uint32_t)__builtin_bit_cast(unsigned short, x);
  asm volatile("ds_write_b16 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
EA_DEV void st64_asm(char* p, uint2 v) {
  const u32x2 x = {v.x, v.y};
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(x) : "memory");
}
EA_DEV void st128_asm(char* p, uint4 v) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(x) : "memory");
}
EA_DEV bf16x8 km_frag_asm(const char* img, int r0, int ks, int lane) {
  return ld128_asm(img + km_off(r0 + (lane & 15), ks * 4 + (lane >> 4)));
}
EA_DEV bf16x8 band_frag_asm(const char* img, int ks, int lane) {
  const int r = lane & 15, c = ks * 4 + (lane >> 4);
  return ld128_asm(img + r * 192 + ((c ^ ((r >> 2) & 3)) << 4));
}
// wait for the asm LDS reads; the sched_barrier keeps their consumers (MFMAs the compiler sees
// no memory dependence for) from being scheduled above the wait
EA_DEV void lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
EA_DEV uint2 gld64_asm(const void* p) {  // untracked global load: the caller waits vmcnt itself
  __attribute__((ext_vector_type(2))) unsigned v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return make_uint2(v.x, v.y);
}
template <int N>
EA_DEV void vmcnt_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
EA_DEV void vmcnt_le_rt(int n) {  // n in {0, 2, 4, 6}
  if (n >= 6) vmcnt_le<6>();
  else if (n >= 4) vmcnt_le<4>();
  else if (n >= 2) vmcnt_le<2>();
  else vmcnt_le<0>();
}
EA_DEV void bar() {
  lgkm0();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// km_frag_tr over image rows {k0 + 8(g&1) + 4h + q : g < 2} and {k1 + ... : g >= 2} (two 16-row
// groups that need not be adjacent: ring wrap)
EA_DEV bf16x8 km_tr_rows(const char* img, int k0, int k1, int n0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  const int col = n0 + 4 * p;
  const int kb = (g >> 1) ? k1 : k0;
  union { bf16x8 v; s16x4 h[2]; } out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = kb + 8 * (g & 1) + 4 * h + q;
    out.h[h] = tr_asm(img + km_off(row, col >> 3) + (col & 7) * 2);
  }
  return out.v;
}
// [64 keys][16 queries] bf16 image (dS^T / Pd^T), 32-B rows of four 8-B slots (4 queries each):
// row r at physical row r ^ (bit 3 of r ? 4 : 0), slot s at s ^ ((physical row >> 2) & 3) —
// the 8-B stores of 16 consecutive rows and the transposed reads of rows kb + 8g + 4h + q are
// both conflict-free (plain rows: 4-way stores, 2-way reads)
EA_DEV int dst_off(int row, int slot) {
  const int ph = row ^ (((row >> 3) & 1) << 2);
  return ph * 32 + ((slot ^ ((ph >> 2) & 3)) << 3);
}
EA_DEV bf16x8 dst_frag_asm(const char* img, int kb, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  union { bf16x8 v; s16x4 h[2]; } out;
#pragma unroll
  for (int h = 0; h < 2; ++h) out.h[h] = tr_asm(img + dst_off(kb + 8 * g + 4 * h + q, p));
  return out.v;
}
// LDS-DMA of km-image rows [ir, ir+8) (ir % 8 == 0) from global rows src + (r0 + 0..7)*ld (64
// bf16 columns), rows clamped into [0, rlim): one instruction per wave, lane L fills row
// ir + (L >> 3), 16-B slot L & 7 (= logical chunk (L & 7) ^ km_swz(row))
EA_DEV void km_dma8(char* img, int ir, const bf16* src, long ld, int r0, int rlim, int lane) {
  const int rr = lane >> 3, ch = (lane & 7) ^ km_swz(ir + rr);
  const int r = min(max(r0 + rr, 0), rlim - 1);
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + (long)r * ld + ch * 8),
                                   (__attribute__((address_space(3))) void*)(img + ir * 128), 16, 0, 0);
}

// 16-lane max / sum of four values with the DPP modifier on the VALU op itself (no separate
// v_mov_b32_dpp, no NaN canonicalisation: the operands are never NaN).  Same pairings in the
// same order as max16 / sum16; the rows are interleaved so that every DPP read comes at least
// two instructions after its operand's write (the leading s_nop covers the caller's write).
#define EA_DPP4(OP, CTRL)                                                   \
  OP " %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n\t" OP " %1, %1, %1 " CTRL \
  " row_mask:0xf bank_mask:0xf\n\t" OP " %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf\n\t" OP \
  " %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf\n\t"
EA_DEV void max16x4(float (&v)[4]) {
  asm("s_nop 1\n\t" EA_DPP4("v_max_f32_dpp", "quad_perm:[1,0,3,2]") EA_DPP4("v_max_f32_dpp", "quad_perm:[2,3,0,1]")
          EA_DPP4("v_max_f32_dpp", "row_half_mirror") EA_DPP4("v_max_f32_dpp", "row_mirror")
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
EA_DEV void sum16x4(float (&v)[4]) {
  asm("s_nop 1\n\t" EA_DPP4("v_add_f32_dpp", "quad_perm:[1,0,3,2]") EA_DPP4("v_add_f32_dpp", "quad_perm:[2,3,0,1]")
          EA_DPP4("v_add_f32_dpp", "row_half_mirror") EA_DPP4("v_add_f32_dpp", "row_mirror")
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
#undef EA_DPP4

// LDS-DMA of the 8 km-image rows [ir, ir+8) at image byte `dst` (ir % 8 == 0) from the rows
// r0 + (lane >> 3) of `src` clamped into [0, rlim), 32-bit byte offsets (the caller checked that
// rlim rows of ldb bytes fit): one instruction per wave, lane L fills 16-B slot L & 7 of row
// ir + (L >> 3) with logical chunk (L & 7) ^ km_swz(ir + (L >> 3)).  `chx` = km_chx(L), the
// swizzle's part that depends on L (ir's own part, 5 * bit 3 of ir, is applied here).
EA_DEV void km_dma8u(char* dst, int ir, const char* src, uint32_t ldb, int r0, int rlim, int chx, int lane) {
  const int r = min(max(r0 + (lane >> 3), 0), rlim - 1);
  const uint32_t off = __umul24((uint32_t)r, ldb) + ((uint32_t)(chx ^ (((ir >> 3) & 1) * 5)) << 4);
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + off),
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// MM: dropout keep decisions — 0 none (p = 0), 1 the forward's bit mask, 2 the counter hash
template <bool REL, int MM>
__global__ __launch_bounds__(256, 2) void attn_bwdq2_kernel(AttnP a) {
  using L = Q2<REL>;
  __shared__ __attribute__((aligned(16))) char sm[L::LDS];
  const int nqb = (a.T1 + QB - 1) / QB;
  const int z = blockIdx.x / nqb, qb = blockIdx.x % nqb;
  const int b = z / a.H, h = z % a.H;
  const int i0 = qb * QB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: ring / image offsets stay scalar
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = a.p > 0.f ? ea_salted(a.seed, a.salt) : 0;
  const bool with_dqv = REL && (a.flags & 1);
  char* win = sm + L::WS + w * L::WSZ;  // band window (REL)
  char* dst = win + L::WIN;
  float* Dv = (float*)(sm + L::D);
  float* Lv = Dv + QB;
  const int kend = a.causal ? min(kl, i0 + QB) : kl;
  const int nch = (kend + KC - 1) / KC;
  const int rlimP = 2 * a.T1 - 1;
  const int rb0 = a.T1 - 1 - (i0 + QB - 1);  // chunk 0's first positional row (ring position 0)
  const char* kh_ = (const char*)(a.k + (long)b * a.T2 * a.ldk + h * DK);
  const char* vh_ = (const char*)(a.v + (long)b * a.T2 * a.ldv + h * DK);
  const char* ph_ = REL ? (const char*)(a.pp + h * DK) : nullptr;
  const uint32_t ldkb = (uint32_t)a.ldk * 2, ldvb = (uint32_t)a.ldv * 2, ldpb = REL ? (uint32_t)a.ldp * 2 : 0;
  const int chx = km_chx(lane);
  // chunk c's K / V rows into buffer c & 1; ring rows [x0, x0 + 8n) (relative to rb0) by groups
  // (32-bit source offsets: the launcher checked the head slices' byte ranges)
  auto dma_kv = [&](int c) {
    char* kb = sm + L::K + (c & 1) * KC * 128;
    char* vb = sm + L::V + (c & 1) * KC * 128;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ir = 8 * (w + 4 * u);
      km_dma8u(kb + ir * 128, ir, kh_, ldkb, 64 * c + ir, a.T2, chx, lane);
      km_dma8u(vb + ir * 128, ir, vh_, ldvb, 64 * c + ir, a.T2, chx, lane);
    }
  };
  auto dma_ring = [&](int x0, int ngrp) {  // groups gi = w, w+4, ... < ngrp
    for (int gi = w; gi < ngrp; gi += 4) {
      const int x = x0 + 8 * gi, ir = x % RING;
      km_dma8u(sm + L::P + ir * 128, ir, ph_, ldpb, rb0 + x, rlimP, chx, lane);
    }
  };
  // lane offsets of the 16 x 32 fragments of a km image at a 16-row boundary (row 16t + r has
  // r's swizzle): fragment (16t rows on, k-step ks) = image + 2048 t + loff[ks]
  int loff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) loff[ks] = lc * 128 + (((ks * 4 + g) ^ km_swz(lc)) << 4);
  if (nch > 0) {
    dma_kv(0);
    if (REL) dma_ring(0, 18);
  }

  // this wave's 16 rows of Q + u, Q + v and dO as A fragments; D_i and lse_i.  Setup images in
  // the second K / V buffers and the window area (free until chunk 1's DMA / chunk 0's window)
  char* img_qu = sm + L::K + KC * 128;
  char* img_qv = sm + L::V + KC * 128;
  char* img_do = sm + L::WS;  // the per-wave areas: 4 x 5 KiB (rel-pos) or 4 x 2 KiB
  static_assert(NWAVE * L::WSZ >= QB * 128, "dO image fits the per-wave areas");
  bf16x8 qa[2], qv[2], doa[2];
  {
    const bf16* qsrc = a.q + (long)b * a.T1 * a.ldq + h * DK;
    km_stage_out(img_qu, qsrc, a.ldq, i0, QB, a.T1, a.bu ? a.bu + h * DK : nullptr,
                 a.wsQu + (long)b * a.T1 * a.ldqu + h * DK, a.ldqu, tid, 256);
    if (REL)
      km_stage_out(img_qv, qsrc, a.ldq, i0, QB, a.T1, a.bv + h * DK,
                   a.wsQv + (long)b * a.T1 * a.ldqvw + h * DK, a.ldqvw, tid, 256);
    km_stage(img_do, a.dO + (long)b * a.T1 * a.lddo + h * DK, a.lddo, i0, QB, a.T1, tid, 256);
    {  // D_i = dO_i . O_i: 4 threads per row, 16 columns each
      const int row = tid >> 2, qd = tid & 3, i = i0 + row;
      float d = 0.f;
      if (i < a.T1) {
        const bf16* dr = a.dO + ((long)b * a.T1 + i) * a.lddo + h * DK + qd * 16;
        const bf16* orow = a.o + ((long)b * a.T1 + i) * a.ldo + h * DK + qd * 16;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          union { uint4 u; bf16 e[8]; } x, y;
          x.u = *(const uint4*)(dr + hf * 8);
          y.u = *(const uint4*)(orow + hf * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) d += (float)x.e[e] * (float)y.e[e];
        }
      }
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      if (qd == 0) {
        Dv[row] = d;
        Lv[row] = i < a.T1 ? a.lse[(long)z * a.T1 + i] * LOG2E : INFINITY;
        if (i < a.T1) a.wsD[(long)z * a.T1 + i] = d;
      }
    }
    bar();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qa[ks] = km_frag(img_qu, 16 * w, ks, lane);
      if (REL) qv[ks] = km_frag(img_qv, 16 * w, ks, lane);
      doa[ks] = km_frag(img_do, 16 * w, ks, lane);
    }
  }
  const int ibase = i0 + 16 * w + 4 * g;  // query row of register r: ibase + r
  float Dr[4], Lr[4];
  int lim[4];  // key j of row r is valid iff j < lim[r]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ibase + r;
    Dr[r] = Dv[16 * w + 4 * g + r];
    Lr[r] = Lv[16 * w + 4 * g + r];
    lim[r] = i < a.T1 ? (a.causal ? min(kl, i + 1) : kl) : 0;
  }
  bar();  // setup images read: the window area and the second buffers are free
  if (REL) {  // zero this wave's window
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int c = 0; c < 3; ++c) *(uint4*)(win + (c * 64 + lane) * 16) = zero;
  }
  const float sl2 = a.scale * LOG2E;
  bf16* dbd_h = REL && a.dbd ? a.dbd + ((long)h * a.B + b) * a.T1 * a.lddbd : nullptr;
  // window start (physical dbd column) of chunk 0 for this wave's rows: Rw + shift, 8-aligned
  const int shift = REL ? ea_attn_dbd_shift_dev(a.T1) : 0;
  const int W0 = a.T1 - 16 - (i0 + 16 * w) + shift;
  const float dsc = MM ? 1.f / (1.f - a.p) : 1.f;
  // keep words of rows ibase + r (clamped to the last row: always four loads per chunk)
  const uint32_t* mrow = a.dmask + ((long)z * a.T1 + min(ibase, a.T1 - 1)) * a.ldm;
  // dbd stores per chunk: two 16-B pieces per lane (out-of-range rows to the dummy sink)
  const int nst = dbd_h ? 2 : 0;

  f32x4 dqu[4], dqv[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) dqu[n] = dqv[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int pb = 48 - 16 * w;  // this wave's first band row relative to the chunk's band start
  for (int c = 0; c < nch; ++c) {
    const int j0 = c * KC;
    // this chunk's images landed (older than the mask loads of this chunk and the previous
    // chunk's dbd stores), all waves done with the previous chunk
    // this chunk's images landed (only the previous chunk's dbd stores are younger), all waves
    // done with the previous chunk
    vmcnt_le_rt(c == 0 ? 0 : nst);
    bar();
    uint2 mw[4];
    if (MM == 1) {  // issued before the prefetch: the dS phase waits for these four only
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ro = ibase + r < a.T1 ? r * a.ldm : (a.T1 - 1 - min(ibase, a.T1 - 1)) * a.ldm;
        mw[r] = gld64_asm(mrow + ro + (j0 >> 5));
      }
    }
    const int ndma = c + 1 < nch ? (REL ? 6 : 4) : 0;  // LDS-DMA issued after the mask loads
    if (c + 1 < nch) {
      dma_kv(c + 1);
      if (REL) dma_ring(64 * c + 144, 8);
    }
    if (MM == 2) {
      const uint32_t key = ea_seed_key(seed), thr = ea_drop_thr(a.p);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint64_t row = (uint64_t)z * a.T1 + ibase + r;
        uint32_t x = 0u, y = 0u;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t bit = (uint32_t)attn_keep(key, thr, row, a.T2, j0 + 16 * t + lc) << (16 * (t & 1) + lc);
          if (t < 2) x |= bit; else y |= bit;
        }
        mw[r] = make_uint2(x, y);
      }
    }
    const char* kimg = sm + L::K + (c & 1) * KC * 128;
    const char* vimg = sm + L::V + (c & 1) * KC * 128;
    const char* ring = sm + L::P;
    f32x4 s[4], dp[4];
    {
      bf16x8 kf[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) kf[t][ks] = ld128_asm(kimg + 2048 * t + loff[ks]);
      lgkm0();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) s[t] = mfma(qa[ks], kf[t][ks], s[t]);
      }
    }
    if (REL) {
      // BDfull (16 x 80) over ring rows 64c + pb + [0, 80), gathered onto the diagonal
      f32x4 bd[5];
      {
        bf16x8 pf[5][2];
        const int rb = (64 * c + pb) % RING;  // wave-uniform, a multiple of 16
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int rp = rb + 16 * t < RING ? rb + 16 * t : rb + 16 * t - RING;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) pf[t][ks] = ld128_asm(ring + rp * 128 + loff[ks]);
        }
        lgkm0();
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          bd[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) bd[t] = mfma(qv[ks], pf[t][ks], bd[t]);
        }
      }
      // (one bpermute per band tile and register: the two calls of neighbouring t are the same
      // expression; no array of gathered values, which hipcc turned into a scratch-indexed load)
      // output (il = 4g + r, jl = 16t + lc) reads BDfull column 16t + lc + 15 - il: tile t (or
      // t + 1 past a tile edge) of lane 16g + ((lc + 15 - il) & 15)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sft = lc + 15 - 4 * g - r;
        const int src = (16 * g + (sft & 15)) * 4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float lo = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[t][r])));
          const float hi = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[t + 1][r])));
          s[t][r] += sft >= 16 ? hi : lo;
        }
      }
    }
    {
      bf16x8 vf[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) vf[t][ks] = ld128_asm(vimg + 2048 * t + loff[ks]);
      lgkm0();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) dp[t] = mfma(doa[ks], vf[t][ks], dp[t]);
      }
    }
    // dS (scaled), in place of s
    if (MM == 1) vmcnt_le_rt(ndma);  // the mask words (older than this chunk's prefetch)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = j0 + 16 * t + lc;
        const float e = __builtin_amdgcn_exp2f(fmaf(s[t][r], sl2, -Lr[r]));
        const float P = j < lim[r] ? e : 0.f;
        float kp = 1.f;
        if (MM) kp = (((t < 2 ? mw[r].x : mw[r].y) >> (16 * (t & 1) + lc)) & 1u) ? dsc : 0.f;
        s[t][r] = (P * a.scale) * fmaf(dp[t][r], kp, -Dr[r]);
      }
    // dS^T image (4 queries per 8-B write); (rel-pos) dS onto the window, column 15 - il + jl
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint2 v = make_uint2(pack_bf16x2(s[t][0], s[t][1]), pack_bf16x2(s[t][2], s[t][3]));
      st64_asm(dst + dst_off(16 * t + lc, g), v);
      if (REL && (with_dqv || dbd_h)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = 4 * g + r;
          st16_asm(win + band_off(il, 15 - il + 16 * t + lc), (bf16)s[t][r]);
        }
      }
    }
    // dQu += dS . K
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 af = dst_frag_asm(dst, 32 * ks, lane);
      bf16x8 bf[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) bf[n] = km_tr_rows(kimg, 32 * ks, 32 * ks + 16, 16 * n, lane);
      lgkm0();
#pragma unroll
      for (int n = 0; n < 4; ++n) dqu[n] = mfma(af, bf[n], dqu[n]);
    }
    if (REL && (with_dqv || dbd_h)) {
      if (with_dqv) {  // dQv += window[:, 0:64] . p[ring rows 64c + pb + 0..63]
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 af = band_frag_asm(win, ks, lane);
          const int rbq = (64 * c + pb) % RING, x0 = rbq + 32 * ks, x1 = x0 + 16;  // wave-uniform
          const int r0 = x0 < RING ? x0 : x0 - RING, r1 = x1 < RING ? x1 : x1 - RING;
          bf16x8 bf[4];
#pragma unroll
          for (int n = 0; n < 4; ++n) bf[n] = km_tr_rows(ring, r0, r1, 16 * n, lane);
          lgkm0();
#pragma unroll
          for (int n = 0; n < 4; ++n) dqv[n] = mfma(af, bf[n], dqv[n]);
        }
      }
      if (dbd_h) {  // the window's first 64 columns are final: rows i0 + 16w + (q >> 3)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int q = lane + 64 * u, row = q >> 3, ch = q & 7;
          const bf16x8 vb = ld128_asm(win + row * 192 + ((ch ^ ((row >> 2) & 3)) << 4));
          lgkm0();
          const uint4 v = *(const uint4*)&vb;
          const int i = i0 + 16 * w + row, col = W0 + j0 + 8 * ch;
          // (32-bit row offsets: the head's dbd block is far below 4 GiB)
          bf16* dstp = (i < a.T1 && col < a.lddbd)
                           ? (bf16*)((char*)dbd_h + __umul24((uint32_t)i, (uint32_t)a.lddbd * 2u) + 2u * (uint32_t)col)
                           : (bf16*)((char*)a.wsDummy + lane * 16);
          *(uint4*)dstp = v;
        }
      }
      // carry columns [64, 80) to [0, 16), zero [16, 96)
      {
        const int row = lane >> 2, cq = 4 * (lane & 3);
        const uint2 tail = ld64_asm(win + band_off(row, 64 + cq));
        lgkm0();
        const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int q = lane + 64 * u;
          if (u < 2 || q < 160) {
            const int zr = (int)(__umul24((uint32_t)q, 205u) >> 11), zc = 2 + q - 10 * zr;  // q / 10 (q < 192)
            st128_asm(win + zr * 192 + ((zc ^ ((zr >> 2) & 3)) << 4), zero);
          }
        }
        st64_asm(win + band_off(row, cq), tail);
      }
    }
  }
  if (REL && nch > 0 && (with_dqv || dbd_h)) {
    // the last window's carried tail: columns [0, 16) = positional rows of virtual chunk nch
    if (with_dqv) {
      const bf16x8 af = band_frag(win, 0, lane);
      const int r0 = (64 * nch + pb) % RING, r1 = (64 * nch + pb + 16) % RING;
      bf16x8 bf[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) bf[n] = km_tr_rows(sm + L::P, r0, r1, 16 * n, lane);
      lgkm0();
#pragma unroll
      for (int n = 0; n < 4; ++n) dqv[n] = mfma(af, bf[n], dqv[n]);
    }
    if (dbd_h && lane < 32) {
      const int row = lane >> 1, ch = lane & 1;
      const uint4 v = *(const uint4*)(win + row * 192 + ((ch ^ ((row >> 2) & 3)) << 4));
      const int i = i0 + 16 * w + row, col = W0 + nch * KC + 8 * ch;
      if (i < a.T1 && col < a.lddbd) *(uint4*)(dbd_h + (long)i * a.lddbd + col) = v;
    }
  }
  if (dbd_h) {
    // zeros outside the windows written above: columns [0, W0) and [W0 + 64 nch + 16, lddbd)
    const int lo = W0, hi = W0 + nch * KC + (nch > 0 ? 16 : 0);
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (int il = 0; il < 16; ++il) {
      const int i = i0 + 16 * w + il;
      if (i >= a.T1) break;
      bf16* drow = dbd_h + (long)i * a.lddbd;
      for (int c0 = 8 * lane; c0 < a.lddbd; c0 += 512)
        if (c0 < lo || c0 >= hi) *(uint4*)(drow + c0) = zero;
    }
  }
  // dQ (bf16) = dS.K (+ dBD.p); column sums of both terms over this block's rows
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ibase + r;
    if (i >= a.T1) continue;
    bf16* qrow = a.dq + ((long)b * a.T1 + i) * a.lddq + h * DK;
#pragma unroll
    for (int n = 0; n < 4; ++n) qrow[16 * n + lc] = (bf16)(dqu[n][r] + (with_dqv ? dqv[n][r] : 0.f));
  }
  if (a.bias_part) {
    bar();  // chunk images no longer read: the column-sum exchange reuses the K buffers
    float* red = (float*)(sm + L::K);  // [2][NWAVE][64]
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      float su = (dqu[n][0] + dqu[n][1]) + (dqu[n][2] + dqu[n][3]);
      float sv = (dqv[n][0] + dqv[n][1]) + (dqv[n][2] + dqv[n][3]);
      su += __shfl_xor(su, 16, 64);
      sv += __shfl_xor(sv, 16, 64);
      su += __shfl_xor(su, 32, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (g == 0) {
        red[w * DK + 16 * n + lc] = su;
        red[(NWAVE + w) * DK + 16 * n + lc] = sv;
      }
    }
    bar();
    if (tid < 2 * DK) {
      const int which = tid / DK, c = tid % DK;
      const float* rr = red + which * NWAVE * DK;
      const float v = (rr[c] + rr[DK + c]) + (rr[2 * DK + c] + rr[3 * DK + c]);
      const long prow = (long)which * a.B * nqb + (long)b * nqb + qb;
      if (which == 0 || REL) a.bias_part[prow * a.ldpart + h * DK + c] = v;
    }
  }
}

// ---------------------------------------------------------- attn forward, pipelined (v2)
// attn_fwd_kernel with the dQ pass's pipelining: K / V chunks double-buffered and the
// positional band (128 rows per chunk) in a 192-row ring, all filled by LDS-DMA one chunk
// ahead (one barrier per chunk, no staging registers); the BD diagonal gather by ds_bpermute;
// Pd written as a [64 keys][16 queries] image with one 8-B store per key tile (4 queries of a
// lane) instead of 16 two-byte stores, read back as the PV MFMA's A operand with transposed
// reads.  Same arithmetic in the same order as attn_fwd_kernel: O, lse and the keep bits are
// bit-identical.  MM: 0 no dropout, 1 dropout + keep bits to dmask, 2 dropout only.
template <bool REL>
struct F2 {
  static constexpr int RINGF = 192;
  static constexpr int K = 0, V = K + 2 * KC * 128, P = V + 2 * KC * 128;
  static constexpr int PT = P + (REL ? RINGF * 128 : 0);  // per wave: Pd^T image [64][16] bf16
  static constexpr int LDS = PT + NWAVE * 64 * 32;
};
static_assert(F2<true>::LDS <= 80 * 1024, "two workgroups per CU");

template <bool REL, int MM>
__global__ __launch_bounds__(256, 2) void attn_fwd2_kernel(AttnP a) {
  using L = F2<REL>;
  constexpr int RF = L::RINGF;
  __shared__ __attribute__((aligned(16))) char sm[L::LDS];
  const int nqb = (a.T1 + QB - 1) / QB;
  const int z = blockIdx.x / nqb, qb = blockIdx.x % nqb;
  const int b = z / a.H, h = z % a.H;
  const int i0 = qb * QB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: ring / image offsets stay scalar
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = MM == 1 || MM == 2 ? ea_salted(a.seed, a.salt) : 0;
  char* pt = sm + L::PT + w * 64 * 32;
  const int kend = a.causal ? min(kl, i0 + QB) : kl;
  const int nch = (kend + KC - 1) / KC;
  const int rlimP = 2 * a.T1 - 1;
  const int rb0 = a.T1 - 1 - (i0 + QB - 1);  // chunk 0's first positional row (ring position 0)
  const char* kh_ = (const char*)(a.k + (long)b * a.T2 * a.ldk + h * DK);
  const char* vh_ = (const char*)(a.v + (long)b * a.T2 * a.ldv + h * DK);
  const char* ph_ = REL ? (const char*)(a.pp + h * DK) : nullptr;
  const uint32_t ldkb = (uint32_t)a.ldk * 2, ldvb = (uint32_t)a.ldv * 2, ldpb = REL ? (uint32_t)a.ldp * 2 : 0;
  const int chx = km_chx(lane);
  auto dma_kv = [&](int c) {
    char* kb = sm + L::K + (c & 1) * KC * 128;
    char* vb = sm + L::V + (c & 1) * KC * 128;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ir = 8 * (w + 4 * u);
      km_dma8u(kb + ir * 128, ir, kh_, ldkb, 64 * c + ir, a.T2, chx, lane);
      km_dma8u(vb + ir * 128, ir, vh_, ldvb, 64 * c + ir, a.T2, chx, lane);
    }
  };
  auto dma_ring = [&](int x0, int ngrp) {  // ring rows x0 + [0, 8 ngrp) (x0 % 8 == 0)
    for (int gi = w; gi < ngrp; gi += 4) {
      const int x = x0 + 8 * gi, ir = x % RF;
      km_dma8u(sm + L::P + ir * 128, ir, ph_, ldpb, rb0 + x, rlimP, chx, lane);
    }
  };
  if (nch > 0) {
    dma_kv(0);
    if (REL) dma_ring(0, 16);
  }
  // lane offsets of the 16 x 32 A/B fragments of a km image at a 16-row boundary (the swizzle of
  // row 16t + r is that of r): fragment (16t rows on, k-step ks) = image + 2048 t + loff[ks]
  int loff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) loff[ks] = lc * 128 + (((ks * 4 + g) ^ km_swz(lc)) << 4);
  // this wave's 16 query rows as A fragments (q + u, q + v), from images in the second buffers
  bf16x8 qa[2], qv[2];
  {
    char* img_qu = sm + L::K + KC * 128;
    char* img_qv = sm + L::V + KC * 128;
    const bf16* qsrc = a.q + (long)b * a.T1 * a.ldq + h * DK;
    km_stage_bias(img_qu, qsrc, a.ldq, i0, QB, a.T1, a.bu ? a.bu + h * DK : nullptr, tid, 256);
    if (REL) km_stage_bias(img_qv, qsrc, a.ldq, i0, QB, a.T1, a.bv + h * DK, tid, 256);
    bar();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qa[ks] = km_frag(img_qu, 16 * w, ks, lane);
      if (REL) qv[ks] = km_frag(img_qv, 16 * w, ks, lane);
    }
  }
  f32x4 oacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) oacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float mrun[4], lrun[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrun[r] = -INFINITY; lrun[r] = 0.f; }
  const int ibase = i0 + 16 * w + 4 * g;  // query row of register rr: ibase + rr
  const int odd = lc & 1;
  const uint64_t npair = (uint64_t)((a.T2 + 1) >> 1);
  const uint64_t prA = ((uint64_t)z * a.T1 + ibase + odd) * npair, prB = prA + 2 * npair;
  // every pair index of the launch below 2^32: the hash input is the pair's low word + key, so a
  // lane's input for key pair (j0 + 16t + lc) >> 1 is aA / aB + j0 / 2 + 8t (ea_pair_hash's value)
  // (rows run up to nqb * 64 + 2 past a head's first and key pairs up to nch * 32: a margin)
  const bool pair32 = ((uint64_t)a.B * a.H * a.T1 + 2 * QB + 4) * npair + a.T2 + 2 * KC < (1ull << 32);
  const uint32_t key = MM == 1 || MM == 2 ? ea_seed_key(seed) : 0u;
  const uint32_t aA = (uint32_t)prA + key + (uint32_t)(lc >> 1), aB = (uint32_t)prB + key + (uint32_t)(lc >> 1);
  const int pb = 48 - 16 * w;
  for (int c = 0; c < nch; ++c) {
    const int j0 = c * KC;
    vmcnt_le<0>();  // this chunk's images (and the previous chunk's keep-bit stores) landed
    bar();          // all waves done with the previous chunk (and, at c = 0, the setup images)
    if (c + 1 < nch) {
      dma_kv(c + 1);
      if (REL) dma_ring(64 * c + 128, 8);
    }
    const char* kimg = sm + L::K + (c & 1) * KC * 128;
    const char* vimg = sm + L::V + (c & 1) * KC * 128;
    f32x4 s[4];
    {
      bf16x8 kf[4][2];
      const uint32_t ka0 = lds_addr(kimg) + loff[0], ka1 = lds_addr(kimg) + loff[1];
      kf[0][0] = ld128_at<0>(ka0);    kf[0][1] = ld128_at<0>(ka1);
      kf[1][0] = ld128_at<2048>(ka0); kf[1][1] = ld128_at<2048>(ka1);
      kf[2][0] = ld128_at<4096>(ka0); kf[2][1] = ld128_at<4096>(ka1);
      kf[3][0] = ld128_at<6144>(ka0); kf[3][1] = ld128_at<6144>(ka1);
      lgkm0();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) s[t] = mfma(qa[ks], kf[t][ks], s[t]);
      }
    }
    if (REL) {
      // BDfull (16 x 80) over ring rows 64c + pb + [0, 80), gathered onto the diagonal
      f32x4 bd[5];
      {
        bf16x8 pf[5][2];
        const int rb = (64 * c + pb) % RF;  // wave-uniform, a multiple of 16
        const uint32_t pa0 = lds_addr(sm) + loff[0], pa1 = lds_addr(sm) + loff[1];
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int rp = rb + 16 * t < RF ? rb + 16 * t : rb + 16 * t - RF;
          pf[t][0] = ld128_at<L::P>(pa0 + rp * 128);
          pf[t][1] = ld128_at<L::P>(pa1 + rp * 128);
        }
        lgkm0();
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          bd[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) bd[t] = mfma(qv[ks], pf[t][ks], bd[t]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sft = lc + 15 - 4 * g - r;
        const int src = (16 * g + (sft & 15)) * 4;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float lo = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[t][r])));
          const float hi = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[t + 1][r])));
          s[t][r] += sft >= 16 ? hi : lo;
        }
      }
    }
    // mask (only a chunk that reaches past the key length, or a causal one), online softmax
    float pv[4][4], mx[4];
    if (!a.causal && j0 + KC <= kl) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mx[r] = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          pv[t][r] = s[t][r] * a.scale;
          mx[r] = fmaxf(mx[r], pv[t][r]);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ibase + r;
        mx[r] = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = j0 + 16 * t + lc;
          const bool ok = j < kl && (!a.causal || j <= i);
          pv[t][r] = ok ? s[t][r] * a.scale : -INFINITY;
          mx[r] = fmaxf(mx[r], pv[t][r]);
        }
      }
    }
    max16x4(mx);
    float sum[4], alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mnew = fmax_nn(mrun[r], mx[r]);
      alpha[r] = mnew == -INFINITY ? 1.f : __expf(mrun[r] - mnew);
      // a masked score is -inf: exp(-inf - m) = 0 for finite m; m = -inf only if the whole row so
      // far is masked, then every exponent is exp(-inf - 0) = 0
      const float ms = mnew == -INFINITY ? 0.f : mnew;
#pragma unroll
      for (int t = 0; t < 4; ++t) pv[t][r] = __expf(pv[t][r] - ms);
      sum[r] = ((pv[0][r] + pv[1][r]) + pv[2][r]) + pv[3][r];
      mrun[r] = mnew;
#pragma unroll
      for (int t = 0; t < 4; ++t) oacc[t][r] *= alpha[r];
    }
    sum16x4(sum);
#pragma unroll
    for (int r = 0; r < 4; ++r) lrun[r] = lrun[r] * alpha[r] + sum[r];
    // dropout (keep bits -> dmask for the backward)
    if (MM == 1 || MM == 2) {
      const uint32_t thr = ea_drop_thr(a.p);
      const float sc = 1.f / (1.f - a.p);
      uint64_t bal[4][4];
      uint32_t hAt[4], hBt[4];
      if (pair32) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          hAt[t] = ea_pair_mix(aA + (uint32_t)((j0 >> 1) + 8 * t));
          hBt[t] = ea_pair_mix(aB + (uint32_t)((j0 >> 1) + 8 * t));
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint64_t jp = (uint64_t)((j0 + 16 * t + lc) >> 1);  // shared by the lane pair
          hAt[t] = ea_pair_hash(key, prA + jp);
          hBt[t] = ea_pair_hash(key, prB + jp);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t hA = hAt[t], hB = hBt[t];
        const uint32_t pA = (uint32_t)__builtin_amdgcn_mov_dpp((int)hA, 0xB1, 0xF, 0xF, false);
        const uint32_t pB = (uint32_t)__builtin_amdgcn_mov_dpp((int)hB, 0xB1, 0xF, 0xF, false);
        const uint32_t hh[4] = {odd ? pA : hA, odd ? hA : pA, odd ? pB : hB, odd ? hB : pB};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool kept = (odd ? hh[r] >> 16 : hh[r] & 0xffffu) >= thr;  // key parity = lane parity
          pv[t][r] *= kept ? sc : 0.f;
          bal[t][r] = __ballot(kept);
        }
      }
      if (MM == 1 && lc < 2) {  // lane lc = u writes word u of each of its group's 4 rows
        const bool hiw = g >= 2;   // the group's 16 ballot bits sit in the high dword
        const uint32_t sh = 16u * (uint32_t)(g & 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = ibase + r;
          const uint64_t lo = lc ? bal[2][r] : bal[0][r], hi = lc ? bal[3][r] : bal[1][r];
          const uint32_t x0 = hiw ? (uint32_t)(lo >> 32) : (uint32_t)lo, x1 = hiw ? (uint32_t)(hi >> 32) : (uint32_t)hi;
          const uint32_t word = __builtin_amdgcn_ubfe(x0, sh, 16) | (__builtin_amdgcn_ubfe(x1, sh, 16) << 16);
          if (i < a.T1) a.dmask[((long)z * a.T1 + i) * a.ldm + (j0 >> 5) + lc] = word;
        }
      }
    }
    // Pd^T image: key 16t + lc, queries 4g .. 4g+3 in one 8-B store
#pragma unroll
    for (int t = 0; t < 4; ++t)
      st64_asm(pt + dst_off(16 * t + lc, g),
               make_uint2(pack_bf16x2(pv[t][0], pv[t][1]), pack_bf16x2(pv[t][2], pv[t][3])));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = dst_frag_asm(pt, 32 * ks, lane);
      bf16x8 vf[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) vf[t] = km_tr_rows(vimg, 32 * ks, 32 * ks + 16, 16 * t, lane);
      lgkm0();
#pragma unroll
      for (int t = 0; t < 4; ++t) oacc[t] = mfma(pa, vf[t], oacc[t]);
    }
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

// attn_bwdkv shared memory
constexpr int V_QU = 0, V_QV = V_QU + BQ * 128, V_DO = V_QV + BQ * 128, V_P = V_DO + BQ * 128;
constexpr int V_D = V_P + 96 * 128;               // D_i, lse_i*log2e (32 each), keep words [2][32]
constexpr int V_XLD = 97;                         // BDfull row stride (floats)
constexpr int V_XS = V_D + 4 * BQ * 4;            // BDfull [32][97] f32, shared by the waves
constexpr int V_LDS = V_XS + BQ * V_XLD * 4;

template <bool REL>
__global__ __launch_bounds__(256, 2) void attn_bwdkv_kernel(AttnP a) {
  __shared__ __attribute__((aligned(16))) char sm[V_LDS];
  const int nkb = (a.T2 + 63) / 64;
  const int z = blockIdx.x / nkb, kb = blockIdx.x % nkb;
  const int b = z / a.H, h = z % a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = a.p > 0.f ? ea_salted(a.seed, a.salt) : 0;
  const int j0 = 64 * kb, jw = j0 + 16 * w;
  char* quimg = sm + V_QU;
  char* qvimg = sm + V_QV;
  char* doimg = sm + V_DO;
  char* pimg = sm + V_P;
  float* Dv = (float*)(sm + V_D);
  float* Lv = Dv + BQ;
  uint32_t* Mw = (uint32_t*)(Lv + BQ);  // [word u][32 rows]
  float* xs = (float*)(sm + V_XS);

  f32x4 dka[4], dva[4];  // rows = keys jw + 4g + r, columns 16n + lc
#pragma unroll
  for (int n = 0; n < 4; ++n) dka[n] = dva[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (j0 < kl) {
    // this wave's 16 keys as B fragments (key jw + lc, dims 32ks + 8g ..+7)
    const int j = jw + lc;
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = vf[ks] = (bf16x8){};
      if (j < kl) {
        kf[ks] = *(const bf16x8*)(a.k + ((long)b * a.T2 + j) * a.ldk + h * DK + 32 * ks + 8 * g);
        vf[ks] = *(const bf16x8*)(a.v + ((long)b * a.T2 + j) * a.ldv + h * DK + 32 * ks + 8 * g);
      }
    }
    const int prow = tid >> 3, pch = tid & 7;
    const bool use_mask = a.p > 0.f && a.dmask != nullptr;
    const float dsc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
    const float sl2 = a.scale * LOG2E;
    // thread tid owns row tid>>3, chunk tid&7 of the Q+u / Q+v / dO tiles, band rows
    // (tid>>3) + 32u (u < 3) of the 96-row band image, (tid < 32) D / lse of row tid and
    // (tid < 64) keep word tid>>5 of row tid&31; per-thread bases at row 0, uniform row offsets
    const long cofs = h * DK + pch * 8;
    const bf16* gQu = a.wsQu + ((long)b * a.T1 + prow) * a.ldqu + cofs;
    const bf16* gQv = REL ? a.wsQv + ((long)b * a.T1 + prow) * a.ldqvw + cofs : nullptr;
    const bf16* gdO = a.dO + ((long)b * a.T1 + prow) * a.lddo + cofs;
    const bf16* gP = REL ? a.pp + (long)prow * a.ldp + cofs : nullptr;
    const int lofs = km_off(prow, pch);
    struct Pre { uint4 qu, qv, dO, p[3]; float D, L; uint32_t mw; };
    auto fetch = [&](int i0n, Pre& pr) {
      const int i = i0n + prow;
      pr.qu = pr.qv = pr.dO = make_uint4(0u, 0u, 0u, 0u);
      if (i < a.T1) {
        pr.qu = *(const uint4*)(gQu + (long)i0n * a.ldqu);
        if (REL) pr.qv = *(const uint4*)(gQv + (long)i0n * a.ldqvw);
        pr.dO = *(const uint4*)(gdO + (long)i0n * a.lddo);
      }
      if (tid < BQ) {
        const int ir = i0n + tid;
        pr.D = ir < a.T1 ? a.wsD[(long)z * a.T1 + ir] : 0.f;
        pr.L = ir < a.T1 ? a.lse[(long)z * a.T1 + ir] * LOG2E : INFINITY;
      }
      if (use_mask && tid < 64) {
        const int im = min(i0n + (tid & 31), a.T1 - 1);
        pr.mw = a.dmask[((long)z * a.T1 + im) * a.ldm + (j0 >> 5) + (tid >> 5)];
      }
      if (REL) {
        const int rs = a.T1 - 1 - (i0n + BQ - 1) + j0;
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int r = rs + prow + 32 * u;
          pr.p[u] = make_uint4(0u, 0u, 0u, 0u);
          if (r >= 0 && r < 2 * a.T1 - 1) pr.p[u] = *(const uint4*)(gP + (long)(rs + 32 * u) * a.ldp);
        }
      }
    };
    // queries before the key block see none of its keys under the causal mask
    const int istart = a.causal ? (j0 / BQ) * BQ : 0;
    const int imin = a.causal ? j : 0;  // rows i in [imin, T1) see key j (if j < kl)
    const int bpos = 16 * (w & 1) + lc;  // this lane's bit in keep word w>>1
    Pre pre;
    fetch(istart, pre);
    for (int i0 = istart; i0 < a.T1; i0 += BQ) {
      __syncthreads();  // previous tile's readers of the images / BDfull are done
      *(uint4*)(quimg + lofs) = pre.qu;
      if (REL) *(uint4*)(qvimg + lofs) = pre.qv;
      *(uint4*)(doimg + lofs) = pre.dO;
      if (REL) {
#pragma unroll
        for (int u = 0; u < 3; ++u) *(uint4*)(pimg + lofs + 4096 * u) = pre.p[u];
      }
      if (tid < BQ) {
        Dv[tid] = pre.D;
        Lv[tid] = pre.L;
      }
      if (use_mask && tid < 64) Mw[(tid >> 5) * BQ + (tid & 31)] = pre.mw;
      __syncthreads();
      if (i0 + BQ < a.T1) fetch(i0 + BQ, pre);
      // S (32 queries x this wave's 16 keys): s[mi] rows 16mi + 4g + r, key column jw + lc
      f32x4 s[2], dp[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        s[mi] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) s[mi] = mfma(km_frag(quimg, 16 * mi, ks, lane), kf[ks], s[mi]);
      }
      if (REL) {
        // BDfull (32 x 96) over band rows rs + [0, 96): the 12 (mi, t) tiles split over the waves
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int idx = w + 4 * u, mi = idx / 6, t = idx % 6;
          f32x4 bd = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) bd = mfma(km_frag(qvimg, 16 * mi, ks, lane), km_frag(pimg, 16 * t, ks, lane), bd);
#pragma unroll
          for (int r = 0; r < 4; ++r) xs[(16 * mi + 4 * g + r) * V_XLD + 16 * t + lc] = bd[r];
        }
        __syncthreads();
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int il = 16 * mi + 4 * g + r, jl = 16 * w + lc;
            s[mi][r] += xs[il * V_XLD + (BQ - 1 - il) + jl];
          }
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        dp[mi] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) dp[mi] = mfma(km_frag(doimg, 16 * mi, ks, lane), vf[ks], dp[mi]);
      }
      // keep words of rows 16mi + 4g + r (this lane's bit bpos): staged mask, else rebuilt from
      // the counter hash, else all kept
      uint32_t mr[2][4];
      if (use_mask) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const uint4 m4 = *(const uint4*)(Mw + (w >> 1) * BQ + 16 * mi + 4 * g);
          mr[mi][0] = m4.x; mr[mi][1] = m4.y; mr[mi][2] = m4.z; mr[mi][3] = m4.w;
        }
      } else if (a.p > 0.f) {
        const uint32_t key = ea_seed_key(seed), thr = ea_drop_thr(a.p);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = i0 + 16 * mi + 4 * g + r;
            mr[mi][r] = (uint32_t)attn_keep(key, thr, (uint64_t)z * a.T1 + i, a.T2, j) << bpos;
          }
      } else {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) mr[mi][r] = ~0u;
      }
      union { bf16x8 v; bf16 e[8]; } ap, as;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const float4 D4 = *(const float4*)(Dv + 16 * mi + 4 * g);
        const float4 L4 = *(const float4*)(Lv + 16 * mi + 4 * g);
        const float Dm[4] = {D4.x, D4.y, D4.z, D4.w}, Lm[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + 16 * mi + 4 * g + r;
          const bool ok = j < kl && (unsigned)(i - imin) < (unsigned)(a.T1 - imin);
          const float e = __builtin_amdgcn_exp2f(fmaf(s[mi][r], sl2, -Lm[r]));
          const float P = ok ? e : 0.f;
          const float kp = ((mr[mi][r] >> bpos) & 1u) ? dsc : 0.f;
          as.e[4 * mi + r] = (bf16)((P * a.scale) * fmaf(dp[mi][r], kp, -Dm[r]));
          ap.e[4 * mi + r] = (bf16)(P * kp);
        }
      }
      // dV += Pd^T dO, dK += dS^T (Q+u): A = (key, 8 queries {4g..4g+3, 16+4g..16+4g+3}),
      // B = dO / Q+u rows in the same order (transposed reads)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        dva[n] = mfma(ap.v, km_frag_tr2(doimg, 4 * g, 16 + 4 * g, 16 * n, lane), dva[n]);
        dka[n] = mfma(as.v, km_frag_tr2(quimg, 4 * g, 16 + 4 * g, 16 * n, lane), dka[n]);
      }
    }
  }
  // dK, dV rows jw + 4g + r (zero for keys at or past klen)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = jw + 4 * g + r;
    if (j >= a.T2) continue;
    bf16* dkr = a.dk + ((long)b * a.T2 + j) * a.lddk + h * DK;
    bf16* dvr = a.dv + ((long)b * a.T2 + j) * a.lddv + h * DK;
    const bool ok = j < kl;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      dkr[16 * n + lc] = (bf16)(ok ? dka[n][r] : 0.f);
      dvr[16 * n + lc] = (bf16)(ok ? dva[n][r] : 0.f);
    }
  }
}

// ------------------------------------------------------------ attn_bwdkv, pipelined (v2)
// attn_bwdkv_kernel with the same treatment: the 32-query tiles (q + u, q + v, dO images), their
// D_i / lse_i / keep words and the positional rows (a 128-row ring: a tile's band is 96 rows,
// the next tile's 32 new rows lie below it) are filled by LDS-DMA one tile ahead, so a tile
// costs one barrier; each wave computes the three BD tiles its 16 keys read and gathers them by
// ds_bpermute (no shared BDfull image, no second barrier).  dK, dV stay in registers.
constexpr int RINGK = 128;
template <bool REL>
struct KV2 {
  static constexpr int IMG = BQ * 128;                          // one 32-row km image
  static constexpr int QU = 0, QV = QU + 2 * IMG, DO = QV + (REL ? 2 * IMG : 0), P = DO + 2 * IMG;
  static constexpr int SM = P + (REL ? RINGK * 128 : 0);        // [2][D 32 | L 32 | mask 2 x 32]
  static constexpr int LDS = SM + 2 * 128 * 4;
};
static_assert(KV2<true>::LDS <= 80 * 1024, "two workgroups per CU");

// km_frag_tr2 via asm (rows k0 + q for half 0, k1 + q for half 1)
EA_DEV bf16x8 km_tr2_asm(const char* img, int k0, int k1, int n0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = n0 + 4 * p;
  union { bf16x8 v; s16x4 h[2]; } out;
  out.h[0] = tr_asm(img + km_off(k0 + q, col >> 3) + (col & 7) * 2);
  out.h[1] = tr_asm(img + km_off(k1 + q, col >> 3) + (col & 7) * 2);
  return out.v;
}
EA_DEV void dma_dword(char* lds, const void* src) {  // lane L writes lds + 4L
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

template <bool REL, int MM>
__global__ __launch_bounds__(256, 2) void attn_bwdkv2_kernel(AttnP a) {
  using L = KV2<REL>;
  __shared__ __attribute__((aligned(16))) char sm[L::LDS];
  const int nkb = (a.T2 + 63) / 64;
  const int z = blockIdx.x / nkb, kb = blockIdx.x % nkb;
  const int b = z / a.H, h = z % a.H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: ring / image offsets stay scalar
  const int g = lane >> 4, lc = lane & 15;
  const int kl = a.klen ? (int)min((long long)a.T2, a.klen[b]) : a.T2;
  const uint64_t seed = MM == 2 ? ea_salted(a.seed, a.salt) : 0;
  const int j0 = 64 * kb, jw = j0 + 16 * w;
  f32x4 dka[4], dva[4];  // rows = keys jw + 4g + r, columns 16n + lc
#pragma unroll
  for (int n = 0; n < 4; ++n) dka[n] = dva[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (j0 < kl) {
    const int j = jw + lc;
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = vf[ks] = (bf16x8){};
      if (j < kl) {
        kf[ks] = *(const bf16x8*)(a.k + ((long)b * a.T2 + j) * a.ldk + h * DK + 32 * ks + 8 * g);
        vf[ks] = *(const bf16x8*)(a.v + ((long)b * a.T2 + j) * a.ldv + h * DK + 32 * ks + 8 * g);
      }
    }
    const float dsc = MM ? 1.f / (1.f - a.p) : 1.f;
    const float sl2 = a.scale * LOG2E;
    const int istart = a.causal ? (j0 / BQ) * BQ : 0;
    const int imin = a.causal ? j : 0;  // rows i in [imin, T1) see key j (if j < kl)
    const int bpos = 16 * (w & 1) + lc;  // this lane's bit in keep word w>>1
    const int ntile = (a.T1 - istart + BQ - 1) / BQ;
    const int rs0 = a.T1 - 1 - (istart + BQ - 1) + j0;  // first tile's first band row
    const char* quh = (const char*)(a.wsQu + (long)b * a.T1 * a.ldqu + h * DK);
    const char* qvh = REL ? (const char*)(a.wsQv + (long)b * a.T1 * a.ldqvw + h * DK) : nullptr;
    const char* doh = (const char*)(a.dO + (long)b * a.T1 * a.lddo + h * DK);
    const char* ph_ = REL ? (const char*)(a.pp + h * DK) : nullptr;
    // 32-bit LDS-DMA source offsets (the launcher checked the head slices' byte ranges)
    const uint32_t ldqub = (uint32_t)a.ldqu * 2, ldqvb = (uint32_t)a.ldqvw * 2, lddob = (uint32_t)a.lddo * 2;
    const uint32_t ldpb = REL ? (uint32_t)a.ldp * 2 : 0;
    const int chx = km_chx(lane);
    // lane offsets of the 16 x 32 fragments of a km image at a 16-row boundary
    int loff[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) loff[ks] = lc * 128 + (((ks * 4 + g) ^ km_swz(lc)) << 4);
    // tile m: images at buffer m & 1; ring rows rs0 - 32m + [0, 96) at positions
    // (row - rs0) mod 128; small arrays: D, lse (log2 scaled at use), keep words of 32 rows
    auto dma_tile = [&](int m, bool first) {
      const int i0 = istart + BQ * m;
      const int buf = m & 1;
      const int ir = 8 * w;
      km_dma8u(sm + L::QU + buf * L::IMG + ir * 128, ir, quh, ldqub, i0 + ir, a.T1, chx, lane);
      if (REL) km_dma8u(sm + L::QV + buf * L::IMG + ir * 128, ir, qvh, ldqvb, i0 + ir, a.T1, chx, lane);
      km_dma8u(sm + L::DO + buf * L::IMG + ir * 128, ir, doh, lddob, i0 + ir, a.T1, chx, lane);
      if (REL) {
        // first tile: all 96 rows (12 groups); later: the 32 new rows below the previous band
        const int x0 = first ? 0 : -32 * m, ng = first ? 12 : 4;
        for (int gi = w; gi < ng; gi += 4) {
          const int x = x0 + 8 * gi;  // relative to rs0; position x mod 128
          const int xr = ((x % RINGK) + RINGK) % RINGK;
          km_dma8u(sm + L::P + xr * 128, xr, ph_, ldpb, rs0 + x, 2 * a.T1 - 1, chx, lane);
        }
      }
      if (w == 0) {
        char* s = sm + L::SM + buf * 512;
        const int ir = min(i0 + (lane & 31), a.T1 - 1);
        const float* src = lane < 32 ? a.wsD + (long)z * a.T1 + ir : a.lse + (long)z * a.T1 + ir;
        dma_dword(s, src);
        if (MM == 1) dma_dword(s + 256, a.dmask + ((long)z * a.T1 + ir) * a.ldm + (j0 >> 5) + (lane >> 5));
      }
    };
    if (ntile > 0) dma_tile(0, true);
    for (int m = 0; m < ntile; ++m) {
      const int i0 = istart + BQ * m;
      vmcnt_le<0>();
      bar();
      if (m + 1 < ntile) dma_tile(m + 1, false);
      const int buf = m & 1;
      const char* quimg = sm + L::QU + buf * L::IMG;
      const char* qvimg = sm + L::QV + buf * L::IMG;
      const char* doimg = sm + L::DO + buf * L::IMG;
      const char* smv = sm + L::SM + buf * 512;
      // S (32 queries x this wave's 16 keys): s[mi] rows 16mi + 4g + r, key column jw + lc
      f32x4 s[2], dp[2];
      {
        bf16x8 qf[2][2], df[2][2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            qf[mi][ks] = ld128_asm(quimg + 2048 * mi + loff[ks]);
            df[mi][ks] = ld128_asm(doimg + 2048 * mi + loff[ks]);
          }
        lgkm0();
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          s[mi] = dp[mi] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            s[mi] = mfma(qf[mi][ks], kf[ks], s[mi]);
            dp[mi] = mfma(df[mi][ks], vf[ks], dp[mi]);
          }
        }
      }
      if (REL) {
        // BDfull tiles (mi, t) for t in {w, w+1, w+2}: band rows rs + 16t + [0, 16) with
        // rs = rs0 - 32m (ring position (16t - 32m) mod 128)
        f32x4 bd[2][3];
        {
          bf16x8 vq[2][2], pf[3][2];
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) vq[mi][ks] = ld128_asm(qvimg + 2048 * mi + loff[ks]);
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int rp = (((16 * (w + u) - 32 * m) % RINGK) + RINGK) % RINGK;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) pf[u][ks] = ld128_asm(sm + L::P + rp * 128 + loff[ks]);  // rp % 16 == 0
          }
          lgkm0();
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int u = 0; u < 3; ++u) {
              bd[mi][u] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int ks = 0; ks < 2; ++ks) bd[mi][u] = mfma(vq[mi][ks], pf[u][ks], bd[mi][u]);
            }
        }
        // (il = 16mi + 4g + r, jl = 16w + lc) reads BDfull column 31 - il + jl = 16(w + u) +
        // ((lc + 31 - 16mi - 4g - r) & 15), u = (lc + 31 - 16mi - 4g - r) >> 4
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int sft = lc + 31 - 16 * mi - 4 * g - r;
            const int src = (16 * g + (sft & 15)) * 4;
            const float x0 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[mi][0][r])));
            const float x1 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[mi][1][r])));
            const float x2 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bd[mi][2][r])));
            const int u = sft >> 4;
            s[mi][r] += u == 0 ? x0 : (u == 1 ? x1 : x2);
          }
      }
      // keep words of rows 16mi + 4g + r (this lane's bit bpos), D_i, lse_i
      float Dm[2][4], Lm[2][4];
      uint32_t mr[2][4];
      {
        bf16x8 dv[2], lv[2], mv[2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          dv[mi] = ld128_asm(smv + (16 * mi + 4 * g) * 4);
          lv[mi] = ld128_asm(smv + 128 + (16 * mi + 4 * g) * 4);
          if (MM == 1) mv[mi] = ld128_asm(smv + 256 + (w >> 1) * 128 + (16 * mi + 4 * g) * 4);
        }
        lgkm0();
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const float4 D4 = __builtin_bit_cast(float4, dv[mi]);
          const float4 L4 = __builtin_bit_cast(float4, lv[mi]);
          Dm[mi][0] = D4.x; Dm[mi][1] = D4.y; Dm[mi][2] = D4.z; Dm[mi][3] = D4.w;
          Lm[mi][0] = L4.x * LOG2E; Lm[mi][1] = L4.y * LOG2E; Lm[mi][2] = L4.z * LOG2E; Lm[mi][3] = L4.w * LOG2E;
          if (MM == 1) {
            const uint4 m4 = __builtin_bit_cast(uint4, mv[mi]);
            mr[mi][0] = m4.x; mr[mi][1] = m4.y; mr[mi][2] = m4.z; mr[mi][3] = m4.w;
          }
        }
      }
      if (MM == 2) {
        const uint32_t key = ea_seed_key(seed), thr = ea_drop_thr(a.p);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = i0 + 16 * mi + 4 * g + r;
            mr[mi][r] = (uint32_t)attn_keep(key, thr, (uint64_t)z * a.T1 + i, a.T2, j) << bpos;
          }
      }
      union { bf16x8 v; bf16 e[8]; } ap, as;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + 16 * mi + 4 * g + r;
          const bool ok = j < kl && (unsigned)(i - imin) < (unsigned)(a.T1 - imin);
          const float e = __builtin_amdgcn_exp2f(fmaf(s[mi][r], sl2, -Lm[mi][r]));
          const float P = ok ? e : 0.f;
          const float kp = MM ? (((mr[mi][r] >> bpos) & 1u) ? dsc : 0.f) : 1.f;
          as.e[4 * mi + r] = (bf16)((P * a.scale) * fmaf(dp[mi][r], kp, -Dm[mi][r]));
          ap.e[4 * mi + r] = (bf16)(P * kp);
        }
      // dV += Pd^T dO, dK += dS^T (Q+u): A = (key, 8 queries {4g..4g+3, 16+4g..16+4g+3}),
      // B = dO / Q+u rows in the same order (transposed reads)
      {
        bf16x8 bo[4], bu[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          bo[n] = km_tr2_asm(doimg, 4 * g, 16 + 4 * g, 16 * n, lane);
          bu[n] = km_tr2_asm(quimg, 4 * g, 16 + 4 * g, 16 * n, lane);
        }
        lgkm0();
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          dva[n] = mfma(ap.v, bo[n], dva[n]);
          dka[n] = mfma(as.v, bu[n], dka[n]);
        }
      }
    }
  }
  // dK, dV rows jw + 4g + r (zero for keys at or past klen)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = jw + 4 * g + r;
    if (j >= a.T2) continue;
    bf16* dkr = a.dk + ((long)b * a.T2 + j) * a.lddk + h * DK;
    bf16* dvr = a.dv + ((long)b * a.T2 + j) * a.lddv + h * DK;
    const bool ok = j < kl;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      dkr[16 * n + lc] = (bf16)(ok ? dka[n][r] : 0.f);
      dvr[16 * n + lc] = (bf16)(ok ? dva[n][r] : 0.f);
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

extern "C" int ea_attn_fused_fwd2(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                                  long ldk, const void* v, long ldv, const float* bu, const float* bv,
                                  const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                                  unsigned long long seed, void* o, long ldo, float* lse, unsigned* dmask, int ldm,
                                  void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(dk == DK && B >= 1 && H >= 1 && T1 >= 1 && T2 >= 1);
  EA_CHECK_ARG(!pp || (T1 == T2 && bv != nullptr));
  EA_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && (!pp || ldp % 8 == 0));
  EA_CHECK_ARG(!dmask || ldm >= 2 * ((T2 + 63) / 64));
  AttnP a = make_p(B, H, T1, T2, q, ldq, k, ldk, v, ldv, bu, bv, pp, ldp, klen, causal, scale, p, seed);
  a.o = (bf16*)o; a.ldo = ldo; a.lse = lse;
  a.dmask = (uint32_t*)dmask; a.ldm = ldm;
  dim3 grid(B * H * ((T1 + QB - 1) / QB));
  const hipStream_t st = (hipStream_t)stream;
  const char* ev = getenv("EA_ATTN_FWD_V1");  // A/B: the original forward kernel
  // the pipelined kernel's LDS-DMA sources are 32-bit byte offsets (__umul24(row, row bytes))
  // from each head's base: beyond that range the original kernel runs
  const auto fits = [](long rows, long ld) { return ld * 2 < (1L << 24) && rows * ld * 2 + 128 < (1L << 32); };
  const bool off32 = fits(T2, ldk) && fits(T2, ldv) && (!pp || fits(2L * T1, ldp));
  const bool v1 = (ev && ev[0] == '1') || !off32;
  const int mm = p > 0.f ? (dmask ? 1 : 2) : 0;
  if (v1) {
    if (pp) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(256), 0, st, a);
  } else if (pp) {
    if (mm == 0) hipLaunchKernelGGL((attn_fwd2_kernel<true, 0>), grid, dim3(256), 0, st, a);
    else if (mm == 1) hipLaunchKernelGGL((attn_fwd2_kernel<true, 1>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_fwd2_kernel<true, 2>), grid, dim3(256), 0, st, a);
  } else {
    if (mm == 0) hipLaunchKernelGGL((attn_fwd2_kernel<false, 0>), grid, dim3(256), 0, st, a);
    else if (mm == 1) hipLaunchKernelGGL((attn_fwd2_kernel<false, 1>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_fwd2_kernel<false, 2>), grid, dim3(256), 0, st, a);
  }
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_attn_fused_fwd(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                                 long ldk, const void* v, long ldv, const float* bu, const float* bv,
                                 const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                                 unsigned long long seed, void* o, long ldo, float* lse, void* stream) {
  return ea_attn_fused_fwd2(B, H, T1, T2, dk, q, ldq, k, ldk, v, ldv, bu, bv, pp, ldp, klen, causal, scale, p, seed,
                            o, ldo, lse, nullptr, 0, stream);
}

static int attn_bwd_launch(AttnP& a, bool rel, bool v2, hipStream_t st) {
  const int nqb = (a.T1 + QB - 1) / QB, nkb = (a.T2 + 63) / 64;
  // the pipelined dQ pass addresses K / V / positional rows with 32-bit byte offsets from each
  // head's base (__umul24(row, row bytes))
  const auto fits = [](long rows, long ld) { return ld * 2 < (1L << 24) && rows * ld * 2 + 128 < (1L << 32); };
  EA_CHECK_ARG(!v2 || (fits(a.T2, a.ldk) && fits(a.T2, a.ldv) && (!rel || fits(2L * a.T1, a.ldp)) &&
                       (!a.dbd || fits(a.T1, a.lddbd))));
  // the pipelined dK / dV pass likewise (else the original one runs)
  const bool kv32 = fits(a.T1, a.ldqu) && fits(a.T1, a.lddo) && (!rel || (fits(a.T1, a.ldqvw) && fits(2L * a.T1, a.ldp)));
  const dim3 gq(a.B * a.H * nqb), gkv(a.B * a.H * nkb);
  const int mm = a.p > 0.f ? (a.dmask ? 1 : 2) : 0;
  const char* ev = getenv("EA_ATTN_BWDKV_V1");  // A/B: the original dK/dV pass
  const bool kv1 = ev && ev[0] == '1';
  if (rel) {
    if (v2 && mm == 0) hipLaunchKernelGGL((attn_bwdq2_kernel<true, 0>), gq, dim3(256), 0, st, a);
    else if (v2 && mm == 1) hipLaunchKernelGGL((attn_bwdq2_kernel<true, 1>), gq, dim3(256), 0, st, a);
    else if (v2) hipLaunchKernelGGL((attn_bwdq2_kernel<true, 2>), gq, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(attn_bwdq_kernel<true>, gq, dim3(256), 0, st, a);
    if (kv1 || !kv32) hipLaunchKernelGGL(attn_bwdkv_kernel<true>, gkv, dim3(256), 0, st, a);
    else if (mm == 0) hipLaunchKernelGGL((attn_bwdkv2_kernel<true, 0>), gkv, dim3(256), 0, st, a);
    else if (mm == 1) hipLaunchKernelGGL((attn_bwdkv2_kernel<true, 1>), gkv, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_bwdkv2_kernel<true, 2>), gkv, dim3(256), 0, st, a);
  } else {
    if (v2 && mm == 0) hipLaunchKernelGGL((attn_bwdq2_kernel<false, 0>), gq, dim3(256), 0, st, a);
    else if (v2 && mm == 1) hipLaunchKernelGGL((attn_bwdq2_kernel<false, 1>), gq, dim3(256), 0, st, a);
    else if (v2) hipLaunchKernelGGL((attn_bwdq2_kernel<false, 2>), gq, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(attn_bwdq_kernel<false>, gq, dim3(256), 0, st, a);
    if (kv1 || !kv32) hipLaunchKernelGGL(attn_bwdkv_kernel<false>, gkv, dim3(256), 0, st, a);
    else if (mm == 0) hipLaunchKernelGGL((attn_bwdkv2_kernel<false, 0>), gkv, dim3(256), 0, st, a);
    else if (mm == 1) hipLaunchKernelGGL((attn_bwdkv2_kernel<false, 1>), gkv, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_bwdkv2_kernel<false, 2>), gkv, dim3(256), 0, st, a);
  }
  EA_LAUNCH_CHECK();
  return 0;
}

static long attn_ws_layout(int B, int H, int T1, long* qu_off, long* qv_off, long* dummy_off = nullptr) {
  const long d = (long)B * H * T1 * 4, q = (long)B * T1 * H * DK * 2;
  *qu_off = (d + 255) / 256 * 256;
  *qv_off = *qu_off + (q + 255) / 256 * 256;
  const long du = *qv_off + (q + 255) / 256 * 256;
  if (dummy_off) *dummy_off = du;
  return du + 1024;
}

extern "C" int ea_attn_fused_bwd_ws_bytes(int B, int H, int T1, long* bytes) {
  EA_CHECK_ARG(B >= 1 && H >= 1 && T1 >= 1 && bytes != nullptr);
  long qu, qv;
  *bytes = attn_ws_layout(B, H, T1, &qu, &qv);
  return 0;
}

extern "C" int ea_attn_fused_bwd2(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                                  long ldk, const void* v, long ldv, const float* bu, const float* bv,
                                  const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                                  unsigned long long seed, const void* o, long ldo, const float* lse, const void* dO,
                                  long lddo, void* dq, long lddq, void* dkout, long lddk, void* dvout, long lddv,
                                  void* dbd, long lddbd, float* bias_part, long ldpart, void* qv_out, long ldqv,
                                  const unsigned* dmask, int ldm, void* ws, long ws_bytes, int flags, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(dk == DK && B >= 1 && H >= 1 && T1 >= 1 && T2 >= 1);
  EA_CHECK_ARG(!pp || (T1 == T2 && bv != nullptr));
  EA_CHECK_ARG(flags >= 0 && flags <= 7 && !((flags & 2) && (flags & 4)));
  // flags bit 1: pipelined dQ pass, dbd in the shifted layout; bit 2: the original dQ pass
  // (A/B); neither: the original pass when dbd is given (unshifted layout), else the pipelined
  const bool v2 = (flags & 2) || (!(flags & 4) && !dbd);
  const long ldmin = (flags & 2) ? ea_attn_dbd_ld(T1) : 2L * T1 - 1;
  EA_CHECK_ARG(!dbd || (pp && lddbd >= ldmin && lddbd % 8 == 0 && (uintptr_t)dbd % 16 == 0));
  EA_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 8 == 0 && lddo % 8 == 0 &&
               (!pp || ldp % 8 == 0) && (!qv_out || (pp && ldqv % 8 == 0)));
  EA_CHECK_ARG(!bias_part || ldpart >= (long)H * DK);
  EA_CHECK_ARG(!(flags & 1) || pp);
  EA_CHECK_ARG(!dmask || ldm >= 2 * ((T2 + 63) / 64));
  long qu_off, qv_off, du_off;
  EA_CHECK_ARG(ws != nullptr && (uintptr_t)ws % 256 == 0 &&
               ws_bytes >= attn_ws_layout(B, H, T1, &qu_off, &qv_off, &du_off));
  AttnP a = make_p(B, H, T1, T2, q, ldq, k, ldk, v, ldv, bu, bv, pp, ldp, klen, causal, scale, p, seed);
  a.o = (bf16*)o; a.ldo = ldo; a.lse = (float*)lse;
  a.dO = (const bf16*)dO; a.lddo = lddo;
  a.dq = (bf16*)dq; a.lddq = lddq; a.dk = (bf16*)dkout; a.lddk = lddk; a.dv = (bf16*)dvout; a.lddv = lddv;
  a.dbd = (bf16*)dbd; a.lddbd = lddbd;
  a.bias_part = bias_part; a.ldpart = ldpart;
  a.flags = flags;
  a.dmask = (uint32_t*)dmask; a.ldm = ldm;
  a.wsD = (float*)ws;
  a.wsDummy = (char*)ws + du_off;
  a.wsQu = (bf16*)((char*)ws + qu_off); a.ldqu = (long)H * DK;
  if (qv_out) { a.wsQv = (bf16*)qv_out; a.ldqvw = ldqv; }
  else { a.wsQv = (bf16*)((char*)ws + qv_off); a.ldqvw = (long)H * DK; }
  return attn_bwd_launch(a, pp != nullptr, v2, (hipStream_t)stream);
}

extern "C" int ea_attn_dbd_layout(int T1, int* shift, long* lddbd) {
  EA_CHECK_ARG(T1 >= 1 && shift != nullptr && lddbd != nullptr);
  *shift = ea_attn_dbd_shift_dev(T1);
  *lddbd = ea_attn_dbd_ld(T1);
  return 0;
}
