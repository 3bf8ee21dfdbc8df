// MFMA GEMM for gfx950 with fused epilogues (see include/espnet_amd.h: ea_gemm).
//
// Tile 128x128, 256 threads = 4 wave64s in 2x2, each wave owns a 64x64 sub-tile
// (4x4 MFMA 16x16 blocks).  K-tiles of 64 (bf16) / 32 (f32) are staged
// global -> registers -> LDS (double buffered, one barrier per K-tile); the next
// tile's global loads are issued before the current tile's MFMAs so HBM latency
// hides under the math.
//
// LDS images keep the operand's global orientation:
//  * K-contiguous operand  -> [mn][K-tile] rows of 128 B, 16-B chunk XOR-swizzled by
//    (row>>1)&7; bf16 fragments are one ds_read_b128 (conflict-free for the
//    ds_read_b128 lane groups), f32 fragments one ds_read_b32.
//  * MN-contiguous operand -> [k][128] rows; bf16 fragments come from two
//    ds_read_b64_tr_b16 (hardware transpose), chunk swizzle 2*((k&3)|((k>>3)&1)<<2) so
//    the 8 rows of a 32-lane half land on 8 distinct 32-B bank windows.
// So Linear forward (A K-major, W K-major), dX = dY.W (B N-major) and
// dW = dY^T.X (A M-major, B N-major) all run without explicit transposes.
// Shared by the GEMM translation units (gemm.hip: host dispatch and the register-staged
// kernel; gemm_pipe*.hip / gemm_lds*.hip: the LDS-DMA kernels; gemm_grouped.hip), so the
// kernel instantiations compile in parallel.  Types and launchers live in namespace eag; the
// device code stays in an anonymous namespace (each unit instantiates only what it launches).
#pragma once
#include "common.h"


namespace eag {

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int TILE_BYTES = 16384;

template <typename T> struct KCfg;
template <> struct KCfg<bf16> { static constexpr int KT = 64, KS = 32, E = 8, NKS = 2; };
template <> struct KCfg<float> { static constexpr int KT = 32, KS = 4, E = 4, NKS = 8; };

struct GemmP {
  int M, N, K;
  const void* A; long lda, sAb, sAh;
  const void* B; long ldb, sBb, sBh;
  int nh, splitk, kchunk;
  void* C; int c_dtype; long ldc, sCb, sCh;
  ea_epilogue epi;
  float* ws;  // split-K partial slabs [z][s][M][N]
  int tiles_m, tiles_n;
  int vec_a, vec_b;  // 16-B vector loads allowed (aligned base, ld and batch strides)
  int vec_c;         // 4-column vector epilogue allowed (aligned C/aux/resid/bias, N % 4 == 0)
  int vec8;          // 8-column (16-B) epilogue allowed (N % 8 == 0, 16-B aligned rows of C/aux/resid)
  int lds;           // bf16 LDS-DMA kernel eligible (aligned operands < 4 GB)
  int bm, bn;        // output tile (LDS-DMA bf16 kernel: 64/128/256 x 128/256; else 128 x 128)
  const unsigned long long* salt;  // per-step dropout salt (device), see ea_set_rng_salt
  unsigned long long* stamp;       // kernel-span probe [first block start, last block end] or null
  ea_conv_geo g;                   // implicit-GEMM operand geometry (g.mode 0: dense operands)
  unsigned long long* diag;        // ea_gemm_set_diag: per-block [start, main loop done, end] s_memtime
  const float* w1x;                // ea_gemm_conv_w1: conv1 input (B, w1T, w1F) f32, or null
  float* w1part;                   //   per-M-tile conv1 weight / bias gradient partials
  const uint8_t* w1pos;            //   ReLU support bits (N/8 bytes per row) instead of aux, or null
  int w1T, w1F;
  // ea_gemm_conv_w1b_all: the four parity classes of the conv2 input gradient in ONE grid,
  // items ordered by class (longest K first), each class's tiles at cls_item0[c] ..; 0 = one class
  int ncls;
  int cls_item0[5], cls_M[4], cls_K[4], cls_a[4], cls_e[4], cls_tile0[4];
  long cls_pos[4];                 //   byte offset of the class plane's first row in w1pos
};

// launchers of the LDS-DMA kernels (grid = tiles x 1 x (batch * split-K slices))
int launch_pipe(GemmP& p, int a_k, int b_k, dim3 grid, hipStream_t st);  // gemm_pipe.hip: 256 / 128 tiles
int launch_k128(GemmP& p, dim3 grid, hipStream_t st);                     // gemm_k128.hip: 128x128 K-major
int launch_pipe_conv(GemmP& p, dim3 grid, hipStream_t st);               // gemm_pipe_conv.hip: conv2 modes
int launch_lds_dense(GemmP& p, int a_k, int b_k, dim3 grid, hipStream_t st);  // gemm_lds.hip
int launch_lds_conv(GemmP& p, dim3 grid, hipStream_t st);                     // gemm_lds_conv.hip
int launch_skinny(GemmP& p, hipStream_t st);  // gemm_skinny.hip: few-row bf16, K split over waves
int launch_skinny_ln(GemmP& p, const float* gamma, const float* beta, float eps, hipStream_t st);  // + LayerNorm
extern int g_k128_slots;     // ring depth of gemm_k128 (3 or 4)
}  // namespace eag

namespace {
using namespace eag;

// Diagnostic timeline (ea_gemm_set_diag): thread 0 of each block stamps the shader clock at
// the block's start, after its main loop and at its end; off (null) in normal runs.
EA_DEV void diag_stamp(const GemmP& p, int slot) {
  if (p.diag && threadIdx.x == 0) {
    const long b = blockIdx.x + (long)gridDim.x * blockIdx.z;
    p.diag[b * 4 + slot] = __builtin_amdgcn_s_memtime();
    if (slot == 0) p.diag[b * 4 + 3] = __builtin_amdgcn_s_memrealtime();
  }
}

// In-kernel span probe (ea_gemm_set_probe): s_memrealtime is the GPU's constant 100 MHz
// clock; the first block to start and the last to finish bound the launch's execution.
EA_DEV void probe_start(const GemmP& p) {
  if (p.stamp && threadIdx.x == 0) atomicMin(&p.stamp[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
EA_DEV void probe_end(const GemmP& p) {
  if (p.stamp) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&p.stamp[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

EA_DEV int swz_k(int row) { return (row >> 1) & 7; }                         // K-major rows
EA_DEV int swz_mn_bf16(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }  // [k][128] bf16
EA_DEV int swz_mn_f32(int k) { return (k & 1) * 4; }                         // [k][128] f32

// ---------------------------------------------------------------- global -> registers
template <typename T, bool KMAJ>
EA_DEV void load_tile(const T* __restrict__ base, long ld, int mn0, int MN, int k0, int K,
                      int vec, uint4 (&v)[4]) {
  constexpr int E = KCfg<T>::E;
  constexpr int CPR = KMAJ ? 8 : (128 * (int)sizeof(T)) / 16;  // 16-B chunks per LDS row
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = threadIdx.x + NT * i;
    const int row = c / CPR, ch = c % CPR;
    int mn, k;
    if (KMAJ) { mn = mn0 + row; k = k0 + ch * E; }
    else      { k = k0 + row; mn = mn0 + ch * E; }
    const T* p = KMAJ ? base + (long)mn * ld + k : base + (long)k * ld + mn;
    const bool full = vec && (KMAJ ? (mn < MN && k + E <= K) : (k < K && mn + E <= MN));
    if (full) {
      v[i] = *(const uint4*)p;
    } else {
      union { uint4 u; T e[E]; } t;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const bool ok = KMAJ ? (mn < MN && k + e < K) : (k < K && mn + e < MN);
        t.e[e] = ok ? p[e] : (T)0.f;
      }
      v[i] = t.u;
    }
  }
}

template <typename T, bool KMAJ>
EA_DEV void store_tile(char* lds, const uint4 (&v)[4]) {
  constexpr int CPR = KMAJ ? 8 : (128 * (int)sizeof(T)) / 16;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = threadIdx.x + NT * i;
    const int row = c / CPR, ch = c % CPR;
    int off;
    if (KMAJ) off = row * 128 + ((ch ^ swz_k(row)) << 4);
    else if (sizeof(T) == 2) off = row * 256 + ((ch ^ swz_mn_bf16(row)) << 4);
    else off = row * 512 + ((ch ^ swz_mn_f32(row)) << 4);
    *(uint4*)(lds + off) = v[i];
  }
}

// ---------------------------------------------------------------- LDS -> fragments
// bf16: fragment = 8 consecutive k of row/col (lane&15), k-block 8*(lane>>4)
template <bool KMAJ>
EA_DEV bf16x8 frag_bf16(const char* lds, int r0, int ks, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    const int ch = ks * 4 + (lane >> 4);
    return *(const bf16x8*)(lds + row * 128 + ((ch ^ swz_k(row)) << 4));
  } else {
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const int col = r0 + 4 * p;
    const int ch = col >> 3, within = (col & 7) * 2;
    union { bf16x8 v; s16x4 h[2]; } out;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = ks * 32 + 8 * (lane >> 4) + 4 * half + q;
      const char* a = lds + row * 256 + ((ch ^ swz_mn_bf16(row)) << 4) + within;
      out.h[half] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(a));
    }
    return out.v;
  }
}
// f32: fragment = element (row/col lane&15, k = ks*4 + lane>>4)
template <bool KMAJ>
EA_DEV float frag_f32(const char* lds, int r0, int ks, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    return *(const float*)(lds + row * 128 + ((ks ^ swz_k(row)) << 4) + (lane >> 4) * 4);
  } else {
    const int k = ks * 4 + (lane >> 4);
    const int col = r0 + (lane & 15);
    return *(const float*)(lds + k * 512 + (((col >> 2) ^ swz_mn_f32(k)) << 4) + (col & 3) * 4);
  }
}

// ---------------------------------------------------------------- epilogue
template <int KIND>
EA_DEV void epi_one(const GemmP& p, int z, int zb, int zh, int row, int col, float acc) {
  const ea_epilogue& e = p.epi;
  const long cidx = zb * p.sCb + zh * p.sCh + (long)row * p.ldc + col;
  const uint64_t didx = ((uint64_t)z * p.M + row) * (uint64_t)p.N + col;
  const uint64_t seed = e.drop_p > 0.f ? ea_salted(e.seed, p.salt) : 0;
  float v = e.alpha * acc;
  if constexpr (KIND == EA_EPI_STORE) {
    if (e.bias) v += e.bias[col];
    v *= e.post_scale;
    if (e.drop_p > 0.f) v *= drop_scale(seed, didx, e.drop_p);
    if (e.beta != 0.f) v += e.beta * load_as_f(p.C, cidx, p.c_dtype);
    store_from_f(p.C, cidx, p.c_dtype, v);
  } else if constexpr (KIND == EA_EPI_ACT) {
    if (e.bias) v += e.bias[col];
    if (e.aux) store_from_f(e.aux, (long)row * e.ldaux + col, e.aux_dtype, v);
    float a = act_fwd(e.act, v);
    if (e.drop_p > 0.f) a *= drop_scale(seed, didx, e.drop_p);
    store_from_f(p.C, cidx, p.c_dtype, a);
  } else if constexpr (KIND == EA_EPI_RESID) {
    if (e.bias) v += e.bias[col];
    if (e.drop_p > 0.f) v *= drop_scale(seed, didx, e.drop_p);
    const float r = e.resid ? e.resid[(long)row * e.ldr + col] : 0.f;
    ((float*)p.C)[cidx] = r + e.rscale * v;
  } else {  // EA_EPI_DACT
    if (e.drop_p > 0.f) v *= drop_scale(seed, didx, e.drop_p);
    v *= act_bwd(e.act, load_as_f(e.aux, (long)row * e.ldaux + col, e.aux_dtype));
    store_from_f(p.C, cidx, p.c_dtype, v);
  }
}

EA_DEV void epi_apply(const GemmP& p, int z, int zb, int zh, int row, int col, float acc) {
  switch (p.epi.kind) {
    case EA_EPI_STORE: epi_one<EA_EPI_STORE>(p, z, zb, zh, row, col, acc); break;
    case EA_EPI_ACT: epi_one<EA_EPI_ACT>(p, z, zb, zh, row, col, acc); break;
    case EA_EPI_RESID: epi_one<EA_EPI_RESID>(p, z, zb, zh, row, col, acc); break;
    default: epi_one<EA_EPI_DACT>(p, z, zb, zh, row, col, acc); break;
  }
}

template <int KIND>
EA_DEV void epi_tile(const GemmP& p, int z, int zb, int zh, int r0, int c0, int lane,
                     const f32x4 (&acc)[4][4]) {
  const int rq = (lane >> 4) * 4, cc = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = r0 + i * 16 + rq + rr, col = c0 + j * 16 + cc;
        if (row < p.M && col < p.N) epi_one<KIND>(p, z, zb, zh, row, col, acc[i][j][rr]);
      }
}


// ---------------------------------------------------------------- vectorised epilogue
// 4 consecutive columns per lane: 16-B f32 / 8-B bf16 loads and stores instead of the
// MFMA layout's 2-4-B scattered accesses.  The accumulator tile is transposed through
// LDS (each wave its own 64 x 68-float region) before this runs.
EA_DEV void ld4(const void* p, long i, int dt, float (&v)[4]) {
  if (dt == EA_BF16) {
    const uint2 u = *(const uint2*)((const bf16*)p + i);
    const bf16* b = (const bf16*)&u;
    v[0] = (float)b[0]; v[1] = (float)b[1]; v[2] = (float)b[2]; v[3] = (float)b[3];
  } else {
    const float4 f = *(const float4*)((const float*)p + i);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  }
}
EA_DEV void st4(void* p, long i, int dt, const float (&v)[4]) {
  if (dt == EA_BF16) {
    uint2 u;
    bf16* b = (bf16*)&u;
    b[0] = (bf16)v[0]; b[1] = (bf16)v[1]; b[2] = (bf16)v[2]; b[3] = (bf16)v[3];
    *(uint2*)((bf16*)p + i) = u;
  } else {
    *(float4*)((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Launch-uniform dropout parameters, computed once per block: the salt is read from device
// memory here and nowhere else in the epilogue (a per-element re-read would be ordered after
// every preceding C store, which the compiler must assume may alias it).
struct EpiK {
  uint32_t key, thr;
  float sc;
  bool drop;
};
EA_DEV EpiK make_epik(const GemmP& p) {
  EpiK k;
  k.drop = p.epi.drop_p > 0.f;
  k.key = k.drop ? ea_seed_key(ea_salted(p.epi.seed, p.salt)) : 0u;
  k.thr = ea_drop_thr(p.epi.drop_p);
  k.sc = k.drop ? 1.f / (1.f - p.epi.drop_p) : 1.f;
  return k;
}
EA_DEV void drop4k(const EpiK& k, uint64_t idx, float (&v)[4]) {  // idx even
  if (!k.drop) return;
  const uint32_t h0 = ea_pair_hash(k.key, idx >> 1), h1 = ea_pair_hash(k.key, (idx >> 1) + 1);
  v[0] *= (h0 & 0xffffu) >= k.thr ? k.sc : 0.f;
  v[1] *= (h0 >> 16) >= k.thr ? k.sc : 0.f;
  v[2] *= (h1 & 0xffffu) >= k.thr ? k.sc : 0.f;
  v[3] *= (h1 >> 16) >= k.thr ? k.sc : 0.f;
}

// The operand an epilogue kind reads besides the accumulator (4 columns at (row, col)):
// STORE with beta != 0 reads C, RESID reads resid, DACT reads aux.  Returns false if none.
template <int KIND>
EA_DEV bool epi_src(const GemmP& p, int zb, int zh, int row, int col, float (&o)[4]) {
  const ea_epilogue& e = p.epi;
  if constexpr (KIND == EA_EPI_STORE) {
    if (e.beta == 0.f) return false;
    ld4(p.C, zb * p.sCb + zh * p.sCh + (long)row * p.ldc + col, p.c_dtype, o);
    return true;
  } else if constexpr (KIND == EA_EPI_RESID) {
    if (!e.resid) return false;
    ld4(e.resid, (long)row * e.ldr + col, EA_F32, o);
    return true;
  } else if constexpr (KIND == EA_EPI_DACT) {
    ld4(e.aux, (long)row * e.ldaux + col, e.aux_dtype, o);
    return true;
  }
  return false;
}

// acc (4 columns) + the preloaded operand `o` -> stored outputs
template <int KIND>
EA_DEV void epi_four_pre(const GemmP& p, const EpiK& k, int z, int zb, int zh, int row, int col,
                         const float (&acc)[4], const float (&bias)[4], bool has_o, const float (&o)[4]) {
  const ea_epilogue& e = p.epi;
  const long cidx = zb * p.sCb + zh * p.sCh + (long)row * p.ldc + col;
  const uint64_t didx = ((uint64_t)z * p.M + row) * (uint64_t)p.N + col;
  float v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = e.alpha * acc[c] + (KIND != EA_EPI_DACT ? bias[c] : 0.f);
  if constexpr (KIND == EA_EPI_STORE) {
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] *= e.post_scale;
    drop4k(k, didx, v);
    if (has_o) {
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] += e.beta * o[c];
    }
    st4(p.C, cidx, p.c_dtype, v);
  } else if constexpr (KIND == EA_EPI_ACT) {
    if (e.aux) st4(e.aux, (long)row * e.ldaux + col, e.aux_dtype, v);
    act_fwd_n<4>(e.act, v);
    drop4k(k, didx, v);
    st4(p.C, cidx, p.c_dtype, v);
  } else if constexpr (KIND == EA_EPI_RESID) {
    drop4k(k, didx, v);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (has_o ? o[c] : 0.f) + e.rscale * v[c];
    st4(p.C, cidx, EA_F32, v);
  } else {
    drop4k(k, didx, v);
    act_bwd_mul_n<4>(e.act, v, o);
    st4(p.C, cidx, p.c_dtype, v);
  }
}

// 8 consecutive columns (16-B bf16 / 2 x 16-B f32 accesses): the epilogue's stores are
// issue-bound with 8-B bf16 stores (MI355X: ~7 B/cycle/CU), so bf16 outputs and operands
// move 16 B per lane per instruction here
EA_DEV void ld8(const void* p, long i, int dt, float (&v)[8]) {
  if (dt == EA_BF16) {
    const uint4 u = *(const uint4*)((const bf16*)p + i);
    const bf16* b = (const bf16*)&u;
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = (float)b[c];
  } else {
    const float4 f0 = *(const float4*)((const float*)p + i), f1 = *(const float4*)((const float*)p + i + 4);
    v[0] = f0.x; v[1] = f0.y; v[2] = f0.z; v[3] = f0.w; v[4] = f1.x; v[5] = f1.y; v[6] = f1.z; v[7] = f1.w;
  }
}
EA_DEV void st8(void* p, long i, int dt, const float (&v)[8]) {
  if (dt == EA_BF16) {
    union { uint4 u; bf16 b[8]; } t;
#pragma unroll
    for (int c = 0; c < 8; ++c) t.b[c] = (bf16)v[c];
    *(uint4*)((bf16*)p + i) = t.u;
  } else {
    *(float4*)((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)((float*)p + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}
EA_DEV void drop8k(const EpiK& k, uint64_t idx, float (&v)[8]) {  // idx even
  if (!k.drop) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t h = ea_pair_hash(k.key, (idx >> 1) + q);
    v[2 * q] *= (h & 0xffffu) >= k.thr ? k.sc : 0.f;
    v[2 * q + 1] *= (h >> 16) >= k.thr ? k.sc : 0.f;
  }
}
template <int KIND>
EA_DEV void epi_eight_pre(const GemmP& p, const EpiK& k, int z, int zb, int zh, int row, int col,
                          const float (&acc)[8], const float (&bias)[8], bool has_o, const float (&o)[8]) {
  const ea_epilogue& e = p.epi;
  const long cidx = zb * p.sCb + zh * p.sCh + (long)row * p.ldc + col;
  const uint64_t didx = ((uint64_t)z * p.M + row) * (uint64_t)p.N + col;
  float v[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) v[c] = e.alpha * acc[c] + (KIND != EA_EPI_DACT ? bias[c] : 0.f);
  if constexpr (KIND == EA_EPI_STORE) {
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] *= e.post_scale;
    drop8k(k, didx, v);
    if (has_o) {
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] += e.beta * o[c];
    }
    st8(p.C, cidx, p.c_dtype, v);
  } else if constexpr (KIND == EA_EPI_ACT) {
    if (e.aux) st8(e.aux, (long)row * e.ldaux + col, e.aux_dtype, v);
    act_fwd_n<8>(e.act, v);
    drop8k(k, didx, v);
    st8(p.C, cidx, p.c_dtype, v);
  } else if constexpr (KIND == EA_EPI_RESID) {
    drop8k(k, didx, v);
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = (has_o ? o[c] : 0.f) + e.rscale * v[c];
    st8(p.C, cidx, EA_F32, v);
  } else {
    drop8k(k, didx, v);
    act_bwd_mul_n<8>(e.act, v, o);
    st8(p.C, cidx, p.c_dtype, v);
  }
}

template <int KIND>
EA_DEV void epi_four(const GemmP& p, const EpiK& k, int z, int zb, int zh, int row, int col, const float (&acc)[4]) {
  float bias[4] = {0.f, 0.f, 0.f, 0.f}, o[4];
  if (p.epi.bias) {
    const float4 bb = *(const float4*)(p.epi.bias + col);
    bias[0] = bb.x; bias[1] = bb.y; bias[2] = bb.z; bias[3] = bb.w;
  }
  const bool has_o = epi_src<KIND>(p, zb, zh, row, col, o);
  epi_four_pre<KIND>(p, k, z, zb, zh, row, col, acc, bias, has_o, o);
}

// NB independent 4-column groups (rows[i], cols[i]) of one thread: every operand load is
// issued before the first store so their latencies overlap (stores to C may alias the
// operands, so the compiler cannot hoist a later group's loads above an earlier store).
// Out-of-range groups are skipped.  Vector path only (p.vec_c, which implies N % 4 == 0, so
// a group is wholly inside or wholly outside); callers run epi_one element-wise otherwise.
template <int KIND, int NB>
EA_DEV void epi_batch(const GemmP& p, const EpiK& k, int z, int zb, int zh, const int (&rows)[NB],
                      const int (&cols)[NB], const float (&v)[NB][4]) {
  float o[NB][4];
  bool has[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    has[i] = false;
    if (rows[i] < p.M && cols[i] < p.N) has[i] = epi_src<KIND>(p, zb, zh, rows[i], cols[i], o[i]);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    if (rows[i] >= p.M || cols[i] >= p.N) continue;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (KIND != EA_EPI_DACT && p.epi.bias) {
      const float4 bb = *(const float4*)(p.epi.bias + cols[i]);
      bias[0] = bb.x; bias[1] = bb.y; bias[2] = bb.z; bias[3] = bb.w;
    }
    epi_four_pre<KIND>(p, k, z, zb, zh, rows[i], cols[i], v[i], bias, has[i], o[i]);
  }
}

constexpr int EPI_LDT = 68;  // floats per LDS row of a wave's 64x64 accumulator tile

// ---------------------------------------------------------------- kernel
template <typename T, bool AK, bool BKM>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmP p) {
  constexpr int KT = KCfg<T>::KT, NKS = KCfg<T>::NKS;
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE_BYTES];

  // XCD-aware tile order: blocks b, b+8, ... share an XCD; give each XCD a contiguous
  // run of tiles (bijective remap), then walk tiles in column-groups of 8 row-tiles
  // so neighbouring tiles on one XCD share A rows / B columns in its L2.
  const int nt = p.tiles_m * p.tiles_n;
  const int b = blockIdx.x;
  const int q = nt / 8, r = nt % 8, xcd = b % 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
  const int GM = 8;
  const int grp = t / (GM * p.tiles_n);
  const int gm0 = grp * GM;
  const int gsz = min(GM, p.tiles_m - gm0);
  const int tm = gm0 + (t % (GM * p.tiles_n)) % gsz;
  const int tn = (t % (GM * p.tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int z = blockIdx.z / p.splitk, s = blockIdx.z % p.splitk;
  const int zb = z / p.nh, zh = z % p.nh;
  const T* A = (const T*)p.A + zb * p.sAb + zh * p.sAh;
  const T* B = (const T*)p.B + zb * p.sBb + zh * p.sBh;
  const int kbeg = s * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nkt = (kend - kbeg + KT - 1) / KT;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  if (nkt > 0) {
    load_tile<T, AK>(A, p.lda, m0, p.M, kbeg, kend, p.vec_a, ra);
    load_tile<T, BKM>(B, p.ldb, n0, p.N, kbeg, kend, p.vec_b, rb);
    store_tile<T, AK>(smem[0][0], ra);
    store_tile<T, BKM>(smem[0][1], rb);
  }
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      load_tile<T, AK>(A, p.lda, m0, p.M, kbeg + (kt + 1) * KT, kend, p.vec_a, ra);
      load_tile<T, BKM>(B, p.ldb, n0, p.N, kbeg + (kt + 1) * KT, kend, p.vec_b, rb);
    }
    const char* la = smem[cur][0];
    const char* lb = smem[cur][1];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if constexpr (sizeof(T) == 2) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_bf16<AK>(la, wm + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag_bf16<BKM>(lb, wn + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      } else {
        float fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag_f32<AK>(la, wm + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = frag_f32<BKM>(lb, wn + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      store_tile<T, AK>(smem[cur ^ 1][0], ra);
      store_tile<T, BKM>(smem[cur ^ 1][1], rb);
    }
    __syncthreads();
  }

  // epilogue: C/D map of 16x16 MFMA: col = lane&15, row = 4*(lane>>4) + reg
  const int rq = (lane >> 4) * 4, cc = lane & 15;
  if (p.splitk > 1) {
    float* slab = p.ws + ((long)z * p.splitk + s) * (long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int row = m0 + wm + i * 16 + rq + rr, col = n0 + wn + j * 16 + cc;
          if (row < p.M && col < p.N) slab[(long)row * p.N + col] = acc[i][j][rr];
        }
    return;
  }
  switch (p.epi.kind) {
    case EA_EPI_STORE: epi_tile<EA_EPI_STORE>(p, z, zb, zh, m0 + wm, n0 + wn, lane, acc); break;
    case EA_EPI_ACT: epi_tile<EA_EPI_ACT>(p, z, zb, zh, m0 + wm, n0 + wn, lane, acc); break;
    case EA_EPI_RESID: epi_tile<EA_EPI_RESID>(p, z, zb, zh, m0 + wm, n0 + wn, lane, acc); break;
    default: epi_tile<EA_EPI_DACT>(p, z, zb, zh, m0 + wm, n0 + wn, lane, acc); break;
  }
}


// ---------------------------------------------------------------- bf16 LDS-DMA kernel
// Same tile/fragment/epilogue scheme as gemm_kernel, but operands move HBM -> LDS with
// global_load_lds_dwordx4 (no staging registers) into a STAGES-deep ring: the tile kt+S-1
// is in flight while tile kt is multiplied; one raw s_barrier per K-tile, counted
// vmcnt waits (never a vmcnt(0) inside the loop).  The LDS image is the same swizzled
// image as gemm_kernel: the swizzle is applied to each lane's SOURCE address since an
// LDS-DMA writes lane-linearly.  M/N edges clamp the source row (results discarded);
// a K remainder (< 64) is loaded once through registers with zero fill.
template <int N>
EA_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most `newer` groups of G DMA instructions (the ones issued last) are still
// in flight; newer in [0, MAXN] (runtime value, compile-time counts)
template <int G, int MAXN>
EA_DEV void wait_newer(int newer) {
  if (MAXN >= 6 && newer >= 6) wait_vmcnt<(MAXN >= 6 ? 6 : 0) * G>();
  else if (MAXN >= 5 && newer == 5) wait_vmcnt<(MAXN >= 5 ? 5 : 0) * G>();
  else if (MAXN >= 4 && newer == 4) wait_vmcnt<(MAXN >= 4 ? 4 : 0) * G>();
  else if (MAXN >= 3 && newer == 3) wait_vmcnt<(MAXN >= 3 ? 3 : 0) * G>();
  else if (MAXN >= 2 && newer == 2) wait_vmcnt<(MAXN >= 2 ? 2 : 0) * G>();
  else if (newer == 1) wait_vmcnt<G>();
  else wait_vmcnt<0>();
}
EA_DEV void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Operand images are built from 128-wide panels of one 64-deep K-tile (16 KB bf16):
//  * K-major operand, R rows: [R][64] (128-B rows, chunk swizzle swz_k)  = R*128 bytes
//  * MN-major operand, R = 128*P cols: [P][64 k][128] panels (swz_mn_bf16)
// A 16-B chunk index c (0 .. R*8-1) maps to (row, chunk) / (panel, k, chunk) the same way
// for the LDS-DMA sources and for the register tail path.
template <bool KMAJ>
EA_DEV int img_off(int c) {  // byte offset of chunk c's LDS slot (the swizzled position)
  if (KMAJ) {
    const int row = c >> 3, ch = c & 7;
    return row * 128 + ((ch ^ swz_k(row)) << 4);
  } else {
    const int pnl = c >> 10, cj = c & 1023, k = cj >> 4, ch = cj & 15;
    return pnl * 16384 + k * 256 + ((ch ^ swz_mn_bf16(k)) << 4);
  }
}

// register tail loader/storer for a K remainder (< 64), zero-filled
template <bool KMAJ, int ROWS, int NTT>
EA_DEV void load_tile_r(const bf16* __restrict__ base, long ld, int mn0, int MN, int k0, int K,
                        uint4 (&v)[ROWS * 8 / NTT]) {
  constexpr int NCH = ROWS * 8 / NTT;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = threadIdx.x + NTT * i;
    int mn, k;
    if (KMAJ) { mn = mn0 + (c >> 3); k = k0 + (c & 7) * 8; }
    else      { const int cj = c & 1023; k = k0 + (cj >> 4); mn = mn0 + (c >> 10) * 128 + (cj & 15) * 8; }
    const bf16* pp = KMAJ ? base + (long)mn * ld + k : base + (long)k * ld + mn;
    union { uint4 u; bf16 e[8]; } t;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = KMAJ ? (mn < MN && k + e < K) : (k < K && mn + e < MN);
      t.e[e] = ok ? pp[e] : (bf16)0.f;
    }
    v[i] = t.u;
  }
}
template <bool KMAJ, int ROWS, int NTT>
EA_DEV void store_tile_r(char* lds, const uint4 (&v)[ROWS * 8 / NTT]) {
#pragma unroll
  for (int i = 0; i < ROWS * 8 / NTT; ++i) {
    const int c = threadIdx.x + NTT * i;
    *(uint4*)(lds + img_off<KMAJ>(c)) = v[i];
  }
}

// fragment of 16 rows/cols starting at r (multiple of 16) from an operand image
template <bool KMAJ>
EA_DEV bf16x8 frag_img(const char* img, int r, int ks, int lane) {
  if (KMAJ) return frag_bf16<true>(img, r, ks, lane);
  return frag_bf16<false>(img + (r >> 7) * 16384, r & 127, ks, lane);
}

// Block -> (output tile, batch slice z, K split sk).  Work items w = (z, sk)-major over the
// grid's nt tiles; each XCD (blocks dispatched round-robin over the linear block id, so XCD =
// id % 8 — a speed assumption only) takes a contiguous range of w, so the blocks sharing a
// slice's A / B panels (every tile of one split, or of one batch slice) share one L2; inside a
// slice, GM-row groups keep the N-tiles of one M panel together.
struct TileIdx { int tm, tn, z, sk; };
EA_DEV TileIdx tile_index(const GemmP& p) {
  const int nt = p.tiles_m * p.tiles_n;
  const int total = gridDim.x * gridDim.z;
  const int bid = blockIdx.x + gridDim.x * blockIdx.z;
  const int q = total / 8, r = total % 8, xcd = bid % 8;
  const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  const int zz = w / nt, t = w - zz * nt;
  const int GM = 8;
  const int grp = t / (GM * p.tiles_n);
  const int gm0 = grp * GM;
  const int gsz = min(GM, p.tiles_m - gm0);
  TileIdx ti;
  ti.tm = gm0 + (t % (GM * p.tiles_n)) % gsz;
  ti.tn = (t % (GM * p.tiles_n)) / gsz;
  ti.z = zz / p.splitk;
  ti.sk = zz % p.splitk;
  return ti;
}

// Epilogue of one wave's (MI*16) x (NJ*16) accumulator tile, in 64 x 64 chunks transposed
// through the wave's private LDS region (64 x EPI_LDT floats); each lane then owns 4
// consecutive columns of 16 rows per chunk.  The operand the epilogue kind reads (aux /
// resid / C for beta != 0) is loaded in batches of 8 row groups, all of a batch's loads in
// flight together (one round trip per batch); bias is read once per batch.  With split-K (p.splitk > 1) the chunk goes to this slice's f32 slab.
template <int KIND, int MI, int NJ>
EA_DEV void epi_wave(const GemmP& p, const EpiK& k, char* smem, int z, int zb, int zh, int r0, int c0, int lane,
                     int w, const f32x4 (&acc)[MI][NJ], int sk = 0) {
  constexpr int RC = MI < 4 ? MI : 4;  // row blocks per chunk
  constexpr int NG = RC * 4;           // row groups (of 4 lanes' rows) per lane per chunk
  constexpr int HB = NG < 8 ? NG : 8;  // row groups per operand-load batch
  constexpr int NCH = (MI / RC) * (NJ / 4), NBC = NG / HB, NU = NCH * NBC;  // chunks, batches, units
  float* t = (float*)smem + w * (RC * 16) * EPI_LDT;
  const int rq = (lane >> 4) * 4, cc = lane & 15, lc = (lane & 15) * 4;
  float* slab = p.splitk > 1 ? p.ws + ((long)z * p.splitk + sk) * (long)p.M * p.N : nullptr;
  const bool reads = p.vec_c && !slab &&
                     (KIND == EA_EPI_DACT || (KIND == EA_EPI_RESID && p.epi.resid) ||
                      (KIND == EA_EPI_STORE && p.epi.beta != 0.f));
  // the operand the kind reads (aux / resid / C for beta != 0), dtype dispatched once
  const void* src = nullptr;
  long sld = 0, sbase = 0;
  int sdt = EA_F32;
  if constexpr (KIND == EA_EPI_STORE) {
    src = p.C; sld = p.ldc; sbase = zb * p.sCb + zh * p.sCh; sdt = p.c_dtype;
  } else if constexpr (KIND == EA_EPI_RESID) {
    src = p.epi.resid; sld = p.epi.ldr;
  } else if constexpr (KIND == EA_EPI_DACT) {
    src = p.epi.aux; sld = p.epi.ldaux; sdt = p.epi.aux_dtype;
  }
  auto ch_rb = [&](int ch) { return r0 + (ch / (NJ / 4)) * RC * 16; };
  auto ch_col = [&](int ch) { return c0 + (ch % (NJ / 4)) * 64 + lc; };
  // one batch of operand loads: unconditional, at clamped (in-range) indices, with the dtype
  // branch outside the batch — a branch around each load makes hipcc drain vmcnt(0) after
  // every one of them (out-of-range groups are never stored)
  auto load_unit = [&](int u, float (&o)[HB][4]) {
    if (!reads) return;
    const int ch = u / NBC, h0 = (u % NBC) * HB;
    const int rb = ch_rb(ch), cl = min(ch_col(ch), p.N - 4);
    if (sdt == EA_BF16) {
#pragma unroll
      for (int it = 0; it < HB; ++it)
        vld4((const bf16*)src + sbase + (long)min(rb + (h0 + it) * 4 + (lane >> 4), p.M - 1) * sld + cl, o[it]);
    } else {
#pragma unroll
      for (int it = 0; it < HB; ++it)
        vld4((const float*)src + sbase + (long)min(rb + (h0 + it) * 4 + (lane >> 4), p.M - 1) * sld + cl, o[it]);
    }
  };
  auto transpose = [&](int ch) {  // a chunk's accumulators -> the wave's LDS image
    const int ri = ch / (NJ / 4), cj = ch % (NJ / 4);
    if (ch > 0) {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < RC; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          t[(i * 16 + rq + rr) * EPI_LDT + j * 16 + cc] = acc[ri * RC + i][cj * 4 + j][rr];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  };
  if (!p.vec_c) {  // cold path (unaligned C / N % 4): element-wise straight from the LDS image
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      transpose(ch);
      const int rb = ch_rb(ch), col = ch_col(ch);
#pragma unroll 1
      for (int it = 0; it < NG; ++it) {
        const int lr = it * 4 + (lane >> 4), row = rb + lr;
        if (row >= p.M) continue;
#pragma unroll 1
        for (int c = 0; c < 4; ++c) {
          if (col + c >= p.N) break;
          const float x = t[lr * EPI_LDT + lc + c];
          if (slab) slab[(long)row * p.N + col + c] = x;
          else epi_one<KIND>(p, z, zb, zh, row, col + c, x);
        }
      }
    }
    return;
  }
  if (p.vec8) {  // 8 consecutive columns per lane: 16-B bf16 stores / operand loads
    constexpr int NG8 = RC * 2;  // row groups of 8 rows per chunk
    constexpr int HB8 = NG8 < 4 ? NG8 : 4;
    const int lc8 = (lane & 7) * 8, rl = lane >> 3;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      transpose(ch);
      const int rb = ch_rb(ch), col = c0 + (ch % (NJ / 4)) * 64 + lc8;
      float bias[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (!slab && KIND != EA_EPI_DACT && p.epi.bias && col < p.N) {
        const float4 b0 = *(const float4*)(p.epi.bias + col), b1 = *(const float4*)(p.epi.bias + col + 4);
        bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
        bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
      }
#pragma unroll
      for (int h0 = 0; h0 < NG8; h0 += HB8) {
        float o[HB8][8];
        if (reads) {  // unconditional, clamped, dtype branch outside the batch (see load_unit)
          const int cl = min(col, p.N - 8);
          if (sdt == EA_BF16) {
#pragma unroll
            for (int it = 0; it < HB8; ++it)
              ld8(src, sbase + (long)min(rb + (h0 + it) * 8 + rl, p.M - 1) * sld + cl, EA_BF16, o[it]);
          } else {
#pragma unroll
            for (int it = 0; it < HB8; ++it)
              ld8(src, sbase + (long)min(rb + (h0 + it) * 8 + rl, p.M - 1) * sld + cl, EA_F32, o[it]);
          }
        }
#pragma unroll
        for (int it = 0; it < HB8; ++it) {
          const int lr = (h0 + it) * 8 + rl, row = rb + lr;
          const float4 f0 = *(const float4*)(t + lr * EPI_LDT + lc8), f1 = *(const float4*)(t + lr * EPI_LDT + lc8 + 4);
          if (row >= p.M || col >= p.N) continue;
          if (slab) {
            *(float4*)(slab + (long)row * p.N + col) = f0;
            *(float4*)(slab + (long)row * p.N + col + 4) = f1;
            continue;
          }
          const float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
          epi_eight_pre<KIND>(p, k, z, zb, zh, row, col, v, bias, reads, o[it]);
        }
      }
    }
    return;
  }
  // per chunk: transpose, then batches of HB row groups whose operand loads are all issued
  // before any of them is used (software pipelining across batches measured slower: the
  // second buffer of live operands costs more registers than the latency it hides)
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int ch = u / NBC, h0 = (u % NBC) * HB;
    const int rb = ch_rb(ch), col = ch_col(ch);
    if (u % NBC == 0) transpose(ch);
    float ob[HB][4];
    load_unit(u, ob);
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (!slab && KIND != EA_EPI_DACT && p.epi.bias && col < p.N) {
      const float4 bb = *(const float4*)(p.epi.bias + col);
      bias[0] = bb.x; bias[1] = bb.y; bias[2] = bb.z; bias[3] = bb.w;
    }
#pragma unroll
    for (int it = 0; it < HB; ++it) {
      const int lr = (h0 + it) * 4 + (lane >> 4), row = rb + lr;
      const float4 f = *(const float4*)(t + lr * EPI_LDT + lc);
      if (row >= p.M || col >= p.N) continue;
      const float v[4] = {f.x, f.y, f.z, f.w};
      if (slab) *(float4*)(slab + (long)row * p.N + col) = f;
      else epi_four_pre<KIND>(p, k, z, zb, zh, row, col, v, bias, reads, ob[it]);
    }
  }
}

// ---------------------------------------------------------------- implicit-GEMM gathers
// Conv2dSubsampling's conv2 (3x3, stride 2) over the phase-split conv1 output x1p: class
// plane (a, e) holds pixels t1 = 2i + a, f1 = 2j + e as a dense [b][i][j][C] block, so
// every tap of every output pixel is one contiguous C-row of one plane (see ea_conv_geo).
EA_DEV int fdiv(int n, int d) {  // exact n / d for 0 <= n < 2^24 (float estimate + fix-up)
  int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
  if (q * d > n) --q;
  if ((q + 1) * d <= n) ++q;
  return q;
}
// element offset of x1p[pixel (b, t2, f2) shifted by tap (kh, kw)] (conv2 input row)
EA_DEV long x1p_row(const ea_conv_geo& g, int b, int t2, int f2, int kh, int kw) {
  const int a = kh & 1, e = kw & 1;
  return g.plane[a * 2 + e] + (((long)b * g.nI[a] + t2 + (kh >> 1)) * g.nJ[e] + f2 + (kw >> 1)) * g.C;
}
// DGRAD tap q of class (a, e): kh in {0,2} (a = 0) or {1}; kw likewise
EA_DEV void dgrad_tap2(int a, int e, int q, int& kh, int& kw) {
  const int nkw = e ? 1 : 2;
  const int qh = q / nkw, qw = q - qh * nkw;
  kh = a ? 1 : 2 * qh;
  kw = e ? 1 : 2 * qw;
}
EA_DEV void dgrad_tap(const ea_conv_geo& g, int q, int& kh, int& kw) {
  const int nkw = g.e ? 1 : 2;
  const int qh = q / nkw, qw = q - qh * nkw;
  kh = g.a ? 1 : 2 * qh;
  kw = g.e ? 1 : 2 * qw;
}

// BM x BN output tile, 2 x WN wave64s, each (BM/2) x (BN/WN) = MI x NJ MFMA 16x16 blocks.
// (BM, BN, WN) in {(64,128,2) K-major A only, (128,128,2), (256,256,4)}.
// Small wave tiles read the fragments of both k-steps up front (register double buffer);
// 128-row wave tiles read one k-step at a time.
template <int BM_, int BN_, int WN, bool AK, bool BKM, int STAGES, int MODE = 0>
__global__ __launch_bounds__(128 * WN, 1) void gemm_bf16_lds(GemmP p) {
  static_assert(MODE == 0 || (MODE == EA_CONV_FWD && AK && BKM) || (MODE == EA_CONV_DGRAD && AK && !BKM) ||
                (MODE == EA_CONV_WGRAD && !AK && !BKM), "conv gather layouts");
  constexpr int NW = 2 * WN, NTT = 64 * NW;
  static_assert(AK || BM_ >= 128, "MN-major A needs 128-wide panels");
  static_assert(BKM || BN_ >= 128, "MN-major B needs 128-wide panels");
  constexpr int BK = 64;
  constexpr int A_BYTES = BM_ * BK * 2, B_BYTES = BN_ * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int MI = BM_ / 32, NJ = BN_ / (16 * WN);
  constexpr int ACH = A_BYTES / (NTT * 16), BCH = B_BYTES / (NTT * 16);  // DMA chunks/thread/K-tile
  constexpr int EPI_BYTES = NW * (MI < 4 ? MI : 4) * 16 * EPI_LDT * 4;
  constexpr int SMEM = STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES;
  constexpr bool DB = MI * NJ <= 16;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  probe_start(p);

  const TileIdx ti = tile_index(p);
  const int tm = ti.tm, m0 = ti.tm * BM_, n0 = ti.tn * BN_;
  const int z = ti.z, sk = ti.sk;
  const int zb = z / p.nh, zh = z % p.nh;
  const bf16* A = (const bf16*)p.A + zb * p.sAb + zh * p.sAh;
  const bf16* B = (const bf16*)p.B + zb * p.sBb + zh * p.sBh;
  const int kbeg = sk * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nfull = max(0, (kend - kbeg) / BK);
  const bool tail = kbeg + nfull * BK < kend;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = (w / WN) * (BM_ / 2), wn = (w % WN) * (BN_ / WN);

  // per-lane DMA sources: chunk ci = (i*NW + w)*64 + lane lands lane-linearly at ci*16;
  // the source is the global chunk whose swizzled slot that is.  Sources are 32-bit byte
  // offsets from a wave-uniform base (scalar base + vector offset addressing; the host
  // keeps operands < 4 GB on this path).
  auto src = [&](long ld, int mn0, int MN, bool kmaj, int ci) -> uint32_t {
    if (kmaj) {
      const int row = ci >> 3, c = (ci & 7) ^ swz_k(ci >> 3);
      return (uint32_t)(((long)min(mn0 + row, MN - 1) * ld + c * 8) * 2);
    }
    const int pnl = ci >> 10, cj = ci & 1023, k = cj >> 4, c = (cj & 15) ^ swz_mn_bf16(k);
    return (uint32_t)(((long)k * ld + min((long)(mn0 + pnl * 128 + c * 8), (long)((MN - 1) & ~7))) * 2);
  };
  const char* abase = (const char*)(A + (AK ? (long)kbeg : (long)kbeg * p.lda));
  const char* bbase = (const char*)(B + (BKM ? (long)kbeg : (long)kbeg * p.ldb));
  uint32_t aoff[ACH], boff[BCH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) aoff[i] = src(p.lda, m0, p.M, AK, (i * NW + w) * 64 + lane);
#pragma unroll
  for (int i = 0; i < BCH; ++i) boff[i] = src(p.ldb, n0, p.N, BKM, (i * NW + w) * 64 + lane);
  const long astep = (AK ? BK : (long)BK * p.lda) * 2;  // bytes per K-tile
  const long bstep = (BKM ? BK : (long)BK * p.ldb) * 2;
  constexpr int GPT = ACH + BCH;  // DMA instructions per thread per K-tile (vmcnt unit)

  // gather modes.  A rows (FWD / DGRAD): each chunk's row decoded once; its source offset
  // (elements, < 2^31) is rebuilt only when the K-tile enters a new tap, so a K-tile costs
  // one add per chunk.  B rows (WGRAD, k = pixel): each chunk's pixel advances by 64 per
  // K-tile with an incremental (b, t2, f2) carry instead of divisions.
  int gb[ACH], gt[ACH], gf[ACH], cur[ACH];
  const int ktg0 = kbeg / BK;  // global K-tile index of this split's first tile
  const int CT = p.g.C / BK;   // K-tiles per tap (gather modes)
  if constexpr (MODE == EA_CONV_FWD || MODE == EA_CONV_DGRAD) {
    const int n2 = MODE == EA_CONV_FWD ? p.g.T2 : p.g.nI[p.g.a];
    const int n3 = MODE == EA_CONV_FWD ? p.g.F2 : p.g.nJ[p.g.e];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int m = min(m0 + (((i * NW + w) * 64 + lane) >> 3), p.M - 1);
      const int bt = fdiv(m, n3);
      gf[i] = m - bt * n3;
      gb[i] = fdiv(bt, n2);
      gt[i] = bt - gb[i] * n2;
      cur[i] = 0;
    }
  }
  auto a_tap = [&](int q) {  // rebuild the A chunk offsets for tap q (FWD / DGRAD)
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int ci = (i * NW + w) * 64 + lane;
      const int cc = ((ci & 7) ^ swz_k(ci >> 3)) * 8;
      if constexpr (MODE == EA_CONV_FWD) {
        const int kh = q / 3, kw = q - 3 * (q / 3);
        cur[i] = (int)x1p_row(p.g, gb[i], gt[i], gf[i], kh, kw) + cc;
      } else {
        int kh, kw;
        dgrad_tap(p.g, q, kh, kw);
        const int t2 = gt[i] - (kh >> 1), f2 = gf[i] - (kw >> 1);  // t1 = 2*t2 + kh
        cur[i] = (t2 >= 0 && t2 < p.g.T2 && f2 >= 0 && f2 < p.g.F2)
                     ? ((gb[i] * p.g.T2 + t2) * p.g.F2 + f2) * p.g.C + cc
                     : (int)p.g.zero + (i * 8 + lane / 8) % 64 * p.g.C + cc;  // spread over 64 zero rows
      }
    }
  };
  // WGRAD B chunks: fixed column (tap, ci) per chunk, pixel state advanced per K-tile
  int wb[BCH], wt[BCH], wf[BCH], wpix[BCH], wbase[BCH], wnI[BCH], wnJ[BCH];
  if constexpr (MODE == EA_CONV_WGRAD) {
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int ci = (i * NW + w) * 64 + lane;
      const int pnl = ci >> 10, cj = ci & 1023, k = cj >> 4, c = (cj & 15) ^ swz_mn_bf16(k);
      const int n = min(n0 + pnl * 128 + c * 8, p.N - 8);
      const int tap = n / p.g.C, cin = n - tap * p.g.C;
      const int kh = tap / 3, kw = tap - 3 * kh, a = kh & 1, e = kw & 1;
      wnI[i] = p.g.nI[a];
      wnJ[i] = p.g.nJ[e];
      // row (b*nI + t2 + kh/2)*nJ + f2 + kw/2 of plane (a, e): fold the tap shift into the base
      wbase[i] = (int)p.g.plane[a * 2 + e] + ((kh >> 1) * wnJ[i] + (kw >> 1)) * p.g.C + cin;
      const int pix = ktg0 * BK + k;
      wpix[i] = pix;
      const int bt = fdiv(pix, p.g.F2);
      wf[i] = pix - bt * p.g.F2;
      wb[i] = fdiv(bt, p.g.T2);
      wt[i] = bt - wb[i] * p.g.T2;
    }
  }
  const int dF = BK % max(p.g.F2, 1), dT = BK / max(p.g.F2, 1);

  auto issue = [&](int kt, int stg) {
    char* base = smem + stg * STAGE_BYTES;
    const char* ak = abase + kt * astep;
    const char* bk = bbase + kt * bstep;
    if constexpr (MODE == EA_CONV_FWD || MODE == EA_CONV_DGRAD) {
      // FWD: k = (64-channel block, tap, channel) — one tap per K-tile, the 9 taps of a block
      // back to back; DGRAD: k = (tap of the class, channel)
      const int ktg = ktg0 + kt;
      const int q = MODE == EA_CONV_FWD ? ktg % 9 : ktg / CT;
      const int c0 = MODE == EA_CONV_FWD ? (ktg / 9) * BK : (ktg - q * CT) * BK;
      if (MODE == EA_CONV_FWD || c0 == 0 || kt == 0) a_tap(q);
#pragma unroll
      for (int i = 0; i < ACH; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)((const char*)A + (long)(cur[i] + c0) * 2),
                                         (__attribute__((address_space(3))) void*)(base + (i * NW + w) * 1024), 16, 0, 0);
      if constexpr (MODE == EA_CONV_DGRAD) {  // W2t [9][co][ci]: k-tile = 64 co of one tap
        int kh, kw;
        dgrad_tap(p.g, q, kh, kw);
        bk = (const char*)(B + ((long)(kh * 3 + kw) * p.g.C + c0) * p.g.C);
      }
    } else {
#pragma unroll
      for (int i = 0; i < ACH; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(ak + aoff[i]),
                                         (__attribute__((address_space(3))) void*)(base + (i * NW + w) * 1024), 16, 0, 0);
    }
    if constexpr (MODE == EA_CONV_WGRAD) {  // B[k = pixel][n = (tap, ci)] gathered from x1p
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int off = wpix[i] < p.g.P ? wbase[i] + ((wb[i] * wnI[i] + wt[i]) * wnJ[i] + wf[i]) * p.g.C
                                        : (int)p.g.zero + (lane & 63) * p.g.C + (wbase[i] % p.g.C);
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)((const char*)B + (long)off * 2),
                                         (__attribute__((address_space(3))) void*)(base + A_BYTES + (i * NW + w) * 1024),
                                         16, 0, 0);
        // advance this chunk's pixel by one K-tile (64 pixels)
        wpix[i] += BK;
        wf[i] += dF;
        wt[i] += dT;
        if (wf[i] >= p.g.F2) { wf[i] -= p.g.F2; ++wt[i]; }
        while (wt[i] >= p.g.T2) { wt[i] -= p.g.T2; ++wb[i]; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(bk + boff[i]),
                                         (__attribute__((address_space(3))) void*)(base + A_BYTES + (i * NW + w) * 1024),
                                         16, 0, 0);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stg) {
    const char* la = smem + stg * STAGE_BYTES;
    const char* lb = la + A_BYTES;
    if constexpr (DB) {
      bf16x8 fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa0[i] = frag_img<AK>(la, wm + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb0[j] = frag_img<BKM>(lb, wn + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) fa1[i] = frag_img<AK>(la, wm + i * 16, 1, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb1[j] = frag_img<BKM>(lb, wn + j * 16, 1, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[i], fb0[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 fb[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[j] = frag_img<BKM>(lb, wn + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const bf16x8 fa = frag_img<AK>(la, wm + i * 16, ks, lane);
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  const int npre = min(STAGES - 1, nfull);
  for (int kt = 0; kt < npre; ++kt) issue(kt, kt);
  for (int kt = 0; kt < nfull; ++kt) {
    const int after = min(STAGES - 2, nfull - 1 - kt);  // newer tiles allowed in flight
    if (after >= 2) wait_vmcnt<2 * GPT>();
    else if (after == 1) wait_vmcnt<GPT>();
    else wait_vmcnt<0>();
    lds_barrier();
    if (kt + STAGES - 1 < nfull) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    compute(kt % STAGES);
  }
  if (tail) {
    uint4 ra[BM_ * 8 / NTT], rb[BN_ * 8 / NTT];
    const int k0 = kbeg + nfull * BK;
    load_tile_r<AK, BM_, NTT>(A, p.lda, m0, p.M, k0, kend, ra);
    load_tile_r<BKM, BN_, NTT>(B, p.ldb, n0, p.N, k0, kend, rb);
    __syncthreads();
    char* base = smem + (nfull % STAGES) * STAGE_BYTES;
    store_tile_r<AK, BM_, NTT>(base, ra);
    store_tile_r<BKM, BN_, NTT>(base + A_BYTES, rb);
    __syncthreads();
    compute(nfull % STAGES);
  }

  __syncthreads();  // every wave is done reading the operand ring: reuse it for the epilogue
  const EpiK ek = make_epik(p);
  switch (p.splitk > 1 ? EA_EPI_STORE : p.epi.kind) {
    case EA_EPI_STORE: epi_wave<EA_EPI_STORE, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    case EA_EPI_ACT: epi_wave<EA_EPI_ACT, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    case EA_EPI_RESID: epi_wave<EA_EPI_RESID, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    default: epi_wave<EA_EPI_DACT, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
  }
  probe_end(p);
}

// ---------------------------------------------------------------- 128x128, K-major, K-split wave groups
// gemm_k128: the narrow-N GEMMs of the step (M = 7,968 tokens, N = 512: the Linear input
// gradients over the transposed weight shadow and the forward projections — both operands
// K-major) as ONE 128 x 128 tile per CU (252 blocks: the fewest operand bytes per CU for this
// output size, 1 MiB at K = 2,048 against 1.5 MiB for two 64 x 128 tiles).  Eight waves in two
// K groups: every wave owns a 64 x 64 quarter of the tile, and group g = w / 4 multiplies only
// the g-th 32-deep half of each 64-deep K-tile, so every SIMD holds one wave of each group and
// one wave's LDS reads and waits overlap the other's MFMAs (the one-wave-per-SIMD form of this
// tile left every barrier and read latency exposed).  The two groups' partial sums are added
// through LDS before the epilogue.  K-tiles stream through an S-slot LDS ring filled S-1 tiles
// ahead by buffer_load ... lds (per-lane 32-bit source offsets fixed for the whole loop, the
// K-tile advance in the scalar offset: no address arithmetic per load); one barrier per
// K-tile, counted vmcnt, fragment reads as inline asm with immediate offsets (hipcc would put
// a vmcnt(0) in front of an LDS read it can see while an LDS-DMA is in flight).  Image format,
// tile mapping and epilogue as gemm_bf16_lds<128, 128>; the host guarantees K % 64 == 0 per
// split and operands < 4 GB.
template <int OFF>
EA_DEV bf16x8 ds_read_b128_at(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}

template <int S>
__global__ __launch_bounds__(512, 1) void gemm_k128(GemmP p) {
  constexpr int BK = 64, NTT = 512, NW = 8, MI = 4, NJ = 4;
  constexpr int A_BYTES = 128 * BK * 2, B_BYTES = 128 * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int ACH = A_BYTES / (NTT * 16), BCH = B_BYTES / (NTT * 16), G = ACH + BCH;  // 2 + 2
  constexpr int EPI_BYTES = 4 * 4 * 16 * EPI_LDT * 4;  // group 0's four transposition images
  constexpr int HAND = EPI_BYTES;                      // group 1's partial sums: 4 x 16 KiB
  constexpr int SMEM = S * STAGE > HAND + 65536 ? S * STAGE : HAND + 65536;
  static_assert(S >= 3 && S <= 4, "ring depth");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  probe_start(p);

  const TileIdx ti = tile_index(p);
  const int m0 = ti.tm * 128, n0 = ti.tn * 128;
  const int z = ti.z, sk = ti.sk;
  const int zb = z / p.nh, zh = z % p.nh;
  const bf16* A = (const bf16*)p.A + zb * p.sAb + zh * p.sAh;
  const bf16* B = (const bf16*)p.B + zb * p.sBb + zh * p.sBh;
  const int kbeg = sk * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nt = max(0, (kend - kbeg) / BK);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, q = w & 3;                    // K group, quarter of the tile
  const int wm = (q >> 1) * 64, wn = (q & 1) * 64;

  // buffer descriptors over this split's operand rows; per-lane source offsets (bytes) of the
  // lane-linear DMA chunks: chunk ci = (i*NW + w)*64 + lane lands at ci*16 and reads the
  // global chunk whose swizzled slot that is
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + kbeg), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B + kbeg), (short)0, 0x7fffffff, 0x00020000);
  auto src = [&](long ld, int mn0, int MN, int ci) -> uint32_t {
    const int row = ci >> 3, c = (ci & 7) ^ swz_k(ci >> 3);
    return (uint32_t)(((long)min(mn0 + row, MN - 1) * ld + c * 8) * 2);
  };
  uint32_t aoff[ACH], boff[BCH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) aoff[i] = src(p.lda, m0, p.M, (i * NW + w) * 64 + lane);
#pragma unroll
  for (int i = 0; i < BCH; ++i) boff[i] = src(p.ldb, n0, p.N, (i * NW + w) * 64 + lane);

  auto issue = [&](int t) {
    char* base = smem + (t % S) * STAGE;
    const int so = t * BK * 2;  // K-tile advance (bytes), scalar
#pragma unroll
    for (int i = 0; i < ACH; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(base + (i * NW + w) * 1024),
                                               16, aoff[i], so, 0, 0);
#pragma unroll
    for (int i = 0; i < BCH; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(base + A_BYTES + (i * NW + w) * 1024), 16, boff[i], so, 0, 0);
  };

  // fragment addresses: row r0 + (lane & 15) of a 16-row block starting at a multiple of 16
  // swizzles by (lane & 15) only, so the blocks of a wave are immediate offsets of one base
  const int ch = g * 4 + (lane >> 4);
  const uint32_t lane_off = (uint32_t)((lane & 15) * 128 + ((ch ^ (((lane & 15) >> 1) & 7)) << 4));
  const uint32_t smem0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  const uint32_t a_off = smem0 + lane_off + wm * 128, b_off = smem0 + A_BYTES + lane_off + wn * 128;
  bf16x8 fa[MI], fb[NJ];
  auto rd = [&](int t) {
    const uint32_t sb = (uint32_t)((t % S) * STAGE);
    const uint32_t pa = a_off + sb, pb = b_off + sb;
    fa[0] = ds_read_b128_at<0>(pa);
    fa[1] = ds_read_b128_at<2048>(pa);
    fa[2] = ds_read_b128_at<4096>(pa);
    fa[3] = ds_read_b128_at<6144>(pa);
    fb[0] = ds_read_b128_at<0>(pb);
    fb[1] = ds_read_b128_at<2048>(pb);
    fb[2] = ds_read_b128_at<4096>(pb);
    fb[3] = ds_read_b128_at<6144>(pb);
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
    const int npre = min(S - 1, nt);
    for (int t = 0; t < npre; ++t) issue(t);
    for (int t = 0; t < nt; ++t) {
      // own share of tile t landed (tiles issued after it may stay in flight), then everyone's;
      // every wave is past its reads of tile t-1, whose slot the refill below reuses
      wait_newer<G, S - 2>(min(S - 2, nt - 1 - t));
      lds_barrier();
      if (t + S - 1 < nt) issue(t + S - 1);
      rd(t);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();  // every wave is done reading the ring: the epilogue reuses it
  // group 1 hands its partial sums to group 0 (same quarter, same lane: conflict-free b128)
  f32x4* hand = (f32x4*)(smem + HAND) + q * (MI * NJ * 64);
  if (g == 1) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) hand[(i * NJ + j) * 64 + lane] = acc[i][j];
  }
  __syncthreads();
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] += hand[(i * NJ + j) * 64 + lane];
    const EpiK ek = make_epik(p);
    switch (p.splitk > 1 ? EA_EPI_STORE : p.epi.kind) {
      case EA_EPI_STORE: epi_wave<EA_EPI_STORE, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, q, acc, sk); break;
      case EA_EPI_ACT: epi_wave<EA_EPI_ACT, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, q, acc, sk); break;
      case EA_EPI_RESID: epi_wave<EA_EPI_RESID, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, q, acc, sk); break;
      default: epi_wave<EA_EPI_DACT, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, q, acc, sk); break;
    }
  }
  probe_end(p);
}

// ---------------------------------------------------------------- ping-pong 256x256 kernel
// gemm_pipe: the 256x256 tile of gemm_bf16_lds with a ping-pong schedule.  K moves in 32-deep
// slices through a 4-slot LDS ring (32 KiB per slot: A 256x32 + B 256x32 bf16), DMA issued
// three slices ahead.  The eight wave64s form two groups, G0 = waves 0-3 (tile rows 0-127)
// and G1 = waves 4-7 (rows 128-255); every SIMD holds one wave of each.  Each wave alternates
// a LOAD segment (read its slice fragments LDS -> registers, issue its share of the DMA three
// slices ahead, counted vmcnt for the next slice, lgkmcnt(0)) and a COMPUTE segment (32 MFMAs
// over its 128 x 64 sub-tile), one s_barrier after each.  G1 runs one barrier behind G0, so
// on every SIMD one wave's MFMAs overlap the other wave's loads:
//
//   segment:   2s          2s+1          2s+2
//   G0:        LOAD(s)     COMPUTE(s)    LOAD(s+1)
//   G1:        COMPUTE(s-1) LOAD(s)      COMPUTE(s)
//
// Slice s is readable once every wave has waited for its own DMA share of s (at the end of
// its LOAD(s-1)) and a barrier has passed; the DMA of slice s+3 goes to the slot of slice s-1,
// whose last reads (G1's LOAD(s-1)) retired before the barrier that opens G0's LOAD(s).
//
// LDS images of a 32-deep slice (16-B chunks, lane-linear DMA: the swizzle is applied to the
// per-lane SOURCE address):
//  * K-major operand: [256 rows][4 chunks] (64-B rows); logical chunk c of row r is stored at
//    c ^ (((r >> 3) & 1) << 1), which makes every ds_read_b128 lane group of a 16-row
//    fragment read 16 distinct 16-B bank slots (conflict-free).
//  * MN-major operand: two [32 k][128] panels of 8 KiB with gemm_bf16_lds's swz_mn_bf16
//    chunk swizzle, read with ds_read_b64_tr_b16.
EA_DEV int swz32(int r) { return ((r >> 3) & 1) << 1; }

template <bool KMAJ>
EA_DEV int img32_off(int c) {  // byte offset of (logical) chunk c's LDS slot
  if (KMAJ) {
    const int row = c >> 2, ch = c & 3;
    return row * 64 + ((ch ^ swz32(row)) << 4);
  } else {
    const int pnl = c >> 9, cj = c & 511, k = cj >> 4, ch = cj & 15;
    return pnl * 8192 + k * 256 + ((ch ^ swz_mn_bf16(k)) << 4);
  }
}

// ds_read_b64_tr_b16 as inline asm: hipcc's waitcnt pass puts a vmcnt(0) in front of every
// tr-read builtin while an LDS-DMA is in flight (it cannot tell the two apart), which would
// drain the DMA pipeline every slice.  The caller waits lgkmcnt(0) itself (then a
// sched_barrier) before any use of the result.
EA_DEV s16x4 tr_read_asm(const char* p) {
  s16x4 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

template <bool KMAJ>
EA_DEV bf16x8 frag32(const char* img, int r, int lane) {  // 16 rows/cols from r (mult. of 16)
  if (KMAJ) {
    const int row = r + (lane & 15), ch = lane >> 4;
    return *(const bf16x8*)(img + row * 64 + ((ch ^ swz32(row)) << 4));
  }
  // as frag_bf16<false> (8 consecutive k of column (lane&15) via two transposed 4 x 4 reads)
  const char* pnl = img + (r >> 7) * 8192;
  const int i = lane & 15, q = i >> 2, pp = i & 3;
  const int col = (r & 127) + 4 * pp;
  const int ch = col >> 3, within = (col & 7) * 2;
  union { bf16x8 v; s16x4 h[2]; } out;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int row = 8 * (lane >> 4) + 4 * half + q;
    out.h[half] = tr_read_asm(pnl + row * 256 + ((ch ^ swz_mn_bf16(row)) << 4) + within);
  }
  return out.v;
}

// Tile geometry of gemm_pipe: BT x BT output tiles, 8 waves in two ping-pong groups of 4.
//  * BT = 256: each wave owns a 128 x 64 sub-tile (G0 rows 0-127, G1 rows 128-255), one
//    block per CU (128 KiB ring).
//  * BT = 128: each wave owns a 32 x 64 sub-tile (G0 rows 0-63 as 2 x 2 waves, G1 rows
//    64-127), 64 KiB ring + 70 KiB epilogue staging -> two blocks per CU, so one block's
//    epilogue overlaps the other's main loop (the N = 512 / short-K GEMMs of the step).
template <int BT, int NS = 4>
struct PipeT {
  static constexpr int BK = 32, NSLOT = NS, NW = 8, NTT = 512;
  static constexpr int A_BYTES = BT * BK * 2, B_BYTES = BT * BK * 2, SLOT = A_BYTES + B_BYTES;
  static constexpr int RING = NSLOT * SLOT;
  static constexpr int MI = BT == 256 ? 8 : 2;  // 16-row fragments per wave
  static constexpr int EPI_BYTES = NW * (MI < 4 ? MI : 4) * 16 * EPI_LDT * 4;
  static constexpr int SMEM = RING > EPI_BYTES ? RING : EPI_BYTES;
  static constexpr int ACH = A_BYTES / (NTT * 16), BCH = B_BYTES / (NTT * 16);  // DMA per thread
  static constexpr int G = ACH + BCH;
  static constexpr int OCC = BT == 256 ? 1 : 2;
  static_assert(BT == 256 || BT == 128, "pipe tiles");
  static_assert(NS == 4, "ring depth: 4 slots (5- and 6/8-slot rings measured slower, round 3/4)");
  EA_DEV static int wm(int w) { return BT == 256 ? (w >> 2) * 128 : (w >> 2) * 64 + ((w >> 1) & 1) * 32; }
  EA_DEV static int wn(int w) { return BT == 256 ? (w & 3) * 64 : (w & 1) * 64; }
};

// The per-tile values the merged conv2 input-gradient launch (GemmP.ncls) varies by parity
// class: rows, the class (a, e), and the class's partial-tile / mask-bit bases.  Kept apart
// from GemmP so that the kernel argument is never copied (its conv geometry is indexed at run
// time, which would put a copy in scratch memory).
struct TileOv {
  int M, a, e;
  float* w1part;
  const uint8_t* w1pos;
};
EA_DEV TileOv tile_ov(const GemmP& p) { return TileOv{p.M, p.g.a, p.g.e, p.w1part, p.w1pos}; }

// One BT x BT output tile over K range [kbeg, kend) into acc (the wave's sub-tile, PipeT);
// A / B point at this tile's batch slice.  Returns with every wave done reading smem.
template <bool AK, bool BKM, int MODE = 0, int BT = 256, int NS = 4>
EA_DEV void pipe_tile(const GemmP& p, const TileOv& ov, char* smem, const bf16* A, const bf16* B, int m0, int n0, int kbeg,
                      int kend, f32x4 (&acc)[PipeT<BT, NS>::MI][4]) {
  static_assert(MODE == 0 || (MODE == EA_CONV_FWD && AK && BKM) || (MODE == EA_CONV_DGRAD && AK) ||
                (MODE == EA_CONV_WGRAD && !AK && !BKM), "conv gather layouts");
  static_assert(MODE == 0 || BT == 256, "conv gathers run on 256-wide tiles");
  using PC = PipeT<BT, NS>;
  constexpr int BK = PC::BK, NSLOT = PC::NSLOT, NW = PC::NW, NTT = PC::NTT, MI = PC::MI;
  constexpr int A_BYTES = PC::A_BYTES, B_BYTES = PC::B_BYTES, SLOT = PC::SLOT;
  constexpr int ACH = PC::ACH, BCH = PC::BCH, G = PC::G;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = PC::wm(w), wn = PC::wn(w);
  const int nsl = max(0, (kend - kbeg) / BK);
  const bool tail = kbeg + nsl * BK < kend;


  // per-lane DMA sources (32-bit byte offsets from the slice base): LDS chunk ci lands at
  // ci*16; its source is the global chunk whose swizzled slot that is
  auto src = [&](long ld, int mn0, int MN, bool kmaj, int ci) -> uint32_t {
    if (kmaj) {
      const int row = ci >> 2, c = (ci & 3) ^ swz32(ci >> 2);
      return (uint32_t)(((long)min(mn0 + row, MN - 1) * ld + c * 8) * 2);
    }
    const int pnl = ci >> 9, cj = ci & 511, k = cj >> 4, c = (cj & 15) ^ swz_mn_bf16(k);
    return (uint32_t)(((long)k * ld + min((long)(mn0 + pnl * 128 + c * 8), (long)((MN - 1) & ~7))) * 2);
  };
  const char* abase = (const char*)(A + (AK ? (long)kbeg : (long)kbeg * p.lda));
  const char* bbase = (const char*)(B + (BKM ? (long)kbeg : (long)kbeg * p.ldb));
  uint32_t aoff[ACH], boff[BCH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) aoff[i] = src(p.lda, m0, ov.M, AK, (i * NW + w) * 64 + lane);
#pragma unroll
  for (int i = 0; i < BCH; ++i) boff[i] = src(p.ldb, n0, p.N, BKM, (i * NW + w) * 64 + lane);
  const long astep = (AK ? BK : (long)BK * p.lda) * 2;  // bytes per slice
  const long bstep = (BKM ? BK : (long)BK * p.ldb) * 2;

  // implicit-GEMM gathers (gemm_bf16_lds's scheme on 32-deep slices; the host guarantees
  // C % 64 == 0, so a slice never straddles two taps and K has no remainder).  A rows
  // (FWD / DGRAD): each chunk's pixel decoded once, its source rebuilt when a slice enters a
  // new tap.  B rows (WGRAD, k = pixel): each chunk's pixel advanced by 32 per slice.
  const int ksl0 = kbeg / BK;                  // global slice index of this range's first slice
  const int CS = MODE ? p.g.C / BK : 1;        // slices per tap
  int gb[ACH], gt[ACH], gf[ACH], cur[ACH];
  if constexpr (MODE == EA_CONV_FWD || MODE == EA_CONV_DGRAD) {
    const int n2 = MODE == EA_CONV_FWD ? p.g.T2 : p.g.nI[ov.a];
    const int n3 = MODE == EA_CONV_FWD ? p.g.F2 : p.g.nJ[ov.e];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int m = min(m0 + ((((i * NW + w) * 64 + lane)) >> 2), ov.M - 1);
      const int bt = fdiv(m, n3);
      gf[i] = m - bt * n3;
      gb[i] = fdiv(bt, n2);
      gt[i] = bt - gb[i] * n2;
      cur[i] = 0;
    }
  }
  auto a_tap = [&](int q) {  // A chunk sources (elements) for tap q
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int ci = (i * NW + w) * 64 + lane;
      const int cc = ((ci & 3) ^ swz32(ci >> 2)) * 8;
      if constexpr (MODE == EA_CONV_FWD) {
        const int kh = q / 3, kw = q - 3 * (q / 3);
        cur[i] = (int)x1p_row(p.g, gb[i], gt[i], gf[i], kh, kw) + cc;
      } else {
        int kh, kw;
        dgrad_tap2(ov.a, ov.e, q, kh, kw);
        const int t2 = gt[i] - (kh >> 1), f2 = gf[i] - (kw >> 1);  // t1 = 2*t2 + kh
        cur[i] = (t2 >= 0 && t2 < p.g.T2 && f2 >= 0 && f2 < p.g.F2)
                     ? ((gb[i] * p.g.T2 + t2) * p.g.F2 + f2) * p.g.C + cc
                     : (int)p.g.zero + ((ci >> 2) & 63) * p.g.C + cc;  // spread over 64 zero rows
      }
    }
  };
  int wb[BCH], wt[BCH], wf[BCH], wpix[BCH], wbase[BCH], wnI[BCH], wnJ[BCH];
  if constexpr (MODE == EA_CONV_WGRAD) {
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int ci = (i * NW + w) * 64 + lane;
      const int pnl = ci >> 9, cj = ci & 511, k = cj >> 4, c = (cj & 15) ^ swz_mn_bf16(k);
      const int n = min(n0 + pnl * 128 + c * 8, p.N - 8);
      const int tap = n / p.g.C, cin = n - tap * p.g.C;
      const int kh = tap / 3, kw = tap - 3 * kh, a = kh & 1, e = kw & 1;
      wnI[i] = p.g.nI[a];
      wnJ[i] = p.g.nJ[e];
      // row (b*nI + t2 + kh/2)*nJ + f2 + kw/2 of plane (a, e): the tap shift folded into the base
      wbase[i] = (int)p.g.plane[a * 2 + e] + ((kh >> 1) * wnJ[i] + (kw >> 1)) * p.g.C + cin;
      const int pix = ksl0 * BK + k;
      wpix[i] = pix;
      const int bt = fdiv(pix, p.g.F2);
      wf[i] = pix - bt * p.g.F2;
      wb[i] = fdiv(bt, p.g.T2);
      wt[i] = bt - wb[i] * p.g.T2;
    }
  }
  const int dF = BK % max(p.g.F2, 1), dT = BK / max(p.g.F2, 1);

  auto issue = [&](int sl) {  // called for sl = 0, 1, 2, ... in order (gather state advances)
    char* base = smem + (sl % NSLOT) * SLOT;
    const char* ak = abase + sl * astep;
    const char* bk = bbase + sl * bstep;
    if constexpr (MODE == EA_CONV_FWD || MODE == EA_CONV_DGRAD) {
      // FWD: k = (64-channel block, tap, channel): 2 slices per tap, the 9 taps of a block back
      // to back, so a tile's x1p footprint for one block stays in cache across its taps;
      // DGRAD: k = (tap of the class, channel)
      const int ks = ksl0 + sl;
      int q, c0;
      bool newtap;
      if constexpr (MODE == EA_CONV_FWD) {
        const int cb = ks / 18, r = ks - 18 * cb;
        q = r >> 1;
        c0 = cb * 64 + (r & 1) * BK;
        newtap = (r & 1) == 0;
      } else {
        q = ks / CS;
        c0 = (ks - q * CS) * BK;
        newtap = c0 == 0;
      }
      if (newtap || sl == 0) a_tap(q);
#pragma unroll
      for (int i = 0; i < ACH; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)((const char*)A + (long)(cur[i] + c0) * 2),
                                         (__attribute__((address_space(3))) void*)(base + (i * NW + w) * 1024), 16, 0, 0);
      if constexpr (MODE == EA_CONV_DGRAD) {  // W2t [9][co][ci]: a slice = 32 co of one tap
        int kh, kw;
        dgrad_tap2(ov.a, ov.e, q, kh, kw);
        // K-major W2k [ci][tap][co] (ldb = 9C): the slice is 32 co of tap (kh, kw) in every row
        bk = BKM ? (const char*)(B + (long)(kh * 3 + kw) * p.g.C + c0)
                 : (const char*)(B + ((long)(kh * 3 + kw) * p.g.C + c0) * p.g.C);
      }
    } else {
#pragma unroll
      for (int i = 0; i < ACH; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(ak + aoff[i]),
                                         (__attribute__((address_space(3))) void*)(base + (i * NW + w) * 1024), 16, 0, 0);
    }
    if constexpr (MODE == EA_CONV_WGRAD) {  // B[k = pixel][n = (tap, ci)] gathered from x1p
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int off = wpix[i] < p.g.P ? wbase[i] + ((wb[i] * wnI[i] + wt[i]) * wnJ[i] + wf[i]) * p.g.C
                                        : (int)p.g.zero + (lane & 63) * p.g.C + (wbase[i] % p.g.C);
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)((const char*)B + (long)off * 2),
                                         (__attribute__((address_space(3))) void*)(base + A_BYTES + (i * NW + w) * 1024),
                                         16, 0, 0);
        wpix[i] += BK;  // next slice: 32 pixels on
        wf[i] += dF;
        wt[i] += dT;
        if (wf[i] >= p.g.F2) { wf[i] -= p.g.F2; ++wt[i]; }
        while (wt[i] >= p.g.T2) { wt[i] -= p.g.T2; ++wb[i]; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(bk + boff[i]),
                                         (__attribute__((address_space(3))) void*)(base + A_BYTES + (i * NW + w) * 1024),
                                         16, 0, 0);
    }
  };

  auto rd_b = [&](int sl, bf16x8 (&fb)[4]) {
    const char* lb = smem + (sl % NSLOT) * SLOT + A_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag32<BKM>(lb, wn + j * 16, lane);
  };
  auto rd_a = [&](int sl, bf16x8 (&fa)[MI]) {
    const char* la = smem + (sl % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = frag32<AK>(la, wm + i * 16, lane);
  };

  const int g1 = w >> 2;  // wave group: G1 runs one barrier behind G0
  const int npre = min(NSLOT - 1, nsl);
  for (int sl = 0; sl < npre; ++sl) issue(sl);
  // own share of slice 0 landed (slices 1 .. npre-1 may stay in flight), then everyone's
  wait_newer<G, NSLOT - 2>(npre - 1);
  lds_barrier();
  if (g1) lds_barrier();  // the stagger
  bf16x8 fa[MI], fb[4];
  for (int sl = 0; sl < nsl; ++sl) {
    // ---- LOAD(sl)
    __builtin_amdgcn_sched_barrier(0);
    rd_b(sl, fb);
    rd_a(sl, fa);
    if (sl + NSLOT - 1 < nsl) issue(sl + NSLOT - 1);
    // own share of slice sl+1 landed: the groups issued after it (sl+2 .. sl+NSLOT-1) may stay
    // in flight
    wait_newer<G, NSLOT - 2>(min(NSLOT - 2, nsl - 2 - sl));
    // fragments in registers before the barrier: the COMPUTE segment never waits on LDS, and
    // this wave is done reading slot sl when the barrier releases its refill
    if (!AK || !BKM) {  // asm tr-reads are invisible to the waitcnt pass
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(fb[j]));
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
    // ---- COMPUTE(sl), at raised issue priority (the other group's LOAD waits for it)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
  }
  if (!g1) lds_barrier();  // balance G1's extra barrier
  if (tail) {  // K remainder (< 32) through registers, zero-filled, into slot 0
    constexpr int NCH = (A_BYTES + B_BYTES) / 16 / NTT;  // 4 chunks per thread
    uint4 v[NCH];
    const int k0 = kbeg + nsl * BK;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + NTT * i;
      const bool isa = c < A_BYTES / 16;
      const int cc = isa ? c : c - A_BYTES / 16;
      const bool km = isa ? AK : BKM;
      const bf16* base = isa ? A : B;
      const long ld = isa ? p.lda : p.ldb;
      const int MN = isa ? ov.M : p.N, mn0 = isa ? m0 : n0;
      int mn, k;
      if (km) { mn = mn0 + (cc >> 2); k = k0 + (cc & 3) * 8; }
      else    { const int cj = cc & 511; k = k0 + (cj >> 4); mn = mn0 + (cc >> 9) * 128 + (cj & 15) * 8; }
      union { uint4 u; bf16 e[8]; } tv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = km ? (mn < MN && k + e < kend) : (k < kend && mn + e < MN);
        tv.e[e] = ok ? (km ? base[(long)mn * ld + k + e] : base[(long)k * ld + mn + e]) : (bf16)0.f;
      }
      v[i] = tv.u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + NTT * i;
      const bool isa = c < A_BYTES / 16;
      const int cc = isa ? c : c - A_BYTES / 16;
      const int off = isa ? (AK ? img32_off<true>(cc) : img32_off<false>(cc))
                          : A_BYTES + (BKM ? img32_off<true>(cc) : img32_off<false>(cc));
      *(uint4*)(smem + off) = v[i];
    }
    __syncthreads();
    rd_b(0, fb);
    rd_a(0, fa);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }

  __syncthreads();  // every wave is done reading the ring
}

// ---------------------------------------------------------------- conv1 weight gradient, fused
// ea_gemm_conv_w1: the EA_CONV_DGRAD GEMM of Conv2dSubsampling's backward whose ReLU-masked
// output g = d(conv1 pre-activation) (bf16-rounded, as the unfused path stores it) never goes
// to HBM: each 256-row tile contributes its share of conv1's weight / bias gradient
//   part[tm][t*C + c] = sum_{rows m of tile tm} g[m][c] * X[m][t],
//   X[m][t] = x[b][2*t1 + t/3][2*f1 + t%3] (t < 9, pixel (b, t1, f1) of class-plane row m), 1 (t = 9)
// as one more small MFMA product per wave: A = g^T (64 channels x 32 pixels, read from the
// epilogue's f32 image), B = X (32 pixels x 16 taps) from an LDS image staged before the main
// loop as bf16 hi + lo halves (x = hi + lo to 2^-16 relative).  The two wave groups' sums
// are combined in fixed order; ea_conv1_wgrad_reduce sums the tiles.
constexpr int W1_TS = 264;                              // X image tap row: 256 pixels + 8 (528 B)
constexpr int W1_IMG = 16 * W1_TS * 2;                  // one half (hi or lo), bytes
constexpr int W1_SMEM = PipeT<256>::SMEM + 2 * W1_IMG;  // 152 KiB

// The conv1 input patches of the tile's 256 pixels: loaded into registers before the main
// loop (w1_load_x; the loads land while it runs) and written to the LDS image after it
// (w1_stage_x), so their latency is off the tile's critical path.
EA_DEV void w1_load_x(const GemmP& p, const TileOv& ov, int m0, float (&xv)[5]) {
  const int tid = threadIdx.x;
  const int row = tid >> 1, t0 = (tid & 1) * 5;  // 512 threads: 256 rows x 2 halves of taps 0..9
  const int m = m0 + row;
#pragma unroll
  for (int u = 0; u < 5; ++u) xv[u] = 0.f;
  if (m < ov.M) {
    const int a = ov.a, e = ov.e, nI = p.g.nI[a], nJ = p.g.nJ[e];
    const int bi = fdiv(m, nJ), j = m - bi * nJ;
    const int b = fdiv(bi, nI), i = bi - b * nI;
    const float* xp = p.w1x + ((long)b * p.w1T + 2 * (2 * i + a)) * p.w1F + 2 * (2 * j + e);
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int t = t0 + u;
      xv[u] = t < 9 ? xp[(t / 3) * p.w1F + t % 3] : 1.f;
    }
  }
}
EA_DEV void w1_stage_x(char* xs, const float (&xv)[5]) {
  bf16* hi = (bf16*)xs;
  bf16* lo = (bf16*)(xs + W1_IMG);
  const int tid = threadIdx.x;
  const int row = tid >> 1, t0 = (tid & 1) * 5;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const bf16 h = (bf16)xv[u];
    hi[(t0 + u) * W1_TS + row] = h;
    lo[(t0 + u) * W1_TS + row] = (bf16)(xv[u] - (float)h);
  }
  for (int q = tid; q < 6 * 256; q += 512) {  // taps 10..15: zero
    const int t = 10 + (q >> 8), r = q & 255;
    hi[t * W1_TS + r] = (bf16)0.f;
    lo[t * W1_TS + r] = (bf16)0.f;
  }
}

// one wave's 128 x 64 (rows wm.., channels wn..) share; acc as pipe_tile leaves it
EA_DEV void w1_epilogue(const GemmP& p, const TileOv& ov, char* smem, int m0, int n0, int wm, int wn, int lane, int w, int tm,
                        const f32x4 (&acc)[8][4]) {
  float* t = (float*)smem + w * 64 * EPI_LDT;  // the wave's 64 x 64 f32 image
  const char* xh = smem + PipeT<256>::SMEM;
  const char* xl = xh + W1_IMG;
  const int g = lane >> 4, lc = lane & 15, rq = g * 4;
  const int lc8 = (lane & 7) * 8, rl = lane >> 3;
  const bf16* aux = (const bf16*)p.epi.aux;
  f32x4 out[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) out[cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {  // 64-row chunks
    if (ch) {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) t[(i * 16 + rq + rr) * EPI_LDT + j * 16 + lc] = acc[ch * 4 + i][j][rr];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    // ReLU mask (support bits, else aux = conv1 output) and bf16 rounding, in place: lane = 8
    // columns of a row
    const int rb = m0 + wm + ch * 64, col = n0 + wn + lc8;
    if (ov.w1pos) {
      uint32_t mb[8];
#pragma unroll
      for (int it = 0; it < 8; ++it)
        mb[it] = ov.w1pos[(long)min(rb + it * 8 + rl, ov.M - 1) * (p.N >> 3) + min(col, p.N - 8) / 8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        float* tr = t + (it * 8 + rl) * EPI_LDT + lc8;
        float4 f0 = *(const float4*)tr, f1 = *(const float4*)(tr + 4);
        float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = (float)(bf16)(((mb[it] >> c) & 1u) ? v[c] : 0.f);
        *(float4*)tr = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(tr + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    } else {
#pragma unroll
      for (int h0 = 0; h0 < 8; h0 += 4) {
        float o[4][8];
#pragma unroll
        for (int it = 0; it < 4; ++it)
          ld8(aux, (long)min(rb + (h0 + it) * 8 + rl, ov.M - 1) * p.epi.ldaux + col, EA_BF16, o[it]);
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          float* tr = t + ((h0 + it) * 8 + rl) * EPI_LDT + lc8;
          float4 f0 = *(const float4*)tr, f1 = *(const float4*)(tr + 4);
          float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
          for (int c = 0; c < 8; ++c) v[c] = (float)(bf16)(o[it][c] > 0.f ? v[c] : 0.f);
          *(float4*)tr = make_float4(v[0], v[1], v[2], v[3]);
          *(float4*)(tr + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    // out[cb][co, tap] += g^T . X over the chunk's 64 pixels (2 k-steps of 32)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int pl = wm + ch * 64 + 32 * ks + 8 * g;  // tile-local pixel of k = 8g
      const bf16x8 bh = *(const bf16x8*)(xh + (lc * W1_TS + pl) * 2);
      const bf16x8 bl = *(const bf16x8*)(xl + (lc * W1_TS + pl) * 2);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        union { bf16x8 v; bf16 e[8]; } af;
#pragma unroll
        for (int e = 0; e < 8; ++e) af.e[e] = (bf16)t[(32 * ks + 8 * g + e) * EPI_LDT + 16 * cb + lc];
        out[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bh, out[cb], 0, 0, 0);
        out[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af.v, bl, out[cb], 0, 0, 0);
      }
    }
  }
  // G1 (rows 128..255) hands its sums to G0 (same channels) through LDS; G0 writes the tile's
  // partial: rows co = 16cb + 4g + r of the wave's 64 channels, column tap lc
  __syncthreads();
  float* cmb = (float*)smem;  // [4][64][16], over the (now free) epilogue images
  if (w >= 4) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) cmb[((w - 4) * 64 + 16 * cb + 4 * g + r) * 16 + lc] = out[cb][r];
  }
  __syncthreads();
  if (w < 4 && lc < 10) {
    float* prow = ov.w1part + (long)tm * 10 * p.N + (long)lc * p.N;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = n0 + wn + 16 * cb + 4 * g + r;
        if (co < p.N) prow[co] = out[cb][r] + cmb[(w * 64 + 16 * cb + 4 * g + r) * 16 + lc];
      }
  }
}

// The four parity classes of the conv2 input gradient as one grid (GemmP.ncls): block -> item
// so that the tiles_n N-tiles of one M panel run on one XCD (blocks bid and bid + 8 share an
// XCD) and consecutive panels go round-robin over the XCDs; items are ordered class by class,
// longest K first, so the long tiles start first and the short ones fill the tail.  Patches the
// class's geometry into q; returns false for the padding blocks past the last item.
EA_DEV bool dgrad_class_item(const GemmP& p, TileOv& ov, TileIdx& ti) {
  const int bid = blockIdx.x, x = bid & 7, sq = bid >> 3, tn_n = p.tiles_n;
  const int item = ((sq / tn_n) * 8 + x) * tn_n + sq % tn_n;
  if (item >= p.cls_item0[p.ncls]) return false;
  int c = 0;
#pragma unroll
  for (int k = 1; k < 4; ++k) c += (k < p.ncls && item >= p.cls_item0[k]) ? 1 : 0;
  const int local = item - p.cls_item0[c];
  ov.M = p.cls_M[c];
  ov.a = p.cls_a[c];
  ov.e = p.cls_e[c];
  ov.w1part = p.w1part + (long)p.cls_tile0[c] * 10 * p.N;
  ov.w1pos = p.w1pos + p.cls_pos[c];
  ti.tm = local / tn_n;
  ti.tn = local % tn_n;
  ti.z = 0;
  ti.sk = p.cls_K[c];  // (the class's K, read by pipe_body for ncls launches)
  return true;
}

template <bool AK, bool BKM, int MODE, int BT, int NS>
EA_DEV void pipe_body(const GemmP& p, const TileOv& ov, const TileIdx& ti, char* smem) {
  using PC = PipeT<BT, NS>;
  constexpr int MI = PC::MI;
  const int tm = ti.tm, m0 = ti.tm * BT, n0 = ti.tn * BT;
  const bool cls = MODE == EA_CONV_DGRAD && p.ncls;  // merged parity classes: ti.sk holds K
  const int z = ti.z, sk = cls ? 0 : ti.sk;
  const int zb = z / p.nh, zh = z % p.nh;
  const bf16* A = (const bf16*)p.A + zb * p.sAb + zh * p.sAh;
  const bf16* B = (const bf16*)p.B + zb * p.sBb + zh * p.sBh;
  const int kbeg = sk * p.kchunk;
  const int kend = cls ? ti.sk : min(p.K, kbeg + p.kchunk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = PC::wm(w), wn = PC::wn(w);
  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  diag_stamp(p, 0);
  float w1x[5];
  if constexpr (MODE == EA_CONV_DGRAD) {
    if (p.w1part) w1_load_x(p, ov, m0, w1x);
  }
  pipe_tile<AK, BKM, MODE, BT, NS>(p, ov, smem, A, B, m0, n0, kbeg, kend, acc);
  diag_stamp(p, 1);
  if constexpr (MODE == EA_CONV_DGRAD) {
    if (p.w1part) {
      w1_stage_x(smem + PC::SMEM, w1x);  // its own region: read across waves by w1_epilogue
      __syncthreads();
      w1_epilogue(p, ov, smem, m0, n0, wm, wn, lane, w, tm, acc);
      return;
    }
  }
  const EpiK ek = make_epik(p);
  switch (p.splitk > 1 ? EA_EPI_STORE : p.epi.kind) {
    case EA_EPI_STORE: epi_wave<EA_EPI_STORE, MI, 4>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    case EA_EPI_ACT: epi_wave<EA_EPI_ACT, MI, 4>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    case EA_EPI_RESID: epi_wave<EA_EPI_RESID, MI, 4>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    default: epi_wave<EA_EPI_DACT, MI, 4>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
  }
  if (p.diag) {
    __syncthreads();
    diag_stamp(p, 2);
  }
}

template <bool AK, bool BKM, int MODE = 0, int BT = 256, int NS = 4>
__global__ __launch_bounds__(512, (PipeT<BT, NS>::OCC)) void gemm_pipe(GemmP p) {
  using PC = PipeT<BT, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[MODE == EA_CONV_DGRAD ? W1_SMEM : PC::SMEM];
  probe_start(p);
  TileOv ov = tile_ov(p);
  TileIdx ti;
  bool run = true;
  if (MODE == EA_CONV_DGRAD && p.ncls) run = dgrad_class_item(p, ov, ti);
  else ti = tile_index(p);
  if (run) pipe_body<AK, BKM, MODE, BT, NS>(p, ov, ti, smem);
  probe_end(p);
}

}  // namespace
