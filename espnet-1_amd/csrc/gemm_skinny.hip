// Few-row bf16 GEMM (ea_gemm_set_skinny): C (M <= a few 16-row blocks, N) = A (M, K) . W (N, K)^T
// with the fused epilogues — the incremental decoder's per-step Linears (one row per running
// hypothesis, ~10) and anything else of that shape.
//
// The tile kernels give such a GEMM ceil(N / 128) blocks that each walk the whole K serially
// (a 2048-deep K at N = 512 is 4 blocks), so the launch is one HBM round trip per K slice.
// Here a block owns 16 (or 32) rows x 32 columns and its 8 waves split K among themselves (wave w
// takes the 32-deep slices w, w + 8, ...), each wave issuing the loads of up to 8 slices before
// its first MFMA: both operands go global -> registers in MFMA fragment order (16-B loads, no
// LDS staging — W is read exactly once per 16-row block and A is a few KB), so a launch costs
// about one memory latency plus the cross-wave sum through LDS and the epilogue.
// N = 512 -> 16 blocks x 8 waves; the output Linear (N = 5000) 157 blocks.
#include "gemm_kern.h"

namespace {
using namespace eag;

constexpr int SK_W = 8;  // waves per block (K split)

template <int KIND>
EA_DEV void skinny_epi(const GemmP& p, const EpiK& ek, int row, int col, const float (&v)[4]) {
  if (row >= p.M) return;
  if (p.vec_c && col + 3 < p.N) {
    epi_four<KIND>(p, ek, 0, 0, 0, row, col, v);
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (col + c < p.N) epi_one<KIND>(p, 0, 0, 0, row, col + c, v[c]);
  }
}

// MT 16-row x NJ 16-column MFMA tiles per block; U 32-deep slices per wave with loads in flight
template <int MT, int NJ, int U>
__global__ __launch_bounds__(64 * SK_W) void gemm_skinny_kernel(GemmP p) {
  constexpr int BR = 16 * MT, BC = 16 * NJ, LD = BC + 4;
  __shared__ __attribute__((aligned(16))) float red[SK_W][BR][LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = blockIdx.y * BR, c0 = blockIdx.x * BC;
  const bf16* __restrict__ A = (const bf16*)p.A;
  const bf16* __restrict__ B = (const bf16*)p.B;
  const int nks = p.K / 32;
  const int kq = 8 * (lane >> 4);
  const bf16* ap[MT];
  bool aok[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = r0 + i * 16 + (lane & 15);
    aok[i] = row < p.M;
    ap[i] = A + (long)(aok[i] ? row : 0) * p.lda + kq;
  }
  const bf16* bp[NJ];
  bool bok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = c0 + j * 16 + (lane & 15);
    bok[j] = col < p.N;
    bp[j] = B + (long)(bok[j] ? col : 0) * p.ldb + kq;
  }
  f32x4 acc[MT][NJ];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero = {};
  for (int ks0 = w; ks0 < nks; ks0 += SK_W * U) {
    bf16x8 a[U][MT], b[U][NJ];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ks = ks0 + u * SK_W;
      const bool in = ks < nks;
#pragma unroll
      for (int i = 0; i < MT; ++i) a[u][i] = in && aok[i] ? *(const bf16x8*)(ap[i] + ks * 32) : zero;
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[u][j] = in && bok[j] ? *(const bf16x8*)(bp[j] + ks * 32) : zero;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
  }
  // partial tiles -> LDS (D layout: lane holds rows 4*(lane>>4)+r of column lane&15)
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][i * 16 + 4 * (lane >> 4) + r][j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  constexpr int GROUPS = BR * BC / 4;  // 4-column output groups of the block
  const EpiK ek = make_epik(p);
  for (int gi = threadIdx.x; gi < GROUPS; gi += 64 * SK_W) {
    const int row = gi / (BC / 4), cg = (gi % (BC / 4)) * 4;
    float v[4];
    float4 s = *(const float4*)&red[0][row][cg];
#pragma unroll
    for (int q = 1; q < SK_W; ++q) {
      const float4 t = *(const float4*)&red[q][row][cg];
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    v[0] = s.x; v[1] = s.y; v[2] = s.z; v[3] = s.w;
    switch (p.epi.kind) {
      case EA_EPI_STORE: skinny_epi<EA_EPI_STORE>(p, ek, r0 + row, c0 + cg, v); break;
      case EA_EPI_ACT: skinny_epi<EA_EPI_ACT>(p, ek, r0 + row, c0 + cg, v); break;
      case EA_EPI_RESID: skinny_epi<EA_EPI_RESID>(p, ek, r0 + row, c0 + cg, v); break;
      default: skinny_epi<EA_EPI_DACT>(p, ek, r0 + row, c0 + cg, v); break;
    }
  }
}

// LayerNorm fused in front (ea_gemm_ln): A is the f32 residual stream x (M x K); each block
// normalises its 16 rows itself — the waves' fragments of a row are summed across lanes and
// waves for the mean, then for the variance of the deviations (the LayerNorm kernel's formula,
// ln_fwd_vec_kernel), and (x - mean) * rstd * gamma + beta is rounded to bf16 in the MFMA
// fragment registers.  One batch of loads: K <= 32 * SK_W * 8 = 2,048.
__global__ __launch_bounds__(64 * SK_W) void gemm_skinny_ln_kernel(GemmP p, const float* __restrict__ gam,
                                                                   const float* __restrict__ bet, float eps) {
  constexpr int NJ = 2, U = 8, BC = 16 * NJ, LD = BC + 4;
  __shared__ __attribute__((aligned(16))) float red[SK_W][16][LD];
  __shared__ float st[2][SK_W][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = blockIdx.y * 16, c0 = blockIdx.x * BC;
  const float* __restrict__ X = (const float*)p.A;
  const bf16* __restrict__ B = (const bf16*)p.B;
  const int nks = p.K / 32;
  const int kq = 8 * (lane >> 4);
  const int row = r0 + (lane & 15);
  const bool aok = row < p.M;
  const float* xp = X + (long)(aok ? row : 0) * p.lda + kq;
  const bf16* bp[NJ];
  bool bok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = c0 + j * 16 + (lane & 15);
    bok[j] = col < p.N;
    bp[j] = B + (long)(bok[j] ? col : 0) * p.ldb + kq;
  }
  float xv[U][8];
  bf16x8 b[U][NJ];
  const bf16x8 zero = {};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int ks = w + u * SK_W;
    const bool in = ks < nks;
    if (in && aok) {
      const float4 v0 = *(const float4*)(xp + ks * 32), v1 = *(const float4*)(xp + ks * 32 + 4);
      xv[u][0] = v0.x; xv[u][1] = v0.y; xv[u][2] = v0.z; xv[u][3] = v0.w;
      xv[u][4] = v1.x; xv[u][5] = v1.y; xv[u][6] = v1.z; xv[u][7] = v1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[u][e] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[u][j] = in && bok[j] ? *(const bf16x8*)(bp[j] + ks * 32) : zero;
  }
  // row mean, then the variance of the deviations, over all K (lanes of a row: lane & 15
  // across the four 16-lane groups; waves through LDS)
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += xv[u][e];
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  if (lane < 16) st[0][w][lane] = s;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int q = 0; q < SK_W; ++q) tot += st[0][q][lane & 15];
  const float mu = tot / p.K;
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (w + u * SK_W >= nks) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dlt = xv[u][e] - mu;
      ss += dlt * dlt;
    }
  }
  ss += __shfl_xor(ss, 16);
  ss += __shfl_xor(ss, 32);
  if (lane < 16) st[1][w][lane] = ss;
  __syncthreads();
  float tss = 0.f;
#pragma unroll
  for (int q = 0; q < SK_W; ++q) tss += st[1][q][lane & 15];
  const float rs = rsqrtf(tss / p.K + eps);
  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int ks = w + u * SK_W;
    if (ks >= nks) continue;
    const int k0 = ks * 32 + kq;
    const float4 g0 = *(const float4*)(gam + k0), g1 = *(const float4*)(gam + k0 + 4);
    const float4 b0 = *(const float4*)(bet + k0), b1 = *(const float4*)(bet + k0 + 4);
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    union { bf16x8 v; bf16 e[8]; } a;
#pragma unroll
    for (int e = 0; e < 8; ++e) a.e[e] = (bf16)((xv[u][e] - mu) * rs * gg[e] + bb[e]);
    if (!aok) a.v = zero;
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b[u][j], acc[j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][4 * (lane >> 4) + r][j * 16 + (lane & 15)] = acc[j][r];
  __syncthreads();
  constexpr int GROUPS = 16 * BC / 4;
  if (threadIdx.x >= GROUPS) return;
  const int orow = threadIdx.x / (BC / 4), cg = (threadIdx.x % (BC / 4)) * 4;
  float4 sm = *(const float4*)&red[0][orow][cg];
#pragma unroll
  for (int q = 1; q < SK_W; ++q) {
    const float4 t = *(const float4*)&red[q][orow][cg];
    sm.x += t.x; sm.y += t.y; sm.z += t.z; sm.w += t.w;
  }
  const float v[4] = {sm.x, sm.y, sm.z, sm.w};
  const EpiK ek = make_epik(p);
  switch (p.epi.kind) {
    case EA_EPI_STORE: skinny_epi<EA_EPI_STORE>(p, ek, r0 + orow, c0 + cg, v); break;
    case EA_EPI_ACT: skinny_epi<EA_EPI_ACT>(p, ek, r0 + orow, c0 + cg, v); break;
    case EA_EPI_RESID: skinny_epi<EA_EPI_RESID>(p, ek, r0 + orow, c0 + cg, v); break;
    default: skinny_epi<EA_EPI_DACT>(p, ek, r0 + orow, c0 + cg, v); break;
  }
}

}  // namespace

namespace eag {
int launch_skinny_ln(GemmP& p, const float* gamma, const float* beta, float eps, hipStream_t st) {
  dim3 grid(ea_cdiv(p.N, 32), ea_cdiv(p.M, 16), 1);
  hipLaunchKernelGGL(gemm_skinny_ln_kernel, grid, dim3(64 * SK_W), 0, st, p, gamma, beta, eps);
  EA_LAUNCH_CHECK();
  return 0;
}
int launch_skinny(GemmP& p, hipStream_t st) {
  dim3 grid(ea_cdiv(p.N, 32), ea_cdiv(p.M, 16), 1);
  hipLaunchKernelGGL((gemm_skinny_kernel<1, 2, 8>), grid, dim3(64 * SK_W), 0, st, p);
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
