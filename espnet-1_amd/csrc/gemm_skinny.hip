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

}  // namespace

namespace eag {
int launch_skinny(GemmP& p, hipStream_t st, int rows32) {
  if (rows32) {  // 32 x 32 blocks (M beyond a few 16-row blocks: the decoder's 1,312 tokens)
    dim3 grid(ea_cdiv(p.N, 32), ea_cdiv(p.M, 32), 1);
    hipLaunchKernelGGL((gemm_skinny_kernel<2, 2, 4>), grid, dim3(64 * SK_W), 0, st, p);
  } else {
    dim3 grid(ea_cdiv(p.N, 32), ea_cdiv(p.M, 16), 1);
    hipLaunchKernelGGL((gemm_skinny_kernel<1, 2, 8>), grid, dim3(64 * SK_W), 0, st, p);
  }
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
