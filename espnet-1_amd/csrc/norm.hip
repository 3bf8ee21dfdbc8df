// LayerNorm (eps 1e-12, transformer/layer_norm.py:12-42) and the conv-module BatchNorm1d
// (conformer/convolution.py:45,75) forward/backward, plus the shared partial-sum reducer.
//
// LayerNorm: one wave64 per row, the row held in registers (d <= 64*MAXE), two-pass
// mean/variance in f32; backward fuses dgamma/dbeta per-block partials (deterministic
// second pass, ea_reduce_partials) and accumulates dx into the f32 residual gradient.
#include "common.h"

namespace {

template <int MAXE, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int d, const float* __restrict__ x, long ldx,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float eps, TO* __restrict__ y, long ldy,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < rows; r += nw) {
    const float* xr = x + (long)r * ldx;
    float v[MAXE];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      const int c = i * 64 + lane;
      v[i] = c < d ? xr[c] : 0.f;
      s += v[i];
    }
    const float mean = wave_sum(s) / d;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      const int c = i * 64 + lane;
      const float t = c < d ? v[i] - mean : 0.f;
      ss += t * t;
    }
    const float rstd = rsqrtf(wave_sum(ss) / d + eps);
    TO* yr = y + (long)r * ldy;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      const int c = i * 64 + lane;
      if (c < d) yr[c] = from_f<TO>((v[i] - mean) * rstd * g[c] + b[c]);
    }
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// dx (+)= rstd*(dxh - mean(dxh) - xh*mean(dxh*xh)),  dxh = dy*gamma
// part[blk][0:d] = sum dy*xh, part[blk][d:2d] = sum dy   (this block's rows)
template <int MAXE, typename TI>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int d, const TI* __restrict__ dy, long lddy,
                                                     const float* __restrict__ x, long ldx,
                                                     const float* __restrict__ g, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, float* __restrict__ dx,
                                                     long lddx, int accumulate, float* __restrict__ part) {
  __shared__ float red[4][2][64 * MAXE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = gridDim.x * 4;
  float pg[MAXE], pb[MAXE];
#pragma unroll
  for (int i = 0; i < MAXE; ++i) pg[i] = pb[i] = 0.f;
  for (int r = blockIdx.x * 4 + w; r < rows; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    float xh[MAXE], dg[MAXE];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      const int c = i * 64 + lane;
      if (c < d) {
        const float dyv = to_f(dy[(long)r * lddy + c]);
        xh[i] = (x[(long)r * ldx + c] - mu) * rs;
        dg[i] = dyv * g[c];
        s1 += dg[i];
        s2 += dg[i] * xh[i];
        pg[i] += dyv * xh[i];
        pb[i] += dyv;
      } else {
        xh[i] = dg[i] = 0.f;
      }
    }
    s1 = wave_sum(s1) / d;
    s2 = wave_sum(s2) / d;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      const int c = i * 64 + lane;
      if (c < d) {
        float v = rs * (dg[i] - s1 - xh[i] * s2);
        float* o = dx + (long)r * lddx + c;
        *o = accumulate ? *o + v : v;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXE; ++i) {
    red[w][0][i * 64 + lane] = pg[i];
    red[w][1][i * 64 + lane] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float a = 0.f, bb = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a += red[k][0][c];
      bb += red[k][1][c];
    }
    part[(long)blockIdx.x * 2 * d + c] = a;
    part[(long)blockIdx.x * 2 * d + d + c] = bb;
  }
}

// out[c] (+)= sum_p part[p*stride + c], c < n.  Block = RP_CW columns x RP_PL part-lanes; each
// lane sums a fixed strided subset of the parts (8 loads in flight per lane: the loop is
// latency-, not bandwidth-bound, so the parts are spread over many lanes and blocks), lanes
// combine in fixed order through LDS (deterministic).
// tr_rows > 0: column j = k*tr_rows + c is written to out[c*tr_cols + k] (transposed output).
constexpr int RP_CW = 16, RP_PL = 16;
__global__ __launch_bounds__(256) void reduce_partials_kernel(int nparts, int n, const float* __restrict__ part,
                                                              long stride, float* __restrict__ out, int accumulate,
                                                              int tr_rows = 0, int tr_cols = 0) {
  __shared__ double red[RP_PL][RP_CW];
  const int cx = threadIdx.x % RP_CW, py = threadIdx.x / RP_CW;
  const int c = blockIdx.x * RP_CW + cx;
  double a = 0.0;
  if (c < n) {
    int p = py;
    for (; p + 7 * RP_PL < nparts; p += 8 * RP_PL) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long)(p + RP_PL * j) * stride + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) a += v[j];
    }
    for (; p < nparts; p += RP_PL) a += part[(long)p * stride + c];
  }
  red[py][cx] = a;
  __syncthreads();
  if (py == 0 && c < n) {
    double t = 0.0;
#pragma unroll
    for (int l = 0; l < RP_PL; ++l) t += red[l][cx];
    // columns [0, tr_rows * tr_cols) written transposed, any after them straight
    const long o = tr_rows > 0 && c < tr_rows * tr_cols ? (long)(c % tr_rows) * tr_cols + c / tr_rows : c;
    out[o] = accumulate ? out[o] + (float)t : (float)t;
  }
}

// column partial sums of x (rows x n, dtype) : part[blk][c] = sum over this block's rows
template <typename T>
__global__ void colsum_partial_kernel(int rows, int n, const T* __restrict__ x, long ld, int rows_per_blk,
                                      float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const int r0 = blockIdx.y * rows_per_blk;
  const int r1 = min(rows, r0 + rows_per_blk);
  float a = 0.f;
  for (int r = r0; r < r1; ++r) a += to_f(x[(long)r * ld + c]);
  part[(long)blockIdx.y * n + c] = a;
}


// Column partial sums, 4 columns per lane (8-B bf16 / 16-B f32 loads): a wave covers 256
// columns of one row, the 4 waves of a block interleave rows, the block writes one
// partial row.  LN=true computes the LayerNorm parameter grads instead:
// part[p][c] = sum dy*xhat, part[p][n + c] = sum dy.
template <typename T, bool LN>
__global__ __launch_bounds__(256) void colsum_vec_kernel(int rows, int n, const T* __restrict__ x, long ld,
                                                         const float* __restrict__ xin, long ldxin,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         int rows_per_part, float* __restrict__ part) {
  __shared__ float red[4][2][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.y * rows_per_part, r1 = min(rows, r0 + rows_per_part);
  float a[4] = {0.f, 0.f, 0.f, 0.f}, g[4] = {0.f, 0.f, 0.f, 0.f};
  auto load4 = [&](int r, float (&v)[4]) {
    if (sizeof(T) == 2) {
      const uint2 u = *(const uint2*)(x + (long)r * ld + c);
      const bf16* b = (const bf16*)&u;
      v[0] = (float)b[0]; v[1] = (float)b[1]; v[2] = (float)b[2]; v[3] = (float)b[3];
    } else {
      const float4 f = *(const float4*)(x + (long)r * ld + c);
      v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    }
  };
  auto acc_row = [&](int r, const float (&v)[4], float4 xv) {
    if (LN) {
      const float mu = mean[r], rs = rstd[r];
      g[0] += v[0] * (xv.x - mu) * rs;
      g[1] += v[1] * (xv.y - mu) * rs;
      g[2] += v[2] * (xv.z - mu) * rs;
      g[3] += v[3] * (xv.w - mu) * rs;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += v[k];
  };
  if (c < n) {
    int r = r0 + w;
    for (; r + 12 < r1; r += 16) {  // 4 rows per wave in flight
      float v[4][4];
      float4 xv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        load4(r + 4 * j, v[j]);
        if (LN) xv[j] = *(const float4*)(xin + (long)(r + 4 * j) * ldxin + c);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc_row(r + 4 * j, v[j], LN ? xv[j] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
    for (; r < r1; r += 4) {
      float v[4];
      load4(r, v);
      acc_row(r, v, LN ? *(const float4*)(xin + (long)r * ldxin + c) : make_float4(0.f, 0.f, 0.f, 0.f));
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[w][0][lane * 4 + k] = a[k];
    red[w][1][lane * 4 + k] = g[k];
  }
  __syncthreads();
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc < n) {
    const int t = threadIdx.x;
    const float sa = (red[0][0][t] + red[1][0][t]) + (red[2][0][t] + red[3][0][t]);
    if (LN) {
      const float sg = (red[0][1][t] + red[1][1][t]) + (red[2][1][t] + red[3][1][t]);
      part[(long)blockIdx.y * 2 * n + cc] = sg;
      part[(long)blockIdx.y * 2 * n + n + cc] = sa;
    } else {
      part[(long)blockIdx.y * n + cc] = sa;
    }
  }
}

// LayerNorm backward, dx only (one wave per row, max parallelism)
template <int MAXE, typename TI>
__global__ __launch_bounds__(256) void ln_bwd_dx_kernel(int rows, int d, const TI* __restrict__ dy, long lddy,
                                                        const float* __restrict__ x, long ldx,
                                                        const float* __restrict__ g, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, float* __restrict__ dx,
                                                        long lddx, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float mu = mean[r], rs = rstd[r];
  float xh[MAXE], dg[MAXE];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXE; ++i) {
    const int c = i * 64 + lane;
    if (c < d) {
      xh[i] = (x[(long)r * ldx + c] - mu) * rs;
      dg[i] = to_f(dy[(long)r * lddy + c]) * g[c];
      s1 += dg[i];
      s2 += dg[i] * xh[i];
    } else {
      xh[i] = dg[i] = 0.f;
    }
  }
  s1 = wave_sum(s1) / d;
  s2 = wave_sum(s2) / d;
#pragma unroll
  for (int i = 0; i < MAXE; ++i) {
    const int c = i * 64 + lane;
    if (c < d) {
      const float v = rs * (dg[i] - s1 - xh[i] * s2);
      float* o = dx + (long)r * lddx + c;
      *o = accumulate ? *o + v : v;
    }
  }
}

// y = dropout(scale * x) (the residual-branch gradient entering a Linear's backward, same
// element index (r*cols + c) and mask as ea_scale_dropout) fused with the column partial
// sums of the stored y (the Linear's bias gradient): one read of x instead of two passes.
// Layout as colsum_vec_kernel: 256 columns per block (4 per lane), the 4 waves interleave the
// block's rows, part[blockIdx.y][c] = this row range's sum (waves combined in fixed order).
template <typename TO>
__global__ __launch_bounds__(256) void scale_drop_colsum_kernel(int rows, int n, const float* __restrict__ x, long ldx,
                                                                TO* __restrict__ y, long ldy, float scale, float p,
                                                                uint64_t seed, const unsigned long long* salt,
                                                                int rows_per_part, float* __restrict__ part) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.y * rows_per_part, r1 = min(rows, r0 + rows_per_part);
  if (p > 0.f) seed = ea_salted(seed, salt);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < n) {
    for (int r = r0 + w; r < r1; r += 4) {
      float v[4];
      vld4(x + (long)r * ldx + c, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] *= scale;
      drop_scale4(seed, (uint64_t)r * n + c, p, v);
      TO* yp = y + (long)r * ldy + c;
      vst4(yp, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += to_f(from_f<TO>(v[k]));  // sum what was stored
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[w][lane * 4 + k] = a[k];
  __syncthreads();
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc < n)
    part[(long)blockIdx.y * n + cc] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// ---------------------------------------------------------------- vectorised LayerNorm
// One wave64 per row; lane l owns the 8-column chunks c = l + 64*j (j < NJ), moved with
// 16-B loads/stores (f32: 2 x float4, bf16: 1 x uint4).  d % 8 == 0, d <= 512*NJ.
template <typename T> EA_DEV void ld8(const T* p, float (&v)[8]);
template <> EA_DEV void ld8<float>(const float* p, float (&v)[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <> EA_DEV void ld8<bf16>(const bf16* p, float (&v)[8]) {
  const uint4 u = *(const uint4*)p;
  const bf16* e = (const bf16*)&u;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)e[i];
}
template <typename T> EA_DEV void st8(T* p, const float (&v)[8]);
template <> EA_DEV void st8<float>(float* p, const float (&v)[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <> EA_DEV void st8<bf16>(bf16* p, const float (&v)[8]) {
  union { uint4 u; bf16 e[8]; } t;
#pragma unroll
  for (int i = 0; i < 8; ++i) t.e[i] = (bf16)v[i];
  *(uint4*)p = t.u;
}

template <int NJ, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(int rows, int d, const float* __restrict__ x, long ldx,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, TO* __restrict__ y, long ldy,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + (long)r * ldx;
  float v[NJ][8], gg[NJ][8], bb[NJ][8];
  float s = 0.f;
  // gamma / beta loaded with the row (not after the two reductions: one latency fewer)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < d) {
      ld8(g + c, gg[j]);
      ld8(b + c, bb[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < d) {
      ld8(xr + c, v[j]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[j][i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[j][i];
  }
  const float mu = wave_sum(s) / d;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (lane + 64 * j) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float t = c < d ? v[j][i] - mu : 0.f;
      ss += t * t;
    }
  }
  const float rs = rsqrtf(wave_sum(ss) / d + eps);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c >= d) continue;
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[j][i] - mu) * rs * gg[j][i] + bb[j][i];
    st8(y + (long)r * ldy + c, o);
  }
  if (lane == 0) {
    mean_out[r] = mu;
    rstd_out[r] = rs;
  }
}

// dx (+)= rstd*(dxh - mean(dxh) - xh*mean(dxh*xh)) with dxh = dy*gamma, and this block's
// partial dgamma = sum dy*xh, dbeta = sum dy over its rows (part[blk][0:d], part[blk][d:2d];
// the 4 waves' sums combined in fixed order), all from one read of dy and x.
// DROP: also y = dropout(yscale * dx_new) in bf16 (element index r*d + c, the law and salt
// of ea_scale_dropout): the next residual site's dropout backward, without re-reading dx;
// with ypart, the block's column sums of the stored y (that site's bias gradient) go to
// ypart[blk][0:d] the same way.
struct LnDrop {
  bf16* y; long ldy; float scale, p; uint64_t seed; const unsigned long long* salt; float* ypart;
  bool want_ycol; float* ycol;  // host side: column sums requested; their final target (direct mode)
};
template <int NJ, typename TI, bool DROP = false, int UR = 2>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(int rows, int d, const TI* __restrict__ dy, long lddy,
                                                         const float* __restrict__ x, long ldx,
                                                         const float* __restrict__ g, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ dx,
                                                         long lddx, int accumulate, int rows_per_blk,
                                                         float* __restrict__ part, LnDrop dr = LnDrop{}) {
  constexpr int NS = DROP ? 3 : 2;
  __shared__ float red[4][NS][512 * NJ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (DROP && dr.p > 0.f) dr.seed = ea_salted(dr.seed, dr.salt);
  float gg[NJ][8], pg[NJ][8], pb[NJ][8], py[DROP ? NJ : 1][8];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (lane + 64 * j) * 8;
    if (c < d) ld8(g + c, gg[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) pg[j][i] = pb[j][i] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < (DROP ? NJ : 1); ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) py[j][i] = 0.f;
  const int r0 = blockIdx.x * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
  // U rows per wave step (rows rb and rb + 4): every load of both rows is issued before
  // either row is computed (the grid is ~2 waves per SIMD: latency, not bandwidth, bounds a
  // one-row step).  Rows are still folded into the partials in order rb, rb + 4.
  constexpr int U = NJ == 1 ? UR : 1;
  for (int rb = r0 + w; rb < r1; rb += 4 * U) {
    float xv[U][NJ][8], dv[U][NJ][8], pv[U][NJ][8], mu[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rb + 4 * u < r1 ? rb + 4 * u : rb;  // no second row: reload the first (unused)
      mu[u] = mean[r];
      rs[u] = rstd[r];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = (lane + 64 * j) * 8;
        if (c < d) {
          ld8(x + (long)r * ldx + c, xv[u][j]);
          ld8(dy + (long)r * lddy + c, dv[u][j]);
          if (accumulate) ld8(dx + (long)r * lddx + c, pv[u][j]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const int r = rb + 4 * u;
    if (r >= r1) break;
    float xh[NJ][8], dg[NJ][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = (lane + 64 * j) * 8;
      if (c < d) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[j][i] = (xv[u][j][i] - mu[u]) * rs[u];
          dg[j][i] = dv[u][j][i] * gg[j][i];
          s1 += dg[j][i];
          s2 += dg[j][i] * xh[j][i];
          pg[j][i] += dv[u][j][i] * xh[j][i];
          pb[j][i] += dv[u][j][i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) xh[j][i] = dg[j][i] = 0.f;
      }
    }
    s1 = wave_sum(s1) / d;
    s2 = wave_sum(s2) / d;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = (lane + 64 * j) * 8;
      if (c >= d) continue;
      float* o = dx + (long)r * lddx + c;
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = rs[u] * (dg[j][i] - s1 - xh[j][i] * s2) + (accumulate ? pv[u][j][i] : 0.f);
      st8(o, v);
      if constexpr (DROP) {
        float lo[4], hi[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { lo[i] = v[i] * dr.scale; hi[i] = v[i + 4] * dr.scale; }
        const uint64_t e = (uint64_t)r * d + c;
        drop_scale4(dr.seed, e, dr.p, lo);
        drop_scale4(dr.seed, e + 4, dr.p, hi);
        bf16* yo = dr.y + (long)r * dr.ldy + c;
        vst4(yo, lo);
        vst4(yo + 4, hi);
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // sums of the stored (rounded) values
          py[DROP ? j : 0][i] += (float)(bf16)lo[i];
          py[DROP ? j : 0][i + 4] += (float)(bf16)hi[i];
        }
      }
    }
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = (lane + 64 * j) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (c + i < 512 * NJ) {
        red[w][0][c + i] = pg[j][i];
        red[w][1][c + i] = pb[j][i];
        if constexpr (DROP) red[w][NS - 1][c + i] = py[DROP ? j : 0][i];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    part[(long)blockIdx.x * 2 * d + c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    part[(long)blockIdx.x * 2 * d + d + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
    if (DROP && dr.ypart)
      dr.ypart[(long)blockIdx.x * d + c] = (red[0][NS - 1][c] + red[1][NS - 1][c]) + (red[2][NS - 1][c] + red[3][NS - 1][c]);
  }
}

// ---------------------------------------------------------------- BatchNorm1d (train)
// Stats over all rows (padding included, as the reference's BatchNorm1d sees them).
// Pass 1: per-block shifted sums (shift = row 0) -> fp64 combine in bn_finalize.
__global__ void bn_partial_kernel(int rows, int C, const float* __restrict__ y, int rows_per_blk,
                                  float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sh = y[c];
  const int r0 = blockIdx.y * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
  float s = 0.f, ss = 0.f;
  for (int r = r0; r < r1; ++r) {
    const float t = y[(long)r * C + c] - sh;
    s += t;
    ss += t * t;
  }
  part[(long)blockIdx.y * 2 * C + c] = s;
  part[(long)blockIdx.y * 2 * C + C + c] = ss;
}

__global__ void bn_finalize_kernel(int rows, int C, int nparts, const float* __restrict__ y,
                                   const float* __restrict__ part, float eps, float momentum,
                                   float* __restrict__ mean, float* __restrict__ rstd,
                                   float* __restrict__ run_mean, float* __restrict__ run_var,
                                   long long* __restrict__ nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  double s = 0.0, ss = 0.0;
  for (int p = 0; p < nparts; ++p) {
    s += part[(long)p * 2 * C + c];
    ss += part[(long)p * 2 * C + C + c];
  }
  const double n = rows;
  const double m = s / n;
  double var = ss / n - m * m;
  if (var < 0) var = 0;
  const double mu = m + (double)y[c];
  mean[c] = (float)mu;
  rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * var * n / (n > 1 ? n - 1 : 1));
  }
}

__global__ void bn_eval_stats_kernel(int C, const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                     float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  rstd[c] = rsqrtf(rv[c] + eps);
}

// z = act(xhat*gamma + beta) (train: batch mean/rstd; eval: running stats passed in)
template <typename TO>
__global__ void bn_apply_act_kernel(long total, int C, const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ g,
                                    const float* __restrict__ b, int act, TO* __restrict__ z) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float h = (y[i] - mean[c]) * rstd[c] * g[c] + b[c];
    z[i] = from_f<TO>(act_fwd(act, h));
  }
}

// backward pass 1: dh = dz*act'(h); part = [sum dh*xhat | sum dh] per block
template <typename TI>
__global__ void bn_bwd_partial_kernel(int rows, int C, const TI* __restrict__ dz, const float* __restrict__ y,
                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                      const float* __restrict__ g, const float* __restrict__ b, int act,
                                      int rows_per_blk, float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
  const float mu = mean[c], rs = rstd[c], gg = g[c], bb = b[c];
  float s1 = 0.f, s2 = 0.f;
  for (int r = r0; r < r1; ++r) {
    const long i = (long)r * C + c;
    const float xh = (y[i] - mu) * rs;
    const float dh = to_f(dz[i]) * act_bwd(act, xh * gg + bb);
    s1 += dh * xh;
    s2 += dh;
  }
  part[(long)blockIdx.y * 2 * C + c] = s1;
  part[(long)blockIdx.y * 2 * C + C + c] = s2;
}

// backward pass 2: dy = gamma*rstd/N * (N*dh - sum(dh) - xhat*sum(dh*xhat))
template <typename TI>
__global__ void bn_bwd_apply_kernel(long total, int C, int rows, const TI* __restrict__ dz, const float* __restrict__ y,
                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                    const float* __restrict__ g, const float* __restrict__ b, int act,
                                    const float* __restrict__ dgamma, const float* __restrict__ dbeta,
                                    float* __restrict__ dy) {
  const float invn = 1.f / rows;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float xh = (y[i] - mean[c]) * rstd[c];
    const float dh = to_f(dz[i]) * act_bwd(act, xh * g[c] + b[c]);
    dy[i] = g[c] * rstd[c] * (dh - dbeta[c] * invn - xh * dgamma[c] * invn);
  }
}

// ---- vectorised BatchNorm passes (C % 4 == 0, 16-B aligned rows): 4 channels per lane,
// the 4 waves of a block interleave rows, 4 rows per wave in flight; one partial row per block.
__global__ __launch_bounds__(256) void bn_partial_vec_kernel(int rows, int C, const float* __restrict__ y,
                                                             int rows_per_blk, float* __restrict__ part) {
  __shared__ float red[4][2][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.y * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
  float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    const float4 sh = *(const float4*)(y + c);
    const float shv[4] = {sh.x, sh.y, sh.z, sh.w};
    int r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      float4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *(const float4*)(y + (long)(r + 4 * j) * C + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t[4] = {v[j].x - shv[0], v[j].y - shv[1], v[j].z - shv[2], v[j].w - shv[3]};
#pragma unroll
        for (int k = 0; k < 4; ++k) { s[k] += t[k]; ss[k] += t[k] * t[k]; }
      }
    }
    for (; r < r1; r += 4) {
      const float4 v = *(const float4*)(y + (long)r * C + c);
      const float t[4] = {v.x - shv[0], v.y - shv[1], v.z - shv[2], v.w - shv[3]};
#pragma unroll
      for (int k = 0; k < 4; ++k) { s[k] += t[k]; ss[k] += t[k] * t[k]; }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) { red[w][0][lane * 4 + k] = s[k]; red[w][1][lane * 4 + k] = ss[k]; }
  __syncthreads();
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc < C) {
    const int t = threadIdx.x;
    part[(long)blockIdx.y * 2 * C + cc] = (red[0][0][t] + red[1][0][t]) + (red[2][0][t] + red[3][0][t]);
    part[(long)blockIdx.y * 2 * C + C + cc] = (red[0][1][t] + red[1][1][t]) + (red[2][1][t] + red[3][1][t]);
  }
}

// parallel finalize: BNF_C channels x BNF_P part-lanes per block (C / 16 blocks: the <= 256
// partial rows are summed 16 lanes wide), fp64 combine in fixed order
constexpr int BNF_C = 16, BNF_P = 16;
__global__ __launch_bounds__(256) void bn_finalize_par_kernel(int rows, int C, int nparts, const float* __restrict__ y,
                                                              const float* __restrict__ part, float eps, float momentum,
                                                              float* __restrict__ mean, float* __restrict__ rstd,
                                                              float* __restrict__ run_mean, float* __restrict__ run_var,
                                                              long long* __restrict__ nbt,
                                                              const float* __restrict__ shift = nullptr) {
  __shared__ double red[2][BNF_P][BNF_C];
  const int cx = threadIdx.x % BNF_C, py = threadIdx.x / BNF_C;
  const int c = blockIdx.x * BNF_C + cx;
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) nbt[0] += 1;
  double s = 0.0, ss = 0.0;
  if (c < C) {
    int p = py;
    for (; p + 3 * BNF_P < nparts; p += 4 * BNF_P) {
      float a[4], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = part[(long)(p + BNF_P * j) * 2 * C + c];
        b[j] = part[(long)(p + BNF_P * j) * 2 * C + C + c];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) { s += a[j]; ss += b[j]; }
    }
    for (; p < nparts; p += BNF_P) {
      s += part[(long)p * 2 * C + c];
      ss += part[(long)p * 2 * C + C + c];
    }
  }
  red[0][py][cx] = s;
  red[1][py][cx] = ss;
  __syncthreads();
  if (py != 0 || c >= C) return;
  s = 0.0;
  ss = 0.0;
#pragma unroll
  for (int l = 0; l < BNF_P; ++l) { s += red[0][l][cx]; ss += red[1][l][cx]; }
  const double n = rows;
  const double m = s / n;
  double var = ss / n - m * m;
  if (var < 0) var = 0;
  const double mu = m + (double)(shift ? shift[c] : y[c]);  // the partials' shift: row 0 of y, or given
  mean[c] = (float)mu;
  rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * var * n / (n > 1 ? n - 1 : 1));
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void bn_apply_act_vec_kernel(int rows, int C, const float* __restrict__ y,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ g, const float* __restrict__ b,
                                                               int act, TO* __restrict__ z) {
  const int c4 = C / 4;
  const long total4 = (long)rows * c4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4) * 4;
    const float4 v = *(const float4*)(y + i * 4);
    const float4 mu = *(const float4*)(mean + c), rs = *(const float4*)(rstd + c);
    const float4 gg = *(const float4*)(g + c), bb = *(const float4*)(b + c);
    float o[4];
    o[0] = (v.x - mu.x) * rs.x * gg.x + bb.x;
    o[1] = (v.y - mu.y) * rs.y * gg.y + bb.y;
    o[2] = (v.z - mu.z) * rs.z * gg.z + bb.z;
    o[3] = (v.w - mu.w) * rs.w * gg.w + bb.w;
    act_fwd_n<4>(act, o);
    vst4(z + i * 4, o);
  }
}

template <typename TI>
__global__ __launch_bounds__(256) void bn_bwd_partial_vec_kernel(int rows, int C, const TI* __restrict__ dz,
                                                                 const float* __restrict__ y,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd,
                                                                 const float* __restrict__ g,
                                                                 const float* __restrict__ b, int act,
                                                                 int rows_per_blk, float* __restrict__ part) {
  __shared__ float red[4][2][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.y * rows_per_blk, r1 = min(rows, r0 + rows_per_blk);
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    float mu[4], rs[4], gg[4], bb[4];
    vld4(mean + c, mu); vld4(rstd + c, rs); vld4(g + c, gg); vld4(b + c, bb);
    auto accum = [&](const float (&yv)[4], const float (&dv)[4]) {
      float xh[4], h[4], dh[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xh[k] = (yv[k] - mu[k]) * rs[k];
        h[k] = xh[k] * gg[k] + bb[k];
        dh[k] = dv[k];
      }
      act_bwd_mul_n<4>(act, dh, h);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s1[k] += dh[k] * xh[k];
        s2[k] += dh[k];
      }
    };
    int r = r0 + w;
    // four rows per wave step, every load issued before any is consumed (the grid is ~2
    // blocks per CU: memory latency, not bandwidth, bounds a one- or two-row step)
    for (; r + 12 < r1; r += 16) {
      float yv[4][4], dv[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vld4(y + (long)(r + 4 * j) * C + c, yv[j]);
        vld4(dz + (long)(r + 4 * j) * C + c, dv[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) accum(yv[j], dv[j]);
    }
    for (; r < r1; r += 4) {
      float yv[4], dv[4];
      vld4(y + (long)r * C + c, yv);
      vld4(dz + (long)r * C + c, dv);
      accum(yv, dv);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) { red[w][0][lane * 4 + k] = s1[k]; red[w][1][lane * 4 + k] = s2[k]; }
  __syncthreads();
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc < C) {
    const int t = threadIdx.x;
    part[(long)blockIdx.y * 2 * C + cc] = (red[0][0][t] + red[1][0][t]) + (red[2][0][t] + red[3][0][t]);
    part[(long)blockIdx.y * 2 * C + C + cc] = (red[0][1][t] + red[1][1][t]) + (red[2][1][t] + red[3][1][t]);
  }
}

template <typename TI>
__global__ __launch_bounds__(256) void bn_bwd_apply_vec_kernel(int rows, int C, const TI* __restrict__ dz,
                                                               const float* __restrict__ y,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ g,
                                                               const float* __restrict__ b, int act,
                                                               const float* __restrict__ dgamma,
                                                               const float* __restrict__ dbeta,
                                                               float* __restrict__ dy,
                                                               float* __restrict__ pgrad, int acc_params) {
  const float invn = 1.f / rows;
  const int c4 = C / 4;
  // the parameter gradients (gamma | beta, adjacent) (+)= the batch sums (dgamma | dbeta
  // adjacent in `sums`), from block 0 instead of a separate reduce launch
  if (pgrad != nullptr && blockIdx.x == 0)
    for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) pgrad[c] = acc_params ? pgrad[c] + dgamma[c] : dgamma[c];
  const long total4 = (long)rows * c4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4) * 4;
    float yv[4], dv[4], mu[4], rs[4], gg[4], bb[4], dg[4], db[4], o[4];
    vld4(y + i * 4, yv); vld4(dz + i * 4, dv);
    vld4(mean + c, mu); vld4(rstd + c, rs); vld4(g + c, gg); vld4(b + c, bb);
    vld4(dgamma + c, dg); vld4(dbeta + c, db);
    float xh[4], h[4], dh[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xh[k] = (yv[k] - mu[k]) * rs[k];
      h[k] = xh[k] * gg[k] + bb[k];
      dh[k] = dv[k];
    }
    act_bwd_mul_n<4>(act, dh, h);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = gg[k] * rs[k] * (dh[k] - db[k] * invn - xh[k] * dg[k] * invn);
    vst4(dy + i * 4, o);
  }
}

int ln_blocks(int rows) { return ea_grid_cap(ea_cdiv(rows, 4), 2048); }

}  // namespace

#define EA_LN_DISPATCH(KER, TYPE, ...)                                                        \
  do {                                                                                        \
    if (d <= 64) hipLaunchKernelGGL((KER<1, TYPE>), __VA_ARGS__);                             \
    else if (d <= 256) hipLaunchKernelGGL((KER<4, TYPE>), __VA_ARGS__);                       \
    else if (d <= 512) hipLaunchKernelGGL((KER<8, TYPE>), __VA_ARGS__);                       \
    else if (d <= 1024) hipLaunchKernelGGL((KER<16, TYPE>), __VA_ARGS__);                     \
    else return EA_ERR_BAD_ARG;                                                               \
  } while (0)

extern "C" int ea_layernorm_fwd(int rows, int d, const float* x, long ldx, const float* gamma,
                                const float* beta, float eps, void* y, int y_dtype, long ldy,
                                float* mean, float* rstd, void* stream) {
  EA_ENTRY();
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = d % 8 == 0 && d <= 1024 && ldx % 4 == 0 && ldy % 8 == 0 && ((uintptr_t)x % 16) == 0 &&
                   ((uintptr_t)y % 16) == 0 && ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0;
  if (vec) {
    dim3 g1(ea_cdiv(rows, 4)), b1(256);
#define EA_LNF(NJ)                                                                                       \
  if (y_dtype == EA_BF16)                                                                                \
    hipLaunchKernelGGL((ln_fwd_vec_kernel<NJ, bf16>), g1, b1, 0, st, rows, d, x, ldx, gamma, beta, eps, (bf16*)y, ldy, mean, rstd); \
  else                                                                                                   \
    hipLaunchKernelGGL((ln_fwd_vec_kernel<NJ, float>), g1, b1, 0, st, rows, d, x, ldx, gamma, beta, eps, (float*)y, ldy, mean, rstd);
    if (d <= 512) { EA_LNF(1) } else { EA_LNF(2) }
#undef EA_LNF
    EA_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid(ln_blocks(rows)), blk(256);
  if (y_dtype == EA_BF16)
    EA_LN_DISPATCH(ln_fwd_kernel, bf16, grid, blk, 0, st, rows, d, x, ldx, gamma, beta, eps, (bf16*)y, ldy, mean, rstd);
  else
    EA_LN_DISPATCH(ln_fwd_kernel, float, grid, blk, 0, st, rows, d, x, ldx, gamma, beta, eps, (float*)y, ldy, mean, rstd);
  EA_LAUNCH_CHECK();
  return 0;
}

// LayerNorm backward: dx (+)= ..., and per-row-block partial sums of (dgamma | dbeta) in
// workspace [nparts][2d]; with dgamma != nullptr the ordered reducer then sums them into
// dgamma/dbeta, otherwise *nparts_out reports the partial count (deferred reduction).
static int ln_bwd_impl(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x, long ldx,
                       const float* gamma, const float* mean, const float* rstd, float* dx, long lddx, int accumulate,
                       float* dgamma, int accumulate_params, float* workspace, long ws_elems, int* nparts_out,
                       hipStream_t st, const LnDrop* drop = nullptr) {
  if (nparts_out) *nparts_out = 0;
  if (rows == 0) return 0;
  // the dropout output in-kernel: vectorized path, bf16 dy and y, 16-B aligned y rows
  const bool kdrop = drop && drop->ldy % 8 == 0 && ((uintptr_t)drop->y % 16) == 0;
  const bool vec = d % 4 == 0 && lddy % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x % 16) == 0 &&
                   ((uintptr_t)dy % (dy_dtype == EA_BF16 ? 8 : 16)) == 0;
  if (!vec) {  // generic fused path (row kernel + per-block partials)
    const int nb = min(ln_blocks(rows), 128);
    EA_CHECK_ARG(ws_elems >= (long)nb * 2 * d);
    dim3 grid(nb), blk(256);
    if (dy_dtype == EA_BF16)
      EA_LN_DISPATCH(ln_bwd_kernel, bf16, grid, blk, 0, st, rows, d, (const bf16*)dy, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, workspace);
    else
      EA_LN_DISPATCH(ln_bwd_kernel, float, grid, blk, 0, st, rows, d, (const float*)dy, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, workspace);
    EA_LAUNCH_CHECK();
    if (!dgamma) { *nparts_out = nb; return 0; }
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(2 * d, RP_CW)), dim3(256), 0, st, nb, 2 * d,
                       workspace, (long)2 * d, dgamma, accumulate_params);
    EA_LAUNCH_CHECK();
    return 0;
  }
  const bool vec8 = d % 8 == 0 && d <= 1024 && lddy % 8 == 0 && ldx % 4 == 0 && lddx % 4 == 0 &&
                    ((uintptr_t)x % 16) == 0 && ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dx % 16) == 0 &&
                    ((uintptr_t)gamma % 16) == 0;
  if (vec8) {  // one pass: dx + per-block dgamma/dbeta partials, then the ordered reducer
    // with the dropout output's column sums: [nb][d] y partials after the [nb][2d] LN partials
    const bool ycs = kdrop && drop->want_ycol;
    const long per = ycs ? 3L * d : 2L * d;
    const int rpb = max(16, ea_cdiv(rows, (int)max(1L, ws_elems / per)));
    const int nb = ea_cdiv(rows, rpb);
    EA_CHECK_ARG(ws_elems >= (long)nb * per);
    LnDrop dd = kdrop ? *drop : LnDrop{};
    dd.ypart = ycs ? workspace + (long)nb * 2 * d : nullptr;
#define EA_LNB(NJ, U)                                                                                     \
  if (kdrop && dy_dtype == EA_BF16)                                                                       \
    hipLaunchKernelGGL((ln_bwd_vec_kernel<NJ, bf16, true, U>), dim3(nb), dim3(256), 0, st, rows, d, (const bf16*)dy, lddy, \
                       x, ldx, gamma, mean, rstd, dx, lddx, accumulate, rpb, workspace, dd);               \
  else if (kdrop)                                                                                         \
    hipLaunchKernelGGL((ln_bwd_vec_kernel<NJ, float, true, U>), dim3(nb), dim3(256), 0, st, rows, d, (const float*)dy, lddy, \
                       x, ldx, gamma, mean, rstd, dx, lddx, accumulate, rpb, workspace, dd);               \
  else if (dy_dtype == EA_BF16)                                                                           \
    hipLaunchKernelGGL((ln_bwd_vec_kernel<NJ, bf16, false, U>), dim3(nb), dim3(256), 0, st, rows, d, (const bf16*)dy, lddy, x, ldx, \
                       gamma, mean, rstd, dx, lddx, accumulate, rpb, workspace);                           \
  else                                                                                                    \
    hipLaunchKernelGGL((ln_bwd_vec_kernel<NJ, float, false, U>), dim3(nb), dim3(256), 0, st, rows, d, (const float*)dy, lddy, x, \
                       ldx, gamma, mean, rstd, dx, lddx, accumulate, rpb, workspace);
    // two rows in flight per wave step for d <= 512 (four measured neutral, round 4)
    if (d > 512) { EA_LNB(2, 1) } else { EA_LNB(1, 2) }
#undef EA_LNB
    EA_LAUNCH_CHECK();
    if (!dgamma) { *nparts_out = nb; return 0; }
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(2 * d, RP_CW)), dim3(256), 0, st, nb, 2 * d,
                       workspace, (long)2 * d, dgamma, accumulate_params);
    EA_LAUNCH_CHECK();
    if (ycs) {
      hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(d, RP_CW)), dim3(256), 0, st, nb, d, dd.ypart, (long)d,
                         drop->ycol, 1);
      EA_LAUNCH_CHECK();
    }
    return 0;
  }
  dim3 g1(ea_cdiv(rows, 4)), blk(256);
  if (dy_dtype == EA_BF16)
    EA_LN_DISPATCH(ln_bwd_dx_kernel, bf16, g1, blk, 0, st, rows, d, (const bf16*)dy, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate);
  else
    EA_LN_DISPATCH(ln_bwd_dx_kernel, float, g1, blk, 0, st, rows, d, (const float*)dy, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate);
  EA_LAUNCH_CHECK();
  const int rpp = max(32, ea_cdiv(rows, 128));
  const int nparts = ea_cdiv(rows, rpp);
  EA_CHECK_ARG(ws_elems >= (long)nparts * 2 * d);
  dim3 g2(ea_cdiv(d, 256), nparts);
  if (dy_dtype == EA_BF16)
    hipLaunchKernelGGL((colsum_vec_kernel<bf16, true>), g2, blk, 0, st, rows, d, (const bf16*)dy, lddy, x, ldx, mean, rstd, rpp, workspace);
  else
    hipLaunchKernelGGL((colsum_vec_kernel<float, true>), g2, blk, 0, st, rows, d, (const float*)dy, lddy, x, ldx, mean, rstd, rpp, workspace);
  EA_LAUNCH_CHECK();
  if (!dgamma) { *nparts_out = nparts; return 0; }
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(2 * d, RP_CW)), dim3(256), 0, st, nparts, 2 * d,
                     workspace, (long)2 * d, dgamma, accumulate_params);
  EA_LAUNCH_CHECK();
  return 0;
}

// ln_bwd_impl + the dropout output: in the LN kernel when it can (kdrop above, vectorized
// rows), otherwise as an ea_scale_dropout pass over the finished dx.  ycol (optional): its
// column sums added into ycol, from the LN kernel's own partials when in-kernel (direct mode:
// reduced here; partials mode: left after the LN partials, *ycol_parts = 1, for the caller),
// else by ea_colsum (*ycol_parts = 0).
static int ln_bwd_drop_impl(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x, long ldx,
                            const float* gamma, const float* mean, const float* rstd, float* dx, long lddx,
                            int accumulate, float* dgamma, int accumulate_params, float* workspace, long ws_elems,
                            int* nparts_out, void* y, int y_dtype, long ldy, float yscale, float p,
                            unsigned long long seed, float* ycol, int* ycol_parts, hipStream_t st) {
  if (ycol_parts) *ycol_parts = 0;
  const LnDrop dr{(bf16*)y, ldy, yscale, p, (uint64_t)seed, ea_g_rng_salt, nullptr, ycol != nullptr, ycol};
  const bool vec8 = d % 8 == 0 && d <= 1024 && lddy % 8 == 0 && ldx % 4 == 0 && lddx % 4 == 0 &&
                    ((uintptr_t)x % 16) == 0 && ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dx % 16) == 0 &&
                    ((uintptr_t)gamma % 16) == 0;
  const bool in_kernel = vec8 && y_dtype == EA_BF16 && ldy % 8 == 0 && ((uintptr_t)y % 16) == 0;
  int rc = ln_bwd_impl(rows, d, dy, dy_dtype, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, dgamma,
                       accumulate_params, workspace, ws_elems, nparts_out, st, in_kernel ? &dr : nullptr);
  if (rc || rows == 0) return rc;
  if (in_kernel) {
    if (ycol && ycol_parts) *ycol_parts = 1;
    return 0;
  }
  rc = ea_scale_dropout(rows, d, dx, EA_F32, lddx, y, y_dtype, ldy, yscale, p, seed, st);
  if (rc || !ycol) return rc;
  // column sums through ea_colsum on the workspace left after the LN partials
  const long used = nparts_out ? (long)*nparts_out * 2 * d : 0;
  return ea_colsum(rows, d, y, y_dtype, ldy, ycol, 1, workspace + used, ws_elems - used, st);
}

extern "C" int ea_layernorm_bwd_drop(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x,
                                     long ldx, const float* gamma, const float* mean, const float* rstd, float* dx,
                                     long lddx, int accumulate, float* dgamma, float* dbeta, int accumulate_params,
                                     float* workspace, long ws_elems, void* y, int y_dtype, long ldy, float yscale,
                                     float p, unsigned long long seed, float* ycol, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(dgamma != nullptr && dbeta == dgamma + d && y != nullptr && (y_dtype == EA_BF16 || y_dtype == EA_F32));
  return ln_bwd_drop_impl(rows, d, dy, dy_dtype, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, dgamma,
                          accumulate_params, workspace, ws_elems, nullptr, y, y_dtype, ldy, yscale, p, seed, ycol,
                          nullptr, (hipStream_t)stream);
}

extern "C" int ea_layernorm_bwd_partials_drop(int rows, int d, const void* dy, int dy_dtype, long lddy,
                                              const float* x, long ldx, const float* gamma, const float* mean,
                                              const float* rstd, float* dx, long lddx, int accumulate, float* part,
                                              long part_elems, int* nparts, void* y, int y_dtype, long ldy,
                                              float yscale, float p, unsigned long long seed, float* ycol,
                                              int* ycol_parts, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(part != nullptr && nparts != nullptr && y != nullptr && (y_dtype == EA_BF16 || y_dtype == EA_F32));
  EA_CHECK_ARG(ycol == nullptr || ycol_parts != nullptr);
  return ln_bwd_drop_impl(rows, d, dy, dy_dtype, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, nullptr, 0,
                          part, part_elems, nparts, y, y_dtype, ldy, yscale, p, seed, ycol, ycol_parts,
                          (hipStream_t)stream);
}

extern "C" int ea_layernorm_bwd(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x,
                                long ldx, const float* gamma, const float* mean, const float* rstd,
                                float* dx, long lddx, int accumulate, float* dgamma, float* dbeta,
                                int accumulate_params, float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(dgamma != nullptr && dbeta == dgamma + d);  // grads of (weight, bias) are adjacent in the arena
  return ln_bwd_impl(rows, d, dy, dy_dtype, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, dgamma,
                     accumulate_params, workspace, ws_elems, nullptr, (hipStream_t)stream);
}

extern "C" int ea_layernorm_bwd_partials(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x,
                                         long ldx, const float* gamma, const float* mean, const float* rstd,
                                         float* dx, long lddx, int accumulate, float* part, long part_elems,
                                         int* nparts, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(part != nullptr && nparts != nullptr);
  return ln_bwd_impl(rows, d, dy, dy_dtype, lddy, x, ldx, gamma, mean, rstd, dx, lddx, accumulate, nullptr, 0,
                     part, part_elems, nparts, (hipStream_t)stream);
}

extern "C" int ea_reduce_partials(int nparts, int n, const float* part, long stride, float* out,
                                  int accumulate, void* stream) {
  EA_ENTRY();
  if (n == 0) return 0;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(n, RP_CW)), dim3(256), 0, (hipStream_t)stream,
                     nparts, n, part, stride, out, accumulate);
  EA_LAUNCH_CHECK();
  return 0;
}

// internal (not exported): transposed-output variant used by the depthwise-conv backward
int ea_reduce_partials_tr(int nparts, int n, const float* part, long stride, float* out, int accumulate,
                          int tr_rows, int tr_cols, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(n, RP_CW)), dim3(256), 0, (hipStream_t)stream,
                     nparts, n, part, stride, out, accumulate, tr_rows, tr_cols);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_colsum(int rows, int n, const void* x, int x_dtype, long ld, float* out, int accumulate,
                         float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = n % 4 == 0 && ld % 4 == 0 && ((uintptr_t)x % (x_dtype == EA_BF16 ? 8 : 16)) == 0 && rows > 0;
  if (vec) {
    const int rpp = max(32, ea_cdiv(rows, 128));
    const int np = ea_cdiv(rows, rpp);
    EA_CHECK_ARG((long)np * n <= ws_elems);
    dim3 g(ea_cdiv(n, 256), np);
    if (x_dtype == EA_BF16)
      hipLaunchKernelGGL((colsum_vec_kernel<bf16, false>), g, dim3(256), 0, st, rows, n, (const bf16*)x, ld, nullptr, 0L, nullptr, nullptr, rpp, workspace);
    else
      hipLaunchKernelGGL((colsum_vec_kernel<float, false>), g, dim3(256), 0, st, rows, n, (const float*)x, ld, nullptr, 0L, nullptr, nullptr, rpp, workspace);
    EA_LAUNCH_CHECK();
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(n, RP_CW)), dim3(256), 0, st, np, n, workspace, (long)n, out,
                       accumulate);
    EA_LAUNCH_CHECK();
    return 0;
  }
  int rpb = max(16, ea_cdiv(rows, 64));
  int nparts = ea_cdiv(rows, rpb);
  while ((long)nparts * n > ws_elems && rpb < (1 << 20)) {
    rpb *= 2;
    nparts = ea_cdiv(rows, rpb);
  }
  EA_CHECK_ARG((long)nparts * n <= ws_elems);
  if (rows == 0) nparts = 0;
  dim3 grid(ea_cdiv(n, 256), max(nparts, 1));
  if (nparts > 0) {
    if (x_dtype == EA_BF16)
      hipLaunchKernelGGL(colsum_partial_kernel<bf16>, grid, dim3(256), 0, st, rows, n, (const bf16*)x, ld, rpb, workspace);
    else
      hipLaunchKernelGGL(colsum_partial_kernel<float>, grid, dim3(256), 0, st, rows, n, (const float*)x, ld, rpb, workspace);
    EA_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(n, RP_CW)), dim3(256), 0, st, nparts, n, workspace,
                     (long)n, out, accumulate);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_scale_dropout_colsum(long rows, int cols, const float* x, long ldx, void* y, int y_dtype, long ldy,
                                       float scale, float p, unsigned long long seed, float* colsum, int accumulate,
                                       float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  if (rows == 0 || cols == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int ya = y_dtype == EA_BF16 ? 8 : 16;
  const bool vec = cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % ya == 0 &&
                   rows * (long)cols < (1L << 31);
  if (!vec) {
    int rc = ea_scale_dropout(rows, cols, x, EA_F32, ldx, y, y_dtype, ldy, scale, p, seed, stream);
    if (rc) return rc;
    return ea_colsum((int)rows, cols, y, y_dtype, ldy, colsum, accumulate, workspace, ws_elems, stream);
  }
  const int rpp = max(32, ea_cdiv(rows, 128));
  const int np = ea_cdiv(rows, rpp);
  EA_CHECK_ARG((long)np * cols <= ws_elems);
  dim3 g(ea_cdiv(cols, 256), np);
  if (y_dtype == EA_BF16)
    hipLaunchKernelGGL(scale_drop_colsum_kernel<bf16>, g, dim3(256), 0, st, (int)rows, cols, x, ldx, (bf16*)y, ldy, scale,
                       p, (uint64_t)seed, ea_g_rng_salt, rpp, workspace);
  else
    hipLaunchKernelGGL(scale_drop_colsum_kernel<float>, g, dim3(256), 0, st, (int)rows, cols, x, ldx, (float*)y, ldy,
                       scale, p, (uint64_t)seed, ea_g_rng_salt, rpp, workspace);
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(cols, RP_CW)), dim3(256), 0, st, np, cols, workspace, (long)cols,
                     colsum, accumulate);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_batchnorm_fwd_parts(int rows, int C, const float* y, const float* part, int nparts,
                                      const float* shift, const float* gamma, const float* beta, float eps,
                                      float momentum, float* mean, float* rstd, float* running_mean,
                                      float* running_var, long long* num_batches_tracked, int act, void* z,
                                      int z_dtype, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(rows > 0 && nparts > 0 && part && shift && C % 4 == 0 && ((uintptr_t)y % 16) == 0 &&
               ((uintptr_t)z % (z_dtype == EA_BF16 ? 8 : 16)) == 0);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_finalize_par_kernel, dim3(ea_cdiv(C, BNF_C)), dim3(256), 0, st, rows, C, nparts, y, part, eps,
                     momentum, mean, rstd, running_mean, running_var, num_batches_tracked, shift);
  EA_LAUNCH_CHECK();
  const long total = (long)rows * C;
  dim3 g4(ea_grid_cap(ea_cdiv(total / 4, 256)));
  if (z_dtype == EA_BF16)
    hipLaunchKernelGGL(bn_apply_act_vec_kernel<bf16>, g4, dim3(256), 0, st, rows, C, y, mean, rstd, gamma, beta, act, (bf16*)z);
  else
    hipLaunchKernelGGL(bn_apply_act_vec_kernel<float>, g4, dim3(256), 0, st, rows, C, y, mean, rstd, gamma, beta, act, (float*)z);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_batchnorm_fwd(int rows, int C, const float* y, const float* gamma, const float* beta,
                                float eps, float momentum, int training, float* mean, float* rstd,
                                float* running_mean, float* running_var, long long* num_batches_tracked,
                                int act, void* z, int z_dtype, float* workspace, long ws_elems,
                                void* stream) {
  EA_ENTRY();
  hipStream_t st = (hipStream_t)stream;
  const long total = (long)rows * C;
  const bool vec = C % 4 == 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)z % (z_dtype == EA_BF16 ? 8 : 16)) == 0;
  if (training) {
    // <= 256 row blocks of >= 16 rows (as the backward: 64 blocks of 125 rows left half the
    // CUs idle)
    const int rpb = max(16, ea_cdiv(rows, 256));
    const int nparts = ea_cdiv(rows, rpb);
    EA_CHECK_ARG((long)nparts * 2 * C <= ws_elems && rows > 0);
    if (vec)
      hipLaunchKernelGGL(bn_partial_vec_kernel, dim3(ea_cdiv(C, 256), nparts), dim3(256), 0, st, rows, C, y, rpb, workspace);
    else
      hipLaunchKernelGGL(bn_partial_kernel, dim3(ea_cdiv(C, 256), nparts), dim3(256), 0, st, rows, C, y, rpb, workspace);
    EA_LAUNCH_CHECK();
    hipLaunchKernelGGL(bn_finalize_par_kernel, dim3(ea_cdiv(C, BNF_C)), dim3(256), 0, st, rows, C, nparts, y, workspace,
                       eps, momentum, mean, rstd, running_mean, running_var, num_batches_tracked);
    EA_LAUNCH_CHECK();
  } else {
    EA_CHECK_ARG(running_mean && running_var);
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(ea_cdiv(C, 256)), dim3(256), 0, st, C, running_mean, running_var,
                       eps, mean, rstd);
    EA_LAUNCH_CHECK();
  }
  dim3 grid(ea_grid_cap(ea_cdiv(total, 256)));
  if (vec) {
    dim3 g4(ea_grid_cap(ea_cdiv(total / 4, 256)));
    if (z_dtype == EA_BF16)
      hipLaunchKernelGGL(bn_apply_act_vec_kernel<bf16>, g4, dim3(256), 0, st, rows, C, y, mean, rstd, gamma, beta, act, (bf16*)z);
    else
      hipLaunchKernelGGL(bn_apply_act_vec_kernel<float>, g4, dim3(256), 0, st, rows, C, y, mean, rstd, gamma, beta, act, (float*)z);
  } else if (z_dtype == EA_BF16)
    hipLaunchKernelGGL(bn_apply_act_kernel<bf16>, grid, dim3(256), 0, st, total, C, y, mean, rstd, gamma, beta, act, (bf16*)z);
  else
    hipLaunchKernelGGL(bn_apply_act_kernel<float>, grid, dim3(256), 0, st, total, C, y, mean, rstd, gamma, beta, act, (float*)z);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_batchnorm_bwd(int rows, int C, const void* dz, int dz_dtype, const float* y, const float* mean,
                                const float* rstd, const float* gamma, const float* beta, int act, float* dy,
                                float* dgamma, float* dbeta, int accumulate_params, float* workspace,
                                long ws_elems, void* stream) {
  EA_ENTRY();
  hipStream_t st = (hipStream_t)stream;
  const long total = (long)rows * C;
  // <= 256 row blocks of >= 16 rows: ~2 blocks per CU at C = 512 (64 row blocks of 125 rows
  // left half the CUs idle: 16.8 us for 24 MB)
  const int rpb = max(16, ea_cdiv(rows, 256));
  const int nparts = ea_cdiv(rows, rpb);
  EA_CHECK_ARG((long)nparts * 2 * C + 2 * C <= ws_elems && rows > 0);
  EA_CHECK_ARG(dbeta == dgamma + C);
  float* sums = workspace + (long)nparts * 2 * C;  // [sum dh*xhat | sum dh] for this batch
  dim3 g1(ea_cdiv(C, 256), nparts);
  const bool vec = C % 4 == 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)dy % 16) == 0 &&
                   ((uintptr_t)dz % (dz_dtype == EA_BF16 ? 8 : 16)) == 0;
  if (vec && dz_dtype == EA_BF16)
    hipLaunchKernelGGL(bn_bwd_partial_vec_kernel<bf16>, g1, dim3(256), 0, st, rows, C, (const bf16*)dz, y, mean, rstd, gamma, beta, act, rpb, workspace);
  else if (vec)
    hipLaunchKernelGGL(bn_bwd_partial_vec_kernel<float>, g1, dim3(256), 0, st, rows, C, (const float*)dz, y, mean, rstd, gamma, beta, act, rpb, workspace);
  else if (dz_dtype == EA_BF16)
    hipLaunchKernelGGL(bn_bwd_partial_kernel<bf16>, g1, dim3(256), 0, st, rows, C, (const bf16*)dz, y, mean, rstd, gamma, beta, act, rpb, workspace);
  else
    hipLaunchKernelGGL(bn_bwd_partial_kernel<float>, g1, dim3(256), 0, st, rows, C, (const float*)dz, y, mean, rstd, gamma, beta, act, rpb, workspace);
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(2 * C, RP_CW)), dim3(256), 0, st, nparts, 2 * C, workspace,
                     (long)2 * C, sums, 0);
  EA_LAUNCH_CHECK();
  dim3 g2(ea_grid_cap(ea_cdiv(total, 256)));
  if (vec) {
    dim3 g4(ea_grid_cap(ea_cdiv(total / 4, 256)));
    if (dz_dtype == EA_BF16)
      hipLaunchKernelGGL(bn_bwd_apply_vec_kernel<bf16>, g4, dim3(256), 0, st, rows, C, (const bf16*)dz, y, mean, rstd, gamma, beta, act, sums, sums + C, dy, dgamma, accumulate_params);
    else
      hipLaunchKernelGGL(bn_bwd_apply_vec_kernel<float>, g4, dim3(256), 0, st, rows, C, (const float*)dz, y, mean, rstd, gamma, beta, act, sums, sums + C, dy, dgamma, accumulate_params);
    EA_LAUNCH_CHECK();
    return 0;
  } else if (dz_dtype == EA_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16>, g2, dim3(256), 0, st, total, C, rows, (const bf16*)dz, y, mean, rstd, gamma, beta, act, sums, sums + C, dy);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, g2, dim3(256), 0, st, total, C, rows, (const float*)dz, y, mean, rstd, gamma, beta, act, sums, sums + C, dy);
  EA_LAUNCH_CHECK();
  // parameter grads: dgamma = sum dh*xhat, dbeta = sum dh
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(ea_cdiv(2 * C, RP_CW)), dim3(256), 0, st, 1, 2 * C, sums,
                     (long)2 * C, dgamma, accumulate_params);
  EA_LAUNCH_CHECK();
  return 0;
}
