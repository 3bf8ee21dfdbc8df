// Memory-bound kernels of the ASR step: input prep (utterance MVN, subsampled lengths,
// sos/eos), dropout/cast, weight repacking, GLU, q+pos_bias, embeddings, argmax.
// All grid-stride, coalesced along the contiguous (channel) dimension.
// hipcc-flags: -fno-slp-vectorize
#include "common.h"

#include <cstdlib>
#include <cstring>

namespace {

// ---------------------------------------------------------------- input prep
// utterance_mvn(norm_means=True, norm_vars=False), layers/utterance_mvn.py:45-88:
// zero padded frames, subtract the mean over valid frames.  One block per (b, feature tile).
__global__ void mvn_kernel(int B, int T, int F, const float* __restrict__ x, const long long* __restrict__ lens,
                           float* __restrict__ y) {
  const int b = blockIdx.x;
  const int f = threadIdx.x;  // blockDim.x >= F
  __shared__ double red[1024];
  const long long L = lens[b];
  double s = 0.0;
  // each thread owns feature f; rows split across blockDim.y
  const int ty = threadIdx.y, ny = blockDim.y;
  if (f < F)
    for (int t = ty; t < T; t += ny)
      if (t < L) s += x[((long)b * T + t) * F + f];
  red[ty * blockDim.x + f] = s;
  __syncthreads();
  if (ty == 0 && f < F) {
    double a = 0.0;
    for (int k = 0; k < ny; ++k) a += red[k * blockDim.x + f];
    red[f] = a;
  }
  __syncthreads();
  if (f >= F) return;
  // the reference computes the mean in the input dtype: sum (f32) / len
  const float mean = (float)red[f] / (float)L;
  for (int t = ty; t < T; t += ny) {
    const long i = ((long)b * T + t) * F + f;
    y[i] = (t < L ? x[i] : 0.f) - mean;
  }
}

// Same op over a (row chunk, utterance) grid: the one-block-per-utterance kernel above
// leaves most CUs idle and walks T/ny rows serially per thread.  Pass 1 writes each chunk's
// f64 column sums over its valid rows to ws[b][chunk][F]; pass 2 sums an utterance's chunk
// partials in chunk order, then writes its own chunk of y.
constexpr int MVN_TC = 32;  // rows per chunk

__global__ __launch_bounds__(512) void mvn_part_kernel(int T, int F, const float* __restrict__ x,
                                                       const long long* __restrict__ lens, double* __restrict__ ws) {
  const int c = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  const int f = threadIdx.x, ty = threadIdx.y, ny = blockDim.y;
  __shared__ double red[512];
  const long long L = lens[b];
  const int t1 = (int)min((long long)min(T, (c + 1) * MVN_TC), L);
  double s = 0.0;
  if (f < F)
    for (int t = c * MVN_TC + ty; t < t1; t += ny) s += x[((long)b * T + t) * F + f];
  red[ty * blockDim.x + f] = s;
  __syncthreads();
  if (ty == 0 && f < F) {
    double a = 0.0;
    for (int k = 0; k < ny; ++k) a += red[k * blockDim.x + f];
    ws[((long)b * nch + c) * F + f] = a;
  }
}

__global__ __launch_bounds__(512) void mvn_apply_kernel(int T, int F, const float* __restrict__ x,
                                                        const long long* __restrict__ lens,
                                                        const double* __restrict__ ws, float* __restrict__ y) {
  const int c = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  const int f = threadIdx.x, ty = threadIdx.y, ny = blockDim.y;
  __shared__ float mean_s[256];
  const long long L = lens[b];
  if (ty == 0 && f < F) {
    double a = 0.0;
    for (int k = 0; k < nch; ++k) a += ws[((long)b * nch + k) * F + f];
    mean_s[f] = (float)a / (float)L;  // f32 mean like the reference (sum / len)
  }
  __syncthreads();
  if (f >= F) return;
  const float mean = mean_s[f];
  const int t1 = min(T, (c + 1) * MVN_TC);
  for (int t = c * MVN_TC + ty; t < t1; t += ny) {
    const long i = ((long)b * T + t) * F + f;
    y[i] = (t < L ? x[i] : 0.f) - mean;
  }
}

// lengths after Conv2dSubsampling as the reference derives them from the sliced mask
// x_mask[:, :, :-2:2][:, :, :-2:2] (subsampling.py:91): l -> ceil(min(l, T-2)/2) twice.
__global__ void subsample_lens_kernel(int B, int T, const long long* __restrict__ ilens, long long* __restrict__ olens) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  long long l = ilens[b];
  const long long T1 = (T - 1) / 2;  // len(range(0, T-2, 2))
  long long l1 = min(l, (long long)T - 2);
  l1 = l1 > 0 ? (l1 + 1) / 2 : 0;
  long long l2 = min(l1, T1 - 2);
  l2 = l2 > 0 ? (l2 + 1) / 2 : 0;
  olens[b] = l2;
}

// add_sos_eos + pad_list (transformer/add_sos_eos.py:12-31)
__global__ void sos_eos_kernel(int B, int L, const long long* __restrict__ ys, long ldys, const long long* __restrict__ ylens,
                               int sos, int eos, int ignore_id, long long* __restrict__ ys_in,
                               long long* __restrict__ ys_out, long long* __restrict__ ys_in_lens) {
  const int b = blockIdx.x;
  const long long l = ylens[b];
  for (int t = threadIdx.x; t <= L; t += blockDim.x) {
    long long vin, vout;
    if (t == 0) vin = sos;
    else if (t <= l) vin = ys[(long)b * ldys + t - 1];
    else vin = eos;
    if (t < l) vout = ys[(long)b * ldys + t];
    else if (t == l) vout = eos;
    else vout = ignore_id;
    ys_in[(long)b * (L + 1) + t] = vin;
    ys_out[(long)b * (L + 1) + t] = vout;
  }
  if (threadIdx.x == 0) ys_in_lens[b] = l + 1;
}

// ---------------------------------------------------------------- conv1 direct (phase-split out)
// Conv2dSubsampling's first Conv2d(1, C, 3, stride 2) + ReLU (subsampling.py:60-61) as a
// direct kernel: 9 MACs per output, so a GEMM (K = 9) would only move bytes.  Output in the
// phase-split layout of ea_conv_geo: pixel (t1, f1) -> plane (t1&1, f1&1), row (b, t1>>1, f1>>1).
// One thread = 8 channels of one pixel (16-B bf16 stores); weights stay in registers.
struct PhaseGeo {
  int T1, F1, nI0, nI1, nJ0, nJ1;
  long plane[4];
};
EA_DEV long phase_row(const PhaseGeo& g, int b, int t1, int f1) {
  const int a = t1 & 1, e = f1 & 1;
  const int nI = a ? g.nI1 : g.nI0, nJ = e ? g.nJ1 : g.nJ0;
  return g.plane[a * 2 + e] + ((long)(b * nI + (t1 >> 1)) * nJ + (f1 >> 1));
}
template <typename TO>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(int B, int T, int F, PhaseGeo g, int C,
                                                        const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, TO* __restrict__ y,
                                                        uint8_t* __restrict__ pos) {
  const int groups = C / 8;
  const int cg = threadIdx.x % groups;  // blockDim.x is a multiple of C/8
  const int c0 = cg * 8;
  float wr[8][9], br[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    br[k] = bias[c0 + k];
#pragma unroll
    for (int t = 0; t < 9; ++t) wr[k][t] = w[(c0 + k) * 9 + t];
  }
  const long npix = (long)B * g.T1 * g.F1;
  const int ppb = blockDim.x / groups;
  for (long pix = (long)blockIdx.x * ppb + threadIdx.x / groups; pix < npix; pix += (long)gridDim.x * ppb) {
    const int f1 = (int)(pix % g.F1);
    const long bt = pix / g.F1;
    const int t1 = (int)(bt % g.T1), b = (int)(bt / g.T1);
    const float* xp = x + ((long)b * T + 2 * t1) * F + 2 * f1;
    float xv[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) xv[kh * 3 + kw] = xp[kh * F + kw];
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float a = br[k];
#pragma unroll
      for (int t = 0; t < 9; ++t) a = fmaf(wr[k][t], xv[t], a);
      o[k] = a > 0.f ? a : 0.f;
    }
    const long prow = phase_row(g, b, t1, f1);
    TO* yp = y + prow * C + c0;
    float lo[4] = {o[0], o[1], o[2], o[3]}, hi[4] = {o[4], o[5], o[6], o[7]};
    vst4(yp, lo);
    vst4(yp + 4, hi);
    if (pos) {  // ReLU support bits of the stored (rounded) outputs: bit k = channel c0 + k > 0
      uint32_t m = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) m |= (uint32_t)((float)(TO)o[k] > 0.f) << k;
      pos[prow * (C / 8) + cg] = (uint8_t)m;
    }
  }
}

// Same conv as conv1_fwd_kernel for C a multiple of 512 (one wave = one pixel's 512
// channels, 8 per lane): blocks stride over output rows (b, t1), so the index arithmetic is
// per row and wave-uniform (scalar), the 9 taps of a pixel are wave-uniform loads, and the
// per-pixel vector work is the 72 FMAs, ReLU, bf16 packing and the support byte.
template <typename TO, bool NT>
__global__ __launch_bounds__(256) void conv1_fwd_rows_kernel(int B, int T, int F, PhaseGeo g, int C,
                                                             const float* __restrict__ x, const float* __restrict__ w,
                                                             const float* __restrict__ bias, TO* __restrict__ y,
                                                             uint8_t* __restrict__ pos) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwc = C >> 9;                 // waves per pixel
  const int wc = wv % nwc, pw = wv / nwc;  // channel slice, pixel slot of this wave
  const int ppb = 4 / nwc;                // pixels per block per step (C <= 2048)
  const int cg = wc * 64 + lane, c0 = cg * 8;
  float wr[8][9], br[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    br[k] = bias[c0 + k];
#pragma unroll
    for (int t = 0; t < 9; ++t) wr[k][t] = w[(c0 + k) * 9 + t];
  }
  const int rows = B * g.T1;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int b = row / g.T1, t1 = row - b * g.T1;
    const int a = t1 & 1;
    const int nI = a ? g.nI1 : g.nI0;
    const float* xr = x + ((long)b * T + 2 * t1) * F;
    const long rbase = (long)(b * nI + (t1 >> 1));
    // two pixels per step: both pixels' taps are in flight before either is computed
    for (int f0 = pw; f0 < g.F1; f0 += 2 * ppb) {
      const int fb = f0 + ppb < g.F1 ? f0 + ppb : f0;  // odd tail: recompute f0 (same values)
      float xv[2][9];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float* xp = xr + 2 * (u ? fb : f0);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) xv[u][kh * 3 + kw] = xp[kh * F + kw];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int f1 = u ? fb : f0;
        const int e = f1 & 1;
        const long prow = g.plane[a * 2 + e] + rbase * (e ? g.nJ1 : g.nJ0) + (f1 >> 1);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float s = br[k];
#pragma unroll
          for (int t = 0; t < 9; ++t) s = fmaf(wr[k][t], xv[u][t], s);
          o[k] = s > 0.f ? s : 0.f;
        }
        TO* yp = y + prow * C + c0;
        if constexpr (sizeof(TO) == 2) {  // one 16-B store per lane
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          union { u32x4 u; TO h[8]; } pk;
#pragma unroll
          for (int k = 0; k < 8; ++k) pk.h[k] = (TO)o[k];
          if (NT) __builtin_nontemporal_store(pk.u, (u32x4*)yp);
          else *(u32x4*)yp = pk.u;
        } else {
          float lo[4] = {o[0], o[1], o[2], o[3]}, hi[4] = {o[4], o[5], o[6], o[7]};
          vst4(yp, lo);
          vst4(yp + 4, hi);
        }
        if (pos) {
          uint32_t m = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) m |= (uint32_t)((float)(TO)o[k] > 0.f) << k;
          if (NT) __builtin_nontemporal_store((uint8_t)m, pos + prow * (C / 8) + cg);
          else pos[prow * (C / 8) + cg] = (uint8_t)m;
        }
      }
    }
  }
}

// conv1 weight/bias gradient from the (ReLU-masked) phase-split gradient dh (= d conv1
// pre-activation): part[blk][t*C + c] = sum over the block's pixels of dh[p,c]*x_t(p),
// t < 9, and part[blk][9*C + c] = sum dh[p,c]; reduced over blocks in fixed order.
template <typename TI>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(int B, int T, int F, PhaseGeo g, int C,
                                                          const float* __restrict__ x, const TI* __restrict__ dh,
                                                          float* __restrict__ part) {
  __shared__ float red[256 * 10];
  const int groups = C / 8;
  const int cg = threadIdx.x % groups, c0 = cg * 8;
  const int ppb = blockDim.x / groups, pl = threadIdx.x / groups;
  float acc[10][8];
#pragma unroll
  for (int t = 0; t < 10; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[t][k] = 0.f;
  const long npix = (long)B * g.T1 * g.F1;
  for (long pix = (long)blockIdx.x * ppb + pl; pix < npix; pix += (long)gridDim.x * ppb) {
    const int f1 = (int)(pix % g.F1);
    const long bt = pix / g.F1;
    const int t1 = (int)(bt % g.T1), b = (int)(bt / g.T1);
    const float* xp = x + ((long)b * T + 2 * t1) * F + 2 * f1;
    float xv[10];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) xv[kh * 3 + kw] = xp[kh * F + kw];
    xv[9] = 1.f;
    const TI* dp = dh + phase_row(g, b, t1, f1) * C + c0;
    float d[8], lo[4], hi[4];
    vld4(dp, lo);
    vld4(dp + 4, hi);
#pragma unroll
    for (int k = 0; k < 4; ++k) { d[k] = lo[k]; d[k + 4] = hi[k]; }
#pragma unroll
    for (int t = 0; t < 10; ++t)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[t][k] = fmaf(d[k], xv[t], acc[t][k]);
  }
  // combine the block's pixel lanes in fixed order: one (t, k) column at a time via LDS
  for (int t = 0; t < 10; ++t) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      __syncthreads();
      red[threadIdx.x] = acc[t][k];
      __syncthreads();
      if (pl == 0) {
        float a = 0.f;
        for (int q = 0; q < ppb; ++q) a += red[q * groups + cg];
        part[(long)blockIdx.x * 10 * C + (long)t * C + c0 + k] = a;
      }
    }
  }
}

// ---------------------------------------------------------------- dropout / cast / scale
template <typename TI, typename TO>
__global__ void scale_drop_kernel(long n, int cols, const TI* __restrict__ x, long ldx, TO* __restrict__ y, long ldy,
                                  float scale, float p, uint64_t seed, const unsigned long long* salt) {
  if (p > 0.f) seed = ea_salted(seed, salt);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, c = i % cols;
    float v = to_f(x[r * ldx + c]) * scale;
    if (p > 0.f) v *= drop_scale(seed, (uint64_t)i, p);
    y[r * ldy + c] = from_f<TO>(v);
  }
}

// 4 columns per thread (cols, lds % 4 == 0, aligned); same per-element dropout index as above
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void scale_drop_vec_kernel(unsigned n4, unsigned cols4, const TI* __restrict__ x, long ldx,
                                                             TO* __restrict__ y, long ldy, float scale, float p,
                                                             uint64_t seed, const unsigned long long* salt) {
  if (p > 0.f) seed = ea_salted(seed, salt);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const unsigned r = i / cols4, c = (i - r * cols4) * 4;
    float v[4];
    vld4(x + (long)r * ldx + c, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] *= scale;
    drop_scale4(seed, (uint64_t)i * 4, p, v);
    vst4(y + (long)r * ldy + c, v);
  }
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void add2d_vec_kernel(unsigned n4, unsigned cols4, const TI* __restrict__ x, long ldx,
                                                        TO* __restrict__ y, long ldy, float alpha) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const unsigned r = i / cols4, c = (i - r * cols4) * 4;
    float v[4], o[4];
    vld4(x + (long)r * ldx + c, v);
    vld4(y + (long)r * ldy + c, o);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] += alpha * v[k];
    vst4(y + (long)r * ldy + c, o);
  }
}

// y[r,c] += alpha * x[r,c]
template <typename TI, typename TO>
__global__ void add2d_kernel(long n, int cols, const TI* __restrict__ x, long ldx, TO* __restrict__ y, long ldy, float alpha) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, c = i % cols;
    TO* o = y + r * ldy + c;
    *o = from_f<TO>(to_f(*o) + alpha * to_f(x[r * ldx + c]));
  }
}

// dst[a][c][b] (+)= src[a][b][c]  (weight repack: conv (Co,Ci,9)<->(Co,9,Ci), linear (O,C,F)<->(O,F,C))
template <typename TI, typename TO>
__global__ void permute3_kernel(int A, int Bd, int Cd, const TI* __restrict__ src, TO* __restrict__ dst, int accumulate) {
  const long n = (long)A * Bd * Cd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long a = i / ((long)Bd * Cd);
    const long rem = i % ((long)Bd * Cd);
    const long c = rem / Bd, b = rem % Bd;  // i indexes dst[a][c][b]
    const float v = to_f(src[(a * Bd + b) * Cd + c]);
    dst[i] = from_f<TO>(accumulate ? to_f(dst[i]) + v : v);
  }
}

// ---------------------------------------------------------------- subsampling im2col
// conv1 (1->C, k3 s2) as a GEMM: rows = (b, t1, f1), 16 columns (9 taps + zero pad)
template <typename TO>
__global__ void im2col_conv1_kernel(int B, int T, int F, int T1, int F1, const float* __restrict__ x, TO* __restrict__ col) {
  const long n = (long)B * T1 * F1 * 16;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i & 15);
    const long r = i >> 4;
    const int f1 = (int)(r % F1);
    const long bt = r / F1;
    const int t1 = (int)(bt % T1), b = (int)(bt / T1);
    float v = 0.f;
    if (k < 9) {
      const int kh = k / 3, kw = k % 3;
      v = x[((long)b * T + 2 * t1 + kh) * F + 2 * f1 + kw];
    }
    col[i] = from_f<TO>(v);
  }
}

// conv2 (C->C, k3 s2) im2col from NHWC x1 (B,T1,F1,C): row (b,t2,f2), column (kh,kw,c)
template <typename T>
__global__ void im2col_conv2_kernel(int B, int T1, int F1, int C, int T2, int F2, const T* __restrict__ x1, T* __restrict__ col) {
  const int C8 = C / 8;
  const long n = (long)B * T2 * F2 * 9 * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    long r = i / C8;
    const int k = (int)(r % 9);
    r /= 9;
    const int f2 = (int)(r % F2);
    const long bt = r / F2;
    const int t2 = (int)(bt % T2), b = (int)(bt / T2);
    const int kh = k / 3, kw = k % 3;
    const T* src = x1 + (((long)b * T1 + 2 * t2 + kh) * F1 + 2 * f2 + kw) * C + c8 * 8;
    T* dst = col + (r * 9 + k) * (long)C + c8 * 8;
    if (sizeof(T) == 2) *(uint4*)dst = *(const uint4*)src;
    else { *(uint4*)dst = *(const uint4*)src; *(uint4*)(dst + 4) = *(const uint4*)(src + 4); }
  }
}

// col2im for conv2's input gradient, gather form: dx1[b,t1,f1,c] = relu'(x1) *
//   sum over taps (kh,kw) with t1 = 2*t2+kh, f1 = 2*f2+kw of dcol[(b,t2,f2),(kh,kw,c)]
template <typename TI, typename TO>
__global__ void col2im_conv2_kernel(int B, int T1, int F1, int C, int T2, int F2, const TI* __restrict__ dcol,
                                    const TO* __restrict__ x1, TO* __restrict__ dx1) {
  const long n = (long)B * T1 * F1 * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long r = i / C;
    const int f1 = (int)(r % F1);
    const long bt = r / F1;
    const int t1 = (int)(bt % T1), b = (int)(bt / T1);
    float acc = 0.f;
    if (to_f(x1[i]) > 0.f) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int tt = t1 - kh;
        if (tt < 0 || (tt & 1) || (tt >> 1) >= T2) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ff = f1 - kw;
          if (ff < 0 || (ff & 1) || (ff >> 1) >= F2) continue;
          const long row = ((long)b * T2 + (tt >> 1)) * F2 + (ff >> 1);
          acc += to_f(dcol[(row * 9 + kh * 3 + kw) * (long)C + c]);
        }
      }
    }
    dx1[i] = from_f<TO>(acc);
  }
}


// vectorised bf16 col2im: 8 channels per thread (16-B loads/stores)
__global__ void col2im_conv2_bf16x8_kernel(int B, int T1, int F1, int C, int T2, int F2, const bf16* __restrict__ dcol,
                                           const bf16* __restrict__ x1, bf16* __restrict__ dx1) {
  const int C8 = C / 8;
  const long n = (long)B * T1 * F1 * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    long r = i / C8;
    const int f1 = (int)(r % F1);
    const long bt = r / F1;
    const int t1 = (int)(bt % T1), b = (int)(bt / T1);
    const long off = r * C + c8 * 8;
    const uint4 xv = *(const uint4*)(x1 + off);
    const bf16* xb = (const bf16*)&xv;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int tt = t1 - kh;
      if (tt < 0 || (tt & 1) || (tt >> 1) >= T2) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ff = f1 - kw;
        if (ff < 0 || (ff & 1) || (ff >> 1) >= F2) continue;
        const long row = ((long)b * T2 + (tt >> 1)) * F2 + (ff >> 1);
        const uint4 dv = *(const uint4*)(dcol + (row * 9 + kh * 3 + kw) * (long)C + c8 * 8);
        const bf16* db = (const bf16*)&dv;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)db[e];
      }
    }
    uint4 out;
    bf16* ob = (bf16*)&out;
#pragma unroll
    for (int e = 0; e < 8; ++e) ob[e] = (bf16)((float)xb[e] > 0.f ? acc[e] : 0.f);
    *(uint4*)(dx1 + off) = out;
  }
}

// ---------------------------------------------------------------- GLU (conv module)
// out[r,c] = x[r,c] * sigmoid(x[r,c+C])   (nn.functional.glu(dim=channels))
template <typename TI, typename TO>
__global__ void glu_fwd_kernel(long rows, int C, const TI* __restrict__ x, TO* __restrict__ y) {
  const long n = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = (int)(i % C);
    const float a = to_f(x[r * 2 * C + c]), g = to_f(x[r * 2 * C + C + c]);
    y[i] = from_f<TO>(a * sigmoidf_(g));
  }
}
template <typename TI, typename TO>
__global__ void glu_bwd_kernel(long rows, int C, const TI* __restrict__ x, const float* __restrict__ dy, TO* __restrict__ dx) {
  const long n = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = (int)(i % C);
    const float a = to_f(x[r * 2 * C + c]), g = to_f(x[r * 2 * C + C + c]);
    const float s = sigmoidf_(g), d = dy[i];
    dx[r * 2 * C + c] = from_f<TO>(d * s);
    dx[r * 2 * C + C + c] = from_f<TO>(d * a * s * (1.f - s));
  }
}

// ---------------------------------------------------------------- depthwise conv1d
// y[b,t,c] = bias[c] + sum_k w[c,k] x[b, t+k-P, c] (zero padded per utterance)
constexpr int DW_TT = 32;   // time rows per block
constexpr int DW_CT = 64;   // channels per block
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(int B, int T, int C, int K, const float* __restrict__ x,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         float* __restrict__ y) {
  extern __shared__ float tile[];  // (DW_TT + K - 1) x DW_CT
  const int P = (K - 1) / 2;
  const int ntt = ea_cdiv(T, DW_TT);
  const int b = blockIdx.x / ntt, t0 = (blockIdx.x % ntt) * DW_TT;
  const int c0 = blockIdx.y * DW_CT;
  const int rowsL = DW_TT + K - 1;
  for (int i = threadIdx.x; i < rowsL * DW_CT; i += blockDim.x) {
    const int rr = i / DW_CT, cc = i % DW_CT;
    const int t = t0 + rr - P, c = c0 + cc;
    tile[i] = (t >= 0 && t < T && c < C) ? x[((long)b * T + t) * C + c] : 0.f;
  }
  __syncthreads();
  const int cc = threadIdx.x % DW_CT, tq = threadIdx.x / DW_CT;  // 4 time groups of 8
  const int c = c0 + cc;
  if (c >= C) return;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = bias ? bias[c] : 0.f;
  for (int k = 0; k < K; ++k) {
    const float wk = w[c * K + k];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += wk * tile[(tq * 8 + j + k) * DW_CT + cc];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = t0 + tq * 8 + j;
    if (t < T) y[((long)b * T + t) * C + c] = acc[j];
  }
}

// dx[b,t,c] = sum_k w[c,k] dy[b, t-k+P, c];  part[blk][c*K+k] = sum_t dy[b,t,c] x[b,t+k-P,c]
__global__ __launch_bounds__(256) void dwconv_bwd_kernel(int B, int T, int C, int K, const float* __restrict__ x,
                                                         const float* __restrict__ w, const float* __restrict__ dy,
                                                         float* __restrict__ dx, float* __restrict__ part) {
  extern __shared__ float sm[];
  const int P = (K - 1) / 2;
  const int ntt = ea_cdiv(T, DW_TT);
  const int b = blockIdx.x / ntt, t0 = (blockIdx.x % ntt) * DW_TT;
  const int c0 = blockIdx.y * DW_CT;
  const int rowsL = DW_TT + K - 1;
  float* tdy = sm;                    // dy rows t0-(K-1-P) .. t0+DW_TT-1+P
  float* tx = sm + rowsL * DW_CT;     // x rows  t0-P .. t0+DW_TT-1+(K-1-P)
  float* tin = tx + rowsL * DW_CT;    // dy rows t0 .. t0+DW_TT-1 (for dw)
  for (int i = threadIdx.x; i < rowsL * DW_CT; i += blockDim.x) {
    const int rr = i / DW_CT, cc = i % DW_CT, c = c0 + cc;
    const int td = t0 + rr - (K - 1 - P);
    const int tx_ = t0 + rr - P;
    tdy[i] = (td >= 0 && td < T && c < C) ? dy[((long)b * T + td) * C + c] : 0.f;
    tx[i] = (tx_ >= 0 && tx_ < T && c < C) ? x[((long)b * T + tx_) * C + c] : 0.f;
  }
  for (int i = threadIdx.x; i < DW_TT * DW_CT; i += blockDim.x) {
    const int rr = i / DW_CT, cc = i % DW_CT, c = c0 + cc, t = t0 + rr;
    tin[i] = (t < T && c < C) ? dy[((long)b * T + t) * C + c] : 0.f;
  }
  __syncthreads();
  const int cc = threadIdx.x % DW_CT, tq = threadIdx.x / DW_CT;
  const int c = c0 + cc;
  if (c < C) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // dx[t] = sum_k w[k] dy[t - k + P]; tdy row index for dy[t'] is t' - t0 + (K-1-P)
    for (int k = 0; k < K; ++k) {
      const float wk = w[c * K + k];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += wk * tdy[(tq * 8 + j - k + (K - 1)) * DW_CT + cc];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + tq * 8 + j;
      if (t < T) dx[((long)b * T + t) * C + c] = acc[j];
    }
  }
  // dw partials: 4 thread-groups split the K taps
  const long blk = (long)blockIdx.x;
  if (c < C) {
    for (int k = tq; k < K; k += 4) {
      float a = 0.f;
      for (int r = 0; r < DW_TT; ++r) a += tin[r * DW_CT + cc] * tx[(r + k) * DW_CT + cc];
      part[blk * (long)C * K + (long)c * K + k] = a;
    }
  }
}

// Register-window variants for a compile-time kernel width: each thread owns one channel and
// R consecutive time rows (a block: 64 channels x 4R rows), holds the R+K-1 input rows it
// touches in registers (one LDS read per row instead of one per tap) and does the R*K taps
// from registers; the block's taps are staged through LDS by one coalesced pass.
constexpr int DW_R = 16;  // rows per thread (64-row tiles: the K-1 halo costs < 1.5x)

// the conv input x = glu(g2) = a * sigmoid(b) for g2 rows [a | b] (2C bf16; glu_fwd_kernel's
// arithmetic), 4 channels from two 8-B loads: the depthwise conv reads the pointwise conv's
// bf16 output directly and the f32 GLU activation is never stored
EA_DEV float4 glu4(const bf16* __restrict__ g2, long row, int C, int c) {
  const uint2 ua = *(const uint2*)(g2 + row * 2 * C + c), ub = *(const uint2*)(g2 + row * 2 * C + C + c);
  const float a0 = __uint_as_float(ua.x << 16), a1 = __uint_as_float(ua.x & 0xffff0000u);
  const float a2 = __uint_as_float(ua.y << 16), a3 = __uint_as_float(ua.y & 0xffff0000u);
  const float b0 = __uint_as_float(ub.x << 16), b1 = __uint_as_float(ub.x & 0xffff0000u);
  const float b2 = __uint_as_float(ub.y << 16), b3 = __uint_as_float(ub.y & 0xffff0000u);
  return make_float4(a0 * sigmoidf_(b0), a1 * sigmoidf_(b1), a2 * sigmoidf_(b2), a3 * sigmoidf_(b3));
}
EA_DEV float glu1(const bf16* __restrict__ g2, long row, int C, int c) {
  return to_f(g2[row * 2 * C + c]) * sigmoidf_(to_f(g2[row * 2 * C + C + c]));
}

// STATS: also the following BatchNorm's batch-statistics partials of this block's rows
// (conformer/convolution.py:75): part[blockIdx.x][c] = sum (y - bias[c]), part[..][C + c] =
// sum (y - bias[c])^2 (f32, the 4 row groups combined in fixed order) — the shifted sums the
// finalize pass turns into mean / var in fp64, without re-reading y
template <int K, int R, bool G2IN = false, bool STATS = false>
__global__ __launch_bounds__(256) void dwconv_fwd_k_kernel(int B, int T, int C, const float* __restrict__ x,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ bias, float* __restrict__ y,
                                                           const bf16* __restrict__ g2 = nullptr,
                                                           float* __restrict__ part = nullptr) {
  constexpr int P = (K - 1) / 2, TT = 4 * R, RL = TT + K - 1, WIN = R + K - 1;
  __shared__ float tile[RL * DW_CT];
  __shared__ float wsm[K * DW_CT];  // [k][c]
  const int ntt = ea_cdiv(T, TT);
  const int b = blockIdx.x / ntt, t0 = (blockIdx.x % ntt) * TT;
  const int c0 = blockIdx.y * DW_CT;
  const int cc = threadIdx.x % DW_CT, tq = threadIdx.x / DW_CT;
  const int c = c0 + cc;
  for (int i = threadIdx.x; i < DW_CT * K; i += 256) {  // w rows c0.. are one contiguous run
    const int ci = i / K, k = i - ci * K;
    wsm[k * DW_CT + ci] = c0 + ci < C ? w[(long)c0 * K + i] : 0.f;
  }
  if (C % 4 == 0) {  // 16-B loads: 16 lanes cover one 64-channel row; all NL in flight at once
    constexpr int NL = (RL * (DW_CT / 4) + 255) / 256;
    float4 v[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int rr = i / (DW_CT / 4), c4 = (i % (DW_CT / 4)) * 4;
      const int t = t0 + rr - P;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < RL * (DW_CT / 4) && t >= 0 && t < T && c0 + c4 < C) {
        if constexpr (G2IN)
          v[u] = glu4(g2, (long)b * T + t, C, c0 + c4);
        else
          v[u] = *(const float4*)(x + ((long)b * T + t) * C + c0 + c4);
      }
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int i = threadIdx.x + 256 * u;
      if (i < RL * (DW_CT / 4)) *(float4*)(tile + (i / (DW_CT / 4)) * DW_CT + (i % (DW_CT / 4)) * 4) = v[u];
    }
  } else {
    for (int rr = tq; rr < RL; rr += 4) {
      const int t = t0 + rr - P;
      float v = 0.f;
      if (t >= 0 && t < T && c < C) {
        if constexpr (G2IN)
          v = glu1(g2, (long)b * T + t, C, c);
        else
          v = x[((long)b * T + t) * C + c];
      }
      tile[rr * DW_CT + cc] = v;
    }
  }
  __syncthreads();
  if (!STATS && c >= C) return;
  float win[WIN];
#pragma unroll
  for (int i = 0; i < WIN; ++i) win[i] = tile[(tq * R + i) * DW_CT + cc];
  float acc[R];
  const float b0 = bias && c < C ? bias[c] : 0.f;
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = b0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float wk = wsm[k * DW_CT + cc];
#pragma unroll
    for (int j = 0; j < R; ++j) acc[j] += wk * win[j + k];
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int t = t0 + tq * R + j;
    if (t < T && c < C) {
      y[((long)b * T + t) * C + c] = acc[j];
      if constexpr (STATS) {
        const float d = acc[j] - b0;
        s1 += d;
        s2 += d * d;
      }
    }
  }
  if constexpr (STATS) {
    __shared__ float red[2][4][DW_CT];
    red[0][tq][cc] = s1;
    red[1][tq][cc] = s2;
    __syncthreads();
    if (tq == 0 && c < C) {
      part[(long)blockIdx.x * 2 * C + c] = (red[0][0][cc] + red[0][1][cc]) + (red[0][2][cc] + red[0][3][cc]);
      part[(long)blockIdx.x * 2 * C + C + c] = (red[1][0][cc] + red[1][1][cc]) + (red[1][2][cc] + red[1][3][cc]);
    }
  }
}

// dx[t] = sum_k w[k] dy[t-k+P];  part[blk][k*C+c] = sum_t dy[t] x[t+k-P];  part[blk][K*C+c] = sum_t dy[t]
// CK: partials laid out as the parameters are — [c][k] (dw is (C, 1, K)) then [c] (dbias) — so
// their sums are plain row reductions the host can defer into the pass's grouped reduce
// GLU: the GLU backward fused into the dx store (conformer/convolution.py:64-66: the depthwise
// conv's input is glu(g2)): dg2 = (dx * sigmoid(b), dx * a * s * (1 - s)) for g2 = [a | b] rows of
// 2C bf16 — the arithmetic of glu_bwd_kernel, without dx's f32 round trip through HBM
// G2IN: x = glu(g2) recomputed in the tile loader (the forward did not store it)
template <int K, int R, bool CK = false, bool GLU = false, bool G2IN = false>
__global__ __launch_bounds__(256) void dwconv_bwd_k_kernel(int B, int T, int C, const float* __restrict__ x,
                                                           const float* __restrict__ w, const float* __restrict__ dy,
                                                           float* __restrict__ dx, float* __restrict__ part,
                                                           const bf16* __restrict__ g2 = nullptr,
                                                           bf16* __restrict__ dg2 = nullptr) {
  constexpr int P = (K - 1) / 2, TT = 4 * R, RL = TT + K - 1, WIN = R + K - 1;
  constexpr int SM = 2 * RL * DW_CT > 4 * (K + 1) * DW_CT ? 2 * RL * DW_CT : 4 * (K + 1) * DW_CT;
  __shared__ float sm[SM];
  float* tdy = sm;                 // dy rows t0-(K-1-P) .. t0+TT-1+P
  float* tx = sm + RL * DW_CT;     // x rows  t0-P .. t0+TT-1+(K-1-P)
  const int ntt = ea_cdiv(T, TT);
  const int b = blockIdx.x / ntt, t0 = (blockIdx.x % ntt) * TT;
  const int c0 = blockIdx.y * DW_CT;
  const int cc = threadIdx.x % DW_CT, tq = threadIdx.x / DW_CT;
  const int c = c0 + cc;
  // the channel's K taps in registers (an LDS copy cost the block 8 KB: 47 KB fit three blocks
  // per CU, 55 KB two)
  float wr[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wr[k] = c < C ? w[(long)c * K + k] : 0.f;
  // GLU: the gate rows this thread's dx store needs, loaded first (their latency hides behind
  // the tile loads; the LDS budget, not registers, bounds this kernel's occupancy)
  bf16 ga[GLU ? R : 1], gb[GLU ? R : 1];
  if constexpr (GLU) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const long row = (long)b * T + min(t0 + tq * R + j, T - 1);
      const int cl = min(c, C - 1);
      ga[j] = g2[row * 2 * C + cl];
      gb[j] = g2[row * 2 * C + C + cl];
    }
  }
  if (C % 4 == 0) {  // 16-B loads, all NL of both tiles in flight before the LDS stores
    constexpr int NL = (RL * (DW_CT / 4) + 255) / 256;
    float4 va[NL], vb[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int rr = i / (DW_CT / 4), c4 = (i % (DW_CT / 4)) * 4;
      const int td = t0 + rr - (K - 1 - P), tx_ = t0 + rr - P;
      const bool okc = i < RL * (DW_CT / 4) && c0 + c4 < C;
      va[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      vb[u] = va[u];
      if (okc && td >= 0 && td < T) va[u] = *(const float4*)(dy + ((long)b * T + td) * C + c0 + c4);
      if (okc && tx_ >= 0 && tx_ < T) {
        if constexpr (G2IN)
          vb[u] = glu4(g2, (long)b * T + tx_, C, c0 + c4);
        else
          vb[u] = *(const float4*)(x + ((long)b * T + tx_) * C + c0 + c4);
      }
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int i = threadIdx.x + 256 * u;
      if (i < RL * (DW_CT / 4)) {
        const int o = (i / (DW_CT / 4)) * DW_CT + (i % (DW_CT / 4)) * 4;
        *(float4*)(tdy + o) = va[u];
        *(float4*)(tx + o) = vb[u];
      }
    }
  } else {
    for (int rr = tq; rr < RL; rr += 4) {
      const int td = t0 + rr - (K - 1 - P), tx_ = t0 + rr - P;
      const bool okc = c < C;
      tdy[rr * DW_CT + cc] = (okc && td >= 0 && td < T) ? dy[((long)b * T + td) * C + c] : 0.f;
      float xv = 0.f;
      if (okc && tx_ >= 0 && tx_ < T) {
        if constexpr (G2IN)
          xv = glu1(g2, (long)b * T + tx_, C, c);
        else
          xv = x[((long)b * T + tx_) * C + c];
      }
      tx[rr * DW_CT + cc] = xv;
    }
  }
  __syncthreads();
  float aw[K + 1];
  {
    float win[WIN];
#pragma unroll
    for (int i = 0; i < WIN; ++i) win[i] = tdy[(tq * R + i) * DW_CT + cc];
    if (c < C) {
      float acc[R];
#pragma unroll
      for (int j = 0; j < R; ++j) acc[j] = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float wk = wr[k];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] += wk * win[j - k + K - 1];
      }
      if constexpr (GLU) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const int t = t0 + tq * R + j;
          if (t < T) {
            const long row = (long)b * T + t;
            const float a = to_f(ga[j]), g = to_f(gb[j]);
            const float s = sigmoidf_(g), d = acc[j];
            dg2[row * 2 * C + c] = from_f<bf16>(d * s);
            dg2[row * 2 * C + C + c] = from_f<bf16>(d * a * s * (1.f - s));
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const int t = t0 + tq * R + j;
          if (t < T) dx[((long)b * T + t) * C + c] = acc[j];
        }
      }
    }
    // dy[t0 + tq*R + j] = win[j + K-1-P]  (rows past T are zero)
    float xw[WIN];
#pragma unroll
    for (int i = 0; i < WIN; ++i) xw[i] = tx[(tq * R + i) * DW_CT + cc];
#pragma unroll
    for (int k = 0; k <= K; ++k) aw[k] = 0.f;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const float d = win[j + K - 1 - P];
      aw[K] += d;
#pragma unroll
      for (int k = 0; k < K; ++k) aw[k] += d * xw[j + k];
    }
  }
  __syncthreads();  // reuse the tiles for the 4-group reduction
#pragma unroll
  for (int k = 0; k <= K; ++k) sm[(tq * (K + 1) + k) * DW_CT + cc] = aw[k];
  __syncthreads();
  const long blk = (long)blockIdx.x;
  for (int i = threadIdx.x; i < (K + 1) * DW_CT; i += blockDim.x) {
    // [k][c]: k = i / DW_CT (coalesced over c); CK: (c, k) with k fastest over the dw block
    const int k = CK ? (i < K * DW_CT ? i % K : K) : i / DW_CT;
    const int ci = CK ? (i < K * DW_CT ? i / K : i - K * DW_CT) : i % DW_CT;
    const int cg = c0 + ci;
    if (cg >= C) continue;
    const float v = (sm[(0 * (K + 1) + k) * DW_CT + ci] + sm[(1 * (K + 1) + k) * DW_CT + ci]) +
                    (sm[(2 * (K + 1) + k) * DW_CT + ci] + sm[(3 * (K + 1) + k) * DW_CT + ci]);
    const long o = CK ? (k < K ? (long)cg * K + k : (long)C * K + cg) : (long)k * C + cg;
    part[blk * (long)C * (K + 1) + o] = v;  // k == K: dbias
  }
}

// ---------------------------------------------------------------- attention helpers
// qu = q + u[h], qv = q + v[h] for q rows of (N, H*dk) inside a fused qkv buffer
template <typename T>
__global__ void add_pos_bias_kernel(long N, int H, int dk, const T* __restrict__ q, long ldq, const float* __restrict__ u,
                                    const float* __restrict__ v, T* __restrict__ qu, T* __restrict__ qv) {
  const int d = H * dk;
  const long n = N * d;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / d;
    const int c = (int)(i % d);
    const float x = to_f(q[r * ldq + c]);
    qu[i] = from_f<T>(x + u[c]);
    qv[i] = from_f<T>(x + v[c]);
  }
}

// ---------------------------------------------------------------- embeddings (decoder)
// y[r] = dropout(E[tok[r]] * xscale + pe[pos(r)]), pos(r) = r % L
__global__ void embed_fwd_kernel(long rows, int d, int L, const long long* __restrict__ tok, const float* __restrict__ E,
                                 float xscale, const float* __restrict__ pe, float p, uint64_t seed,
                                 const unsigned long long* salt, float* __restrict__ y) {
  if (p > 0.f) seed = ea_salted(seed, salt);
  const long n = rows * d;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / d;
    const int c = (int)(i % d);
    float v = E[tok[r] * d + c] * xscale + pe[(r % L) * d + c];
    if (p > 0.f) v *= drop_scale(seed, (uint64_t)i, p);
    y[i] = v;
  }
}
// y[r] = dropout(y[r] + pe[r % L]) in place: the absolute PositionalEncoding after the
// subsampling Linear (embedding.py:81-92; the Linear's epilogue already applied x*xscale).
// Same per-element dropout index r*d + c as ea_scale_dropout, so the backward is an
// ea_scale_dropout(_colsum) with scale xscale.
__global__ void add_pe_dropout_kernel(long n, int d, int L, const float* __restrict__ pe, float p, uint64_t seed,
                                      const unsigned long long* salt, float* __restrict__ y) {
  if (p > 0.f) seed = ea_salted(seed, salt);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / d;
    const int c = (int)(i % d);
    float v = y[i] + pe[(r % L) * d + c];
    if (p > 0.f) v *= drop_scale(seed, (uint64_t)i, p);
    y[i] = v;
  }
}
// dE[tok[r]] += xscale * dropout_mask * dy[r], deterministic: one block per row r; the
// block of a token's FIRST row sums all of that token's rows in increasing order and owns
// the update of dE[tok] (no atomics, bit-reproducible).  tok staged in LDS (rows <= 4096).
constexpr int EMBED_BWD_MAXROWS = 4096;
__global__ __launch_bounds__(256) void embed_bwd_kernel(int rows, int d, const long long* __restrict__ tok,
                                                        const float* __restrict__ dy, float xscale, float p,
                                                        uint64_t seed, const unsigned long long* salt,
                                                        float* __restrict__ dE) {
  __shared__ int stok[EMBED_BWD_MAXROWS];
  __shared__ int dup;
  if (p > 0.f) seed = ea_salted(seed, salt);
  const int r = blockIdx.x;
  const long long me = tok[r];
  if (threadIdx.x == 0) dup = 0;
  __syncthreads();
  for (int q = threadIdx.x; q < rows; q += blockDim.x) {
    stok[q] = (int)tok[q];
    if (q < r && tok[q] == me) dup = 1;
  }
  __syncthreads();
  if (dup) return;
  // the rows of this token, in increasing order (wave ballots + per-chunk offsets), then one
  // pass per column over that list: the same summation order as scanning every row
  __shared__ int list[EMBED_BWD_MAXROWS];
  __shared__ int wcnt[4], nlist;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) nlist = 0;
  __syncthreads();
  for (int base = r; base < rows; base += 256) {
    const int q = base + threadIdx.x;
    const bool hit = q < rows && stok[q] == (int)me;
    const unsigned long long m = __ballot(hit);
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    int off = nlist;
    for (int v = 0; v < w; ++v) off += wcnt[v];
    if (hit) list[off + __popcll(m & ((1ull << lane) - 1ull))] = q;
    __syncthreads();
    if (threadIdx.x == 0) nlist += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
  const int n = nlist;
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float a = 0.f;
    for (int k = 0; k < n; ++k) {
      const int q = list[k];
      const uint64_t i = (uint64_t)q * d + c;
      float v = dy[i] * xscale;
      if (p > 0.f) v *= drop_scale(seed, i, p);
      a += v;
    }
    dE[me * d + c] += a;
  }
}

// ---------------------------------------------------------------- argmax rows (CTC align)
__global__ void argmax_rows_kernel(long rows, int V, const float* __restrict__ x, long ld, long long* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long r = blockIdx.x * (long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = lane; v < V; v += 64) {
    const float t = xr[v];
    if (t > best || (t == best && v < bi) || (t != t && best == best)) { best = t; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) out[r] = bi;
}

}  // namespace

#define EA_GRID(n) dim3(ea_grid_cap(ea_cdiv((n), 256))), dim3(256), 0, (hipStream_t)stream

extern "C" int ea_utterance_mvn(int B, int T, int F, const float* x, const long long* lens, float* y, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(F <= 256 && F > 0);
  const int bx = F <= 64 ? 64 : (F <= 128 ? 128 : 256);
  const int by = 1024 / bx;
  hipLaunchKernelGGL(mvn_kernel, dim3(B), dim3(bx, by), 0, (hipStream_t)stream, B, T, F, x, lens, y);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_utterance_mvn_ws_bytes(int B, int T, int F, long* bytes) {
  EA_ENTRY();
  EA_CHECK_ARG(bytes != nullptr && B >= 0 && T >= 0 && F > 0);
  *bytes = (long)B * ea_cdiv(T, MVN_TC) * F * (long)sizeof(double);
  return 0;
}

extern "C" int ea_utterance_mvn2(int B, int T, int F, const float* x, const long long* lens, float* y, void* ws,
                                 long ws_bytes, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(F <= 256 && F > 0 && ws != nullptr);
  const int nch = ea_cdiv(T, MVN_TC);
  EA_CHECK_ARG(ws_bytes >= (long)B * nch * F * (long)sizeof(double));
  if (B == 0 || T == 0) return 0;
  const int bx = F <= 64 ? 64 : (F <= 128 ? 128 : 256);
  const int by = 512 / bx;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(mvn_part_kernel, dim3(nch, B), dim3(bx, by), 0, st, T, F, x, lens, (double*)ws);
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(mvn_apply_kernel, dim3(nch, B), dim3(bx, by), 0, st, T, F, x, lens, (const double*)ws, y);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_subsample_lens(int B, int T, const long long* ilens, long long* olens, void* stream) {
  EA_ENTRY();
  hipLaunchKernelGGL(subsample_lens_kernel, dim3(ea_cdiv(B, 64)), dim3(64), 0, (hipStream_t)stream, B, T, ilens, olens);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_add_sos_eos(int B, int L, const long long* ys, long ldys, const long long* ylens, int sos, int eos,
                              int ignore_id, long long* ys_in, long long* ys_out, long long* ys_in_lens, void* stream) {
  EA_ENTRY();
  hipLaunchKernelGGL(sos_eos_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, B, L, ys, ldys, ylens, sos, eos,
                     ignore_id, ys_in, ys_out, ys_in_lens);
  EA_LAUNCH_CHECK();
  return 0;
}

const unsigned long long* ea_g_rng_salt = nullptr;

namespace {
__global__ void rng_advance_kernel(unsigned long long* salt) { salt[0] += 1ull; }
}  // namespace

extern "C" int ea_set_rng_salt(const unsigned long long* salt) {
  EA_ENTRY();
  ea_g_rng_salt = salt;
  return 0;
}

extern "C" int ea_rng_advance(unsigned long long* salt, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(salt != nullptr);
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, salt);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_scale_dropout(long rows, int cols, const void* x, int x_dtype, long ldx, void* y, int y_dtype,
                                long ldy, float scale, float p, unsigned long long seed, void* stream) {
  EA_ENTRY();
  const long n = rows * cols;
  if (n == 0) return 0;
  const int xa = x_dtype == EA_BF16 ? 8 : 16, ya = y_dtype == EA_BF16 ? 8 : 16;
  if (cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (uintptr_t)x % xa == 0 && (uintptr_t)y % ya == 0 &&
      n / 4 < (1L << 31)) {
    const unsigned n4 = (unsigned)(n / 4), c4 = (unsigned)(cols / 4);
#define EA_SDV(TI, TO) hipLaunchKernelGGL((scale_drop_vec_kernel<TI, TO>), EA_GRID(n4), n4, c4, (const TI*)x, ldx, (TO*)y, ldy, scale, p, (uint64_t)seed, ea_g_rng_salt)
    if (x_dtype == EA_BF16 && y_dtype == EA_BF16) EA_SDV(bf16, bf16);
    else if (x_dtype == EA_BF16) EA_SDV(bf16, float);
    else if (y_dtype == EA_BF16) EA_SDV(float, bf16);
    else EA_SDV(float, float);
#undef EA_SDV
    EA_LAUNCH_CHECK();
    return 0;
  }
#define EA_SD(TI, TO) hipLaunchKernelGGL((scale_drop_kernel<TI, TO>), EA_GRID(n), n, cols, (const TI*)x, ldx, (TO*)y, ldy, scale, p, (uint64_t)seed, ea_g_rng_salt)
  if (x_dtype == EA_BF16 && y_dtype == EA_BF16) EA_SD(bf16, bf16);
  else if (x_dtype == EA_BF16) EA_SD(bf16, float);
  else if (y_dtype == EA_BF16) EA_SD(float, bf16);
  else EA_SD(float, float);
#undef EA_SD
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_add_2d(long rows, int cols, const void* x, int x_dtype, long ldx, void* y, int y_dtype,
                          long ldy, float alpha, void* stream) {
  EA_ENTRY();
  const long n = rows * cols;
  if (n == 0) return 0;
  const int xa = x_dtype == EA_BF16 ? 8 : 16, ya = y_dtype == EA_BF16 ? 8 : 16;
  if (cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (uintptr_t)x % xa == 0 && (uintptr_t)y % ya == 0 &&
      n / 4 < (1L << 31)) {
    const unsigned n4 = (unsigned)(n / 4), c4 = (unsigned)(cols / 4);
#define EA_A2V(TI, TO) hipLaunchKernelGGL((add2d_vec_kernel<TI, TO>), EA_GRID(n4), n4, c4, (const TI*)x, ldx, (TO*)y, ldy, alpha)
    if (x_dtype == EA_BF16 && y_dtype == EA_BF16) EA_A2V(bf16, bf16);
    else if (x_dtype == EA_BF16) EA_A2V(bf16, float);
    else if (y_dtype == EA_BF16) EA_A2V(float, bf16);
    else EA_A2V(float, float);
#undef EA_A2V
    EA_LAUNCH_CHECK();
    return 0;
  }
#define EA_A2(TI, TO) hipLaunchKernelGGL((add2d_kernel<TI, TO>), EA_GRID(n), n, cols, (const TI*)x, ldx, (TO*)y, ldy, alpha)
  if (x_dtype == EA_BF16 && y_dtype == EA_BF16) EA_A2(bf16, bf16);
  else if (x_dtype == EA_BF16) EA_A2(bf16, float);
  else if (y_dtype == EA_BF16) EA_A2(float, bf16);
  else EA_A2(float, float);
#undef EA_A2
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_permute3(int A, int Bd, int Cd, const void* src, int src_dtype, void* dst, int dst_dtype,
                           int accumulate, void* stream) {
  EA_ENTRY();
  const long n = (long)A * Bd * Cd;
  if (n == 0) return 0;
#define EA_P3(TI, TO) hipLaunchKernelGGL((permute3_kernel<TI, TO>), EA_GRID(n), A, Bd, Cd, (const TI*)src, (TO*)dst, accumulate)
  if (src_dtype == EA_BF16 && dst_dtype == EA_BF16) EA_P3(bf16, bf16);
  else if (src_dtype == EA_BF16) EA_P3(bf16, float);
  else if (dst_dtype == EA_BF16) EA_P3(float, bf16);
  else EA_P3(float, float);
#undef EA_P3
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_im2col_conv1(int B, int T, int F, const float* x, void* col, int col_dtype, void* stream) {
  EA_ENTRY();
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  const long n = (long)B * T1 * F1 * 16;
  if (col_dtype == EA_BF16)
    hipLaunchKernelGGL(im2col_conv1_kernel<bf16>, EA_GRID(n), B, T, F, T1, F1, x, (bf16*)col);
  else
    hipLaunchKernelGGL(im2col_conv1_kernel<float>, EA_GRID(n), B, T, F, T1, F1, x, (float*)col);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_im2col_conv2(int B, int T1, int F1, int C, const void* x1, void* col, int dtype, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(C % 8 == 0);
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const long n = (long)B * T2 * F2 * 9 * (C / 8);
  if (dtype == EA_BF16)
    hipLaunchKernelGGL(im2col_conv2_kernel<bf16>, EA_GRID(n), B, T1, F1, C, T2, F2, (const bf16*)x1, (bf16*)col);
  else
    hipLaunchKernelGGL(im2col_conv2_kernel<float>, EA_GRID(n), B, T1, F1, C, T2, F2, (const float*)x1, (float*)col);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_col2im_conv2(int B, int T1, int F1, int C, const void* dcol, int dcol_dtype, const void* x1,
                               void* dx1, int dtype, void* stream) {
  EA_ENTRY();
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const long n = (long)B * T1 * F1 * C;
  if (dcol_dtype == EA_BF16 && dtype == EA_BF16 && C % 8 == 0) {
    hipLaunchKernelGGL(col2im_conv2_bf16x8_kernel, EA_GRID(n / 8), B, T1, F1, C, T2, F2, (const bf16*)dcol,
                       (const bf16*)x1, (bf16*)dx1);
    EA_LAUNCH_CHECK();
    return 0;
  }
#define EA_C2I(TI, TO) hipLaunchKernelGGL((col2im_conv2_kernel<TI, TO>), EA_GRID(n), B, T1, F1, C, T2, F2, (const TI*)dcol, (const TO*)x1, (TO*)dx1)
  if (dcol_dtype == EA_BF16 && dtype == EA_BF16) EA_C2I(bf16, bf16);
  else if (dcol_dtype == EA_BF16) EA_C2I(bf16, float);
  else if (dtype == EA_BF16) EA_C2I(float, bf16);
  else EA_C2I(float, float);
#undef EA_C2I
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_glu_fwd(long rows, int C, const void* x, int x_dtype, void* y, int y_dtype, void* stream) {
  EA_ENTRY();
  const long n = rows * C;
#define EA_G(TI, TO) hipLaunchKernelGGL((glu_fwd_kernel<TI, TO>), EA_GRID(n), rows, C, (const TI*)x, (TO*)y)
  if (x_dtype == EA_BF16 && y_dtype == EA_BF16) EA_G(bf16, bf16);
  else if (x_dtype == EA_BF16) EA_G(bf16, float);
  else if (y_dtype == EA_BF16) EA_G(float, bf16);
  else EA_G(float, float);
#undef EA_G
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_glu_bwd(long rows, int C, const void* x, int x_dtype, const float* dy, void* dx, void* stream) {
  EA_ENTRY();
  const long n = rows * C;
  if (x_dtype == EA_BF16)
    hipLaunchKernelGGL((glu_bwd_kernel<bf16, bf16>), EA_GRID(n), rows, C, (const bf16*)x, dy, (bf16*)dx);
  else
    hipLaunchKernelGGL((glu_bwd_kernel<float, float>), EA_GRID(n), rows, C, (const float*)x, dy, (float*)dx);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_dwconv_fwd(int B, int T, int C, int K, const float* x, const float* w, const float* bias, float* y,
                             void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(K % 2 == 1);
  dim3 grid(B * ea_cdiv(T, DW_TT), ea_cdiv(C, DW_CT));
  dim3 gridr(B * ea_cdiv(T, 4 * DW_R), ea_cdiv(C, DW_CT));
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define EA_DWF(KK) case KK: hipLaunchKernelGGL((dwconv_fwd_k_kernel<KK, DW_R>), gridr, dim3(256), 0, st, B, T, C, x, w, bias, y); break;
    EA_DWF(3) EA_DWF(5) EA_DWF(7) EA_DWF(15) EA_DWF(31)
#undef EA_DWF
    default: {
      const size_t sm = (size_t)(DW_TT + K - 1) * DW_CT * sizeof(float);
      hipLaunchKernelGGL(dwconv_fwd_kernel, grid, dim3(256), sm, st, B, T, C, K, x, w, bias, y);
    }
  }
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_dwconv_bwd(int B, int T, int C, int K, const float* x, const float* w, const float* dy, float* dx,
                             float* dw, float* dbias, int accumulate_params, float* workspace, long ws_elems,
                             void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(K % 2 == 1);
  const int nblk = B * ea_cdiv(T, DW_TT);
  dim3 grid(nblk, ea_cdiv(C, DW_CT));
  if (K == 3 || K == 5 || K == 7 || K == 15 || K == 31) {
    // one fused pass: dx, and per-block partials of dw and dbias
    const int nblkr = B * ea_cdiv(T, 4 * DW_R);
    dim3 gridr(nblkr, ea_cdiv(C, DW_CT));
    const long rowlen = (long)C * (K + 1);
    EA_CHECK_ARG((long)nblkr * rowlen <= ws_elems);
    hipStream_t st = (hipStream_t)stream;
    switch (K) {
#define EA_DWB(KK) case KK: hipLaunchKernelGGL((dwconv_bwd_k_kernel<KK, DW_R>), gridr, dim3(256), 0, st, B, T, C, x, w, dy, dx, workspace); break;
      EA_DWB(3) EA_DWB(5) EA_DWB(7) EA_DWB(15) EA_DWB(31)
#undef EA_DWB
    }
    EA_LAUNCH_CHECK();
    // partial columns are [k][c]; dw is (C, 1, K): the reduction writes it transposed
    int rc = ea_reduce_partials_tr(nblkr, C * K, workspace, rowlen, dw, accumulate_params, C, K, stream);
    if (rc || !dbias) return rc;
    return ea_reduce_partials(nblkr, C, workspace + (long)C * K, rowlen, dbias, accumulate_params, stream);
  }
  EA_CHECK_ARG((long)nblk * C * K <= ws_elems);
  const size_t sm = (size_t)(2 * (DW_TT + K - 1) + DW_TT) * DW_CT * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dwconv_bwd_kernel, grid, dim3(256), sm, st, B, T, C, K, x, w, dy, dx, workspace);
  EA_LAUNCH_CHECK();
  int rc = ea_reduce_partials(nblk, C * K, workspace, (long)C * K, dw, accumulate_params, stream);
  if (rc) return rc;
  if (dbias) return ea_colsum(B * T, C, dy, EA_F32, C, dbias, accumulate_params, workspace, ws_elems, stream);
  return 0;
}

extern "C" int ea_dwconv_fwd_glu(int B, int T, int C, int K, const void* g2, const float* w, const float* bias,
                                 float* y, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG((K == 3 || K == 5 || K == 7 || K == 15 || K == 31) && g2 && y && C % 4 == 0 &&
               ((uintptr_t)g2 % 8) == 0);
  dim3 gridr(B * ea_cdiv(T, 4 * DW_R), ea_cdiv(C, DW_CT));
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define EA_DWF(KK)                                                                                          \
  case KK:                                                                                                  \
    hipLaunchKernelGGL((dwconv_fwd_k_kernel<KK, DW_R, true>), gridr, dim3(256), 0, st, B, T, C, (const float*)nullptr, \
                       w, bias, y, (const bf16*)g2);                                                        \
    break;
    EA_DWF(3) EA_DWF(5) EA_DWF(7) EA_DWF(15) EA_DWF(31)
#undef EA_DWF
  }
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_dwconv_fwd_glu_stats(int B, int T, int C, int K, const void* g2, const float* w, const float* bias,
                                       float* y, float* part, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG((K == 3 || K == 5 || K == 7 || K == 15 || K == 31) && g2 && y && part && bias && C % 4 == 0 &&
               ((uintptr_t)g2 % 8) == 0);
  dim3 gridr(B * ea_cdiv(T, 4 * DW_R), ea_cdiv(C, DW_CT));
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
#define EA_DWF(KK)                                                                                            \
  case KK:                                                                                                    \
    hipLaunchKernelGGL((dwconv_fwd_k_kernel<KK, DW_R, true, true>), gridr, dim3(256), 0, st, B, T, C,           \
                       (const float*)nullptr, w, bias, y, (const bf16*)g2, part);                             \
    break;
    EA_DWF(3) EA_DWF(5) EA_DWF(7) EA_DWF(15) EA_DWF(31)
#undef EA_DWF
  }
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_dwconv_stats_parts(int B, int T, int* nparts) {
  EA_ENTRY();
  EA_CHECK_ARG(nparts != nullptr && B > 0 && T > 0);
  *nparts = B * ea_cdiv(T, 4 * DW_R);
  return 0;
}

extern "C" int ea_dwconv_glu_bwd(int B, int T, int C, int K, const float* x, const float* w, const float* dy,
                                 const void* g2, void* dg2, float* dw, float* dbias, int accumulate_params,
                                 float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG((K == 3 || K == 5 || K == 7 || K == 15 || K == 31) && g2 && dg2 && dw && dbias);
  EA_CHECK_ARG(x != nullptr || (C % 4 == 0 && ((uintptr_t)g2 % 8) == 0));
  const int nblkr = B * ea_cdiv(T, 4 * DW_R);
  dim3 gridr(nblkr, ea_cdiv(C, DW_CT));
  const long rowlen = (long)C * (K + 1);
  EA_CHECK_ARG((long)nblkr * rowlen <= ws_elems);
  hipStream_t st = (hipStream_t)stream;
  // dw (C, 1, K) and dbias adjacent (the parameter arena's layout): ONE reduction over the
  // (K + 1) C partial columns, the dw block written transposed and the dbias block straight
  // (the same sums in the same order as the two reductions)
  const bool adj = dbias == dw + (long)C * K;
  switch (K) {
#define EA_DWB(KK)                                                                                              \
  case KK:                                                                                                      \
    if (x)                                                                                                      \
      hipLaunchKernelGGL((dwconv_bwd_k_kernel<KK, DW_R, false, true>), gridr, dim3(256), 0, st, B, T, C, x, w, dy,   \
                         (float*)nullptr, workspace, (const bf16*)g2, (bf16*)dg2);                                    \
    else                                                                                                        \
      hipLaunchKernelGGL((dwconv_bwd_k_kernel<KK, DW_R, false, true, true>), gridr, dim3(256), 0, st, B, T, C,      \
                         (const float*)nullptr, w, dy, (float*)nullptr, workspace, (const bf16*)g2, (bf16*)dg2);      \
    break;
    EA_DWB(3) EA_DWB(5) EA_DWB(7) EA_DWB(15) EA_DWB(31)
#undef EA_DWB
  }
  EA_LAUNCH_CHECK();
  if (adj) return ea_reduce_partials_tr(nblkr, (int)rowlen, workspace, rowlen, dw, accumulate_params, C, K, stream);
  int rc = ea_reduce_partials_tr(nblkr, C * K, workspace, rowlen, dw, accumulate_params, C, K, stream);
  if (rc) return rc;
  return ea_reduce_partials(nblkr, C, workspace + (long)C * K, rowlen, dbias, accumulate_params, stream);
}


extern "C" int ea_add_pos_bias(long N, int H, int dk, const void* q, long ldq, const float* u, const float* v,
                               void* qu, void* qv, int dtype, void* stream) {
  EA_ENTRY();
  const long n = N * H * dk;
  if (dtype == EA_BF16)
    hipLaunchKernelGGL(add_pos_bias_kernel<bf16>, EA_GRID(n), N, H, dk, (const bf16*)q, ldq, u, v, (bf16*)qu, (bf16*)qv);
  else
    hipLaunchKernelGGL(add_pos_bias_kernel<float>, EA_GRID(n), N, H, dk, (const float*)q, ldq, u, v, (float*)qu, (float*)qv);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_embed_fwd(long rows, int d, int L, const long long* tok, const float* E, float xscale,
                            const float* pe, float p, unsigned long long seed, float* y, void* stream) {
  EA_ENTRY();
  const long n = rows * d;
  hipLaunchKernelGGL(embed_fwd_kernel, EA_GRID(n), rows, d, L, tok, E, xscale, pe, p, (uint64_t)seed, ea_g_rng_salt, y);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_add_pe_dropout(long rows, int d, int L, const float* pe, float p, unsigned long long seed,
                                 float* y, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(rows >= 0 && d > 0 && L > 0);
  const long n = rows * d;
  if (n == 0) return 0;
  hipLaunchKernelGGL(add_pe_dropout_kernel, EA_GRID(n), n, d, L, pe, p, (uint64_t)seed, ea_g_rng_salt, y);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_embed_bwd(long rows, int d, const long long* tok, const float* dy, float xscale, float p,
                            unsigned long long seed, float* dE, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(rows >= 0 && rows <= EMBED_BWD_MAXROWS);
  if (rows == 0) return 0;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, (int)rows, d, tok,
                     dy, xscale, p, (uint64_t)seed, ea_g_rng_salt, dE);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_argmax_rows(long rows, int V, const float* x, long ld, long long* out, void* stream) {
  EA_ENTRY();
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(ea_cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, rows, V, x, ld, out);
  EA_LAUNCH_CHECK();
  return 0;
}

static PhaseGeo phase_geo(int B, int T1, int F1, int C) {
  PhaseGeo g;
  g.T1 = T1; g.F1 = F1;
  g.nI0 = (T1 + 1) / 2; g.nI1 = T1 / 2; g.nJ0 = (F1 + 1) / 2; g.nJ1 = F1 / 2;
  // plane offsets in ROWS (pixels); callers scale by C
  g.plane[0] = 0;
  g.plane[1] = (long)B * g.nI0 * g.nJ0;
  g.plane[2] = g.plane[1] + (long)B * g.nI0 * g.nJ1;
  g.plane[3] = g.plane[2] + (long)B * g.nI1 * g.nJ0;
  return g;
}

extern "C" int ea_conv1_fwd2(int B, int T, int F, int C, const float* x, const float* w, const float* bias,
                             void* x1p, int dtype, unsigned char* pos, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(C % 8 == 0 && 256 % (C / 8) == 0 && T >= 3 && F >= 3);
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  const PhaseGeo g = phase_geo(B, T1, F1, C);
  const long npix = (long)B * T1 * F1;
  if ((C == 512 || C == 1024 || C == 2048) && (long)B * T1 < (1L << 31)) {
    // one resident wave of blocks: each loads its 80 weights per lane once and walks rows
    static int resident = 0;
    if (!resident) {
      int per_cu = 0, dev = 0, ncu = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv1_fwd_rows_kernel<bf16, true>, 256, 0);
      resident = std::max(1, per_cu) * std::max(1, ncu);
    }
    dim3 grid((unsigned)std::min<long>((long)B * T1, resident));
    // streaming stores (the 0.6 GB output exceeds L2 + MALL): 210 -> 168 us at the C3 shape
    if (dtype == EA_BF16)
      hipLaunchKernelGGL((conv1_fwd_rows_kernel<bf16, true>), grid, dim3(256), 0, (hipStream_t)stream, B, T, F, g, C,
                         x, w, bias, (bf16*)x1p, pos);
    else
      hipLaunchKernelGGL((conv1_fwd_rows_kernel<float, false>), grid, dim3(256), 0, (hipStream_t)stream, B, T, F, g, C, x, w,
                         bias, (float*)x1p, pos);
    EA_LAUNCH_CHECK();
    return 0;
  }
  const int ppb = 256 / (C / 8);
  dim3 grid(ea_grid_cap(ea_cdiv(npix, ppb), 4096));
  if (dtype == EA_BF16)
    hipLaunchKernelGGL(conv1_fwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, B, T, F, g, C, x, w, bias,
                       (bf16*)x1p, pos);
  else
    hipLaunchKernelGGL(conv1_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, B, T, F, g, C, x, w, bias,
                       (float*)x1p, pos);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_conv1_fwd(int B, int T, int F, int C, const float* x, const float* w, const float* bias,
                            void* x1p, int dtype, void* stream) {
  return ea_conv1_fwd2(B, T, F, C, x, w, bias, x1p, dtype, nullptr, stream);
}

extern "C" int ea_conv1_wgrad(int B, int T, int F, int C, const float* x, const void* dh, int dtype, float* dw,
                              float* dbias, float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(C % 8 == 0 && 256 % (C / 8) == 0 && T >= 3 && F >= 3);
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  const PhaseGeo g = phase_geo(B, T1, F1, C);
  const long npix = (long)B * T1 * F1;
  const int ppb = 256 / (C / 8);
  int nb = ea_grid_cap(ea_cdiv(npix, ppb * 16), 1024);
  if ((long)nb > ws_elems / (10L * C)) nb = (int)(ws_elems / (10L * C));
  EA_CHECK_ARG(nb >= 1);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == EA_BF16)
    hipLaunchKernelGGL(conv1_wgrad_kernel<bf16>, dim3(nb), dim3(256), 0, st, B, T, F, g, C, x, (const bf16*)dh, workspace);
  else
    hipLaunchKernelGGL(conv1_wgrad_kernel<float>, dim3(nb), dim3(256), 0, st, B, T, F, g, C, x, (const float*)dh,
                       workspace);
  EA_LAUNCH_CHECK();
  // weight: partial column t*C + c -> dw[c*9 + t]; bias: columns 9C .. 10C-1
  int rc = ea_reduce_partials_tr(nb, 9 * C, workspace, 10L * C, dw, 1, C, 9, stream);
  if (rc) return rc;
  return ea_reduce_partials(nb, C, workspace + 9L * C, 10L * C, dbias, 1, stream);
}

extern "C" int ea_conv1_wgrad_reduce(int ntiles, int C, const float* part, float* dw, float* dbias, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(ntiles >= 1 && C >= 1 && part && dw && dbias);
  // weight: partial column t*C + c -> dw[c*9 + t]; bias: columns 9C .. 10C-1 (accumulating)
  int rc = ea_reduce_partials_tr(ntiles, 9 * C, part, 10L * C, dw, 1, C, 9, stream);
  if (rc) return rc;
  return ea_reduce_partials(ntiles, C, part + 9L * C, 10L * C, dbias, 1, stream);
}

// ------------------------------------------------------------------ ReLU (f32, in place)
// The ReLU of the legacy Encoder's "linear" input layer (Linear -> LayerNorm -> Dropout -> ReLU,
// espnet/nets/pytorch_backend/transformer/encoder.py:120-127) used by TransformerLM.
namespace {
__global__ void relu_inplace_kernel(long n, float* __restrict__ x) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n / 4; i += (long)gridDim.x * blockDim.x) {
    float4 v = ((float4*)x)[i];
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    ((float4*)x)[i] = v;
  }
  for (long i = (n / 4) * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = fmaxf(x[i], 0.f);
}
}  // namespace

extern "C" int ea_relu_f32_inplace(long n, float* x, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 0 && (n == 0 || (x && (uintptr_t)x % 16 == 0)));
  if (n == 0) return 0;
  hipLaunchKernelGGL(relu_inplace_kernel, dim3(ea_grid_cap(ea_cdiv(n / 4 + 1, 256), 4096)), dim3(256), 0,
                     (hipStream_t)stream, n, x);
  EA_LAUNCH_CHECK();
  return 0;
}
