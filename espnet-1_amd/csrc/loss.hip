// Losses of the hybrid CTC/attention objective (espnet2/asr/espnet_model.py:320-325):
//  * CTC (espnet2/asr/ctc.py:52-97, builtin = torch CTCLoss(reduction=none,
//    zero_infinity=True, blank=0) on log_softmax, then sum / B): row log-sum-exp,
//    alpha/beta lattice in log space (fp64, one workgroup per utterance, states across
//    threads, the previous time step in LDS), and a fused gradient w.r.t. the logits
//    (softmax - occupancy), i.e. CTCLoss backward composed with log_softmax backward.
//  * LabelSmoothingLoss (transformer/label_smoothing_loss.py:41-63: KLDiv(reduction=none)
//    vs the smoothed target, ignore_id rows zeroed, sum / (B or #tokens)) fused with
//    th_accuracy (nets_utils.py:304-324) and its gradient.
#include "common.h"

namespace {

// ---------------------------------------------------------------- row reductions
// One 256-thread block per logits row (V ~ 5000 f32 = 20 KB): the max (and, for the
// label-smoothing loss, its first index and the f64 row sum), then the f64 sum of
// exp(x - max).  16-B loads when the row is 16-B aligned; the second pass re-reads the
// row from L2.  Partial results combine in a fixed order (deterministic).
struct RowRed { float mx; int am; double sx, se; };

template <bool LSM>
EA_DEV RowRed row_reduce(const float* __restrict__ xr, int V) {
  __shared__ float s_m[4];
  __shared__ int s_i[4];
  __shared__ double s_x[4], s_e[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V4 = ((uintptr_t)xr & 15) == 0 ? V >> 2 : 0;
  const float4* x4 = (const float4*)xr;
  float mx = -INFINITY;
  int am = 0x7fffffff;
  double sx = 0.0;
  auto take = [&](float t, int v) {
    if (t > mx || (t == mx && v < am)) { mx = t; am = v; }
    if (LSM) sx += (double)t;
  };
  for (int i = tid; i < V4; i += 256) {
    const float4 q = x4[i];
    take(q.x, 4 * i); take(q.y, 4 * i + 1); take(q.z, 4 * i + 2); take(q.w, 4 * i + 3);
  }
  for (int v = 4 * V4 + tid; v < V; v += 256) take(xr[v], v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oi = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oi < am)) { mx = om; am = oi; }
  }
  if (LSM) sx = wave_sum_d(sx);
  if (lane == 0) { s_m[w] = mx; s_i[w] = am; s_x[w] = sx; }
  __syncthreads();
  RowRed r{s_m[0], s_i[0], s_x[0], 0.0};
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    if (s_m[k] > r.mx || (s_m[k] == r.mx && s_i[k] < r.am)) { r.mx = s_m[k]; r.am = s_i[k]; }
    r.sx += s_x[k];
  }
  double se = 0.0;
  for (int i = tid; i < V4; i += 256) {
    const float4 q = x4[i];
    se += (double)(__expf(q.x - r.mx) + __expf(q.y - r.mx)) + (double)(__expf(q.z - r.mx) + __expf(q.w - r.mx));
  }
  for (int v = 4 * V4 + tid; v < V; v += 256) se += (double)__expf(xr[v] - r.mx);
  se = wave_sum_d(se);
  if (lane == 0) s_e[w] = se;
  __syncthreads();
  r.se = (s_e[0] + s_e[1]) + (s_e[2] + s_e[3]);
  return r;
}

__global__ __launch_bounds__(256) void lse_rows_kernel(long rows, int V, const float* __restrict__ x, long ld,
                                                       float* __restrict__ lse) {
  const long r = blockIdx.x;
  const RowRed s = row_reduce<false>(x + r * ld, V);
  if (threadIdx.x == 0) lse[r] = s.mx + (float)log(s.se);
}

EA_DEV double lae(double a, double b) {  // log(exp a + exp b)
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const double m = fmax(a, b);
  return m + log(exp(a - m) + exp(b - m));
}

struct CtcP {
  int B, T, V, Lmax, Smax;
  const float* logits; long ldt;     // row (b,t) at (b*T + t)*ldt
  const float* lse;                  // [B*T]
  const long long* hlens;            // [B]
  const long long* ys; long ldys;    // [B][ldys]
  const long long* ylens;
  double* alpha; double* beta;       // [B][T][Smax]
  double* nll;                       // [B]
  float* loss_utt;                   // [B]  (0 for infeasible, zero_infinity)
};

EA_DEV int ctc_label(const CtcP& p, int b, int s) {
  return (s & 1) ? (int)p.ys[(long)b * p.ldys + (s >> 1)] : 0;
}
EA_DEV double ctc_lp(const CtcP& p, int b, int t, int lab) {
  const long row = (long)b * p.T + t;
  return (double)p.logits[row * p.ldt + lab] - (double)p.lse[row];
}

__global__ __launch_bounds__(256) void ctc_lattice_kernel(CtcP p) {
  extern __shared__ double sh[];  // 2 x Smax
  const int b = blockIdx.x;
  const int Tb = (int)min((long long)p.T, p.hlens[b]);
  const int L = (int)p.ylens[b];
  const int S = 2 * L + 1;
  double* prev = sh;
  double* cur = sh + p.Smax;
  double* A = p.alpha + (long)b * p.T * p.Smax;
  double* Bt = p.beta + (long)b * p.T * p.Smax;
  if (Tb <= 0) {
    if (threadIdx.x == 0) { p.nll[b] = (L == 0) ? 0.0 : INFINITY; p.loss_utt[b] = 0.f; }
    return;
  }
  // ---- alpha
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    double a = -INFINITY;
    if (s < 2) a = ctc_lp(p, b, 0, ctc_label(p, b, s));
    prev[s] = a;
    A[s] = a;
  }
  __syncthreads();
  for (int t = 1; t < Tb; ++t) {
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const int lab = ctc_label(p, b, s);
      double a = prev[s];
      if (s >= 1) a = lae(a, prev[s - 1]);
      if (s >= 2 && lab != 0 && lab != ctc_label(p, b, s - 2)) a = lae(a, prev[s - 2]);
      a = a == -INFINITY ? a : a + ctc_lp(p, b, t, lab);
      cur[s] = a;
      A[(long)t * p.Smax + s] = a;
    }
    __syncthreads();
    double* tmp = prev; prev = cur; cur = tmp;
  }
  // nll
  __shared__ double ll;
  if (threadIdx.x == 0) {
    double l = prev[S - 1];
    if (S >= 2) l = lae(l, prev[S - 2]);
    ll = -l;
    p.nll[b] = -l;
    p.loss_utt[b] = isinf(-l) ? 0.f : (float)(-l);  // zero_infinity
  }
  __syncthreads();
  // ---- beta
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    double v = -INFINITY;
    if (s >= S - 2) v = ctc_lp(p, b, Tb - 1, ctc_label(p, b, s));
    prev[s] = v;
    Bt[(long)(Tb - 1) * p.Smax + s] = v;
  }
  __syncthreads();
  for (int t = Tb - 2; t >= 0; --t) {
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      const int lab = ctc_label(p, b, s);
      double v = prev[s];
      if (s + 1 < S) v = lae(v, prev[s + 1]);
      if (s + 2 < S && lab != 0 && lab != ctc_label(p, b, s + 2)) v = lae(v, prev[s + 2]);
      v = v == -INFINITY ? v : v + ctc_lp(p, b, t, lab);
      cur[s] = v;
      Bt[(long)t * p.Smax + s] = v;
    }
    __syncthreads();
    double* tmp = prev; prev = cur; cur = tmp;
  }
}

// Same recursion as ctc_lattice_kernel (identical arithmetic, bit-identical results), with
// the serial chain's global loads taken off it: alpha and beta run in two workgroups of
// their own (blockIdx.x = 2b + dir), each state's label / skip rule lives in registers, and
// the emissions (logit of the state's label, row lse) for time steps are staged through LDS
// in chunks of CTC_TC steps, the next chunk's loads in flight while the current chunk's
// steps run.  One state per thread: S = 2L+1 <= 256; longer label sequences take the
// one-workgroup kernel above.
constexpr int CTC_TC = 32, CTC_NR = 16;  // steps per chunk; staged values per thread

__global__ __launch_bounds__(256) void ctc_lattice2_kernel(CtcP p) {
  extern __shared__ double sh[];
  const int b = blockIdx.x >> 1, dir = blockIdx.x & 1, tid = threadIdx.x;
  const int Tb = (int)min((long long)p.T, p.hlens[b]);
  const int L = (int)p.ylens[b];
  const int S = 2 * L + 1, U = p.Lmax + 1;
  double* prev = sh;
  double* cur = sh + 256;
  float* em = (float*)(sh + 512);   // [2][CTC_TC][U] logit of unique label u at step k
  float* ls = em + 2 * CTC_TC * U;  // [2][CTC_TC]    row lse at step k
  double* out = (dir ? p.beta : p.alpha) + (long)b * p.T * p.Smax;
  if (Tb <= 0) {
    if (dir == 0 && tid == 0) { p.nll[b] = (L == 0) ? 0.0 : INFINITY; p.loss_utt[b] = 0.f; }
    return;
  }
  const long long* ys = p.ys + (long)b * p.ldys;
  // this thread's state: unique-label index u (0 = blank), label, skip transition allowed
  const int s = tid;
  const int u = (s & 1) ? (s + 1) >> 1 : 0;
  const int lab = s < S ? ((s & 1) ? (int)ys[s >> 1] : 0) : 0;
  const int s2 = dir ? s + 2 : s - 2;  // skip source state
  const bool skip = s < S && s2 >= 0 && s2 < S && lab != 0 && lab != ((s2 & 1) ? (int)ys[s2 >> 1] : 0);
  const int s1 = dir ? s + 1 : s - 1;
  const bool step1 = s < S && s1 >= 0 && s1 < S;
  auto tmap = [&](int k) { return dir ? Tb - 1 - k : k; };
  // staged element e of a chunk: e < CTC_TC*U -> (kk = e / U, uu = e % U) logit; else lse of kk
  const int NE = CTC_TC * U + CTC_TC;
  auto fetch = [&](int k0, float (&r)[CTC_NR]) {
#pragma unroll
    for (int i = 0; i < CTC_NR; ++i) {
      const int e = tid + 256 * i;
      float v = 0.f;
      if (e < NE) {
        const int kk = e < CTC_TC * U ? e / U : e - CTC_TC * U;
        const int k = k0 + kk;
        if (k < Tb) {
          const long row = (long)b * p.T + tmap(k);
          if (e < CTC_TC * U) {
            const int uu = e - kk * U;
            const int lb = uu == 0 ? 0 : (uu <= L ? (int)ys[uu - 1] : 0);
            v = p.logits[row * p.ldt + lb];
          } else {
            v = p.lse[row];
          }
        }
      }
      r[i] = v;
    }
  };
  auto stash = [&](int buf, const float (&r)[CTC_NR]) {
#pragma unroll
    for (int i = 0; i < CTC_NR; ++i) {
      const int e = tid + 256 * i;
      if (e < CTC_TC * U) em[buf * CTC_TC * U + e] = r[i];
      else if (e < NE) ls[buf * CTC_TC + e - CTC_TC * U] = r[i];
    }
  };
  float r[CTC_NR];
  fetch(0, r);
  stash(0, r);
  __syncthreads();
  const int nchunk = (Tb + CTC_TC - 1) / CTC_TC;
  for (int c = 0; c < nchunk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunk) fetch((c + 1) * CTC_TC, r);  // in flight under this chunk's steps
    const float* emc = em + buf * CTC_TC * U;
    const float* lsc = ls + buf * CTC_TC;
    const int kend = min(CTC_TC, Tb - c * CTC_TC);
    for (int kk = 0; kk < kend; ++kk) {
      const int k = c * CTC_TC + kk, t = tmap(k);
      const double lp = (double)emc[kk * U + u] - (double)lsc[kk];
      double a;
      if (k == 0) {
        a = -INFINITY;
        if (s < S && (dir ? s >= S - 2 : s < 2)) a = lp;
      } else {
        a = prev[s];
        if (step1) a = lae(a, prev[s1]);
        if (skip) a = lae(a, prev[s2]);
        a = a == -INFINITY ? a : a + lp;
      }
      if (s < S) {
        cur[s] = a;
        out[(long)t * p.Smax + s] = a;
      }
      __syncthreads();
      double* tmp = prev; prev = cur; cur = tmp;
    }
    if (c + 1 < nchunk) stash(buf ^ 1, r);
    __syncthreads();
  }
  if (dir == 0 && tid == 0) {
    double l = prev[S - 1];
    if (S >= 2) l = lae(l, prev[S - 2]);
    p.nll[b] = -l;
    p.loss_utt[b] = isinf(-l) ? 0.f : (float)(-l);  // zero_infinity
  }
}

// loss = sum_b loss_utt / B  (ctc.py:58-60); one block
__global__ void ctc_reduce_kernel(int B, const float* __restrict__ loss_utt, float* __restrict__ loss) {
  __shared__ double red[16];
  double a = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) a += loss_utt[b];
  a = block_sum_d(a, red);
  if (threadIdx.x == 0) loss[0] = (float)(a / B);
}

// grad[b,t,v] = g_b * (softmax(x)[v] - sum_{s: l'(s)=v} exp(alpha+beta+nll-lp))
// One block per (b, t) row.  The occupancies of the row's <= L+1 distinct labels go to a small
// LDS table; one vectorized pass writes g*softmax for every column, then (after a barrier) the
// label columns are rewritten with the same expression including their occupancy — the values
// are those of a single pass with a V-wide occupancy array.
template <typename TO>
__global__ __launch_bounds__(256) void ctc_grad_kernel(CtcP p, const float* __restrict__ gscale, float coef,
                                                       TO* __restrict__ grad, long ldg) {
  extern __shared__ float occ_tab[];  // [Lmax] label occupancy, then [Lmax] int label (or -1)
  int* lab_tab = (int*)(occ_tab + p.Lmax);
  const long row = blockIdx.x;
  const int b = (int)(row / p.T), t = (int)(row % p.T);
  const int Tb = (int)min((long long)p.T, p.hlens[b]);
  const double nll = p.nll[b];
  TO* gr = grad + row * ldg;
  const bool vec = (p.V % 4 == 0) && (p.ldt % 4 == 0) && (ldg % 4 == 0);
  if (t >= Tb || isinf(nll) || isnan(nll)) {
    if (vec) {
      const float z4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int v = threadIdx.x * 4; v < p.V; v += blockDim.x * 4) vst4(gr + v, z4);
    } else {
      for (int v = threadIdx.x; v < p.V; v += blockDim.x) gr[v] = from_f<TO>(0.f);
    }
    return;
  }
  __shared__ double red[16];
  const int L = (int)p.ylens[b];
  const int S = 2 * L + 1;
  const double* A = p.alpha + ((long)b * p.T + t) * p.Smax;
  const double* Bt = p.beta + ((long)b * p.T + t) * p.Smax;
  // occupancy per label, summed in a fixed order (no atomics: bit-reproducible):
  // blank (every even s) by a block reduction; a label at odd s by the thread owning its
  // first occurrence, over all its occurrences in increasing s
  auto occ = [&](int s, int lab) -> double {
    const double ab = A[s] + Bt[s];
    return ab != -INFINITY ? exp(ab + nll - ctc_lp(p, b, t, lab)) : 0.0;
  };
  double bsum = 0.0;
  for (int s = 2 * threadIdx.x; s < S; s += 2 * blockDim.x) bsum += occ(s, 0);
  bsum = block_sum_d(bsum, red);
  for (int s = 2 * threadIdx.x + 1; s < S; s += 2 * blockDim.x) {
    const int lab = ctc_label(p, b, s);
    bool first = true;
    for (int q = 1; q < s; q += 2) first = first && ctc_label(p, b, q) != lab;
    double a = 0.0;
    if (first)
      for (int q = s; q < S; q += 2)
        if (ctc_label(p, b, q) == lab) a += occ(q, lab);
    lab_tab[s >> 1] = first ? lab : -1;
    occ_tab[s >> 1] = (float)a;
  }
  const float g = gscale[0] * coef;
  const float* xr = p.logits + row * p.ldt;
  const float l = p.lse[row];
  if (vec) {
    for (int v = threadIdx.x * 4; v < p.V; v += blockDim.x * 4) {
      const float4 x4 = *(const float4*)(xr + v);
      const float o[4] = {g * __expf(x4.x - l), g * __expf(x4.y - l), g * __expf(x4.z - l), g * __expf(x4.w - l)};
      vst4(gr + v, o);
    }
  } else {
    for (int v = threadIdx.x; v < p.V; v += blockDim.x) gr[v] = from_f<TO>(g * (__expf(xr[v] - l) - 0.f));
  }
  __syncthreads();  // the table is complete; this block's softmax writes are visible
  for (int i = threadIdx.x; i <= L; i += blockDim.x) {
    const int lab = i < L ? lab_tab[i] : 0;  // i == L: the blank
    if (lab < 0) continue;
    const float a = i < L ? occ_tab[i] : (float)bsum;
    gr[lab] = from_f<TO>(g * (__expf(xr[lab] - l) - a));
  }
}

// ---------------------------------------------------------------- label smoothing
struct LsmP {
  long rows; int V;
  const float* x; long ldx;
  const long long* tgt;
  float smoothing; int ignore_id;
  float* lse;          // [rows]
  double* loss_row;    // [rows]
  int* stat;           // [0] correct, [1] valid
};

__global__ __launch_bounds__(256) void lsm_fwd_kernel(LsmP p) {
  const long r = blockIdx.x;
  const float* xr = p.x + r * p.ldx;
  const RowRed s = row_reduce<true>(xr, p.V);
  if (threadIdx.x != 0) return;
  const int am = s.am;
  const double sx = s.sx;
  const double lse = (double)s.mx + log(s.se);
  p.lse[r] = (float)lse;
  const long long t = p.tgt[r];
  if (t == p.ignore_id) { p.loss_row[r] = 0.0; return; }
  // true_dist = eps everywhere, conf at target (label_smoothing_loss.py:55-60), in the
  // logits' dtype (f32) like the reference
  const float epsf = p.smoothing / (p.V - 1);
  const float conf = 1.f - p.smoothing;
  const double eps = epsf, cf = conf;
  const double xt = xr[t];
  const double qlogq = (eps > 0 ? (p.V - 1) * eps * log(eps) : 0.0) + (cf > 0 ? cf * log(cf) : 0.0);
  const double qx = eps * (sx - xt) + cf * xt;
  const double qsum = eps * (p.V - 1) + cf;
  p.loss_row[r] = qlogq - (qx - lse * qsum);
  atomicAdd(&p.stat[1], 1);
  if (am == t) atomicAdd(&p.stat[0], 1);
}

// out[0] = loss = sum rows / denom, out[1] = acc, out[2] = 1/denom
__global__ void lsm_finalize_kernel(long rows, const double* __restrict__ loss_row, const int* __restrict__ stat,
                                    int normalize_length, float batch, float* __restrict__ loss_out,
                                    float* __restrict__ acc_out, float* __restrict__ inv_out) {
  __shared__ double red[16];
  double a = 0.0;
  for (long r = threadIdx.x; r < rows; r += blockDim.x) a += loss_row[r];
  a = block_sum_d(a, red);
  if (threadIdx.x == 0) {
    const double denom = normalize_length ? (double)stat[1] : (double)batch;
    loss_out[0] = (float)(a / denom);
    acc_out[0] = stat[1] > 0 ? (float)((double)stat[0] / (double)stat[1]) : 0.f;
    inv_out[0] = (float)(1.0 / denom);
  }
}

template <typename TO>
__global__ void lsm_bwd_kernel(LsmP p, const float* __restrict__ gscale, const float* __restrict__ coef_dev,
                               float coef, TO* __restrict__ grad, long ldg) {
  const long r = blockIdx.x;
  const long long t = p.tgt[r];
  TO* gr = grad + r * ldg;
  if (t == p.ignore_id) {
    for (int v = threadIdx.x; v < p.V; v += blockDim.x) gr[v] = from_f<TO>(0.f);
    return;
  }
  const float g = gscale[0] * coef_dev[0] * coef;
  const float eps = p.smoothing / (p.V - 1), conf = 1.f - p.smoothing;
  const float* xr = p.x + r * p.ldx;
  const float l = p.lse[r];
  for (int v = threadIdx.x; v < p.V; v += blockDim.x) {
    const float q = v == t ? conf : eps;
    gr[v] = from_f<TO>(g * (__expf(xr[v] - l) - q));
  }
}

}  // namespace

extern "C" int ea_ctc_loss_fwd(int B, int T, int V, const float* logits, long ldt, const long long* hlens,
                               const long long* ys, long ldys, const long long* ylens, int Lmax, float* lse,
                               double* alpha, double* beta, double* nll, float* loss_utt, float* loss,
                               void* stream) {
  EA_ENTRY();
  hipStream_t st = (hipStream_t)stream;
  const long rows = (long)B * T;
  hipLaunchKernelGGL(lse_rows_kernel, dim3(rows), dim3(256), 0, st, rows, V, logits, ldt, lse);
  EA_LAUNCH_CHECK();
  const int Smax = 2 * Lmax + 1;
  CtcP p{B, T, V, Lmax, Smax, logits, ldt, lse, hlens, ys, ldys, ylens, alpha, beta, nll, loss_utt};
  const int U = Lmax + 1;
  if (Smax <= 256 && CTC_TC * U + CTC_TC <= 256 * CTC_NR) {
    const size_t sm = 512 * sizeof(double) + (size_t)2 * CTC_TC * (U + 1) * sizeof(float);
    hipLaunchKernelGGL(ctc_lattice2_kernel, dim3(2 * B), dim3(256), sm, st, p);
  } else {
    hipLaunchKernelGGL(ctc_lattice_kernel, dim3(B), dim3(256), 2 * Smax * sizeof(double), st, p);
  }
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(ctc_reduce_kernel, dim3(1), dim3(256), 0, st, B, loss_utt, loss);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_ctc_loss_bwd(int B, int T, int V, const float* logits, long ldt, const long long* hlens,
                               const long long* ys, long ldys, const long long* ylens, int Lmax, const float* lse,
                               const double* alpha, const double* beta, const double* nll,
                               const float* gscale, float coef, void* grad, int grad_dtype, long ldg,
                               void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(V <= 16384);
  const int Smax = 2 * Lmax + 1;
  CtcP p{B, T, V, Lmax, Smax, logits, ldt, lse, hlens, ys, ldys, ylens, (double*)alpha, (double*)beta,
         (double*)nll, nullptr};
  hipStream_t st = (hipStream_t)stream;
  const size_t sm = (size_t)max(Lmax, 1) * (sizeof(float) + sizeof(int));
  if (grad_dtype == EA_BF16)
    hipLaunchKernelGGL(ctc_grad_kernel<bf16>, dim3((long)B * T), dim3(256), sm, st, p, gscale, coef, (bf16*)grad, ldg);
  else
    hipLaunchKernelGGL(ctc_grad_kernel<float>, dim3((long)B * T), dim3(256), sm, st, p, gscale, coef, (float*)grad, ldg);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_lsm_loss_fwd(long rows, int V, const float* x, long ldx, const long long* tgt, float smoothing,
                               int ignore_id, int normalize_length, float batch, float* lse, double* loss_row,
                               int* stat, float* loss, float* acc, float* inv_denom, void* stream) {
  EA_ENTRY();
  hipStream_t st = (hipStream_t)stream;
  hipMemsetAsync(stat, 0, 2 * sizeof(int), st);
  LsmP p{rows, V, x, ldx, tgt, smoothing, ignore_id, lse, loss_row, stat};
  hipLaunchKernelGGL(lsm_fwd_kernel, dim3(rows), dim3(256), 0, st, p);
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(lsm_finalize_kernel, dim3(1), dim3(256), 0, st, rows, loss_row, stat, normalize_length, batch, loss, acc, inv_denom);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_lsm_loss_bwd(long rows, int V, const float* x, long ldx, const long long* tgt, float smoothing,
                               int ignore_id, const float* lse, const float* gscale, const float* inv_denom,
                               float coef, void* grad, int grad_dtype, long ldg, void* stream) {
  EA_ENTRY();
  LsmP p{rows, V, x, ldx, tgt, smoothing, ignore_id, (float*)lse, nullptr, nullptr};
  hipStream_t st = (hipStream_t)stream;
  if (grad_dtype == EA_BF16)
    hipLaunchKernelGGL(lsm_bwd_kernel<bf16>, dim3(rows), dim3(256), 0, st, p, gscale, inv_denom, coef, (bf16*)grad, ldg);
  else
    hipLaunchKernelGGL(lsm_bwd_kernel<float>, dim3(rows), dim3(256), 0, st, p, gscale, inv_denom, coef, (float*)grad, ldg);
  EA_LAUNCH_CHECK();
  return 0;
}
