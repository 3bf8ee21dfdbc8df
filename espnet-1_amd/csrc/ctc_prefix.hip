// CTC prefix scoring for joint CTC/attention beam search:
// espnet/nets/scorers/ctc.py:10-97 (CTCPrefixScorer) over espnet/nets/ctc_prefix_score.py:272-358
// (CTCPrefixScore, Algorithm 2 of Watanabe et al., "Hybrid CTC/attention architecture").
//
// The reference runs the recursion in numpy on the host, one hypothesis at a time, after
// copying the CTC posteriors off the device.  Here the posteriors stay in HBM and ONE launch
// scores every (running hypothesis, pre-beam candidate) pair of a search step: one thread
// per pair walks the T frames (the recursion is serial in t), reading its hypothesis's
// forward variables r_{t}^{n,b}(g) and writing the candidate's r_t^{n,b}(h) for the next
// step.  Arithmetic is float32 with numpy's logaddexp, as in the reference.
#include "common.h"

namespace {

constexpr float kLogZero = -10000000000.0f;  // ctc_prefix_score.py:283

// numpy npy_logaddexpf (float32)
EA_DEV float np_logaddexpf(float x, float y) {
  if (x == y) return x + 0.693147180559945309417232121458176568f;
  const float tmp = x - y;
  if (tmp > 0.f) return x + log1pf(expf(-tmp));
  if (tmp <= 0.f) return y + log1pf(expf(tmp));
  return tmp;  // NaN
}

// logp[t][v] = log_softmax(logits[t]) (one block per frame), then (block 0, thread 0)
// r0[t] = (logzero, cumulative blank log-prob)  — initial_state(), :289-301
template <bool LOG>
__global__ __launch_bounds__(256) void ctc_softmax_rows_kernel(int V, const float* __restrict__ logits, long ldl,
                                                               float* __restrict__ out) {
  __shared__ float red[256];
  const int t = blockIdx.x;
  const float* row = logits + (long)t * ldl;
  float m = -INFINITY;
  for (int v = threadIdx.x; v < V; v += 256) m = fmaxf(m, row[v]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float acc = 0.f;
  for (int v = threadIdx.x; v < V; v += 256) acc += expf(row[v] - m);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const float lz = m + logf(red[0]);
  for (int v = threadIdx.x; v < V; v += 256) out[(long)t * V + v] = LOG ? row[v] - lz : expf(row[v] - lz);
}

__global__ void ctc_prefix_init_kernel(int T, int V, int blank, const float* __restrict__ logp, float* __restrict__ r0) {
  float acc = 0.f;
  for (int t = 0; t < T; ++t) {
    acc = t == 0 ? logp[blank] : acc + logp[(long)t * V + blank];
    r0[2 * t] = kLogZero;
    r0[2 * t + 1] = acc;
  }
}

// log(exp(x) + exp(y)) for the serial recursion of ctc_prefix_score2, branch-free on the
// hardware base-2 exp / log (v_exp_f32 / v_log_f32, ~1 ulp): max + ln2 * log2(1 + 2^-(|x-y| log2 e)).
// x == y gives x + ln 2 and NaN propagates through x - y, as npy_logaddexpf; for |x - y| > ~17
// the 1 + e rounds to 1 where log1p would keep ~e (absolute error < 6e-8, an ulp of any
// log-probability the recursion carries).  (npy_logaddexpf's branches and the libm log1p chain
// made each frame of the serial loop ~1,000 cycles.)
EA_DEV float lae_fast(float x, float y) {
  const float m = fmaxf(x, y);
  const float e = __builtin_amdgcn_exp2f(-fabsf(x - y) * 1.44269504088896341f);
  return m + 0.693147180559945309f * __builtin_amdgcn_logf(1.f + e);
}

// one thread per (hypothesis h, candidate c): __call__ (:303-358)
// ol_arr: per-hypothesis output lengths, or NULL when every hypothesis has ol_uniform
__global__ __launch_bounds__(64) void ctc_prefix_score_kernel(int T, int V, int blank, int eos, int n_hyp,
                                                              int n_cand, const float* __restrict__ logp,
                                                              const unsigned long long* __restrict__ r_prev_ptr,
                                                              const int* __restrict__ ol_arr, int ol_uniform,
                                                              const int* __restrict__ last_arr,
                                                              const int* __restrict__ cand_arr, float* __restrict__ log_psi,
                                                              float* __restrict__ r_new, int wstart, int wend) {
  const int idx = blockIdx.x * 64 + threadIdx.x;
  if (idx >= n_hyp * n_cand) return;
  const int h = idx / n_cand;
  const int ol = ol_arr ? ol_arr[h] : ol_uniform;  // output length (prefix without <sos>)
  const int last = last_arr[h];                     // last label of the prefix
  const int c = cand_arr[idx];                      // candidate label
  const float* rp = (const float*)r_prev_ptr[h];
  float* r = r_new + (long)idx * T * 2;
  const bool same = ol > 0 && c == last;  // log_phi = r^b(g) for a repeated label, else r^n + r^b
  // frames [start, end): max(ol, 1) .. T, or the attention window (wstart > 0)
  const int end = wend > 0 ? min(wend, T) : T;
  const int start = min(wstart > 0 ? wstart : max(ol, 1), max(end, 1));
  for (int t = 0; t < T; ++t)
    if (t < start || t >= end) { r[2 * t] = kLogZero; r[2 * t + 1] = kLogZero; }
  if (ol == 0) r[0] = logp[c];
  // r[start-1] (logzero but for the empty prefix's first frame)
  float psi = ol == 0 && start == 1 ? logp[c] : kLogZero;
  float rn = psi, rb = kLogZero;
  // frames in chunks of CH: the chunk's loads (and its log_phi values, which do not depend on
  // the recursion) are issued together, so one memory latency is exposed per chunk instead of
  // one per frame; the serial recursion then runs from registers
  constexpr int CH = 16;
  for (int t0 = start; t0 < end; t0 += CH) {
    float xc[CH], xb[CH], ph[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int t = min(t0 + k, end - 1);
      xc[k] = logp[(long)t * V + c];
      xb[k] = logp[(long)t * V + blank];
      const float a = rp[2 * (t - 1)], b = rp[2 * (t - 1) + 1];
      ph[k] = same ? b : np_logaddexpf(a, b);  // log_phi[t-1]
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int t = t0 + k;
      if (t < end) {
        const float nrn = np_logaddexpf(rn, ph[k]) + xc[k];
        const float nrb = np_logaddexpf(rn, rb) + xb[k];
        psi = np_logaddexpf(psi, ph[k] + xc[k]);
        rn = nrn;
        rb = nrb;
        r[2 * t] = rn;
        r[2 * t + 1] = rb;
      }
    }
  }
  if (c == eos) psi = np_logaddexpf(rp[2 * (T - 1)], rp[2 * (T - 1) + 1]);
  if (c == blank) psi = kLogZero;
  log_psi[idx] = psi;
}

// The same recursion with one workgroup per hypothesis (ctc_prefix_score2): frames move through
// LDS in chunks of CH — every thread of the block gathers the chunk's emissions of all the
// hypothesis's candidates (logp[t][c], logp[t][blank]) and the parent's log_phi, then each
// candidate's thread runs the serial recursion over the chunk from LDS, and the block writes
// the candidate's forward variables back as contiguous rows.  The serial loop touches no
// global memory (the one-thread-per-pair kernel above waited on scattered loads and stores
// every frame); the recursion is the same, in the same order, with lae_fast.
template <int CH>
__global__ __launch_bounds__(256) void ctc_prefix_score2_kernel(int T, int V, int blank, int eos, int n_cand,
                                                                const float* __restrict__ logp,
                                                                const unsigned long long* __restrict__ r_prev_ptr,
                                                                const int* __restrict__ ol_arr, int ol_uniform,
                                                                const int* __restrict__ last_arr,
                                                                const int* __restrict__ cand_arr,
                                                                float* __restrict__ log_psi, float* __restrict__ r_new,
                                                                int wstart, int wend) {
  extern __shared__ float sm[];
  constexpr int XS = CH + 1, RS = 2 * CH + 1;  // padded row strides (bank spread)
  float* phi = sm;               // [CH]: lae(r^n, r^b) of the parent at frame t-1
  float* pb = phi + CH;          // [CH]: r^b of the parent at frame t-1 (repeated label)
  float* xb = pb + CH;           // [CH]: blank emission at frame t
  float* xc = xb + CH;           // [n_cand][XS]: candidate emissions
  float* ro = xc + n_cand * XS;  // [n_cand][RS]: forward variables out
  const int h = blockIdx.x, tid = threadIdx.x;
  const int ol = ol_arr ? ol_arr[h] : ol_uniform;
  const int last = last_arr[h];
  const float* rp = (const float*)r_prev_ptr[h];
  const int* cand = cand_arr + (long)h * n_cand;
  float* rout = r_new + (long)h * n_cand * T * 2;
  // frames [start, end): max(ol, 1) .. T, or the attention window (wstart > 0)
  const int end = wend > 0 ? min(wend, T) : T;
  const int start = min(wstart > 0 ? wstart : max(ol, 1), max(end, 1));
  // frames before start: logzero (r[0] = (logp[c], logzero) for the empty prefix)
  for (int q = tid; q < n_cand * 2 * min(start, T); q += 256) {
    const int k = q / (2 * min(start, T)), e = q - k * 2 * min(start, T);
    rout[(long)k * T * 2 + e] = (ol == 0 && e == 0) ? logp[cand[k]] : kLogZero;
  }
  // frames from end on (a window ending before the utterance): logzero
  for (int q = tid; q < n_cand * 2 * (T - end); q += 256) {
    const int k = q / (2 * (T - end)), e = q - k * 2 * (T - end);
    rout[(long)k * T * 2 + 2 * end + e] = kLogZero;
  }
  const int k = tid;
  const bool act = k < n_cand;
  const int c = act ? cand[k] : 0;
  __shared__ int cl[256];  // the candidates (n_cand <= 256), for the emission gather
  if (act) cl[k] = c;
  const bool same = ol > 0 && c == last;
  // r[start-1] (logzero but for the empty prefix's first frame)
  float psi = act && ol == 0 && start == 1 ? logp[c] : kLogZero;
  float rn = psi, rb = kLogZero;
  for (int t0 = start; t0 < end; t0 += CH) {
    const int nf = min(CH, end - t0);
    __syncthreads();  // the previous chunk's rows are written out
    for (int i = tid; i < nf; i += 256) {
      const int t = t0 + i;
      const float a = rp[2 * (t - 1)], b = rp[2 * (t - 1) + 1];
      phi[i] = np_logaddexpf(a, b);
      pb[i] = b;
      xb[i] = logp[(long)t * V + blank];
    }
    // candidate emissions: scattered 4-B reads (one row of the posteriors per frame), GU of
    // them in flight per thread before any is stored (a load -> store loop ran them serially)
    {
      constexpr int GU = 16;
      const int nq = n_cand * nf;
      for (int q0 = 0; q0 < nq; q0 += 256 * GU) {
        float v[GU];
        int dst[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {  // clamped, unconditional loads: all GU in flight at once
          const int q = min(q0 + tid + 256 * u, nq - 1);
          const int kk = q / nf, i = q - kk * nf;
          dst[u] = kk * XS + i;
          v[u] = logp[(long)(t0 + i) * V + cl[kk]];
        }
#pragma unroll
        for (int u = 0; u < GU; ++u)
          if (q0 + tid + 256 * u < nq) xc[dst[u]] = v[u];
      }
    }
    __syncthreads();
    if (act) {
      const float* xk = xc + k * XS;
      const float* pk = same ? pb : phi;  // log_phi[t-1]
      float* rk = ro + k * RS;
      // next frame's operands loaded one iteration ahead (LDS latency off the serial chain)
      float ph_n = pk[0], x_n = xk[0], xb_n = xb[0];
      for (int i = 0; i < nf; ++i) {
        const float ph = ph_n, x = x_n, xbb = xb_n;
        const int in = i + 1 < nf ? i + 1 : i;
        ph_n = pk[in];
        x_n = xk[in];
        xb_n = xb[in];
        const float nrn = lae_fast(rn, ph) + x;
        const float nrb = lae_fast(rn, rb) + xbb;
        psi = lae_fast(psi, ph + x);
        rn = nrn;
        rb = nrb;
        rk[2 * i] = rn;
        rk[2 * i + 1] = rb;
      }
    }
    __syncthreads();
    for (int q = tid; q < n_cand * 2 * nf; q += 256) {
      const int kk = q / (2 * nf), e = q - kk * 2 * nf;
      rout[(long)kk * T * 2 + 2 * t0 + e] = ro[kk * RS + e];
    }
  }
  if (act) {
    if (c == eos) psi = np_logaddexpf(rp[2 * (T - 1)], rp[2 * (T - 1) + 1]);
    if (c == blank) psi = kLogZero;
    log_psi[(long)h * n_cand + k] = psi;
  }
}

int launch_prefix2(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                   const unsigned long long* r_prev, const int* ol_arr, int ol_uniform, const int* last,
                   const int* cand, float* log_psi, float* r_new, hipStream_t st, int wstart = 0, int wend = 0) {
  auto bytes = [&](int ch) { return (size_t)(3 * ch + n_cand * (ch + 1) + n_cand * (2 * ch + 1)) * 4; };
  if (bytes(256) <= 64 * 1024)
    hipLaunchKernelGGL(ctc_prefix_score2_kernel<256>, dim3(n_hyp), dim3(256), bytes(256), st, T, V, blank, eos, n_cand,
                       logp, r_prev, ol_arr, ol_uniform, last, cand, log_psi, r_new, wstart, wend);
  else if (bytes(64) <= 64 * 1024)
    hipLaunchKernelGGL(ctc_prefix_score2_kernel<64>, dim3(n_hyp), dim3(256), bytes(64), st, T, V, blank, eos, n_cand,
                       logp, r_prev, ol_arr, ol_uniform, last, cand, log_psi, r_new, wstart, wend);
  else
    hipLaunchKernelGGL(ctc_prefix_score_kernel, dim3(ea_cdiv(n_hyp * n_cand, 64)), dim3(64), 0, st, T, V, blank, eos,
                       n_hyp, n_cand, logp, r_prev, ol_arr, ol_uniform, last, cand, log_psi, r_new, wstart, wend);
  return 0;
}

}  // namespace

extern "C" int ea_ctc_prefix_init(int T, int V, const float* logits, long ld_logits, int blank, float* logp,
                                  float* r0, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(T >= 1 && V >= 1 && blank >= 0 && blank < V && ld_logits >= V);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ctc_softmax_rows_kernel<true>, dim3(T), dim3(256), 0, st, V, logits, ld_logits, logp);
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(ctc_prefix_init_kernel, dim3(1), dim3(1), 0, st, T, V, blank, logp, r0);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_softmax_rows(long rows, int V, const float* logits, long ld, float* out, int log, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(rows >= 0 && rows < (1L << 31) && V >= 1 && ld >= V);
  if (rows == 0) return 0;
  if (log)
    hipLaunchKernelGGL(ctc_softmax_rows_kernel<true>, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, V,
                       logits, ld, out);
  else
    hipLaunchKernelGGL(ctc_softmax_rows_kernel<false>, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, V,
                       logits, ld, out);
  EA_LAUNCH_CHECK();
  return 0;
}

static int prefix_score_meta(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                             const unsigned long long* r_prev, const int* meta, float* log_psi, float* r_new,
                             int wstart, int wend, hipStream_t st) {
  if (n_hyp * n_cand == 0) return 0;
  if (n_cand <= 256)
    launch_prefix2(T, V, blank, eos, n_hyp, n_cand, logp, r_prev, meta, 0, meta + n_hyp, meta + 2 * n_hyp, log_psi,
                   r_new, st, wstart, wend);
  else
    hipLaunchKernelGGL(ctc_prefix_score_kernel, dim3(ea_cdiv(n_hyp * n_cand, 64)), dim3(64), 0, st, T, V, blank,
                       eos, n_hyp, n_cand, logp, r_prev, meta, 0, meta + n_hyp, meta + 2 * n_hyp, log_psi, r_new,
                       wstart, wend);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_ctc_prefix_score(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                                   const unsigned long long* r_prev, const int* meta, float* log_psi, float* r_new,
                                   void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(T >= 1 && V >= 1 && n_hyp >= 0 && n_cand >= 0);
  return prefix_score_meta(T, V, blank, eos, n_hyp, n_cand, logp, r_prev, meta, log_psi, r_new, 0, 0,
                           (hipStream_t)stream);
}

extern "C" int ea_ctc_prefix_score_win(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                                       const unsigned long long* r_prev, const int* meta, int start, int end,
                                       float* log_psi, float* r_new, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(T >= 1 && V >= 1 && n_hyp >= 0 && n_cand >= 0 && start >= 1 && end >= 1);
  return prefix_score_meta(T, V, blank, eos, n_hyp, n_cand, logp, r_prev, meta, log_psi, r_new, start, end,
                           (hipStream_t)stream);
}

// streaming: the forward variables of a hypothesis over T_old frames extended to T frames —
// r^n logzero, r^b accumulating the blank emissions in frame order (ctc_prefix_score.py:244-269)
__global__ void ctc_prefix_extend_kernel(int T_old, int T, int V, int blank, const float* __restrict__ logp,
                                         const float* __restrict__ r_old, float* __restrict__ r) {
  for (int t = 0; t < T_old; ++t) { r[2 * t] = r_old[2 * t]; r[2 * t + 1] = r_old[2 * t + 1]; }
  const int start = max(T_old, 1);
  if (T_old == 0) { r[0] = kLogZero; r[1] = kLogZero; }
  float acc = r[2 * (start - 1) + 1];
  for (int t = start; t < T; ++t) {
    acc = acc + logp[(long)t * V + blank];
    r[2 * t] = kLogZero;
    r[2 * t + 1] = acc;
  }
}

extern "C" int ea_ctc_prefix_extend(int T_old, int T, int V, int blank, const float* logp, const float* r_old,
                                    float* r, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(T_old >= 0 && T >= T_old && T >= 1 && V >= 1 && blank >= 0 && blank < V);
  hipLaunchKernelGGL(ctc_prefix_extend_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, T_old, T, V, blank, logp,
                     r_old, r);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_ctc_prefix_score_dev(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                                       const unsigned long long* r_prev, int out_len, const int* last,
                                       const int* cand, float* log_psi, float* r_new, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(T >= 1 && V >= 1 && n_hyp >= 0 && n_cand >= 0 && out_len >= 0);
  if (n_hyp * n_cand == 0) return 0;
  if (n_cand <= 256)
    launch_prefix2(T, V, blank, eos, n_hyp, n_cand, logp, r_prev, nullptr, out_len, last, cand, log_psi, r_new,
                   (hipStream_t)stream);
  else
    hipLaunchKernelGGL(ctc_prefix_score_kernel, dim3(ea_cdiv(n_hyp * n_cand, 64)), dim3(64), 0, (hipStream_t)stream,
                       T, V, blank, eos, n_hyp, n_cand, logp, r_prev, (const int*)nullptr, out_len, last, cand,
                       log_psi, r_new, 0, 0);
  EA_LAUNCH_CHECK();
  return 0;
}
