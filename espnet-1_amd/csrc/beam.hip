// Beam-search selection on the device for joint CTC/attention decoding (SURVEY.md §8(f)
// row 4): espnet/nets/batch_beam_search.py:81-101 (batch_beam: global top-k over the
// flattened (n_hyps x vocab) weighted scores) and the pre-beam of :170-182 (top-k of the
// weighted full scores per hypothesis, <eos> always CTC-scored: ctc_prefix_score.py:178-179).
//
// The reference builds the (n_hyps, V) weighted-score matrix on the host every step.  Here
// the decoder's log-probabilities stay in HBM: ea_beam_prebeam writes each hypothesis's
// pre-beam candidates straight into the CTC prefix kernel's metadata, and ea_beam_select
// combines decoder, length-bonus, CTC prefix and running scores for those candidates only
// (every other (hypothesis, token) pair carries the CTC score logzero - prefix, about
// -1e10: it can be chosen only when fewer than `beam` candidates exist, which the pre-beam
// rules out), picks the new beam and writes the next step's CTC metadata (last labels,
// forward-variable row pointers, prefix scores) and running scores.  One small record per
// chosen hypothesis goes back to the host.
//
// Arithmetic follows the reference's float32 tensor ops term by term (no contraction):
//   W = w_dec * logp (+ w_lb)          weighted full scores (scorer sum order is immaterial
//                                      for two terms)
//   ctc = psi - prefix                  CTC prefix score increment (scorers/ctc.py:76-79)
//   W = (W + w_ctc * ctc) + score       batch_beam_search.py:190-205
// Ties in a top-k break toward the lower index.
#include "common.h"

namespace {

struct Best {
  float v;
  int i;  // index; ties -> lower index
};

EA_DEV bool better(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi) || (bv != bv && av == av);  // NaN loses
}

template <int NT>
EA_DEV Best block_argmax(Best b, Best* red) {
  // wave level
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(b.v, o);
    const int oi = __shfl_xor(b.i, o);
    if (better(ov, oi, b.v, b.i)) { b.v = ov; b.i = oi; }
  }
  constexpr int NW = NT / 64;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[w] = b;
  __syncthreads();
  if (w == 0) {
    b = lane < NW ? red[lane] : Best{-INFINITY, 0x7fffffff};
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(b.v, o);
      const int oi = __shfl_xor(b.i, o);
      if (better(ov, oi, b.v, b.i)) { b.v = ov; b.i = oi; }
    }
    if (lane == 0) red[NW] = b;
  }
  __syncthreads();
  b = red[NW];
  __syncthreads();
  return b;
}

// one block per hypothesis: the P best tokens of W = w_dec*logp (+ w_lb), descending, then
// <eos>; written at cand[h*(P+1) ...].  Two levels under the total order (value desc, token
// asc): each wave takes the top P of its slice of the vocabulary (its lane values stay in
// registers, P argmax rounds by shuffles), then wave 0 takes the top P of the waves' lists.
constexpr int PB_NT = 1024, PB_NW = PB_NT / 64, PB_PER = 32;  // <= 32 tokens per lane: V <= 32768 (PER
                                                                // per instantiation: 8, 16 or 32)
constexpr int PB_PMAX = 64;

EA_DEV Best wave_argmax(Best b) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(b.v, o);
    const int oi = __shfl_xor(b.i, o);
    if (better(ov, oi, b.v, b.i)) { b.v = ov; b.i = oi; }
  }
  return b;
}

template <int PER>
__global__ __launch_bounds__(PB_NT) void prebeam_kernel(int V, const float* __restrict__ logp, long ld, float w_dec,
                                                        float w_lb, int use_lb, int P, int eos, int* __restrict__ cand) {
  __shared__ Best lst[PB_NW * PB_PMAX];
  const int h = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* row = logp + (long)h * ld;
  const int span = (V + PB_NW - 1) / PB_NW, v0 = wv * span, v1 = min(V, v0 + span);
  float val[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int v = v0 + e * 64 + lane;
    float wvv = -INFINITY;
    if (v < v1) {
      wvv = __fmul_rn(w_dec, row[v]);
      if (use_lb) wvv = __fadd_rn(wvv, w_lb);
    }
    val[e] = wvv;
  }
  uint32_t taken = 0u;
  for (int r = 0; r < P; ++r) {
    Best b{-INFINITY, 0x7fffffff};
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int v = v0 + e * 64 + lane;
      if (v < v1 && !((taken >> e) & 1u) && better(val[e], v, b.v, b.i)) { b.v = val[e]; b.i = v; }
    }
    b = wave_argmax(b);
    if (b.i != 0x7fffffff && b.i >= v0 && b.i < v1 && (b.i - v0) % 64 == lane) taken |= 1u << ((b.i - v0) / 64);
    if (lane == 0) lst[wv * PB_PMAX + r] = b;
  }
  __syncthreads();
  if (wv == 0) {  // (wave 0 alone: a chosen entry is retired in place)
    const int nl = PB_NW * P;
    int* out = cand + (long)h * (P + 1);
    for (int r = 0; r < P; ++r) {
      Best b{-INFINITY, 0x7fffffff};
      int at = -1;
      for (int q = lane; q < nl; q += 64) {
        const Best c = lst[(q / P) * PB_PMAX + (q % P)];
        if (c.i != 0x7fffffff && better(c.v, c.i, b.v, b.i)) {
          b = c;
          at = (q / P) * PB_PMAX + (q % P);
        }
      }
      const Best m = wave_argmax(b);
      if (at >= 0 && m.i == b.i) lst[at].i = 0x7fffffff;  // each token is in one list, once
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) out[r] = m.i;
    }
    if (lane == 0) out[P] = eos;
  }
}

// the new beam over the n*(P+1) candidates (duplicates of <eos> skipped).  Outputs:
//   rec_i[b*4 + {0,1,2,3}] = parent hypothesis, token, candidate column, 0
//   rec_f[b*4 + {0,1,2,3}] = weighted score, decoder log-prob, CTC increment, CTC prefix psi
//   next step: last[b] = token, rptr[b] = &r_new[(h*(P+1)+col)*T*2], prefix[b] = psi,
//   score[b] = weighted score (all already in the new hypothesis order)
constexpr int SEL_NT = 1024;
__global__ __launch_bounds__(SEL_NT) void select_kernel(int n, int V, int P, int beam, int T, const float* __restrict__ logp,
                                                        long ld, const int* __restrict__ cand,
                                                        const float* __restrict__ psi, const float* __restrict__ prefix,
                                                        const float* __restrict__ score, float w_dec, float w_lb,
                                                        int use_lb, float w_ctc, const float* r_new, int* __restrict__ rec_i,
                                                        float* __restrict__ rec_f, int* __restrict__ last_next,
                                                        unsigned long long* __restrict__ rptr_next,
                                                        float* __restrict__ prefix_next, float* __restrict__ score_next) {
  __shared__ Best red[SEL_NT / 64 + 1];
  __shared__ float wsc[4096];
  const int nc = n * (P + 1);
  for (int c = threadIdx.x; c < nc; c += SEL_NT) {
    const int h = c / (P + 1), k = c - h * (P + 1);
    const int j = cand[c];
    bool dup = false;
    if (k == P)
      for (int q = 0; q < P; ++q) dup |= cand[h * (P + 1) + q] == j;
    float wv = __fmul_rn(w_dec, logp[(long)h * ld + j]);
    if (use_lb) wv = __fadd_rn(wv, w_lb);
    const float inc = __fsub_rn(psi[c], prefix[h]);
    wv = __fadd_rn(__fadd_rn(wv, __fmul_rn(w_ctc, inc)), score[h]);
    wsc[c] = dup ? -INFINITY : wv;
  }
  __syncthreads();
  for (int b = 0; b < beam; ++b) {
    Best best{-INFINITY, 0x7fffffff};
    for (int c = threadIdx.x; c < nc; c += SEL_NT) {
      const int h = c / (P + 1);
      const int flat = h * V + cand[c];  // the reference's index into the flattened scores
      if (wsc[c] != -INFINITY && better(wsc[c], flat, best.v, best.i)) { best.v = wsc[c]; best.i = flat; }
    }
    best = block_argmax<SEL_NT>(best, red);
    if (threadIdx.x == 0) {
      // locate the candidate column again (first occurrence of the token in the row)
      const int h = best.i == 0x7fffffff ? 0 : best.i / V, j = best.i == 0x7fffffff ? cand[0] : best.i - h * V;
      int k = 0;
      while (k < P + 1 && cand[h * (P + 1) + k] != j) ++k;
      if (k == P + 1) k = 0;
      const int c = h * (P + 1) + k;
      const float dec = logp[(long)h * ld + j];
      const float inc = __fsub_rn(psi[c], prefix[h]);
      rec_i[b * 4 + 0] = h; rec_i[b * 4 + 1] = j; rec_i[b * 4 + 2] = k; rec_i[b * 4 + 3] = best.i == 0x7fffffff;
      rec_f[b * 4 + 0] = best.v; rec_f[b * 4 + 1] = dec; rec_f[b * 4 + 2] = inc; rec_f[b * 4 + 3] = psi[c];
      last_next[b] = j;
      rptr_next[b] = (unsigned long long)(uintptr_t)(r_new + (long)c * T * 2);
      prefix_next[b] = psi[c];
      score_next[b] = best.v;
      wsc[c] = -INFINITY;  // taken
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int ea_beam_prebeam(int n, int V, const float* logp, long ld, float w_dec, float w_lb, int use_lb, int P,
                               int eos, int* cand, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 0 && V >= 1 && ld >= V && P >= 1 && P < V && P <= PB_PMAX && V <= PB_PER * PB_NT && eos >= 0 &&
               eos < V);
  if (n == 0) return 0;
  const int per = ((V + PB_NW - 1) / PB_NW + 63) / 64;  // tokens per lane
  if (per <= 8)
    hipLaunchKernelGGL(prebeam_kernel<8>, dim3(n), dim3(PB_NT), 0, (hipStream_t)stream, V, logp, ld, w_dec, w_lb,
                       use_lb, P, eos, cand);
  else if (per <= 16)
    hipLaunchKernelGGL(prebeam_kernel<16>, dim3(n), dim3(PB_NT), 0, (hipStream_t)stream, V, logp, ld, w_dec, w_lb,
                       use_lb, P, eos, cand);
  else
    hipLaunchKernelGGL(prebeam_kernel<32>, dim3(n), dim3(PB_NT), 0, (hipStream_t)stream, V, logp, ld, w_dec, w_lb,
                       use_lb, P, eos, cand);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_beam_select(int n, int V, int P, int beam, int T, const float* logp, long ld, const int* cand,
                              const float* psi, const float* prefix, const float* score, float w_dec, float w_lb,
                              int use_lb, float w_ctc, const float* r_new, int* rec_i, float* rec_f, int* last_next,
                              unsigned long long* rptr_next, float* prefix_next, float* score_next, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 1 && V >= 1 && ld >= V && P >= 1 && beam >= 1 && T >= 1 && n * (P + 1) <= 4096 &&
               beam <= n * (P + 1));
  hipLaunchKernelGGL(select_kernel, dim3(1), dim3(SEL_NT), 0, (hipStream_t)stream, n, V, P, beam, T, logp, ld, cand,
                     psi, prefix, score, w_dec, w_lb, use_lb, w_ctc, r_new, rec_i, rec_f, last_next, rptr_next,
                     prefix_next, score_next);
  EA_LAUNCH_CHECK();
  return 0;
}
