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

// one block per hypothesis: the P best tokens of W = w_dec*logp (+ w_lb), descending, then
// <eos>; written at cand[h*(P+1) ...].  Two levels under the total order (value desc, token
// asc): each wave takes the top P of its slice of the vocabulary (its lane values stay in
// registers, P argmax rounds by shuffles), then wave 0 takes the top P of the waves' lists.
constexpr int PB_NT = 1024, PB_NW = PB_NT / 64, PB_PER = 32;  // <= 32 tokens per lane: V <= 32768 (PER
                                                                // per instantiation: 8, 16 or 32)
constexpr int PB_PMAX = 64;

// Wave argmax under `better` (a total order, so the combination order is immaterial): DPP
// within each 16-lane row (quad swaps, then row rotations by 4 and 8: every lane of a row ends
// with the row's best), then the four rows' results by readlane.  A shuffle (ds_bpermute)
// reduction costs an LDS round trip per step; these are VALU moves.
template <int CTRL>
EA_DEV void dpp_step(float& v, int& i) {
  const float ov = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
  const int oi = __builtin_amdgcn_mov_dpp(i, CTRL, 0xF, 0xF, false);
  if (better(ov, oi, v, i)) { v = ov; i = oi; }
}
template <int CTRL>
EA_DEV void dpp_step3(float& v, int& i, int& c) {
  const float ov = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
  const int oi = __builtin_amdgcn_mov_dpp(i, CTRL, 0xF, 0xF, false);
  const int oc = __builtin_amdgcn_mov_dpp(c, CTRL, 0xF, 0xF, false);
  if (better(ov, oi, v, i)) { v = ov; i = oi; c = oc; }
}
EA_DEV Best wave_argmax(Best b) {
  dpp_step<0xB1>(b.v, b.i);   // quad_perm [1,0,3,2]
  dpp_step<0x4E>(b.v, b.i);   // quad_perm [2,3,0,1]
  dpp_step<0x124>(b.v, b.i);  // row_ror:4
  dpp_step<0x128>(b.v, b.i);  // row_ror:8
  Best r{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(b.v), 0)), __builtin_amdgcn_readlane(b.i, 0)};
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    const float ov = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b.v), 16 * q));
    const int oi = __builtin_amdgcn_readlane(b.i, 16 * q);
    if (better(ov, oi, r.v, r.i)) { r.v = ov; r.i = oi; }
  }
  return r;
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
  // each lane sorts its PER (value, token) pairs once (odd-even transposition network under
  // `better`); a selection round is then one wave argmax over the lanes' heads, and the winning
  // lane shifts its list — instead of every lane rescanning all PER values every round (with 4
  // waves per SIMD that rescan was ~2 us per round)
  int idx[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int v = v0 + e * 64 + lane;
    idx[e] = v < v1 ? v : 0x7fffffff;
    if (v >= v1) val[e] = -INFINITY;
  }
#pragma unroll
  for (int pass = 0; pass < PER; ++pass)
#pragma unroll
    for (int e = pass & 1; e + 1 < PER; e += 2)
      if (better(val[e + 1], idx[e + 1], val[e], idx[e])) {
        const float tv = val[e]; val[e] = val[e + 1]; val[e + 1] = tv;
        const int ti = idx[e]; idx[e] = idx[e + 1]; idx[e + 1] = ti;
      }
  for (int r = 0; r < P; ++r) {
    Best b = wave_argmax(Best{val[0], idx[0]});
    if (idx[0] == b.i && b.i != 0x7fffffff) {  // this lane's head was taken: shift its list
#pragma unroll
      for (int e = 0; e + 1 < PER; ++e) { val[e] = val[e + 1]; idx[e] = idx[e + 1]; }
      val[PER - 1] = -INFINITY;
      idx[PER - 1] = 0x7fffffff;
    }
    if (lane == 0) lst[wv * PB_PMAX + r] = b;
  }
  __syncthreads();
  if (wv == 0) {  // 16-way merge of the waves' sorted lists: lane l < PB_NW holds list l's head
    int* out = cand + (long)h * (P + 1);
    int hp = 0;
    Best head = lane < PB_NW ? lst[lane * PB_PMAX] : Best{-INFINITY, 0x7fffffff};
    for (int r = 0; r < P; ++r) {
      const Best m = wave_argmax(head);
      if (lane == 0) out[r] = m.i;
      if (lane < PB_NW && head.i == m.i && m.i != 0x7fffffff) {  // tokens are distinct across lists
        ++hp;
        head = hp < P ? lst[lane * PB_PMAX + hp] : Best{-INFINITY, 0x7fffffff};
      }
    }
    if (lane == 0) out[P] = eos;
  }
}

// the new beam over the n*(P+1) candidates (duplicates of <eos> skipped).  Outputs:
//   rec_i[b*4 + {0,1,2,3}] = parent hypothesis, token, candidate column, 0
//   rec_f[b*4 + {0,1,2,3}] = weighted score, decoder log-prob, CTC increment, CTC prefix psi
//   next step: last[b] = token, rptr[b] = &r_new[(h*(P+1)+col)*T*2], prefix[b] = psi,
//   score[b] = weighted score (all already in the new hypothesis order)
// One wave: every candidate's weighted score, decoder log-prob and psi are computed once into
// LDS, then `beam` wave argmax rounds (shuffles only, no block barriers) pick the winners; the
// winner's record comes from LDS (no global load in the serial part).
constexpr int SEL_NT = 64, SEL_MAX = 4096;
struct BestC {
  float v;
  int i;  // the reference's flat index h*V + token (tie order)
  int c;  // candidate slot
};
EA_DEV BestC wave_argmax_c(BestC b) {
  dpp_step3<0xB1>(b.v, b.i, b.c);
  dpp_step3<0x4E>(b.v, b.i, b.c);
  dpp_step3<0x124>(b.v, b.i, b.c);
  dpp_step3<0x128>(b.v, b.i, b.c);
  BestC r{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(b.v), 0)), __builtin_amdgcn_readlane(b.i, 0),
          __builtin_amdgcn_readlane(b.c, 0)};
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    const float ov = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b.v), 16 * q));
    const int oi = __builtin_amdgcn_readlane(b.i, 16 * q);
    const int oc = __builtin_amdgcn_readlane(b.c, 16 * q);
    if (better(ov, oi, r.v, r.i)) { r.v = ov; r.i = oi; r.c = oc; }
  }
  return r;
}
__global__ __launch_bounds__(SEL_NT) void select_kernel(int n, int V, int P, int beam, int T, const float* __restrict__ logp,
                                                        long ld, const int* __restrict__ cand,
                                                        const float* __restrict__ psi, const float* __restrict__ prefix,
                                                        const float* __restrict__ score, float w_dec, float w_lb,
                                                        int use_lb, float w_ctc, const float* r_new, int* __restrict__ rec_i,
                                                        float* __restrict__ rec_f, int* __restrict__ last_next,
                                                        unsigned long long* __restrict__ rptr_next,
                                                        float* __restrict__ prefix_next, float* __restrict__ score_next) {
  __shared__ float wsc[SEL_MAX], dec_s[SEL_MAX], psi_s[SEL_MAX];
  const int nc = n * (P + 1), lane = threadIdx.x;
  for (int c = lane; c < nc; c += SEL_NT) {
    const int h = c / (P + 1), k = c - h * (P + 1);
    const int j = cand[c];
    bool dup = false;
    if (k == P)
      for (int q = 0; q < P; ++q) dup |= cand[h * (P + 1) + q] == j;
    const float lp = logp[(long)h * ld + j];
    const float ps = psi[c];
    float wv = __fmul_rn(w_dec, lp);
    if (use_lb) wv = __fadd_rn(wv, w_lb);
    const float inc = __fsub_rn(ps, prefix[h]);
    wv = __fadd_rn(__fadd_rn(wv, __fmul_rn(w_ctc, inc)), score[h]);
    wsc[c] = dup ? -INFINITY : wv;
    dec_s[c] = lp;
    psi_s[c] = ps;
  }
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  for (int b = 0; b < beam; ++b) {
    BestC best{-INFINITY, 0x7fffffff, 0};
    for (int c = lane; c < nc; c += SEL_NT) {
      const float w = wsc[c];
      const int flat = (c / (P + 1)) * V + cand[c];
      if (w != -INFINITY && better(w, flat, best.v, best.i)) { best.v = w; best.i = flat; best.c = c; }
    }
    best = wave_argmax_c(best);
    const bool none = best.i == 0x7fffffff;
    const int c = none ? 0 : best.c;
    const int h = c / (P + 1), k = c - h * (P + 1);
    if (lane == 0) {
      const int j = cand[c];
      const float ps = psi_s[c];
      const float inc = __fsub_rn(ps, prefix[h]);
      rec_i[b * 4 + 0] = h; rec_i[b * 4 + 1] = j; rec_i[b * 4 + 2] = k; rec_i[b * 4 + 3] = none;
      rec_f[b * 4 + 0] = best.v; rec_f[b * 4 + 1] = dec_s[c]; rec_f[b * 4 + 2] = inc; rec_f[b * 4 + 3] = ps;
      last_next[b] = j;
      rptr_next[b] = (unsigned long long)(uintptr_t)(r_new + (long)c * T * 2);
      prefix_next[b] = ps;
      score_next[b] = best.v;
      wsc[c] = -INFINITY;  // taken
    }
    __builtin_amdgcn_wave_barrier();
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
  EA_CHECK_ARG(n >= 1 && V >= 1 && ld >= V && P >= 1 && beam >= 1 && T >= 1 && n * (P + 1) <= SEL_MAX &&
               beam <= n * (P + 1));
  hipLaunchKernelGGL(select_kernel, dim3(1), dim3(SEL_NT), 0, (hipStream_t)stream, n, V, P, beam, T, logp, ld, cand,
                     psi, prefix, score, w_dec, w_lb, use_lb, w_ctc, r_new, rec_i, rec_f, last_next, rptr_next,
                     prefix_next, score_next);
  EA_LAUNCH_CHECK();
  return 0;
}
