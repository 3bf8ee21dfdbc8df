// SpecAugment on the device (espnet2/asr/specaug/specaug.py:95-102): TimeWarp
// (layers/time_warp.py:9-88, bicubic, align_corners=False) then MaskAlongAxis along freq and
// along time (layers/mask_along_axis.py:8-68), fused into one pass over the (B, T, F) f32
// features.  The random draws (warp centre / target, mask positions and widths) are made on
// the host in the reference's order (espnet_amd/asr/specaug.py) and passed in as small int
// arrays, so one launch applies a batch's whole augmentation with no per-utterance loop.
//
// Bicubic resampling along time only: the freq axis keeps its size, so its cubic weights
// are (0, 1, 0, 0) and it is the identity (ATen upsample_bicubic2d with scale 1).  The time
// axis follows ATen's UpSample.h: scale = in/out (f32), src = scale*(dst+0.5)-0.5,
// idx = min(floor(src), in-1), t = clamp(src-idx, 0, 1), taps idx-1..idx+2 clamped to the
// segment, A = -0.75 cubic convolution weights.
#include "common.h"

namespace {

EA_DEV float cubic1(float x, float A) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
EA_DEV float cubic2(float x, float A) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; }

// one thread per (t, f) of utterance blockIdx.y; 256 threads cover 256 consecutive elements
__global__ __launch_bounds__(256) void specaug_kernel(int T, int F, const float* __restrict__ x,
                                                      const long long* __restrict__ lens,
                                                      const int* __restrict__ warp, int per_utt,
                                                      const int* __restrict__ fmask, int nf,
                                                      const int* __restrict__ tmask, int nt,
                                                      float* __restrict__ y) {
  const int b = blockIdx.y;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)T * F) return;
  const int t = (int)(i / F), f = (int)(i - (long)t * F);
  const float* xb = x + (long)b * T * F;
  // TimeWarp's per-utterance path warps x[b, :len] and pads with 0 (time_warp.py:76-86);
  // the equal-length path warps the whole padded axis and pads nothing (:73-75)
  const int wlen = per_utt ? (int)min((long long)T, lens[b]) : T;
  float v = 0.f;
  if (t < wlen) {
    const int center = warp[2 * b], warped = warp[2 * b + 1];
    if (center > 0) {
      int base, in_size, out_size, oy;
      if (t < warped) {
        base = 0; in_size = center; out_size = warped; oy = t;
      } else {
        base = center; in_size = wlen - center; out_size = wlen - warped; oy = t - warped;
      }
      const float scale = (float)in_size / (float)out_size;
      const float src = scale * ((float)oy + 0.5f) - 0.5f;
      const int iy = min((int)floorf(src), in_size - 1);
      const float tt = fminf(fmaxf(src - (float)iy, 0.f), 1.f);
      const float A = -0.75f;
      const float c0 = cubic2(tt + 1.f, A), c1 = cubic1(tt, A);
      const float c2 = cubic1(1.f - tt, A), c3 = cubic2(1.f - tt + 1.f, A);
      auto row = [&](int k) {
        const int r = min(max(iy - 1 + k, 0), in_size - 1);
        return xb[(long)(base + r) * F + f];
      };
      v = row(0) * c0;
      v += row(1) * c1;
      v += row(2) * c2;
      v += row(3) * c3;
    } else {
      v = xb[i];
    }
  }
  // masks (replace_with_zero=True): any of the utterance's spans covering t / f
  for (int k = 0; k < nt; ++k) {
    const int p = tmask[(b * nt + k) * 2], w = tmask[(b * nt + k) * 2 + 1];
    if (t >= p && t < p + w) v = 0.f;
  }
  for (int k = 0; k < nf; ++k) {
    const int p = fmask[(b * nf + k) * 2], w = fmask[(b * nf + k) * 2 + 1];
    if (f >= p && f < p + w) v = 0.f;
  }
  y[(long)b * T * F + i] = v;
}

}  // namespace

extern "C" int ea_specaug(int B, int T, int F, const float* x, const long long* lengths, const int* warp,
                          int per_utt, const int* fmask, int nf, const int* tmask, int nt, float* y,
                          void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(B >= 0 && T >= 0 && F > 0 && nf >= 0 && nt >= 0 && x != y);
  EA_CHECK_ARG(warp != nullptr && (nf == 0 || fmask != nullptr) && (nt == 0 || tmask != nullptr));
  EA_CHECK_ARG(!per_utt || lengths != nullptr);
  if (B == 0 || T == 0) return 0;
  dim3 grid(ea_cdiv((long)T * F, 256), B);
  hipLaunchKernelGGL(specaug_kernel, grid, dim3(256), 0, (hipStream_t)stream, T, F, x, lengths, warp, per_utt,
                     fmask, nf, tmask, nt, y);
  EA_LAUNCH_CHECK();
  return 0;
}
