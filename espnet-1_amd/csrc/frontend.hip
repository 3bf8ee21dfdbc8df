// Raw-waveform frontend: espnet2/asr/frontend/default.py:17-140 =
// Stft (layers/stft.py: torch.stft, center=True reflect padding, window) -> power spectrum ->
// LogMel (layers/log_mel.py: matmul with the mel matrix, clamp 1e-10, log, pad mask) ->
// GlobalMVN (layers/global_mvn.py:73-104).
//
// MI355X layout: the STFT is a framing kernel (reflect-padded, windowed frames written as
// rows of an (M = B*nF) x n_fft f32 matrix) followed by ONE exact-f32 MFMA GEMM against the
// real DFT basis [cos | -sin] (n_fft x 2*nbin), the power spectrum is one pass over that
// GEMM's output, the mel projection is a second f32 GEMM, and log + masks + mean/variance
// normalisation are one elementwise pass.  No FFT library, no complex tensors.
#include "common.h"

namespace {

// frames[b*nF + f][k] = window[k] * x[b][reflect(f*hop + k - pad)], pad = center ? n_fft/2 : 0.
// torch.stft pads the batch tensor as a whole (length Ns), so reflection at the end reads the
// batch padding of shorter utterances exactly like the reference.
__global__ __launch_bounds__(256) void stft_frames_kernel(int B, long Ns, int nF, int n_fft, int hop, int pad,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ win,
                                                          float* __restrict__ frames) {
  const long row = blockIdx.y;  // b*nF + f
  const int b = (int)(row / nF), f = (int)(row - (long)b * nF);
  const float* xb = x + (long)b * Ns;
  for (int k = blockIdx.x * 256 + threadIdx.x; k < n_fft; k += gridDim.x * 256) {
    long i = (long)f * hop + k - pad;
    if (i < 0) i = -i;                            // reflect (edge sample not repeated)
    if (i >= Ns) i = 2 * (Ns - 1) - i;
    const float v = (i >= 0 && i < Ns) ? xb[i] : 0.f;
    frames[row * n_fft + k] = v * win[k];
  }
}

// power[m][j] = re^2 + im^2 from the DFT GEMM output spec[m] = [re(0..nb-1) | im(0..nb-1)];
// frames at or beyond the utterance's frame count are zero (stft.py masked_fill of olens)
__global__ __launch_bounds__(256) void power_kernel(long M, int nF, int nb, const float* __restrict__ spec, long lds,
                                                    const long long* __restrict__ flens, float* __restrict__ pw,
                                                    long ldp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * nb) return;
  const long m = i / nb;
  const int j = (int)(i - m * nb);
  const int b = (int)(m / nF), f = (int)(m - (long)b * nF);
  const float re = spec[m * lds + j], im = spec[m * lds + nb + j];
  pw[m * ldp + j] = f < flens[b] ? re * re + im * im : 0.f;
}

// y = log(max(mel, 1e-10)), zero past the frame count (log_mel.py), then GlobalMVN
// (global_mvn.py:84-102): y -= mean; zero padding; y /= std
__global__ __launch_bounds__(256) void logmel_mvn_kernel(long M, int nF, int nm, const float* __restrict__ mel, long ldm,
                                                         const long long* __restrict__ flens,
                                                         const float* __restrict__ mean, const float* __restrict__ std,
                                                         float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * nm) return;
  const long m = i / nm;
  const int j = (int)(i - m * nm);
  const int b = (int)(m / nF), f = (int)(m - (long)b * nF);
  float v = 0.f;
  if (f < flens[b]) {
    v = logf(fmaxf(mel[m * ldm + j], 1e-10f));
    if (mean) v -= mean[j];
    if (std) v /= std[j];
  }
  y[i] = v;
}

// GlobalMVN (global_mvn.py:73-104) on (B, T, D) f32: y = (x - mean) masked past lens, / std
__global__ __launch_bounds__(256) void global_mvn_kernel(long n, int T, int D, const float* __restrict__ x,
                                                         const long long* __restrict__ lens,
                                                         const float* __restrict__ mean, const float* __restrict__ std,
                                                         float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long bt = i / D;
  const int j = (int)(i - bt * D);
  const int b = (int)(bt / T), t = (int)(bt - (long)b * T);
  float v = x[i];
  if (mean) v -= mean[j];
  if (t >= lens[b]) v = 0.f;
  if (std) v /= std[j];
  y[i] = v;
}

}  // namespace

extern "C" int ea_global_mvn(int B, int T, int D, const float* x, const long long* lens, const float* mean,
                             const float* std, float* y, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(B >= 0 && T >= 0 && D >= 1 && lens != nullptr);
  const long n = (long)B * T * D;
  if (n == 0) return 0;
  hipLaunchKernelGGL(global_mvn_kernel, dim3(ea_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, n, T, D, x, lens,
                     mean, std, y);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_stft_frames(int B, long Ns, int nF, int n_fft, int hop, int center, const float* x,
                              const float* window, float* frames, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(B >= 0 && Ns >= 1 && nF >= 0 && n_fft >= 1 && hop >= 1);
  EA_CHECK_ARG(!center || Ns > n_fft / 2);  // reflect padding needs pad < length (torch.stft)
  if (B == 0 || nF == 0) return 0;
  dim3 grid(ea_cdiv(n_fft, 256), (unsigned)((long)B * nF));
  hipLaunchKernelGGL(stft_frames_kernel, grid, dim3(256), 0, (hipStream_t)stream, B, Ns, nF, n_fft, hop,
                     center ? n_fft / 2 : 0, x, window, frames);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_power_spectrum(long M, int nF, int nbins, const float* spec, long ld_spec, const long long* flens,
                                 float* power, long ld_power, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(M >= 0 && nF >= 1 && nbins >= 1 && ld_spec >= 2 * nbins && ld_power >= nbins);
  if (M == 0) return 0;
  hipLaunchKernelGGL(power_kernel, dim3(ea_cdiv(M * nbins, 256)), dim3(256), 0, (hipStream_t)stream, M, nF, nbins,
                     spec, ld_spec, flens, power, ld_power);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_logmel_mvn(long M, int nF, int n_mels, const float* mel, long ld_mel, const long long* flens,
                             const float* mean, const float* std, float* y, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(M >= 0 && nF >= 1 && n_mels >= 1 && ld_mel >= n_mels);
  if (M == 0) return 0;
  hipLaunchKernelGGL(logmel_mvn_kernel, dim3(ea_cdiv(M * n_mels, 256)), dim3(256), 0, (hipStream_t)stream, M, nF,
                     n_mels, mel, ld_mel, flens, mean, std, y);
  EA_LAUNCH_CHECK();
  return 0;
}
