// Optimizer step over the flat parameter arena (one launch for all 615 tensors):
// clip_grad_norm_(max_norm, 2) (trainer.py:653-657) + skip-on-non-finite
// (trainer.py:662-678) + torch.optim.Adam (L2 weight decay, bias correction), plus the
// f32 -> bf16 weight shadow for the AMP GEMMs, and small scalar helpers.
// The clip coefficient and the finite check are read from device memory: no host sync.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(long n, const float* __restrict__ x, double* __restrict__ part,
                                                             int vec) {
  __shared__ double red[16];
  double a = 0.0;
  const long n4 = vec ? n >> 2 : 0, stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = ((const float4*)x)[i];
    a += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (long i = 4 * n4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const double v = x[i];
    a += v * v;
  }
  a = block_sum_d(a, red);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}

__global__ void sqnorm_final_kernel(int nparts, const double* __restrict__ part, float* __restrict__ norm) {
  __shared__ double red[16];
  double a = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) a += part[i];
  a = block_sum_d(a, red);
  if (threadIdx.x == 0) norm[0] = (float)sqrt(a);
}

struct AdamP {
  long n;
  float* p; const float* g; float* m; float* v; bf16* p16;
  float lr, b1, b2, eps, wd;
  float bc1, bc2_sqrt;   // 1-b1^t, sqrt(1-b2^t)
  const float* norm; float max_norm;
  const ea_opt_state* st;  // device step state: lr / bias corrections / skip come from here
};

// Device-resident step bookkeeping (ea_adam_step_dev): runs before the update, one thread.
// A non-finite norm skips both optimizer.step() and scheduler.step() (trainer.py:662-697),
// so the step counter only advances on an applied update.
__global__ void adam_prep_kernel(ea_opt_state* st, ea_lr_schedule sc, float b1, float b2, const float* norm,
                                 float max_norm) {
  const float nrm = norm ? norm[0] : 0.f;
  st->last_norm = nrm;
  auto lr_at = [&](long long t) {  // espnet2/schedulers/warmup_lr.py:40-50, s = t
    double lr = sc.base_lr;
    if (sc.kind == EA_SCHED_WARMUP) {
      const double s = (double)t, w = sc.warmup_steps;
      lr = sc.base_lr * sqrt(w) * fmin(1.0 / sqrt(s), s * pow(w, -1.5));
    }
    return lr;
  };
  if (norm && !isfinite(nrm)) {
    st->skip = 1;
    st->next_lr = (float)lr_at(st->step + 1);
    return;
  }
  st->skip = 0;
  const long long t = st->step + 1;
  st->step = t;
  st->lr = (float)lr_at(t);
  st->next_lr = (float)lr_at(t + 1);
  st->bc1 = (float)(1.0 - pow((double)b1, (double)t));
  st->bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, (double)t));
  st->coef = (norm && max_norm > 0.f) ? fminf(max_norm / (nrm + 1e-6f), 1.f) : 1.f;
}

// coef (grad-clip factor), lr and the bias corrections of this update; false = skip the step
EA_DEV bool adam_prelude(const AdamP& a, float& coef, float& step_size, float& bc2s) {
  float lr = a.lr, bc1 = a.bc1;
  coef = 1.f;
  bc2s = a.bc2_sqrt;
  if (a.st) {
    if (a.st->skip) return false;
    coef = a.st->coef; lr = a.st->lr; bc1 = a.st->bc1; bc2s = a.st->bc2_sqrt;
  } else {
    const float nrm = a.norm ? a.norm[0] : 0.f;
    if (a.norm && !isfinite(nrm)) return false;  // trainer.py:662: skip the update
    if (a.norm && a.max_norm > 0.f) coef = fminf(a.max_norm / (nrm + 1e-6f), 1.f);
  }
  step_size = lr / bc1;
  return true;
}
// one element of torch.optim.Adam (foreach=False arithmetic order)
EA_DEV void adam_elem(const AdamP& a, float coef, float step_size, float bc2s, float& p, float g, float& m, float& v) {
  g *= coef;
  if (a.wd != 0.f) g += a.wd * p;
  m = m + (1.f - a.b1) * (g - m);  // lerp, as torch Adam
  v = v * a.b2 + (1.f - a.b2) * g * g;
  const float denom = sqrtf(v) / bc2s + a.eps;
  p -= step_size * (m / denom);
}

__global__ __launch_bounds__(256) void adam_kernel(AdamP a) {
  float coef, step_size, bc2s;
  if (!adam_prelude(a, coef, step_size, bc2s)) return;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.n; i += (long)gridDim.x * blockDim.x) {
    float p = a.p[i], m = a.m[i], v = a.v[i];
    adam_elem(a, coef, step_size, bc2s, p, a.g[i], m, v);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
    if (a.p16) a.p16[i] = (bf16)p;
  }
}

__global__ void cast_kernel(long n, const float* __restrict__ x, bf16* __restrict__ y) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = (bf16)x[i];
}

__global__ void scale_inplace_kernel(long n, float* __restrict__ x, const float* __restrict__ s, float c) {
  const float k = s[0] * c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= k;
}

__global__ void axpy_dev_kernel(long n, const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ s,
                                float c) {
  const float k = s[0] * c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] += k * x[i];
}

// out = wa*a + wb*b (device scalars; b may be null)
__global__ void axpby_scalar_kernel(const float* a, float wa, const float* b, float wb, float* out) {
  out[0] = wa * a[0] + (b ? wb * b[0] : 0.f);
}

}  // namespace

// one thread per parameter, 4-B accesses: a 16-B vector form measured the same (739 vs 742 us
// at 115 M parameters, 4.7 TB/s of mixed read/write traffic) and nontemporal write-back
// slower (765 us), scripts/adam_bench.py
static void launch_adam(const AdamP& a, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(ea_grid_cap(ea_cdiv(a.n, 256), 4096)), dim3(256), 0, st, a);
}

extern "C" int ea_sqnorm(long n, const float* x, double* workspace, float* norm, void* stream) {
  EA_ENTRY();
  hipStream_t st = (hipStream_t)stream;
  const int nb = ea_grid_cap(ea_cdiv(n, 1024), 2048);
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nb), dim3(256), 0, st, n, x, workspace, (int)(((uintptr_t)x & 15) == 0));
  EA_LAUNCH_CHECK();
  hipLaunchKernelGGL(sqnorm_final_kernel, dim3(1), dim3(256), 0, st, nb, workspace, norm);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_adam_step(long n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                            void* params_bf16, float lr, float beta1, float beta2, float eps, float weight_decay,
                            long step, const float* grad_norm, float max_norm, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(step >= 1);
  AdamP a;
  a.n = n; a.p = params; a.g = grads; a.m = exp_avg; a.v = exp_avg_sq; a.p16 = (bf16*)params_bf16;
  a.lr = lr; a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  a.bc2_sqrt = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  a.norm = grad_norm; a.max_norm = max_norm;
  a.st = nullptr;
  launch_adam(a, (hipStream_t)stream);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_adam_step_dev(long n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                                void* params_bf16, const ea_lr_schedule* sched, float beta1, float beta2, float eps,
                                float weight_decay, ea_opt_state* state, const float* grad_norm, float max_norm,
                                void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(sched != nullptr && state != nullptr);
  EA_CHECK_ARG(sched->kind == EA_SCHED_CONSTANT || (sched->kind == EA_SCHED_WARMUP && sched->warmup_steps > 0.f));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, st, state, *sched, beta1, beta2, grad_norm, max_norm);
  EA_LAUNCH_CHECK();
  AdamP a;
  a.n = n; a.p = params; a.g = grads; a.m = exp_avg; a.v = exp_avg_sq; a.p16 = (bf16*)params_bf16;
  a.lr = 0.f; a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.bc1 = 1.f; a.bc2_sqrt = 1.f;
  a.norm = grad_norm; a.max_norm = max_norm;
  a.st = state;
  launch_adam(a, st);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_cast_f32_bf16(long n, const float* x, void* y, void* stream) {
  EA_ENTRY();
  hipLaunchKernelGGL(cast_kernel, dim3(ea_grid_cap(ea_cdiv(n, 256), 4096)), dim3(256), 0, (hipStream_t)stream, n, x, (bf16*)y);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_scale_by_scalar(long n, float* x, const float* s, float c, void* stream) {
  EA_ENTRY();
  hipLaunchKernelGGL(scale_inplace_kernel, dim3(ea_grid_cap(ea_cdiv(n, 256), 4096)), dim3(256), 0, (hipStream_t)stream, n, x, s, c);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_axpy_dev(long n, const float* x, float* y, const float* s, float c, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 0 && (n == 0 || (x && y && s)));
  if (n == 0) return 0;
  hipLaunchKernelGGL(axpy_dev_kernel, dim3(ea_grid_cap(ea_cdiv(n, 256), 4096)), dim3(256), 0, (hipStream_t)stream, n, x, y, s, c);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_axpby_scalar(const float* a, float wa, const float* b, float wb, float* out, void* stream) {
  EA_ENTRY();
  hipLaunchKernelGGL(axpby_scalar_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, a, wa, b, wb, out);
  EA_LAUNCH_CHECK();
  return 0;
}

// ----------------------------------------------------------------- transposed weight shadow
// bf16 W^T copies of the shadow weights whose Linear input gradient (dX = dY . W, N = K_in) runs
// on narrow-N tiles: read K-major there, the weight panel is one LDS-DMA stream instead of
// 128-wide MN-major panels (about a third of those launches' time).  Problem p: dst[c*R + r] =
// src[off + r*C + c] for an R x C row-major weight; one workgroup per 64 x 64 tile, the tiles
// listed as (problem, tile row, tile col); R, C multiples of 8.
namespace {
struct TrProb {
  long long src_off;
  bf16* dst;
  int R, C;
};
__global__ __launch_bounds__(256) void transpose_grouped_kernel(const int4* __restrict__ tiles,
                                                                const TrProb* __restrict__ probs,
                                                                const bf16* __restrict__ src) {
  __shared__ __attribute__((aligned(16))) bf16 t[64][72];  // 144-B rows
  const int4 tl = tiles[blockIdx.x];
  const TrProb p = probs[tl.x];
  const int r0 = tl.y * 64, c0 = tl.z * 64, tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = tid + 256 * u, rr = q >> 3, ch = q & 7;
    const int r = r0 + rr, c = c0 + ch * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < p.R && c < p.C) v = *(const uint4*)(src + p.src_off + (long)r * p.C + c);
    *(uint4*)&t[rr][ch * 8] = v;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = tid + 256 * u, cc = q >> 3, ch = q & 7;
    const int c = c0 + cc, r = r0 + ch * 8;
    if (c < p.C && r < p.R) {
      union { uint4 u4; bf16 e[8]; } o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.e[e] = t[ch * 8 + e][cc];
      *(uint4*)(p.dst + (long)c * p.R + r) = o.u4;
    }
  }
}
}  // namespace

extern "C" int ea_transpose_bf16_grouped(int ntiles, const int* tiles, const void* probs, const void* src,
                                         void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(ntiles >= 0 && (ntiles == 0 || (tiles && probs && src)));
  if (ntiles == 0) return 0;
  hipLaunchKernelGGL(transpose_grouped_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream,
                     (const int4*)tiles, (const TrProb*)probs, (const bf16*)src);
  EA_LAUNCH_CHECK();
  return 0;
}
