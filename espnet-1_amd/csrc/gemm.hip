// GEMM host side (include/espnet_amd.h: ea_gemm, ea_gemm_conv*): tile choice, split-K, the
// register-staged kernel (f32 parity path / unaligned operands) and the launch dispatch onto
// the LDS-DMA kernels of gemm_kern.h (instantiated in gemm_pipe*.hip and gemm_lds*.hip).

#include "gemm_kern.h"
#include <cstdio>
#include <cstdlib>

namespace {
// split-K combine: C = epi(sum_s slab[s]) (any epilogue kind), 4 columns per thread
__global__ void splitk_reduce(GemmP p) {
  const long MN = (long)p.M * p.N;
  const int z = blockIdx.y;
  const int zb = z / p.nh, zh = z % p.nh;
  const float* base = p.ws + (long)z * p.splitk * MN;
  const bool vec = p.vec_c && (p.N % 4 == 0);
  const EpiK ek = make_epik(p);
  const long n4 = vec ? MN / 4 : MN;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    if (vec) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      int s = 0;
      // 8 slab loads in flight per thread (the combine is latency-bound: a 512 x 64 output
      // is 32 K float4s over 12 slabs), summed in slab order as before
      for (; s + 8 <= p.splitk; s += 8) {
        float4 b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = *(const float4*)(base + (long)(s + j) * MN + i * 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) { a.x += b[j].x; a.y += b[j].y; a.z += b[j].z; a.w += b[j].w; }
      }
      for (; s < p.splitk; ++s) {
        const float4 b = *(const float4*)(base + (long)s * MN + i * 4);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      const int row = (int)(i * 4 / p.N), col = (int)(i * 4 % p.N);
      const float v[4] = {a.x, a.y, a.z, a.w};
      switch (p.epi.kind) {
        case EA_EPI_STORE: epi_four<EA_EPI_STORE>(p, ek, z, zb, zh, row, col, v); break;
        case EA_EPI_ACT: epi_four<EA_EPI_ACT>(p, ek, z, zb, zh, row, col, v); break;
        case EA_EPI_RESID: epi_four<EA_EPI_RESID>(p, ek, z, zb, zh, row, col, v); break;
        default: epi_four<EA_EPI_DACT>(p, ek, z, zb, zh, row, col, v); break;
      }
    } else {
      float a = 0.f;
      for (int s = 0; s < p.splitk; ++s) a += base[s * MN + i];
      epi_apply(p, z, zb, zh, (int)(i / p.N), (int)(i % p.N), a);
    }
  }
}

int g_gemm_stages = 2;
unsigned long long* g_probe = nullptr;  // ea_gemm_set_probe
unsigned long long* g_diag = nullptr;   // ea_gemm_set_diag
int g_gemm_bm64 = 1;
int g_gemm_bm32 = [] { const char* e = std::getenv("EA_GEMM_BM32"); return e ? std::atoi(e) : 1; }();
int g_gemm_pipe = 0;  // ea_gemm_set_pipe bits: 1 = 256x256 tiles on gemm_pipe, 2 = 128x128 tiles too

// gemm_k128 for the N = 512 grids at K >= 1,024 (mode 1, default): 7968x512x2048 23.0 vs 26.3 us
// on the 64x128 tile (RESID epilogue 28.5 vs 31.0), C3 step 1813-1827 vs 1795-1796 utt/s on one
// box (gpurun_out/r5b); at K = 512 the 64x128 tile stays (15.0 vs 15.8 us)
int g_gemm_k128 = [] { const char* e = std::getenv("EA_GEMM_K128"); return e ? std::atoi(e) : 1; }();
// few-row GEMMs (M <= g_gemm_skinny) on gemm_skinny (ea_gemm_set_skinny; 0 = off)
int g_gemm_skinny = [] { const char* e = std::getenv("EA_GEMM_SKINNY"); return e ? std::atoi(e) : 16; }();

int launch_lds(GemmP& p, int a_k, int b_k, int nz, hipStream_t st, bool k128 = false) {
  dim3 grid(p.tiles_m * p.tiles_n, 1, nz * p.splitk);
  if (k128) return launch_k128(p, grid, st);
  if (p.g.mode != 0) {  // implicit-GEMM conv2 modes: fixed layouts, 128x128 or 256x256 tiles
    if (p.bm == 256 && g_gemm_pipe) return launch_pipe_conv(p, grid, st);
    return launch_lds_conv(p, grid, st);
  }
  if ((p.bm == 256 && p.bn == 256 && (g_gemm_pipe & 1)) ||
      (p.bm == 128 && p.bn == 128 && (g_gemm_pipe & 2)))
    return launch_pipe(p, a_k, b_k, grid, st);
  return launch_lds_dense(p, a_k, b_k, grid, st);
}

// Output tile choice by a two-term time model fitted to measured launches on MI355X
// (scripts/gemm_tiles.py): rounds of co-resident blocks each pay a fixed prologue/epilogue
// cost t0 (us), and each CU's share of the flops runs at the tile's steady-state rate
// (TFLOP/s per CU; larger tiles need fewer L2 bytes per flop).  g_force_bm/bn pin a shape.
int g_force_bm = 0, g_force_bn = 0;
void choose_tile(GemmP& p, int a_k, long nz) {
  struct Cfg { int bm, bn, occ; double t0, rcu; bool ak_only; };
  static const Cfg cfgs[] = {{256, 256, 1, 12.4, 4.49, false}, {128, 128, 2, 8.3, 2.9, false},
                             {64, 128, 3, 6.8, 2.8, true}, {32, 128, 2, 6.0, 2.0, true}};
  p.bm = 128; p.bn = 128;
  if (g_force_bm) {
    if (g_force_bm <= 64 && !a_k) return;  // 32/64-row tiles need K-major A: keep 128 x 128
    p.bm = g_force_bm; p.bn = g_force_bn;
    return;
  }
  double best = 1e300;
  for (const Cfg& c : cfgs) {
    if (c.ak_only && (!a_k || !g_gemm_bm64)) continue;
    if (c.bm == 32 && !g_gemm_bm32) continue;
    const long tiles = (long)ea_cdiv(p.M, c.bm) * ea_cdiv(p.N, c.bn) * nz;
    const double rounds = (double)((tiles + 256L * c.occ - 1) / (256L * c.occ));
    const double per_cu = (double)((tiles + 255) / 256) * 2.0 * c.bm * c.bn * (double)p.K * 1e-6;
    const double est = rounds * c.t0 + per_cu / c.rcu;
    if (est < best * 0.999) { best = est; p.bm = c.bm; p.bn = c.bn; }
  }
}

template <typename T>
int launch(GemmP& p, int a_k, int b_k, int nz, hipStream_t st, bool k128 = false) {
  if (sizeof(T) == 2 && p.lds) return launch_lds(p, a_k, b_k, nz, st, k128);
  if (p.bm != 128 || p.bn != 128) return EA_ERR_BAD_ARG;
  dim3 grid(p.tiles_m * p.tiles_n, 1, nz * p.splitk);
#define EA_GEMM_CASE(AKV, BKV)                                                      \
  if (a_k == AKV && b_k == BKV) {                                                   \
    hipLaunchKernelGGL((gemm_kernel<T, AKV, BKV>), grid, dim3(NT), 0, st, p);       \
  }
  EA_GEMM_CASE(true, true)
  else EA_GEMM_CASE(true, false)
  else EA_GEMM_CASE(false, true)
  else EA_GEMM_CASE(false, false)
#undef EA_GEMM_CASE
  EA_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" int ea_gemm_set_pipeline(int stages) {
  EA_ENTRY();
  EA_CHECK_ARG(stages == 0 || stages == 2 || stages == 12);
  g_gemm_bm64 = stages < 10;   // 12/13: same ring, 128-row tiles only (A/B measurements)
  g_gemm_stages = stages % 10;
  return 0;
}

namespace {
__global__ void probe_begin_kernel(unsigned long long* s) { s[0] = ~0ull; s[1] = 0ull; }
__global__ void probe_end_kernel(unsigned long long* s) {
  if (s[1] > s[0]) { s[2] += s[1] - s[0]; s[3] += 1ull; }
}
}  // namespace

// Step phase timer (ea_phase_stamp): st = {last stamp, step counter}; ring[slot][4] =
// {forward, backward, optimizer seconds, extra}.  Stream-ordered single-thread kernels: a
// stamp runs after everything issued before it on the stream, so the differences are the
// device durations of the phases, and a captured step re-measures itself on every replay.
namespace {
__global__ void phase_stamp_kernel(unsigned long long* st, float* ring, int cap, int phase, const float* extra,
                                   const int* skip) {
  const unsigned long long now = __builtin_amdgcn_s_memrealtime();
  if (phase > 0) {
    const long slot = (long)(st[1] % (unsigned long long)cap);
    float dt = (float)((double)(now - st[0]) * 1e-8);  // 100 MHz clock
    // a skipped update (non-finite grad norm) registers no optim_step_time in the reference
    // (trainer.py:662-682); NaN is what its reporter's nanmean then ignores
    if (phase == 3 && skip && skip[0]) dt = __builtin_nanf("");
    ring[slot * 4 + phase - 1] = dt;
    if (phase == 3) {
      ring[slot * 4 + 3] = extra ? extra[0] : 0.f;
      st[1] = st[1] + 1ull;
    }
  }
  st[0] = now;
}
}  // namespace

extern "C" int ea_phase_stamp(unsigned long long* state, float* ring, int cap, int phase, const float* extra,
                              void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(state != nullptr && ring != nullptr && cap > 0 && phase >= 0 && phase <= 3);
  hipLaunchKernelGGL(phase_stamp_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state, ring, cap, phase, extra,
                     (const int*)nullptr);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_phase_stamp_opt(unsigned long long* state, float* ring, int cap, int phase,
                                  const ea_opt_state* opt, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(state != nullptr && ring != nullptr && cap > 0 && phase >= 0 && phase <= 3 && opt != nullptr);
  hipLaunchKernelGGL(phase_stamp_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, state, ring, cap, phase,
                     &opt->next_lr, &opt->skip);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_gemm_set_diag(unsigned long long* buf) {
  EA_ENTRY();
  g_diag = buf;
  return 0;
}

extern "C" int ea_gemm_set_probe(unsigned long long* slots) {
  EA_ENTRY();
  g_probe = slots;
  return 0;
}

extern "C" int ea_probe_begin(unsigned long long* slots, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(slots != nullptr);
  hipLaunchKernelGGL(probe_begin_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, slots);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_probe_end(unsigned long long* slots, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(slots != nullptr);
  hipLaunchKernelGGL(probe_end_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, slots);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_gemm_set_pipe(int on) {
  EA_ENTRY();
  g_gemm_pipe = on;
  return 0;
}

extern "C" int ea_gemm_set_k128(int mode, int slots) {
  EA_ENTRY();
  EA_CHECK_ARG(mode >= 0 && mode <= 3 && (slots == 3 || slots == 4));
  g_gemm_k128 = mode;
  eag::g_k128_slots = slots;
  return 0;
}

extern "C" int ea_gemm_set_skinny(int max_m) {
  EA_ENTRY();
  EA_CHECK_ARG(max_m >= 0 && max_m <= 64);
  g_gemm_skinny = max_m;
  return 0;
}

extern "C" int ea_gemm_set_tile(int bm, int bn) {
  EA_ENTRY();
  EA_CHECK_ARG((bm == 0 && bn == 0) || (bm == 32 && bn == 128) || (bm == 64 && bn == 128) ||
               (bm == 128 && bn == 128) || (bm == 256 && bn == 256));
  g_force_bm = bm;
  g_force_bn = bn;
  return 0;
}

static int gemm_impl(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K,
                     const void* A, long lda, long sAb, long sAh,
                     const void* B, long ldb, long sBb, long sBh,
                     int batch, int nh,
                     void* C, int c_dtype, long ldc, long sCb, long sCh,
                     const ea_epilogue* epi, float* workspace, long ws_elems, void* stream,
                     const ea_conv_geo* geo, const float* w1x = nullptr, int w1T = 0, int w1F = 0,
                     float* w1part = nullptr, const uint8_t* w1pos = nullptr) {
  EA_CHECK_ARG(epi != nullptr && M >= 0 && N >= 0 && K >= 0 && batch >= 1 && nh >= 1);
  EA_CHECK_ARG(dtype == EA_F32 || dtype == EA_BF16);
  if (M == 0 || N == 0) return 0;
  const int E = dtype == EA_BF16 ? 8 : 4;
  const int esz = dtype == EA_BF16 ? 2 : 4;
  (void)esz;
  if (epi->kind == EA_EPI_RESID) EA_CHECK_ARG(c_dtype == EA_F32);
  GemmP p{};
  p.M = M; p.N = N; p.K = K;
  p.A = A; p.lda = lda; p.sAb = sAb; p.sAh = sAh;
  p.B = B; p.ldb = ldb; p.sBb = sBb; p.sBh = sBh;
  p.nh = nh;
  p.C = C; p.c_dtype = c_dtype; p.ldc = ldc; p.sCb = sCb; p.sCh = sCh;
  p.epi = *epi;
  p.ws = workspace;
  p.salt = ea_g_rng_salt;
  p.stamp = g_probe;
  p.diag = g_diag;
  p.g = geo ? *geo : ea_conv_geo{};
  p.w1x = w1x; p.w1part = w1part; p.w1pos = w1pos; p.w1T = w1T; p.w1F = w1F;
  // unaligned operands (odd vocab / leading dims) take the element-wise load path
  p.vec_a = (lda % E == 0 && sAb % E == 0 && sAh % E == 0 && ((uintptr_t)A % 16) == 0);
  p.vec_b = (ldb % E == 0 && sBb % E == 0 && sBh % E == 0 && ((uintptr_t)B % 16) == 0);
  {
    const int ce = c_dtype == EA_BF16 ? 2 : 4;
    bool vc = (N % 4 == 0) && ldc % 4 == 0 && sCb % 4 == 0 && sCh % 4 == 0 && ((uintptr_t)C % (4 * ce)) == 0;
    if (epi->bias) vc = vc && ((uintptr_t)epi->bias % 16) == 0;
    if (epi->aux) vc = vc && epi->ldaux % 4 == 0 && ((uintptr_t)epi->aux % (4 * (epi->aux_dtype == EA_BF16 ? 2 : 4))) == 0;
    if (epi->resid) vc = vc && epi->ldr % 4 == 0 && ((uintptr_t)epi->resid % 16) == 0;
    p.vec_c = vc;
    bool v8 = vc && N % 8 == 0 && ldc % 8 == 0 && sCb % 8 == 0 && sCh % 8 == 0 && ((uintptr_t)C % 16) == 0;
    if (epi->aux) v8 = v8 && epi->ldaux % 8 == 0 && ((uintptr_t)epi->aux % 16) == 0;
    if (epi->resid) v8 = v8 && epi->ldr % 8 == 0;
    p.vec8 = v8;
  }
  p.bm = 128; p.bn = 128;
  // few rows (decoder steps): K split over the waves of a 16 x 32 block instead of a tile
  // walking all of K (gemm_skinny.hip)
  if (dtype == EA_BF16 && M <= g_gemm_skinny && a_kmajor && b_kmajor && !geo && !w1part &&
      batch * nh == 1 && K % 32 == 0 && K > 0 && p.vec_a && p.vec_b) {
    static const bool trace_s = std::getenv("EA_GEMM_TRACE") != nullptr;
    if (trace_s) std::fprintf(stderr, "[ea_gemm] M=%d N=%d K=%d skinny epi=%d\n", M, N, K, (int)epi->kind);
    return launch_skinny(p, (hipStream_t)stream);
  }
  // operand extent per batch slice (bytes) must fit the kernel's 32-bit source offsets
  const double a_ext = 2.0 * ((a_kmajor ? (double)M : (double)K) * lda);
  const double b_ext = 2.0 * ((b_kmajor ? (double)N : (double)K) * ldb);
  const bool lds_path = dtype == EA_BF16 && p.vec_a && p.vec_b && g_gemm_stages > 0 &&
                        a_ext < 4.0e9 && b_ext < 4.0e9;
  p.lds = lds_path;
  if (geo && geo->mode != 0) {
    // gather modes: LDS-DMA path only, K a whole number of 64-deep tiles within taps
    if (!lds_path || K % 64 != 0 || geo->C % 64 != 0 || batch * nh != 1) return EA_ERR_BAD_ARG;
    if ((geo->mode == EA_CONV_WGRAD) == (a_kmajor != 0) || (geo->mode == EA_CONV_FWD) != (b_kmajor != 0))
      return EA_ERR_BAD_ARG;
    choose_tile(p, 0, 1);
    // weight gradient: few output tiles over a huge K (pixels) -> 256x256 tiles (the higher
    // per-CU MFMA rate) split over K to ~one block per CU (split rule below)
    if (geo->mode == EA_CONV_WGRAD && !g_force_bm) { p.bm = 256; p.bn = 256; }
    if (w1part) {  // the fused conv1-gradient epilogue lives in the 256 x 256 ping-pong kernel
      if (!g_gemm_pipe || !p.vec8) return EA_ERR_BAD_ARG;
      p.bm = 256; p.bn = 256;
    }
    if (p.bm != 256 || p.bn != 256) { p.bm = 128; p.bn = 128; }
  } else if (lds_path) {
    choose_tile(p, a_kmajor, (long)batch * nh);
  }
  // gemm_k128 (ea_gemm_set_k128 / EA_GEMM_K128): both operands K-major, K a whole number of
  // 64-deep tiles, a 64x128 / 128x128 choice whose 128x128 grid about fills the CUs (one tile
  // per CU: the N = 512 GEMMs at M = 7,968) and K >= 1,024; mode 2: any such grid of >= 128
  // tiles, any K; mode 3: every eligible GEMM (tests)
  bool k128 = false;
  if (g_gemm_k128 && lds_path && !geo && a_kmajor && b_kmajor && K % 64 == 0 && K > 0) {
    const long t128 = (long)ea_cdiv(M, 128) * ea_cdiv(N, 128) * batch * nh;
    const bool fits = g_gemm_k128 == 3 ||
                      (!g_force_bm && (p.bm == 64 || p.bm == 128) && p.bn == 128 && t128 >= 128 &&
                       (g_gemm_k128 == 2 || (t128 <= 256 && K >= 1024)));
    if (fits) { p.bm = 128; p.bn = 128; k128 = true; }
  }
  if (p.bm <= 64 && !a_kmajor) return EA_ERR_BAD_ARG;
  p.tiles_m = ea_cdiv(M, p.bm);
  p.tiles_n = ea_cdiv(N, p.bn);
  const int KT = dtype == EA_BF16 ? KCfg<bf16>::KT : KCfg<float>::KT;
  const int nz = batch * nh;
  // split-K when the output grid cannot fill the 256 CUs and K is long (dW GEMMs)
  int splitk = 1;
  // 128x128-equivalent tiles: split K only when the grid cannot fill the CUs
  const long tiles = max(1L, (long)p.tiles_m * p.tiles_n * nz * (p.bm * p.bn) / (128 * 128));
  // K >= 1024: a K = 512 GEMM split two ways costs more in the reduce pass than it gains
  // (decoder 1312x2048x512: 23.1 us split vs 10.5 us unsplit, scripts/gemm_splitk_ab.py)
  if (geo && geo->mode == EA_CONV_WGRAD && p.bm == 256) {
    if (workspace) {
      splitk = max(1, 256 / (p.tiles_m * p.tiles_n));  // one 512-thread block per CU
      splitk = min(splitk, K / (4 * KT));
      while (splitk > 1 && (long)splitk * M * N > ws_elems) --splitk;
      splitk = max(splitk, 1);
    }
  } else if (!k128 && workspace && tiles < 200 && K >= 16 * KT && K >= 1024 && (long)p.tiles_m * p.tiles_n * nz < 128) {
    // (a grid already covering half the CUs — e.g. 32-row tiles of a decoder GEMM — runs
    // unsplit: the partial slabs and the combine pass cost more than the extra blocks gain)
    splitk = (int)((384 + tiles - 1) / tiles);
    splitk = min(splitk, K / (4 * KT));
    splitk = min(splitk, 16);
    while (splitk > 1 && (long)splitk * nz * M * N > ws_elems) --splitk;
    if (splitk < 1) splitk = 1;
  }
  int kchunk = K;
  if (splitk > 1) {
    kchunk = ea_cdiv(ea_cdiv(K, splitk), KT) * KT;
    splitk = ea_cdiv(K, kchunk);
  }
  p.splitk = splitk;
  p.kchunk = kchunk;
  static const bool trace = std::getenv("EA_GEMM_TRACE") != nullptr;  // shape census (diagnostics)
  if (trace)
    std::fprintf(stderr, "[ea_gemm] M=%d N=%d K=%d ak=%d bk=%d nz=%d tile=%dx%d%s splitk=%d epi=%d geo=%d lds=%d\n", M,
                 N, K, a_kmajor, b_kmajor, nz, p.bm, p.bn, k128 ? "k" : "", splitk, (int)epi->kind, geo ? geo->mode : 0,
                 (int)p.lds);
  hipStream_t st = (hipStream_t)stream;
  int rc = dtype == EA_BF16 ? launch<bf16>(p, a_kmajor, b_kmajor, nz, st, k128)
                            : launch<float>(p, a_kmajor, b_kmajor, nz, st);
  if (rc) return rc;
  if (splitk > 1) {
    const long MN = (long)M * N;
    dim3 grid(ea_grid_cap(ea_cdiv(MN / 4 + 1, 256), 2048), nz);
    hipLaunchKernelGGL(splitk_reduce, grid, dim3(256), 0, st, p);
    EA_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int ea_gemm(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K,
                       const void* A, long lda, long sAb, long sAh,
                       const void* B, long ldb, long sBb, long sBh,
                       int batch, int nh,
                       void* C, int c_dtype, long ldc, long sCb, long sCh,
                       const ea_epilogue* epi, float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  return gemm_impl(dtype, a_kmajor, b_kmajor, M, N, K, A, lda, sAb, sAh, B, ldb, sBb, sBh, batch, nh, C, c_dtype,
                   ldc, sCb, sCh, epi, workspace, ws_elems, stream, nullptr);
}

extern "C" int ea_gemm_ln(int M, int N, int K, const float* x, long ldx, const float* gamma, const float* beta,
                          float eps, const void* W, long ldw, void* C, int c_dtype, long ldc, const ea_epilogue* epi,
                          void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(epi != nullptr && M >= 0 && N >= 0 && K > 0 && K % 32 == 0 && K <= 32 * 8 * 8);
  EA_CHECK_ARG(x && gamma && beta && W && C && ldx >= K && ldw >= K && ldc >= N);
  EA_CHECK_ARG(ldx % 4 == 0 && ((uintptr_t)x % 16) == 0 && ldw % 8 == 0 && ((uintptr_t)W % 16) == 0 &&
               ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0);
  if (epi->kind == EA_EPI_RESID) EA_CHECK_ARG(c_dtype == EA_F32);
  if (M == 0 || N == 0) return 0;
  GemmP p{};
  p.M = M; p.N = N; p.K = K;
  p.A = x; p.lda = ldx;
  p.B = W; p.ldb = ldw;
  p.nh = 1; p.splitk = 1; p.kchunk = K;
  p.C = C; p.c_dtype = c_dtype; p.ldc = ldc;
  p.epi = *epi;
  p.salt = ea_g_rng_salt;
  const int ce = c_dtype == EA_BF16 ? 2 : 4;
  bool vc = (N % 4 == 0) && ldc % 4 == 0 && ((uintptr_t)C % (4 * ce)) == 0;
  if (epi->bias) vc = vc && ((uintptr_t)epi->bias % 16) == 0;
  if (epi->aux) vc = vc && epi->ldaux % 4 == 0 && ((uintptr_t)epi->aux % (4 * (epi->aux_dtype == EA_BF16 ? 2 : 4))) == 0;
  if (epi->resid) vc = vc && epi->ldr % 4 == 0 && ((uintptr_t)epi->resid % 16) == 0;
  p.vec_c = vc;
  return launch_skinny_ln(p, gamma, beta, eps, (hipStream_t)stream);
}

extern "C" int ea_gemm_conv(const ea_conv_geo* geo, int a_kmajor, int b_kmajor, int M, int N, int K,
                            const void* A, long lda, const void* B, long ldb, void* C, int c_dtype, long ldc,
                            const ea_epilogue* epi, float* workspace, long ws_elems, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(geo != nullptr && geo->mode >= EA_CONV_FWD && geo->mode <= EA_CONV_WGRAD);
  return gemm_impl(EA_BF16, a_kmajor, b_kmajor, M, N, K, A, lda, 0, 0, B, ldb, 0, 0, 1, 1, C, c_dtype, ldc, 0, 0,
                   epi, workspace, ws_elems, stream, geo);
}

extern "C" int ea_gemm_conv_w1(const ea_conv_geo* geo, int M, int N, int K, const void* A, long lda, const void* B,
                               long ldb, const ea_epilogue* epi, const float* x, int T, int Fin, float* part,
                               void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(geo != nullptr && geo->mode == EA_CONV_DGRAD && x != nullptr && part != nullptr);
  EA_CHECK_ARG(epi != nullptr && epi->kind == EA_EPI_DACT && epi->act == EA_ACT_RELU && epi->aux != nullptr &&
               epi->aux_dtype == EA_BF16);
  EA_CHECK_ARG(T >= 3 && Fin >= 3 && M < (1 << 24));
  return gemm_impl(EA_BF16, 1, 0, M, N, K, A, lda, 0, 0, B, ldb, 0, 0, 1, 1, nullptr, EA_BF16, N, 0, 0, epi,
                   nullptr, 0, stream, geo, x, T, Fin, part);
}

extern "C" int ea_gemm_conv_w1b(const ea_conv_geo* geo, int M, int N, int K, const void* A, long lda, const void* B,
                                long ldb, const ea_epilogue* epi, const float* x, int T, int Fin, float* part,
                                const unsigned char* pos, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(geo != nullptr && geo->mode == EA_CONV_DGRAD && x != nullptr && part != nullptr && pos != nullptr);
  EA_CHECK_ARG(epi != nullptr && epi->kind == EA_EPI_DACT && epi->act == EA_ACT_RELU && N % 8 == 0);
  EA_CHECK_ARG(T >= 3 && Fin >= 3 && M < (1 << 24));
  return gemm_impl(EA_BF16, 1, 0, M, N, K, A, lda, 0, 0, B, ldb, 0, 0, 1, 1, nullptr, EA_BF16, N, 0, 0, epi,
                   nullptr, 0, stream, geo, x, T, Fin, part, pos);
}


// The four parity classes of the conv2 input gradient fused with conv1's weight gradient
// (ea_gemm_conv_w1b each) as ONE launch: per-class launches each end in a partly filled round
// of 256x256 tiles (2.3-2.4 rounds per class at C3); one grid ordered longest K first fills it.
// Same tiles, same arithmetic and the same partial-tile layout as the four launches.
extern "C" int ea_gemm_conv_w1b_all(const ea_conv_geo* geo, int N, const void* A, long lda, const void* B, long ldb,
                                    const ea_epilogue* epi, const float* x, int T, int Fin, float* part,
                                    const unsigned char* pos, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(geo != nullptr && geo->mode == EA_CONV_DGRAD && x != nullptr && part != nullptr && pos != nullptr);
  EA_CHECK_ARG(epi != nullptr && epi->kind == EA_EPI_DACT && epi->act == EA_ACT_RELU);
  EA_CHECK_ARG(N >= 8 && N % 8 == 0 && geo->C % 64 == 0 && T >= 3 && Fin >= 3 && g_gemm_pipe != 0);
  EA_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0);
  GemmP p{};
  p.N = N;
  p.A = A; p.lda = lda;
  p.B = B; p.ldb = ldb;
  p.nh = 1; p.splitk = 1;
  p.C = nullptr; p.c_dtype = EA_BF16; p.ldc = N;
  p.epi = *epi;
  p.salt = ea_g_rng_salt;
  p.stamp = g_probe;
  p.diag = g_diag;
  p.g = *geo;
  p.w1x = x; p.w1part = part; p.w1pos = pos; p.w1T = T; p.w1F = Fin;
  p.vec_a = p.vec_b = p.vec_c = p.vec8 = p.lds = 1;
  p.bm = p.bn = 256;
  p.tiles_n = ea_cdiv(N, 256);
  int items = 0, tiles = 0;
  for (int c = 0; c < 4; ++c) {
    const int a = c >> 1, e = c & 1;
    const long rows = (long)geo->B * geo->nI[a] * geo->nJ[e];
    EA_CHECK_ARG(rows < (1L << 24));
    if (rows == 0) continue;
    const int k = p.ncls++;
    p.cls_item0[k] = items;
    p.cls_M[k] = (int)rows;
    p.cls_K[k] = (a ? 1 : 2) * (e ? 1 : 2) * geo->C;
    p.cls_a[k] = a;
    p.cls_e[k] = e;
    p.cls_tile0[k] = tiles;
    p.cls_pos[k] = geo->plane[c] / geo->C * (N / 8);
    tiles += (int)ea_cdiv(rows, 256);
    items += (int)ea_cdiv(rows, 256) * p.tiles_n;
  }
  if (p.ncls == 0) return 0;
  p.cls_item0[p.ncls] = items;
  p.M = p.cls_M[0]; p.K = p.cls_K[0]; p.kchunk = p.K; p.tiles_m = ea_cdiv(p.M, 256);
  const int unit = 8 * p.tiles_n;  // the block -> item map is a bijection on whole units
  const dim3 grid((unsigned)(ea_cdiv(items, unit) * unit));
  static const bool trace = std::getenv("EA_GEMM_TRACE") != nullptr;
  if (trace) std::fprintf(stderr, "[ea_gemm] conv dgrad x%d classes, %d tiles, grid %u\n", p.ncls, items, grid.x);
  return launch_pipe_conv(p, grid, (hipStream_t)stream);
}
