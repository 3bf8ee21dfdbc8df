// Plain bf16 GEMMs through hipBLASLt (ea_gemm_set_blaslt): C = alpha * op(A) op(B) + beta * C
// with no other epilogue — the Linear input-gradient GEMMs of the backward (dX = dY . W, bf16
// out) and the few forward products without bias.  At M = 7,968 tokens and N = 512 outputs
// hipBLASLt's 128x128x64 kernels run the L2-feed-bound main loop faster than the 64x128 tile
// (DESIGN.md §7); everything with a fused epilogue (bias + activation + dropout, residual add,
// activation backward) stays on the MFMA kernels of gemm_kern.h.
//
// Row-major C (M x N, ldc) is hipBLASLt's column-major D (N x M, ldc):
//   D = op(X) . op(Y),  X = our B (N x K after op), Y = our A (K x M after op).
// One plan (descriptors + heuristic algorithm, no workspace) per shape / layout / output type,
// built on first use — in the eager warm-up, before a step is captured — and reused.
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace {

struct LtPlan {
  bool ok = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t x = nullptr, y = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
};

using LtKey = std::tuple<int, int, int, int, int, long, long, long, int>;
hipblasLtHandle_t g_lt = nullptr;
std::map<LtKey, LtPlan> g_plans;
std::mutex g_mu;

LtPlan build_plan(int a_kmajor, int b_kmajor, int M, int N, int K, long lda, long ldb, long ldc, int c_dtype) {
  LtPlan p;
  if (!g_lt && hipblasLtCreate(&g_lt) != HIPBLAS_STATUS_SUCCESS) return p;
  const hipblasOperation_t tx = b_kmajor ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  const hipblasOperation_t ty = a_kmajor ? HIPBLAS_OP_N : HIPBLAS_OP_T;
  const hipDataType cdt = c_dtype == EA_BF16 ? HIP_R_16BF : HIP_R_32F;
  bool ok = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &tx, sizeof(tx)) ==
                 HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ty, sizeof(ty)) ==
                 HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.x, HIP_R_16BF, b_kmajor ? K : N, b_kmajor ? N : K, ldb) ==
                 HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.y, HIP_R_16BF, a_kmajor ? K : M, a_kmajor ? M : K, lda) ==
                 HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.d, cdt, N, M, ldc) == HIPBLAS_STATUS_SUCCESS;
  hipblasLtMatmulPreference_t pref = nullptr;
  ok = ok && hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
  uint64_t ws = 0;  // no workspace: no split-K slabs, nothing to allocate under capture
  ok = ok && hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws,
                                                   sizeof(ws)) == HIPBLAS_STATUS_SUCCESS;
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  ok = ok && hipblasLtMatmulAlgoGetHeuristic(g_lt, p.desc, p.x, p.y, p.d, p.d, pref, 1, res, &n) ==
                 HIPBLAS_STATUS_SUCCESS;
  ok = ok && n > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS && res[0].workspaceSize == 0;
  if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  if (ok) {
    p.algo = res[0].algo;
    p.ok = true;
  }
  return p;
}

}  // namespace

// bit 1: plain GEMMs with N <= 512 and M >= 4096 (the L2-feed-bound family); bit 2: every other
// plain GEMM with M >= 4096; 0 = off (EA_GEMM_BLASLT).  Default 1: C3 step 1775-1776 ->
// 1787-1790 utt/s (mode 3: 1784-1787), profiles/r4_blaslt_ab.txt
int g_gemm_blaslt = [] { const char* e = std::getenv("EA_GEMM_BLASLT"); return e ? std::atoi(e) : 1; }();

extern "C" int ea_gemm_set_blaslt(int mode) {
  EA_ENTRY();
  EA_CHECK_ARG(mode >= 0 && mode <= 3);
  g_gemm_blaslt = mode;
  return 0;
}

// 0: launched on hipBLASLt; 1: not eligible / no algorithm (the caller runs its own kernels)
int ea_blaslt_try(int a_kmajor, int b_kmajor, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                  void* C, int c_dtype, long ldc, float alpha, float beta, hipStream_t st) {
  // M >= 4096: at the decoder's 1,312 tokens hipBLASLt is slower than the tile kernels
  // (1312x512x512: 21.4 vs 11.6 us, 1312x512x2048: 17.4 vs 15.6 us; scripts/gemm_rows_ab.py)
  if (!g_gemm_blaslt || M < 4096 || K < 64) return 1;
  if (!((N <= 512 && (g_gemm_blaslt & 1)) || (N > 512 && (g_gemm_blaslt & 2)))) return 1;
  const LtKey key{a_kmajor, b_kmajor, M, N, K, lda, ldb, ldc, c_dtype};
  LtPlan* p;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) it = g_plans.emplace(key, build_plan(a_kmajor, b_kmajor, M, N, K, lda, ldb, ldc, c_dtype)).first;
    p = &it->second;
  }
  if (!p->ok) return 1;
  const hipblasStatus_t s = hipblasLtMatmul(g_lt, p->desc, &alpha, B, p->x, A, p->y, &beta, C, p->d, C, p->d,
                                            &p->algo, nullptr, 0, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1;
}
