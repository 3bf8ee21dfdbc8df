/*
 * espnet_amd.h — C ABI of the MI355X-native ESPnet2 ASR training-step library.
 *
 * libespnet_amd.so (hand-written HIP for gfx950) is the drop-in boundary for the
 * ESPnetASRModel training step.  The reference binds NO native code
 * on this path: every op below replaces a PyTorch ATen call made by the reference's
 * Python modules; each declaration cites the reference site it replaces.
 *
 * Conventions
 *  - plain device pointers + sizes; no torch types.  `stream` is a hipStream_t.
 *  - element types: EA_F32 (float) / EA_BF16 (bfloat16); "ld" = leading dimension in
 *    elements; all matrices row-major unless stated.
 *  - every entry point returns 0 on success, EA_ERR_BAD_ARG on a bad shape/alignment, or
 *    the hipError_t of the failed launch.  Nothing allocates device memory: callers pass
 *    workspaces, so every call is hipGraph-capturable.
 */
#ifndef ESPNET_AMD_H
#define ESPNET_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

enum { EA_F32 = 0, EA_BF16 = 1 };
enum { EA_OK = 0, EA_ERR_BAD_ARG = 1000 };
enum { EA_ACT_NONE = 0, EA_ACT_SWISH = 1, EA_ACT_RELU = 2 };

/* GEMM epilogues (applied to acc = sum_k A[m,k] B[k,n]):
 *  EA_EPI_STORE : v = (alpha*acc + bias[n]) * post_scale; v = dropout(v);
 *                 C = v + beta*C                                  (Linear, scores, dW)
 *  EA_EPI_ACT   : h = alpha*acc + bias[n]; aux = h; C = dropout(act(h))
 *                 (PositionwiseFeedForward w_1 + activation + dropout)
 *  EA_EPI_RESID : v = dropout(alpha*acc + bias[n]); C(f32) = resid + rscale*v
 *                 (residual `x = residual + ff_scale*dropout(f(x))`, encoder_layer.py:115-168)
 *  EA_EPI_DACT  : v = alpha*acc * dropout_mask(seed) * act'(aux)   (backward of EPI_ACT) */
enum { EA_EPI_STORE = 0, EA_EPI_ACT = 1, EA_EPI_RESID = 2, EA_EPI_DACT = 3 };

typedef struct ea_epilogue {
  int kind;                 /* EA_EPI_* */
  int act;                  /* EA_ACT_* */
  float alpha, beta, post_scale, rscale, drop_p;
  unsigned long long seed;  /* dropout stream; element index = (z*M + m)*N + n */
  const float* bias;        /* [N] or NULL */
  void* aux;                /* pre-activation (ACT: written, DACT: read) */
  int aux_dtype;
  long ldaux;
  const float* resid;       /* RESID: f32 [M, ldr]; may alias C */
  long ldr;
} ea_epilogue;

/* Batched GEMM on MFMA (bf16: v_mfma_f32_16x16x32_bf16, f32: v_mfma_f32_16x16x4_f32 —
 * exact f32 FMA chain).  C[z][m,n] = epi( sum_k A[z][m,k] * B[z][k,n] ).
 *  a_kmajor=1: A[m,k] at A[m*lda + k]   (row-major M x K)   else A[k*lda + m]
 *  b_kmajor=1: B[k,n] at B[n*ldb + k]   (torch Linear weight N x K) else B[k*ldb + n]
 *  z in [0, batch*nh): zb = z / nh, zh = z % nh; operand offset = zb*s?b + zh*s?h.
 *  lda/ldb and the A/B base pointers must be 16-byte aligned in elements.
 *  workspace (f32, ws_elems) enables split-K for EA_EPI_STORE; NULL disables it.
 * Replaces: torch.nn.Linear / torch.matmul in transformer/attention.py:54-93,262-305,
 * positionwise_feed_forward.py:30-32, conformer/convolution.py:71-77 (1x1 convs),
 * subsampling.py:66 and their autograd backward GEMMs. */
int ea_gemm(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K,
            const void* A, long lda, long sAb, long sAh,
            const void* B, long ldb, long sBb, long sBh,
            int batch, int nh,
            void* C, int c_dtype, long ldc, long sCb, long sCh,
            const ea_epilogue* epi, float* workspace, long ws_elems, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ESPNET_AMD_H */
