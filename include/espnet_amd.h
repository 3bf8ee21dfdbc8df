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

#include <stddef.h>

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
 *  16-B aligned bases / leading dims take 16-B vector loads; others an element-wise path.
 *  Contract of the 16-B (LDS-DMA) path for an MN-major bf16 operand whose extent MN (M for
 *  A, N for B) is not a multiple of 8: every row, the last one included, is read in whole
 *  16-B chunks up to MN rounded up to 8, so the caller keeps that many elements readable
 *  past the row start (hip_ops.gemm re-homes a view that ends closer to its allocation's
 *  end; the values read past MN never reach C).
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


/* Implicit GEMMs of Conv2dSubsampling's second Conv2d(C, C, 3, stride 2) (subsampling.py:
 * 60-65) over a phase-split conv1 output x1p: class plane (a, e) = pixels t1 = 2i+a,
 * f1 = 2j+e stored dense as [b][i][j][C] (dims nI[a] x nJ[e]) at element offset
 * plane[a*2+e].  Every tap of every conv2 pixel is then one contiguous C-row, gathered by
 * the LDS-DMA loader (no im2col buffer):
 *  EA_CONV_FWD  : A[m = (b,t2,f2)][k = (cb,kh,kw,c)] = x1p row (64-channel blocks cb, the 9
 *                 taps of a block consecutive in k, c < 64 within the block); B = W2p
 *                 [Co][C/64][9][64] K-major (a_kmajor = b_kmajor = 1); out (P, Co).
 *  EA_CONV_DGRAD: input gradient for one parity class (a, e) (sub-pixel decomposition of the
 *                 transposed conv): A[m = (b,i,j)][k = (tap of class, co)] = dY2 row of
 *                 (t2, f2) = ((2i+a-kh)/2, (2j+e-kw)/2), or one of 64 zero rows at `zero`
 *                 (element offset from A; 64*C zeros: spread so off-grid reads do not all
 *                 hit one L2 channel) off the grid; B = W2t [9][co][ci] (tap-major) N-major
 *                 (b_kmajor = 0, ldb = C); out = the class plane of dx1p (M = B*nI*nJ).
 *  EA_CONV_WGRAD: weight gradient: A = dY2 (P x Co) read M-major (a_kmajor = 0, lda = Co),
 *                 B[k = pixel][n = (tap, ci)] = x1p row gathered (b_kmajor = 0); K = P
 *                 rounded up to 64 with dY2 rows P..K-1 zero and 64 zero rows of x1p at `zero`.
 * bf16 operands only; C % 64 == 0; K % 64 == 0.  Replaces the im2col + GEMM + col2im of the
 * channel-last conv2 (and torch's cudnn/miopen conv) on the AMP path. */
enum { EA_CONV_FWD = 1, EA_CONV_DGRAD = 2, EA_CONV_WGRAD = 3 };
typedef struct ea_conv_geo {
  int mode;              /* EA_CONV_* */
  int B, T2, F2, C, P;   /* conv2 output grid (P = B*T2*F2 pixels), channels */
  int nI[2], nJ[2];      /* class-plane dims: nI[a] = (T1 - a + 1) / 2, nJ[e] = (F1 - e + 1) / 2 */
  int a, e;              /* DGRAD: the parity class */
  long plane[4];         /* element offsets of the 4 class planes in x1p */
  long zero;             /* element offset of 64 zero rows (64*C) in the gathered operand */
} ea_conv_geo;
int ea_gemm_conv(const ea_conv_geo* geo, int a_kmajor, int b_kmajor, int M, int N, int K,
                 const void* A, long lda, const void* B, long ldb, void* C, int c_dtype, long ldc,
                 const ea_epilogue* epi, float* workspace, long ws_elems, void* stream);
/* The EA_CONV_DGRAD launch of one parity class fused with conv1's weight gradient: the
 * ReLU-masked input gradient g (epi: EA_EPI_DACT, EA_ACT_RELU, aux = the class plane of x1p,
 * bf16) is not stored; instead each 256-row tile tm writes
 *   part[tm*10*N + t*N + c] = sum over its rows m of bf16(g[m][c]) * X[m][t],
 *   X = x[b][2*t1 + t/3][2*f1 + t%3] (t < 9) for the pixel (b, t1, f1) of class-plane row m,
 *   X = 1 (t = 9),
 * x = the conv1 input (B, T, Fin) f32 — subsampling.py conv.0's weight / bias gradient
 * (torch Conv2d backward) without the dx1 round trip through HBM.  part holds ceil(M/256)
 * tiles; ea_conv1_wgrad_reduce sums any number of such tiles into dw [N][9] / dbias [N]. */
int ea_gemm_conv_w1(const ea_conv_geo* geo, int M, int N, int K, const void* A, long lda, const void* B,
                    long ldb, const ea_epilogue* epi, const float* x, int T, int Fin, float* part,
                    void* stream);
/* ea_gemm_conv_w1 with the ReLU mask read from ea_conv1_fwd2's support bits of the class plane
 * (pos = bits of the plane's first row, N/8 bytes per row) instead of the bf16 aux rows. */
int ea_gemm_conv_w1b(const ea_conv_geo* geo, int M, int N, int K, const void* A, long lda, const void* B,
                     long ldb, const ea_epilogue* epi, const float* x, int T, int Fin, float* part,
                     const unsigned char* pos, void* stream);
/* The four parity classes (a, e) = (0,0), (0,1), (1,0), (1,1) of ea_gemm_conv_w1b in one
 * launch (geo: EA_CONV_DGRAD with nI / nJ / plane; a, e ignored): class c has
 * M_c = B*nI[a]*nJ[e] rows and K_c = (a ? 1 : 2)*(e ? 1 : 2)*C, its mask bits start at row
 * plane[c]/C of pos, and its ceil(M_c/256) partial tiles follow the previous classes' in part —
 * the same results as the four ea_gemm_conv_w1b calls in that order, bit for bit.  B is conv2's
 * weight as W2t [9][co][ci] (ldb = C) or as W2k [ci][9][co] (ldb = 9*C, K-major fragment reads;
 * the same products in the same order, so the same results). */
int ea_gemm_conv_w1b_all(const ea_conv_geo* geo, int N, const void* A, long lda, const void* B, long ldb,
                         const ea_epilogue* epi, const float* x, int T, int Fin, float* part,
                         const unsigned char* pos, void* stream);
int ea_conv1_wgrad_reduce(int ntiles, int C, const float* part, float* dw, float* dbias, void* stream);

/* Select the bf16 GEMM main loop: 2 = LDS-DMA (global_load_lds) 2-stage ring (default),
 * 0 = register-staged loop; 12 = same ring without 64-row tiles.
 * Process-wide; for A/B measurements. */
int ea_gemm_set_pipeline(int stages);

/* Pin the bf16 LDS-DMA GEMM output tile (bm x bn in {32x128, 64x128, 128x128, 256x256});
 * 0,0 = automatic choice by grid size.  Process-wide; for tests and tuning. */
int ea_gemm_set_tile(int bm, int bn);
/* Route 256x256-tile bf16 GEMMs to the pipelined kernel (gemm_pipe: 4-slot ring of 32-deep
 * K slices, counted vmcnt, one barrier per slice) when on != 0 (A/B switch). */
int ea_gemm_set_pipe(int on);
/* gemm_k128 (128x128 tile, K-major A and B, one block per CU of 8 waves in two K groups, 64-deep
 * K-tiles through a `slots`-deep (3 or 4) LDS ring) for bf16 GEMMs: mode 0 off, 1 =
 * where a 64x128 / 128x128 tile was chosen and the 128x128 grid has 128-256 tiles (the
 * N = 512 GEMMs at M = 7,968), 2 = such grids of any size >= 128 tiles, 3 = every eligible
 * GEMM (K % 64 == 0; tests); mode 1 also needs K >= 1024.  Default 1.  Process-wide (EA_GEMM_K128). */
int ea_gemm_set_k128(int mode, int slots);
/* bf16 GEMMs with M <= max_m rows (K-major A and B, K % 32 == 0, unbatched: the incremental
 * decoder's per-step Linears) on gemm_skinny — 16 x 32 output blocks whose 8 waves split K,
 * operands loaded straight into MFMA fragments, partial tiles summed through LDS before the
 * epilogue.  0 = off; default 16 (EA_GEMM_SKINNY).  Process-wide. */
int ea_gemm_set_skinny(int max_m);
/* C = epi(LayerNorm(x) . W^T): x f32 (M x K, ldx, rows 16-B aligned), gamma / beta f32 (K),
 * W bf16 (N x K, ldw) — the LayerNorm (eps) computed per row inside the few-row GEMM
 * (16 x 32 blocks, 8 waves splitting K) and rounded to bf16 in the MFMA operand registers,
 * as the unfused path stores it.  K % 32 == 0, K <= 2048.  Any epilogue of ea_gemm.
 * Replaces a LayerNorm (layer_norm.py) + Linear pair of the incremental decoder's step. */
int ea_gemm_ln(int M, int N, int K, const float* x, long ldx, const float* gamma, const float* beta, float eps,
               const void* W, long ldw, void* C, int c_dtype, long ldc, const ea_epilogue* epi, void* stream);

/* One problem of a grouped launch: C[M,N] (f32, row stride ldc) = beta*C + op(A) op(B), bf16
 * operands in the layouts of ea_gemm (a_kmajor/b_kmajor shared by the group), lda/ldb
 * multiples of 8 elements, 16-B aligned bases, N and ldc multiples of 4. */
typedef struct ea_group_gemm {
  const void* A;
  const void* B;
  float* C;
  long lda, ldb, ldc;
  int M, N, K;
  float beta;
} ea_group_gemm;
/* n independent GEMMs in ONE launch, every tile 256x256 over the problem's whole K on the
 * pipelined main loop (problems in the given order: put the longest K first).  Replaces the
 * per-Linear weight-gradient GEMMs of a backward pass (torch.nn.Linear weight.grad
 * accumulation, e.g. espnet/nets/pytorch_backend/transformer/positionwise_feed_forward.py:
 * 30-32 w_1/w_2) when they are deferred to one batch.  `ws`: device workspace of at least
 * ea_gemm_grouped_ws_bytes(n, ntiles) bytes (ntiles = sum of ceil(M/256)*ceil(N/256)) holding
 * the problem table; it must stay untouched until the launch has run (stream order).
 * Problems writing overlapping C must not share a call. */
int ea_gemm_grouped(int a_kmajor, int b_kmajor, int n, const ea_group_gemm* probs, void* ws, long ws_bytes,
                    void* stream);
/* *bytes = workspace size ea_gemm_grouped needs for n problems with ntiles output tiles. */
int ea_gemm_grouped_ws_bytes(int n, long ntiles, long* bytes);
/* Tile -> XCD assignment of ea_gemm_grouped: chunks of `chunk` consecutive tiles go to one XCD
 * and successive chunks round-robin over the 8 XCDs, so every XCD walks the longest-K-first
 * order at the same pace (default 4, EA_GROUPED_XCD_CHUNK); 0 = one contiguous 1/8 of the
 * tiles per XCD.  Process-wide; A/B switch. */
int ea_gemm_grouped_set_xcd_chunk(int chunk);

/* Kernel-span probe for measurement (bench.py): slots = 4 device u64
 * {span start, span end, sum of spans, count} in units of the GPU's constant 100 MHz
 * clock (s_memrealtime).  ea_probe_begin resets the span; ea_gemm launches made while
 * ea_gemm_set_probe(slots) is set stamp their first-block start / last-block end into it;
 * ea_probe_end adds the span to the sum.  All three are stream-ordered kernels, so a
 * captured hipGraph re-measures on every replay (torch-ROCm refuses timing events inside
 * captured graphs).  The LDS-DMA bf16 GEMM path only. */
int ea_gemm_set_probe(unsigned long long* slots);
/* Diagnostics only: while buf != NULL, gemm_pipe launches write per block (block b = x + gridDim.x*z)
 * buf[4b..4b+3] = {shader clock at start, after the main loop, at the end, 100 MHz clock at start}.
 * buf must hold 4 * blocks entries. */
int ea_gemm_set_diag(unsigned long long* buf);
/* Device-side step phase timer (Reporter forward_time / backward_time / optim_step_time,
 * espnet2/train/trainer.py:566,623,682): phase 0 marks the step start, phases 1..3 write the
 * seconds since the previous stamp into ring[slot*4 + phase-1] (slot = step counter % cap),
 * phase 3 also copies *extra (e.g. the optimizer's device lr; NULL: 0) into ring[slot*4+3]
 * and advances the counter.  state = {last stamp, step counter} (2 x u64, zeroed). */
int ea_phase_stamp(unsigned long long* state, float* ring, int cap, int phase, const float* extra, void* stream);
/* ea_phase_stamp with the optimizer's device state: phase 3 records opt->next_lr as the extra
 * value and NaN as the optimizer duration when opt->skip (the update was skipped: the
 * reference registers no optim_step_time then, trainer.py:662-682). */
struct ea_opt_state;
int ea_phase_stamp_opt(unsigned long long* state, float* ring, int cap, int phase, const struct ea_opt_state* opt,
                       void* stream);
int ea_probe_begin(unsigned long long* slots, void* stream);
int ea_probe_end(unsigned long long* slots, void* stream);
/* Stream-ordering diagnostic: hold `stream` for ns nanoseconds (0 <= ns <= 1e8) with one
 * sleeping single-lane workgroup.  hip_ops launches it at the head of every side / auxiliary
 * stream segment under EA_DEBUG_DELAY_NS, so a missing cross-stream dependency shows up in
 * every run instead of now and then (tests/test_dp_streams_gpu.py).  Not on the product path. */
int ea_debug_spin(long ns, void* stream);
/* Diagnostic device allocator for torch.cuda.memory.CUDAPluggableAllocator (the pluggable
 * allocator's malloc / free signatures): each allocation is a fresh hipMalloc with a zeroed
 * body and a 64 KiB tail guard of 0xFF bytes (NaN in f32 / bf16), so a kernel reading past
 * the end of a buffer turns its output NaN deterministically; free synchronises the device
 * before hipFree.  Never on the product path (scripts/dp_drift_diag.py --guard). */
void* ea_guard_malloc(size_t size, int device, void* stream);
void ea_guard_free(void* ptr, size_t size, int device, void* stream);

/* ---------------------------------------------------------------- normalisation */

/* LayerNorm(eps) over the last dim, one wave64 per row; y in y_dtype, saves mean/rstd.
 * Replaces torch.nn.LayerNorm in transformer/layer_norm.py:12-42 (eps 1e-12), used
 * 5x per conformer block (encoder_layer.py:61-70), after_norm, decoder norm1-3. */
int ea_layernorm_fwd(int rows, int d, const float* x, long ldx, const float* gamma,
                     const float* beta, float eps, void* y, int y_dtype, long ldy,
                     float* mean, float* rstd, void* stream);

/* LayerNorm backward: dx (+)= ..., dgamma/dbeta (+)= (dbeta must equal dgamma + d:
 * weight and bias grads are adjacent in the parameter arena).
 * workspace >= min(ceil(rows/4),512) * 2d floats. */
int ea_layernorm_bwd(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x,
                     long ldx, const float* gamma, const float* mean, const float* rstd,
                     float* dx, long lddx, int accumulate, float* dgamma, float* dbeta,
                     int accumulate_params, float* workspace, long ws_elems, void* stream);

/* out[c] (+)= sum_p part[p*stride + c] in fixed order (deterministic). */
int ea_reduce_partials(int nparts, int n, const float* part, long stride, float* out,
                       int accumulate, void* stream);

/* out[c] (+)= sum_r x[r*ld + c]  — Linear bias gradients (autograd sum over rows). */
int ea_colsum(int rows, int n, const void* x, int x_dtype, long ld, float* out, int accumulate,
              float* workspace, long ws_elems, void* stream);

/* LayerNorm backward without the parameter-gradient reduction: dx as ea_layernorm_bwd, the
 * per-row-block (dgamma | dbeta) partials written to part ([*nparts][2d]; part_elems sets the
 * row-block size exactly as ea_layernorm_bwd's ws_elems does), to be summed by
 * ea_reduce_grouped (deferred: one launch for a whole backward pass). */
int ea_layernorm_bwd_partials(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x,
                              long ldx, const float* gamma, const float* mean, const float* rstd,
                              float* dx, long lddx, int accumulate, float* part, long part_elems,
                              int* nparts, void* stream);

/* The two entries above plus the next residual site's dropout backward: y = dropout(yscale *
 * dx) after dx is final (ea_scale_dropout's mask law, index r*d + c), written by the LayerNorm
 * kernel itself when dy and y are bf16 (vectorized rows), else by an ea_scale_dropout pass.
 * ycol (optional): ycol += column sums of the stored y (that site's bias gradient) -- from the
 * LayerNorm kernel's own per-block partials when in-kernel.  In partials mode those y partials
 * ([*nparts][d], right after the [*nparts][2d] LayerNorm partials in part; part_elems must hold
 * 3d per row block) are left to the caller when *ycol_parts = 1; *ycol_parts = 0 means ycol was
 * already accumulated.  Saves the f32 dx and bf16 y re-reads of the Conformer block's backward
 * (encoder_layer.py:115-171: every norm_* backward is followed by a dropout backward). */
int ea_layernorm_bwd_drop(int rows, int d, const void* dy, int dy_dtype, long lddy, const float* x,
                          long ldx, const float* gamma, const float* mean, const float* rstd, float* dx,
                          long lddx, int accumulate, float* dgamma, float* dbeta, int accumulate_params,
                          float* workspace, long ws_elems, void* y, int y_dtype, long ldy, float yscale,
                          float p, unsigned long long seed, float* ycol, void* stream);
int ea_layernorm_bwd_partials_drop(int rows, int d, const void* dy, int dy_dtype, long lddy,
                                   const float* x, long ldx, const float* gamma, const float* mean,
                                   const float* rstd, float* dx, long lddx, int accumulate, float* part,
                                   long part_elems, int* nparts, void* y, int y_dtype, long ldy,
                                   float yscale, float p, unsigned long long seed, float* ycol,
                                   int* ycol_parts, void* stream);

/* Grouped reductions of a backward pass's parameter gradients (bias grads of every Linear:
 * torch.nn.Linear bias.grad; LayerNorm weight/bias grads: torch.nn.LayerNorm in
 * espnet/nets/pytorch_backend/transformer/layer_norm.py:12-42).  A column-sum problem writes
 * the row-block partials part[ceil(rows/rpp)][n]; a reduce problem sums out[c] (+)=
 * sum_p part[p*stride + c] in fixed order (f64).  ws: device workspace for the problem table
 * (ea_grouped_table_bytes), untouched until the launch has run. */
typedef struct ea_colsum_prob {
  const void* x;
  float* part;
  long ld;
  int rows, n, dtype, rpp;
} ea_colsum_prob;
typedef struct ea_reduce_prob {
  const float* part;
  float* out;
  long stride;
  int nparts, n, accumulate;
} ea_reduce_prob;
int ea_colsum_grouped(int n, const ea_colsum_prob* probs, void* ws, long ws_bytes, void* stream);
int ea_reduce_grouped(int n, const ea_reduce_prob* probs, void* ws, long ws_bytes, void* stream);
int ea_grouped_table_bytes(int n, long* colsum_bytes, long* reduce_bytes);

/* BatchNorm1d (training: batch stats over ALL rows incl. padding, running stats update
 * with momentum and unbiased var, num_batches_tracked += 1; eval: given mean/rstd) fused
 * with the following activation: z = act(BN(y)).  y, z: (rows, C) channel-last.
 * Replaces conformer/convolution.py:45,75 (norm + Swish).
 * workspace >= min(ceil(rows/16), 256) * 2C floats (training). */
int ea_batchnorm_fwd(int rows, int C, const float* y, const float* gamma, const float* beta,
                     float eps, float momentum, int training, float* mean, float* rstd,
                     float* running_mean, float* running_var, long long* num_batches_tracked,
                     int act, void* z, int z_dtype, float* workspace, long ws_elems, void* stream);

/* ea_batchnorm_fwd (training) from precomputed shifted partial sums part[nparts][2C] of y
 * (sum (y - shift[c]), sum (y - shift[c])^2): fp64 finalize (mean, rstd, running stats,
 * num_batches_tracked) and the BN + activation pass.  C % 4 == 0. */
int ea_batchnorm_fwd_parts(int rows, int C, const float* y, const float* part, int nparts, const float* shift,
                           const float* gamma, const float* beta, float eps, float momentum, float* mean,
                           float* rstd, float* running_mean, float* running_var, long long* num_batches_tracked,
                           int act, void* z, int z_dtype, void* stream);

/* Backward of z = act(BN_train(y)): dy, dgamma/dbeta (dbeta == dgamma + C).
 * workspace >= (min(ceil(rows/16), 256) + 1) * 2C floats. */
int ea_batchnorm_bwd(int rows, int C, const void* dz, int dz_dtype, const float* y, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int act, float* dy,
                     float* dgamma, float* dbeta, int accumulate_params, float* workspace,
                     long ws_elems, void* stream);

/* ---------------------------------------------------------------- elementwise / layout */

/* utterance_mvn(norm_means=True, norm_vars=False), espnet2/layers/utterance_mvn.py:45-88:
 * x (B,T,F) f32 -> y = (x masked to valid frames) - per-utterance mean. F <= 256. */
int ea_utterance_mvn(int B, int T, int F, const float* x, const long long* lens, float* y, void* stream);
/* Same op over a (32-row chunk, utterance) grid in two launches (chunk column sums in f64,
 * then mean + write); ws holds ea_utterance_mvn_ws_bytes(B, T, F) bytes (any alignment of 8). */
int ea_utterance_mvn_ws_bytes(int B, int T, int F, long* bytes);
int ea_utterance_mvn2(int B, int T, int F, const float* x, const long long* lens, float* y, void* ws,
                      long ws_bytes, void* stream);

/* Raw-waveform frontend (espnet2/asr/frontend/default.py:17-140), four launches around two
 * f32 GEMMs (ea_gemm, exact-f32 MFMA):
 *  ea_stft_frames: frames[b*nF + f][k] = window[k] * x[b][reflect(f*hop + k - pad)], pad =
 *    center ? n_fft/2 : 0 (torch.stft center/reflect, layers/stft.py:88-100); window has n_fft
 *    entries (a shorter win_length zero-padded to the centre, as torch.stft does);
 *  [GEMM frames x [cos | -sin] basis (n_fft x 2*nbins) -> spec (M, 2*nbins)]
 *  ea_power_spectrum: power = re^2 + im^2, frames f >= flens[b] zero (stft.py:107-114);
 *  [GEMM power x melmat (nbins x n_mels)]
 *  ea_logmel_mvn: log(max(mel, 1e-10)), frames >= flens zero (layers/log_mel.py:60-84), and
 *    when mean/std are given the GlobalMVN below fused in;
 *  ea_global_mvn: (x - mean) zeroed past lens, / std (layers/global_mvn.py:73-104); mean/std
 *    NULL skip that part (norm_means / norm_vars false). */
int ea_stft_frames(int B, long Ns, int nF, int n_fft, int hop, int center, const float* x,
                   const float* window, float* frames, void* stream);
int ea_power_spectrum(long M, int nF, int nbins, const float* spec, long ld_spec, const long long* flens,
                      float* power, long ld_power, void* stream);
int ea_logmel_mvn(long M, int nF, int n_mels, const float* mel, long ld_mel, const long long* flens,
                  const float* mean, const float* std, float* y, void* stream);
int ea_global_mvn(int B, int T, int D, const float* x, const long long* lens, const float* mean,
                  const float* std, float* y, void* stream);

/* SpecAugment, espnet2/asr/specaug/specaug.py:95-102 = TimeWarp (layers/time_warp.py:9-88,
 * bicubic, align_corners=False) -> MaskAlongAxis(freq) -> MaskAlongAxis(time)
 * (layers/mask_along_axis.py:8-68, replace_with_zero), one pass over x (B,T,F) f32 -> y.
 * The draws are the caller's (the reference's torch.randint calls, in its order):
 *  warp  [B][2] (center, warped): center <= 0 leaves utterance b unwarped;
 *  per_utt = 1: TimeWarp's per-utterance path (lengths differ): utterance b is warped over
 *               its first lengths[b] frames and frames >= lengths[b] are zero (pad_list 0.0);
 *          = 0: the equal-length path: the whole T axis is warped, nothing is zero-filled;
 *  fmask [B][nf][2], tmask [B][nt][2]: (position, width) spans set to 0.
 * Replaces the reference's per-utterance interpolate loop (time_warp.py:78-86). */
int ea_specaug(int B, int T, int F, const float* x, const long long* lengths, const int* warp, int per_utt,
               const int* fmask, int nf, const int* tmask, int nt, float* y, void* stream);

/* encoder_out_lens of Conv2dSubsampling from the sliced mask, subsampling.py:91 +
 * conformer_encoder.py:374. */
int ea_subsample_lens(int B, int T, const long long* ilens, long long* olens, void* stream);

/* add_sos_eos + pad_list (transformer/add_sos_eos.py:12-31); ys_in/ys_out (B, L+1). */
int ea_add_sos_eos(int B, int L, const long long* ys, long ldys, const long long* ylens, int sos,
                   int eos, int ignore_id, long long* ys_in, long long* ys_out,
                   long long* ys_in_lens, void* stream);

/* y = dropout(x * scale) with the counter-based mask (index = r*cols + c). */
int ea_scale_dropout(long rows, int cols, const void* x, int x_dtype, long ldx, void* y,
                     int y_dtype, long ldy, float scale, float p, unsigned long long seed,
                     void* stream);

/* ea_scale_dropout (f32 x) fused with the column sums of the stored y accumulated into
 * colsum[cols] (deterministic two-level sum): the gradient entering a Linear on a dropped-out
 * residual branch and that Linear's bias gradient (encoder_layer.py:115-168 backward) from
 * one read of x.  Needs a workspace of ceil(rows/max(32, rows/128)) * cols floats. */
int ea_scale_dropout_colsum(long rows, int cols, const float* x, long ldx, void* y, int y_dtype, long ldy,
                            float scale, float p, unsigned long long seed, float* colsum, int accumulate,
                            float* workspace, long ws_elems, void* stream);

/* y[r, c] += alpha * x[r, c] (mixed dtypes) — autograd's gradient accumulation of a
 * tensor consumed twice (q + pos_bias_u and q + pos_bias_v, attention.py:287-301). */
int ea_add_2d(long rows, int cols, const void* x, int x_dtype, long ldx, void* y, int y_dtype,
              long ldy, float alpha, void* stream);

/* dst[a][c][b] (+)= src[a][b][c]: weight repacks (Conv2d (Co,Ci,9) <-> (Co,9,Ci); the
 * subsampling Linear's (O, C, F) <-> (O, F, C) for channel-last activations). */
int ea_permute3(int A, int Bd, int Cd, const void* src, int src_dtype, void* dst, int dst_dtype,
                int accumulate, void* stream);

/* Conv2dSubsampling (subsampling.py:60-65) as GEMMs over channel-last activations:
 * conv1 rows (b,t1,f1) x 16 taps (9 used); conv2 rows (b,t2,f2) x (kh,kw,c); the input
 * gradient of conv2 by a gather col2im fused with conv1's ReLU mask. */
int ea_im2col_conv1(int B, int T, int F, const float* x, void* col, int col_dtype, void* stream);
int ea_im2col_conv2(int B, int T1, int F1, int C, const void* x1, void* col, int dtype, void* stream);
int ea_col2im_conv2(int B, int T1, int F1, int C, const void* dcol, int dcol_dtype, const void* x1,
                    void* dx1, int dtype, void* stream);

/* conv1 of Conv2dSubsampling (Conv2d(1, C, 3, stride 2) + ReLU, subsampling.py:60-61) as a
 * direct kernel writing the phase-split layout of ea_conv_geo (x1p, B*T1*F1 rows of C);
 * w (C, 9) f32.  ea_conv1_wgrad: dw[c*9 + t] += sum_p dh[p,c] x_t(p), dbias[c] += sum_p
 * dh[p,c] from the phase-split pre-activation gradient dh (deterministic block partials;
 * workspace >= 10*C floats per block, up to 1024 blocks). */
int ea_conv1_fwd(int B, int T, int F, int C, const float* x, const float* w, const float* bias,
                 void* x1p, int dtype, void* stream);
/* ea_conv1_fwd that also writes the ReLU support of x1p as bits: pos[row*(C/8) + c/8] bit
 * (c & 7) = (x1p[row][c] > 0), rows in x1p's phase-split order (the backward's ReLU mask at
 * 1/16 of x1p's bytes; NULL: none). */
int ea_conv1_fwd2(int B, int T, int F, int C, const float* x, const float* w, const float* bias,
                  void* x1p, int dtype, unsigned char* pos, void* stream);
int ea_conv1_wgrad(int B, int T, int F, int C, const float* x, const void* dh, int dtype, float* dw,
                   float* dbias, float* workspace, long ws_elems, void* stream);

/* GLU over channels (conformer/convolution.py:72): y = x[:, :C] * sigmoid(x[:, C:]). */
int ea_glu_fwd(long rows, int C, const void* x, int x_dtype, void* y, int y_dtype, void* stream);
int ea_glu_bwd(long rows, int C, const void* x, int x_dtype, const float* dy, void* dx, void* stream);

/* Depthwise Conv1d(C, C, K, pad (K-1)/2, groups=C) over time, channel-last (B,T,C) f32
 * (conformer/convolution.py:38-45,75).  bwd: dx, dw (C,K), dbias. */
int ea_dwconv_fwd(int B, int T, int C, int K, const float* x, const float* w, const float* bias,
                  float* y, void* stream);
int ea_dwconv_bwd(int B, int T, int C, int K, const float* x, const float* w, const float* dy,
                  float* dx, float* dw, float* dbias, int accumulate_params, float* workspace,
                  long ws_elems, void* stream);
/* ea_dwconv_bwd (K in {3,5,7,15,31}) with the GLU backward that precedes the depthwise conv in
 * the backward (conformer/convolution.py:64-66, x = glu(g2)) fused into the input-gradient
 * store: g2 = [a | b] (rows x 2C bf16, the pointwise_conv1 output), dg2 (rows x 2C bf16) =
 * (dx * sigmoid(b), dx * a * sigmoid(b) * (1 - sigmoid(b))) — the arithmetic of ea_dwconv_bwd
 * followed by ea_glu_bwd (equal up to the f32 rounding of the tap sums); dx is never stored. */
int ea_dwconv_glu_bwd(int B, int T, int C, int K, const float* x, const float* w, const float* dy,
                      const void* g2, void* dg2, float* dw, float* dbias, int accumulate_params,
                      float* workspace, long ws_elems, void* stream);
/* x == NULL in ea_dwconv_glu_bwd: the conv input is recomputed as glu(g2) (C % 4 == 0, g2 8-B
 * aligned).  ea_dwconv_fwd_glu: ea_dwconv_fwd of x = glu(g2) = a * sigmoid(b) computed from the
 * bf16 pointwise_conv1 output in the tile loader (ea_glu_fwd's arithmetic, f32): the GLU
 * activation (convolution.py:66) is never stored. */
int ea_dwconv_fwd_glu(int B, int T, int C, int K, const void* g2, const float* w, const float* bias,
                      float* y, void* stream);
/* ea_dwconv_fwd_glu that also writes the following BatchNorm's batch-statistics partials
 * (convolution.py:75) of each (utterance, 64-frame tile) block: part[p][c] = sum (y - bias[c]),
 * part[p][C + c] = sum (y - bias[c])^2, p < *nparts (ea_dwconv_stats_parts); ea_batchnorm_fwd_parts
 * then finalizes them (shift = bias) and applies BN + activation without a statistics pass over y. */
int ea_dwconv_fwd_glu_stats(int B, int T, int C, int K, const void* g2, const float* w, const float* bias,
                            float* y, float* part, void* stream);
int ea_dwconv_stats_parts(int B, int T, int* nparts);
/* q + pos_bias_u / q + pos_bias_v (attention.py:287-290) for the fused qkv rows. */
int ea_add_pos_bias(long N, int H, int dk, const void* q, long ldq, const float* u, const float* v,
                    void* qu, void* qv, int dtype, void* stream);

/* Decoder Embedding + PositionalEncoding (x*sqrt(d) + pe, dropout), embedding.py:81-92;
 * backward adds into the embedding gradient in a fixed order (no atomics; rows <= 4096). */
int ea_embed_fwd(long rows, int d, int L, const long long* tok, const float* E, float xscale,
                 const float* pe, float p, unsigned long long seed, float* y, void* stream);
/* y = dropout(y + pe[r % L]) in place over rows x d (f32): the absolute PositionalEncoding
 * added after Conv2dSubsampling's Linear for encoder: transformer (TransformerEncoder,
 * espnet2/asr/encoder/transformer_encoder.py:94 -> subsampling.py:66-69 + embedding.py:81-92;
 * the Linear epilogue applies the x*sqrt(d) scale).  Dropout index r*d + c (ea_scale_dropout's
 * law), so the backward is ea_scale_dropout_colsum with scale sqrt(d). */
int ea_add_pe_dropout(long rows, int d, int L, const float* pe, float p, unsigned long long seed, float* y,
                      void* stream);
int ea_embed_bwd(long rows, int d, const long long* tok, const float* dy, float xscale, float p,
                 unsigned long long seed, float* dE, void* stream);

/* Dropout salt: all later launches read a per-step salt from device memory `salt`
 * (NULL: none) and mix it into their site seeds; ea_rng_advance adds 1 on the stream.
 * A captured hipGraph of a training step thus draws a fresh mask stream on each replay,
 * as the reference's torch.nn.Dropout (bernoulli_) does per call. */
int ea_set_rng_salt(const unsigned long long* salt);
int ea_rng_advance(unsigned long long* salt, void* stream);

/* CTC.argmax (ctc.py:119-127): first maximal index per row (bit-exact alignment). */
int ea_argmax_rows(long rows, int V, const float* x, long ld, long long* out, void* stream);

/* ---------------------------------------------------------------- attention */

/* P = masked_softmax(scale*(S + rel_shift(BD))), Pd = dropout(P) — attention.py:63-93,
 * 262-305.  S [z][i][ldS] (z = b*H + h), BD [h][b][i][ldBD] (rel-pos, T1 == T2) or NULL,
 * key j valid iff j < klen[b] (klen NULL: all) and (!causal || j <= i). */
int ea_attn_softmax_fwd(int B, int H, int T1, int T2, float scale, const float* S, long ldS,
                        const float* BD, long ldBD, const long long* klen, int causal, float p,
                        unsigned long long seed, float* P, long ldP, void* Pd, int pd_dtype,
                        long ldPd, void* stream);

/* dS = scale * P*(dP - rowsum(P*dP)), dP = dropout_bwd(dPd); if dBD != NULL also
 * dBD[h][b][i][r] = dS[i, r-(T1-1-i)] (0 off the band) for r < 2*T1-1. */
int ea_attn_softmax_bwd(int B, int H, int T1, int T2, float scale, const float* dPd, long ldd,
                        const float* P, long ldP, float p, unsigned long long seed, void* dS,
                        int ds_dtype, long ldS, void* dBD, long ldBD, void* stream);

/* Fused attention core, head dim 64, bf16 q/k/v (relattn.hip): per (b, h)
 *   s[i,j] = ((q_i + bu)·k_j + (q_i + bv)·pp[T-1-i+j]) * scale   (pp != NULL: rel-pos,
 *            RelPositionMultiHeadedAttention with rel_shift, attention.py:262-305; T1 == T2)
 *   s[i,j] = ((q_i + bu)·k_j) * scale                            (pp == NULL; bu may be NULL)
 *   key j valid iff j < klen[b] (klen NULL: all) and (!causal || j <= i); P = softmax (fully
 *   masked row: 0); O = dropout(P)·V (mask index (z*T1 + i)*T2 + j, z = b*H + h).
 * q rows b*T1 + i, k/v rows b*T2 + j, pp rows r < 2*T1-1, head h at column h*64 of each.
 * fwd writes O (bf16, rows b*T1 + i) and lse[z*T1 + i] (row log-sum-exp; +inf if masked).
 * Nothing is materialised at (T1, T2) size; any T1, T2.  Backward: ea_attn_fused_bwd2. */
int ea_attn_fused_fwd(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                      long ldk, const void* v, long ldv, const float* bu, const float* bv,
                      const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                      unsigned long long seed, void* o, long ldo, float* lse, void* stream);
/* ea_attn_fused_fwd that also writes the dropout keep decisions (p > 0) as bits for the
 * backward: dmask[(z*T1 + i)*ldm + (j >> 5)] bit (j & 31), ldm >= 2*ceil(T2/64) words (NULL:
 * none; words of key chunks past the row's last valid key are left unwritten). */
int ea_attn_fused_fwd2(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                       long ldk, const void* v, long ldv, const float* bu, const float* bv,
                       const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                       unsigned long long seed, void* o, long ldo, float* lse, unsigned* dmask, int ldm,
                       void* stream);
/* Backward of ea_attn_fused_fwd(2): dq = d(q + bu) (flags bit 0, pp only: + d(q + bv), the
 * rel-pos path dBD·pp computed in-kernel), dk, dv (bf16), and optionally:
 *   dbd (pp only, or NULL): the band dbd[h][b][i][T-1-i+j] = gradient of the raw rel-pos term
 *     (q_i + bv)·pp[r] (bf16, rows written in full: 0 off the band; lddbd >= 2*T1-1, lddbd % 8
 *     == 0, 16-B aligned) — the linear_pos weight gradient's operand;
 *   bias_part (or NULL): [2][B*ceil(T1/64)][ldpart] f32, row (b*ceil(T1/64) + qb) holds the
 *     column sums over queries [64qb, 64qb+64) of d(q+bu) (plane 0) and, with pp, d(q+bv)
 *     (plane 1) at columns h*64 + c — reduce over rows for pos_bias_u / pos_bias_v gradients;
 *   qv_out (or NULL, pp only): q + bv (bf16, rows b*T1 + i, head columns);
 *   dmask (or NULL): the forward's keep bits (ea_attn_fused_fwd2, same p / seed), read
 *     instead of regenerating the dropout hash.
 * ws: ea_attn_fused_bwd_ws_bytes() bytes of device scratch, 256-B aligned (D_i, q + bu, q + bv
 * handed from the dQ pass to the dK/dV pass).  Two launches, any T1, T2, deterministic.
 * flags bit 1 (2): the pipelined dQ pass (LDS-DMA one key chunk ahead, 16-B band stores); dbd
 *   is then in the SHIFTED layout of ea_attn_dbd_layout: logical column r at r + shift, row
 *   stride lddbd >= the returned minimum.  Without dbd the pipelined pass is the default.
 * flags bit 2 (4): force the original dQ pass (A/B measurements; unshifted dbd). */
int ea_attn_fused_bwd_ws_bytes(int B, int H, int T1, long* bytes);
/* Shifted dbd layout of ea_attn_fused_bwd2 flags bit 1: shift >= 15 with (T1 + shift) % 8 == 0,
 * minimum row stride lddbd = roundup8(2*T1 - 1 + shift); columns outside [shift, shift + 2*T1-1)
 * are written as zeros. */
int ea_attn_dbd_layout(int T1, int* shift, long* lddbd);
int ea_attn_fused_bwd2(int B, int H, int T1, int T2, int dk, const void* q, long ldq, const void* k,
                       long ldk, const void* v, long ldv, const float* bu, const float* bv,
                       const void* pp, long ldp, const long long* klen, int causal, float scale, float p,
                       unsigned long long seed, const void* o, long ldo, const float* lse, const void* dO,
                       long lddo, void* dq, long lddq, void* dkout, long lddk, void* dvout, long lddv,
                       void* dbd, long lddbd, float* bias_part, long ldpart, void* qv_out, long ldqv,
                       const unsigned* dmask, int ldm, void* ws, long ws_bytes, int flags, void* stream);

/* ---------------------------------------------------------------- losses */

/* CTC forward (ctc.py:52-97 builtin; torch CTCLoss reduction=none, zero_infinity=True,
 * blank=0, on log_softmax(logits)): per-utterance loss (0 if infeasible) and
 * loss = sum / B.  logits rows (b*T + t)*ldt; alpha/beta [B][T][2*Lmax+1] f64. */
int ea_ctc_loss_fwd(int B, int T, int V, const float* logits, long ldt, const long long* hlens,
                    const long long* ys, long ldys, const long long* ylens, int Lmax, float* lse,
                    double* alpha, double* beta, double* nll, float* loss_utt, float* loss,
                    void* stream);

/* d loss / d logits = gscale[0]*coef*(softmax - occupancy); 0 past hlens or if infeasible. */
int ea_ctc_loss_bwd(int B, int T, int V, const float* logits, long ldt, const long long* hlens,
                    const long long* ys, long ldys, const long long* ylens, int Lmax, const float* lse,
                    const double* alpha, const double* beta, const double* nll,
                    const float* gscale, float coef, void* grad, int grad_dtype, long ldg,
                    void* stream);

/* LabelSmoothingLoss + th_accuracy (label_smoothing_loss.py:41-63, nets_utils.py:304-324):
 * loss[0], acc[0] (correct/valid tokens), inv_denom[0] = 1/(#tokens or batch). */
int ea_lsm_loss_fwd(long rows, int V, const float* x, long ldx, const long long* tgt, float smoothing,
                    int ignore_id, int normalize_length, float batch, float* lse, double* loss_row,
                    int* stat, float* loss, float* acc, float* inv_denom, void* stream);
int ea_lsm_loss_bwd(long rows, int V, const float* x, long ldx, const long long* tgt, float smoothing,
                    int ignore_id, const float* lse, const float* gscale, const float* inv_denom,
                    float coef, void* grad, int grad_dtype, long ldg, void* stream);

/* ---------------------------------------------------------------- optimizer */

/* norm[0] = ||x||_2 (fp64 accumulation); workspace >= 2048 doubles. */
int ea_sqnorm(long n, const float* x, double* workspace, float* norm, void* stream);

/* torch.optim.Adam step (L2 weight decay) over the flat arena with
 * clip_grad_norm_(max_norm) folded in (coef = min(1, max_norm/(norm+1e-6))) and the
 * update skipped on device when norm is not finite (trainer.py:653-678).
 * Optionally refreshes the bf16 weight shadow. */
int ea_adam_step(long n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                 void* params_bf16, float lr, float beta1, float beta2, float eps, float weight_decay,
                 long step, const float* grad_norm, float max_norm, void* stream);

/* Device-resident optimizer step (graph-capturable: nothing on the host changes per step).
 * state (device memory) holds the count of APPLIED updates (torch Adam state['step'] and
 * the batch-step scheduler's last_epoch): a prep kernel reads grad_norm, sets skip on a
 * non-finite norm (trainer.py:662-697 skips optimizer.step() and scheduler.step()), else
 * advances step to t and stores lr(t) from `sched` (EA_SCHED_WARMUP:
 * base*w^0.5*min(t^-0.5, t*w^-1.5), espnet2/schedulers/warmup_lr.py:40-50), the bias
 * corrections and the clip coefficient; the update kernel reads them. */
enum { EA_SCHED_CONSTANT = 0, EA_SCHED_WARMUP = 1 };
typedef struct ea_lr_schedule {
  int kind;            /* EA_SCHED_* */
  float warmup_steps;
  double base_lr;
} ea_lr_schedule;
typedef struct ea_opt_state {  /* device memory, zero-initialised; 40 bytes */
  long long step;      /* applied updates so far */
  float lr;            /* lr of the last applied update */
  float bc1, bc2_sqrt; /* 1-b1^t, sqrt(1-b2^t) */
  float coef;          /* clip coefficient min(1, max_norm/(norm+1e-6)) */
  float last_norm;     /* grad norm seen by the last call */
  int skip;            /* 1: the last call skipped the update (non-finite norm) */
  float next_lr;       /* lr(step + 1): the optimizer's lr after scheduler.step(), what the
                          reference reports as optim0_lr0 (trainer.py:705-712) */
  int pad;
} ea_opt_state;
int ea_adam_step_dev(long n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                     void* params_bf16, const ea_lr_schedule* sched, float beta1, float beta2, float eps,
                     float weight_decay, ea_opt_state* state, const float* grad_norm, float max_norm,
                     void* stream);

int ea_cast_f32_bf16(long n, const float* x, void* y, void* stream);
/* x = max(x, 0) in place (f32, 16-B aligned): the ReLU of the legacy Encoder's "linear" input
 * layer (transformer/encoder.py:120-127), used by TransformerLM (espnet2/lm/transformer_lm.py). */
int ea_relu_f32_inplace(long n, float* x, void* stream);
/* Transposed bf16 weight copies for the Linear input-gradient GEMMs (read K-major): problem
 * table probs[] of {int64 src_off; bf16* dst; int32 R, C} (24 B each, device memory), tile table
 * tiles[] of int32x4 {problem, tile row, tile col, 0} (64 x 64 tiles); dst[c*R + r] =
 * src[src_off + r*C + c].  R, C multiples of 8. */
int ea_transpose_bf16_grouped(int ntiles, const int* tiles, const void* probs, const void* src, void* stream);
/* x *= s[0]*c (device scalar) */
int ea_scale_by_scalar(long n, float* x, const float* s, float c, void* stream);
/* y += s[0]*c * x (f32, s a device scalar): a gradient computed unscaled ahead of the backward,
 * accumulated with the upstream gradient once it exists (the CTC head, layers/losses.py) */
int ea_axpy_dev(long n, const float* x, float* y, const float* s, float c, void* stream);
/* out[0] = wa*a[0] + wb*b[0] (b may be NULL) — loss = w*ctc + (1-w)*att, espnet_model.py:325 */
int ea_axpby_scalar(const float* a, float wa, const float* b, float wb, float* out, void* stream);


/* ---------------------------------------------------------------- joint CTC/attention decoding */

/* out[r][v] = softmax or (log=1) log_softmax over the V entries of logits row r (rows*ld f32,
 * out dense rows x V): CTC.softmax / CTC.log_softmax, espnet2/asr/ctc.py:99-117. */
int ea_softmax_rows(long rows, int V, const float* logits, long ld, float* out, int log, void* stream);

/* CTCPrefixScorer.init_state (espnet/nets/scorers/ctc.py:25-37 + ctc_prefix_score.py:289-301):
 * logp[t][v] = log_softmax(logits[t]) (T x V f32, dense) and the initial forward variables
 * r0[t] = (r_t^n, r_t^b)(<sos>) = (logzero, sum_{s<=t} logp[s][blank]). */
int ea_ctc_prefix_init(int T, int V, const float* logits, long ld_logits, int blank, float* logp,
                       float* r0, void* stream);

/* CTCPrefixScore.__call__ (ctc_prefix_score.py:303-358) for every (hypothesis h < n_hyp,
 * candidate c < n_cand) pair of a beam-search step in one launch.  r_prev: device array of
 * n_hyp device pointers, each to that hypothesis's (T x 2) f32 forward variables; meta:
 * device int32 [n_hyp output lengths | n_hyp last labels | n_hyp*n_cand candidate labels].
 * Writes log_psi[h*n_cand + c] (prefix log-probability; <eos>: full-sequence probability,
 * blank: logzero) and r_new[(h*n_cand + c)][T][2]. */
int ea_ctc_prefix_score(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                        const unsigned long long* r_prev, const int* meta, float* log_psi, float* r_new,
                        void* stream);

/* ea_ctc_prefix_score with the metadata as separate device arrays and one output length
 * out_len shared by every hypothesis (batch beam search: all running prefixes have one
 * length): last[n_hyp] last labels, cand[n_hyp*n_cand] candidates. */
int ea_ctc_prefix_score_dev(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                            const unsigned long long* r_prev, int out_len, const int* last, const int* cand,
                            float* log_psi, float* r_new, void* stream);

/* ea_ctc_prefix_score over the attention window of CTCPrefixScoreTH (margin > 0,
 * ctc_prefix_score.py:143-161): the recursion runs over frames [start, end) only (start >= 1,
 * end clamped to T), r_new frames outside it are logzero (r_new[0][0] = logp[0][c] for the
 * empty prefix) and log_psi sums the window's terms with r[start-1][0]. */
int ea_ctc_prefix_score_win(int T, int V, int blank, int eos, int n_hyp, int n_cand, const float* logp,
                            const unsigned long long* r_prev, const int* meta, int start, int end,
                            float* log_psi, float* r_new, void* stream);

/* CTCPrefixScoreTH.extend_state (ctc_prefix_score.py:244-269, streaming decoding): a
 * hypothesis's forward variables r_old (T_old x 2) extended to r (T x 2): frames < T_old
 * copied, then r^n = logzero and r^b accumulating logp[t][blank] frame by frame. */
int ea_ctc_prefix_extend(int T_old, int T, int V, int blank, const float* logp, const float* r_old, float* r,
                         void* stream);

/* Device-side beam step of joint CTC/attention decoding (espnet/nets/batch_beam_search.py:
 * 170-205 + batch_beam :81-101).  ea_beam_prebeam: per hypothesis h < n, the P best tokens of
 * W = w_dec*logp[h] (+ w_lb when use_lb), descending (ties: lower token), then <eos>, into
 * cand[h*(P+1) ...] (int32, device; the candidate block of ea_ctc_prefix_score's meta).
 * V <= 32768. */
int ea_beam_prebeam(int n, int V, const float* logp, long ld, float w_dec, float w_lb, int use_lb, int P, int eos,
                    int* cand, void* stream);
/* ea_beam_select: the new beam (beam hypotheses) from the n*(P+1) candidates with log_psi =
 * psi (ea_ctc_prefix_score), per-hypothesis CTC prefix scores `prefix` and running scores
 * `score`: total = (w_dec*logp (+ w_lb) + w_ctc*(psi - prefix)) + score, global top-k in
 * descending order (ties: lower flattened index h*V + token; the duplicate <eos> column is
 * skipped).  Writes per chosen hypothesis b: rec_i[4b..] = {parent, token, candidate column,
 * 1 if no candidate was left}, rec_f[4b..] = {total, decoder log-prob, CTC increment, psi},
 * and the next step's inputs last_next[b] = token, rptr_next[b] = &r_new[(parent*(P+1) +
 * column)*T*2], prefix_next[b] = psi, score_next[b] = total.  n*(P+1) <= 4096. */
int ea_beam_select(int n, int V, int P, int beam, int T, const float* logp, long ld, const int* cand,
                   const float* psi, const float* prefix, const float* score, float w_dec, float w_lb, int use_lb,
                   float w_ctc, const float* r_new, int* rec_i, float* rec_f, int* last_next,
                   unsigned long long* rptr_next, float* prefix_next, float* score_next, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ESPNET_AMD_H */
