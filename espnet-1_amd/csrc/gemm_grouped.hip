// Grouped weight-gradient GEMM (include/espnet_amd.h: ea_gemm_grouped): many independent
// f32-output problems in one launch of the ping-pong 256x256 tile (gemm_kern.h: pipe_tile).
#include "gemm_kern.h"

namespace {
// ---------------------------------------------------------------- grouped GEMM
// gemm_grouped: many independent f32-output GEMMs in one launch (ea_gemm_grouped), each tile
// a 256x256 pipe_tile over the problem's whole K (no split-K, no partial slabs): the Linear
// weight gradients of a backward pass (dW = dY^T X, K = tokens) are deferred and issued
// together, so ~1,400 full-K tiles fill the chip instead of ~60-tile launches that need a
// split and a combine pass each.  The problem table and a tile -> problem map live in a
// device workspace written by group_upload launches whose ARGUMENTS carry the descriptors
// (so a captured hipGraph replays the same table); the host orders problems longest-K first.
struct GroupProbD {
  const bf16* A;
  const bf16* B;
  float* C;
  int lda, ldb, ldc;
  int M, N, K;
  int tiles_n, tile0;
  float beta;
};
constexpr int EA_GROUP_CHUNK = 60;
struct GroupChunk {
  int first, n;  // problems [first, first + n) of the table
  GroupProbD pr[EA_GROUP_CHUNK];
};
static_assert(sizeof(GroupChunk) <= 4000, "kernel argument space");

// table layout in the workspace: GroupProbD[nprob] then int map[ntiles]
__global__ void group_upload(GroupChunk c, GroupProbD* table, int* map) {
  for (int i = threadIdx.x; i < c.n; i += blockDim.x) table[c.first + i] = c.pr[i];
  for (int i = 0; i < c.n; ++i) {
    const GroupProbD& d = c.pr[i];
    const int nt = ea_cdiv(d.M, 256) * d.tiles_n;
    for (int t = threadIdx.x; t < nt; t += blockDim.x) map[d.tile0 + t] = c.first + i;
  }
}

template <bool AK, bool BKM, int NS = 4>
__global__ __launch_bounds__(512, 1) void gemm_grouped(const GroupProbD* __restrict__ table,
                                                       const int* __restrict__ map, int ntiles, int xchunk) {
  using PC = PipeT<256, NS>;
  __shared__ __attribute__((aligned(1024))) char smem[PC::SMEM];
  const int nt = ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid % 8;
  int t;
  if (xchunk > 0) {
    // block bid runs on XCD bid % 8 as that XCD's (bid / 8)-th block: chunks of G consecutive
    // tiles (neighbours sharing an A panel) go to one XCD, successive chunks round-robin over
    // the XCDs, so every XCD walks the longest-first order at the same pace (a contiguous
    // 1/8 range per XCD gave XCD 0 only full-K encoder tiles and XCD 7 only decoder tiles)
    const int G = xchunk, full = nt / (8 * G) * (8 * G);
    const int j = bid / 8;
    t = bid < full ? ((j / G) * 8 + xcd) * G + j % G : bid;
  } else {
    const int q8 = nt / 8, r8 = nt % 8;
    t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  }
  const GroupProbD q = table[__builtin_amdgcn_readfirstlane(map[t])];
  const int lt = t - q.tile0;
  const int tm = lt / q.tiles_n, tn = lt - tm * q.tiles_n;  // neighbours share the A panel
  const int m0 = tm * 256, n0 = tn * 256;
  GemmP p{};
  p.M = q.M; p.N = q.N; p.K = q.K;
  p.A = q.A; p.lda = q.lda;
  p.B = q.B; p.ldb = q.ldb;
  p.nh = 1; p.splitk = 1; p.kchunk = q.K;
  p.C = q.C; p.c_dtype = EA_F32; p.ldc = q.ldc;
  p.epi.kind = EA_EPI_STORE; p.epi.alpha = 1.f; p.epi.beta = q.beta; p.epi.post_scale = 1.f;
  p.epi.rscale = 1.f;
  p.vec_c = 1;  // host-checked: N % 4 == 0, ldc % 4 == 0, 16-B aligned C
  p.vec8 = q.N % 8 == 0 && q.ldc % 8 == 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = PC::wm(w), wn = PC::wn(w);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  pipe_tile<AK, BKM, 0, 256, NS>(p, tile_ov(p), smem, q.A, q.B, m0, n0, 0, q.K, acc);
  const EpiK ek = make_epik(p);
  epi_wave<EA_EPI_STORE, 8, 4>(p, ek, smem, 0, 0, 0, m0 + wm, n0 + wn, lane, w, acc);
}

}  // namespace

// tile -> XCD assignment of gemm_grouped: chunks of this many consecutive tiles round-robin
// over the XCDs (0: one contiguous range per XCD, the round-3 mapping); EA_GROUPED_XCD_CHUNK
static int g_xcd_chunk = [] { const char* e = std::getenv("EA_GROUPED_XCD_CHUNK"); return e ? std::atoi(e) : 4; }();

extern "C" int ea_gemm_grouped_set_xcd_chunk(int chunk) {
  EA_ENTRY();
  EA_CHECK_ARG(chunk >= 0 && chunk <= 64);
  g_xcd_chunk = chunk;
  return 0;
}

static long grouped_ws_bytes(int n, long ntiles) { return (long)n * (long)sizeof(GroupProbD) + 4 * ntiles + 256; }

extern "C" int ea_gemm_grouped_ws_bytes(int n, long ntiles, long* bytes) {
  EA_CHECK_ARG(n >= 0 && ntiles >= 0 && bytes != nullptr);
  *bytes = grouped_ws_bytes(n, ntiles);
  return 0;
}

extern "C" int ea_gemm_grouped(int a_kmajor, int b_kmajor, int n, const ea_group_gemm* probs, void* ws,
                               long ws_bytes, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 0 && (n == 0 || (probs != nullptr && ws != nullptr)));
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  long ntiles = 0;
  for (int i = 0; i < n; ++i) {
    const ea_group_gemm& e = probs[i];
    EA_CHECK_ARG(e.M > 0 && e.N > 0 && e.K > 0 && e.A && e.B && e.C);
    // pipe_tile operand rules (16-B rows, 32-bit offsets) and the vector epilogue's
    EA_CHECK_ARG(e.lda % 8 == 0 && e.ldb % 8 == 0 && ((uintptr_t)e.A % 16) == 0 && ((uintptr_t)e.B % 16) == 0);
    EA_CHECK_ARG(e.N % 4 == 0 && e.ldc % 4 == 0 && ((uintptr_t)e.C % 16) == 0);
    EA_CHECK_ARG(e.ldc >= e.N && e.lda >= (a_kmajor ? e.K : e.M) && e.ldb >= (b_kmajor ? e.K : e.N));
    EA_CHECK_ARG(e.lda < (1L << 31) && e.ldb < (1L << 31) && e.ldc < (1L << 31));
    const double a_ext = 2.0 * ((a_kmajor ? (double)e.M : (double)e.K) * e.lda);
    const double b_ext = 2.0 * ((b_kmajor ? (double)e.N : (double)e.K) * e.ldb);
    EA_CHECK_ARG(a_ext < 4.0e9 && b_ext < 4.0e9);
    ntiles += (long)ea_cdiv(e.M, 256) * ea_cdiv(e.N, 256);
  }
  EA_CHECK_ARG(ntiles < (1L << 30) && grouped_ws_bytes(n, ntiles) <= ws_bytes);
  GroupProbD* table = (GroupProbD*)ws;
  int* map = (int*)((char*)ws + (long)n * sizeof(GroupProbD));
  GroupChunk c{};
  int tile0 = 0;
  for (int i = 0; i < n; ++i) {
    const ea_group_gemm& e = probs[i];
    GroupProbD& d = c.pr[c.n++];
    d.A = (const bf16*)e.A; d.B = (const bf16*)e.B; d.C = e.C;
    d.lda = (int)e.lda; d.ldb = (int)e.ldb; d.ldc = (int)e.ldc;
    d.M = e.M; d.N = e.N; d.K = e.K;
    d.tiles_n = ea_cdiv(e.N, 256);
    d.tile0 = tile0;
    d.beta = e.beta;
    tile0 += ea_cdiv(e.M, 256) * d.tiles_n;
    if (c.n == EA_GROUP_CHUNK || i == n - 1) {
      hipLaunchKernelGGL(group_upload, dim3(1), dim3(256), 0, st, c, table, map);
      EA_LAUNCH_CHECK();
      c.first += c.n;
      c.n = 0;
    }
  }
  const dim3 grid((unsigned)ntiles), block(512);
  if (a_kmajor && b_kmajor) hipLaunchKernelGGL((gemm_grouped<true, true>), grid, block, 0, st, table, map, (int)ntiles, g_xcd_chunk);
  else if (a_kmajor) hipLaunchKernelGGL((gemm_grouped<true, false>), grid, block, 0, st, table, map, (int)ntiles, g_xcd_chunk);
  else if (b_kmajor) hipLaunchKernelGGL((gemm_grouped<false, true>), grid, block, 0, st, table, map, (int)ntiles, g_xcd_chunk);
  else hipLaunchKernelGGL((gemm_grouped<false, false>), grid, block, 0, st, table, map, (int)ntiles, g_xcd_chunk);
  EA_LAUNCH_CHECK();
  return 0;
}
