// Grouped parameter-gradient reductions (see include/espnet_amd.h: ea_colsum_grouped,
// ea_reduce_grouped).
//
// A training backward pass produces ~160 bias column sums (torch.nn.Linear bias.grad =
// dY summed over tokens) and ~80 LayerNorm weight/bias gradient reductions, each a
// two-launch "row-block partials, then ordered reduce" pair of a few microseconds.  Deferred
// to the end of the pass (or of a DP bucket), they run as TWO launches: every column-sum
// problem's partials in one grid, then every problem's ordered reduction in another.  The
// problem tables live in a device workspace written by table_upload launches whose
// arguments carry the descriptors, so a captured hipGraph replays the same tables.  Sums are
// deterministic (fixed row-block order, f64 in the final reduction) and equal the per-call
// ea_colsum / ea_layernorm_bwd results bit for bit.
#include "common.h"

namespace {

struct ColsumProbD {
  const void* x;   // rows x n, row stride ld (elements), dtype bf16 or f32
  float* part;     // [nrb][n] partial sums (this problem's slice of the partial buffer)
  long ld;
  int rows, n, dtype, rpp, ncb, item0;  // rpp rows per row block; ncb 256-column blocks
};

struct ReduceProbD {
  const float* part;  // [nparts][stride]
  float* out;         // out[c] (+)= sum_p part[p*stride + c], c < n
  long stride;
  int nparts, n, accumulate, item0;
};

constexpr int CHUNK = 40;
template <typename P>
struct Chunk {
  int first, n;
  P pr[CHUNK];
};
static_assert(sizeof(Chunk<ColsumProbD>) <= 4000 && sizeof(Chunk<ReduceProbD>) <= 4000, "kernel argument space");

template <typename P>
__global__ void table_upload(Chunk<P> c, P* table) {
  for (int i = threadIdx.x; i < c.n; i += blockDim.x) table[c.first + i] = c.pr[i];
}

// problem owning work item t (problems ordered by item0, wave-uniform binary search)
template <typename P>
EA_DEV int find_prob(const P* table, int n, int t) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (__builtin_amdgcn_readfirstlane(table[mid].item0) <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// one work item = (row block, 256-column block) of one problem: 4 columns per lane, the 4
// waves interleave the block's rows (4 rows per wave in flight), combined in fixed order
__global__ __launch_bounds__(256) void colsum_grouped_kernel(const ColsumProbD* __restrict__ table, int nprob) {
  __shared__ float red[4][256];
  const int pi = find_prob(table, nprob, blockIdx.x);
  const ColsumProbD q = table[pi];
  const int it = blockIdx.x - q.item0;
  const int rb = it / q.ncb, cb = it - rb * q.ncb;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = cb * 256 + lane * 4;
  const int r0 = rb * q.rpp, r1 = min(q.rows, r0 + q.rpp);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < q.n) {
    if (q.dtype == EA_BF16) {
      const bf16* x = (const bf16*)q.x;
      int r = r0 + w;
      for (; r + 12 < r1; r += 16) {
        float v[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) vld4(x + (long)(r + 4 * j) * q.ld + c, v[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) a[k] += v[j][k];
      }
      for (; r < r1; r += 4) {
        float v[4];
        vld4(x + (long)r * q.ld + c, v);
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += v[k];
      }
    } else {
      const float* x = (const float*)q.x;
      int r = r0 + w;
      for (; r + 12 < r1; r += 16) {
        float v[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) vld4(x + (long)(r + 4 * j) * q.ld + c, v[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) a[k] += v[j][k];
      }
      for (; r < r1; r += 4) {
        float v[4];
        vld4(x + (long)r * q.ld + c, v);
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += v[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[w][lane * 4 + k] = a[k];
  __syncthreads();
  const int cc = cb * 256 + threadIdx.x;
  const int t = threadIdx.x;  // the waves combined as colsum_vec_kernel does (bit-identical partials)
  if (cc < q.n) q.part[(long)rb * q.n + cc] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

// one work item = 16 columns of one problem x 16 part lanes (reduce_partials_kernel's scheme)
constexpr int RP_CW = 16, RP_PL = 16;
__global__ __launch_bounds__(256) void reduce_grouped_kernel(const ReduceProbD* __restrict__ table, int nprob) {
  __shared__ double red[RP_PL][RP_CW];
  const int pi = find_prob(table, nprob, blockIdx.x);
  const ReduceProbD q = table[pi];
  const int cx = threadIdx.x % RP_CW, py = threadIdx.x / RP_CW;
  const int c = (blockIdx.x - q.item0) * RP_CW + cx;
  double a = 0.0;
  if (c < q.n) {
    int p = py;
    for (; p + 7 * RP_PL < q.nparts; p += 8 * RP_PL) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = q.part[(long)(p + RP_PL * j) * q.stride + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) a += v[j];
    }
    for (; p < q.nparts; p += RP_PL) a += q.part[(long)p * q.stride + c];
  }
  red[py][cx] = a;
  __syncthreads();
  if (py == 0 && c < q.n) {
    double t = 0.0;
#pragma unroll
    for (int l = 0; l < RP_PL; ++l) t += red[l][cx];
    q.out[c] = q.accumulate ? q.out[c] + (float)t : (float)t;
  }
}

template <typename P>
int upload(const P* probs, int n, P* table, hipStream_t st) {
  Chunk<P> c{};
  for (int i = 0; i < n; ++i) {
    c.pr[c.n++] = probs[i];
    if (c.n == CHUNK || i == n - 1) {
      hipLaunchKernelGGL((table_upload<P>), dim3(1), dim3(64), 0, st, c, table);
      EA_LAUNCH_CHECK();
      c.first += c.n;
      c.n = 0;
    }
  }
  return 0;
}

}  // namespace

extern "C" int ea_colsum_grouped(int n, const ea_colsum_prob* probs, void* ws, long ws_bytes, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 0 && (n == 0 || (probs && ws)));
  if (n == 0) return 0;
  EA_CHECK_ARG((long)n * (long)sizeof(ColsumProbD) <= ws_bytes && n <= 4096);
  ColsumProbD* host = (ColsumProbD*)malloc(sizeof(ColsumProbD) * n);
  if (!host) return EA_ERR_BAD_ARG;
  long items = 0;
  int rc = 0;
  for (int i = 0; i < n && !rc; ++i) {
    const ea_colsum_prob& e = probs[i];
    const bool ok = e.x && e.part && e.rows > 0 && e.n > 0 && e.n % 4 == 0 && e.ld % 4 == 0 && e.rpp > 0 &&
                    (e.dtype == EA_BF16 || e.dtype == EA_F32) &&
                    ((uintptr_t)e.x % (e.dtype == EA_BF16 ? 8 : 16)) == 0;
    if (!ok) { rc = EA_ERR_BAD_ARG; break; }
    ColsumProbD& d = host[i];
    d.x = e.x; d.part = e.part; d.ld = e.ld;
    d.rows = e.rows; d.n = e.n; d.dtype = e.dtype; d.rpp = e.rpp;
    d.ncb = ea_cdiv(e.n, 256);
    d.item0 = (int)items;
    items += (long)ea_cdiv(e.rows, e.rpp) * d.ncb;
  }
  if (!rc && items >= (1L << 30)) rc = EA_ERR_BAD_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (!rc) rc = upload(host, n, (ColsumProbD*)ws, st);
  free(host);
  if (rc) return rc;
  hipLaunchKernelGGL(colsum_grouped_kernel, dim3((unsigned)items), dim3(256), 0, st, (const ColsumProbD*)ws, n);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_reduce_grouped(int n, const ea_reduce_prob* probs, void* ws, long ws_bytes, void* stream) {
  EA_ENTRY();
  EA_CHECK_ARG(n >= 0 && (n == 0 || (probs && ws)));
  if (n == 0) return 0;
  EA_CHECK_ARG((long)n * (long)sizeof(ReduceProbD) <= ws_bytes && n <= 4096);
  ReduceProbD* host = (ReduceProbD*)malloc(sizeof(ReduceProbD) * n);
  if (!host) return EA_ERR_BAD_ARG;
  long items = 0;
  int rc = 0;
  for (int i = 0; i < n; ++i) {
    const ea_reduce_prob& e = probs[i];
    if (!(e.part && e.out && e.n > 0 && e.nparts >= 0 && e.stride >= e.n)) { rc = EA_ERR_BAD_ARG; break; }
    ReduceProbD& d = host[i];
    d.part = e.part; d.out = e.out; d.stride = e.stride;
    d.nparts = e.nparts; d.n = e.n; d.accumulate = e.accumulate;
    d.item0 = (int)items;
    items += ea_cdiv(e.n, RP_CW);
  }
  if (!rc && items >= (1L << 30)) rc = EA_ERR_BAD_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (!rc) rc = upload(host, n, (ReduceProbD*)ws, st);
  free(host);
  if (rc) return rc;
  hipLaunchKernelGGL(reduce_grouped_kernel, dim3((unsigned)items), dim3(256), 0, st, (const ReduceProbD*)ws, n);
  EA_LAUNCH_CHECK();
  return 0;
}

extern "C" int ea_grouped_table_bytes(int n, long* colsum_bytes, long* reduce_bytes) {
  EA_CHECK_ARG(n >= 0 && colsum_bytes && reduce_bytes);
  *colsum_bytes = (long)n * (long)sizeof(ColsumProbD);
  *reduce_bytes = (long)n * (long)sizeof(ReduceProbD);
  return 0;
}
