// gemm_quad: 256 x 256 bf16 output tiles computed by FOUR waves of 128 x 128 each (one wave
// per SIMD, accumulators in the AGPR half of the register file), K-major A and B (ea_gemm_set_quad).
//
// gemm_pipe's eight waves own 128 x 64 sub-tiles: per 32-deep slice a wave reads 12 KiB of
// fragments for 32 MFMAs, 96 KiB per CU per slice — with the slice's 32 KiB of LDS-DMA writes
// that is as many LDS cycles as the SIMDs' MFMA cycles (1,024 per slice), so the MFMA pipes
// idle whenever the two drift apart (0.48 MFMA-busy on the conv2 forward, PMC).  A 128 x 128
// wave tile reads 16 KiB for 64 MFMAs: 64 KiB per CU per slice, about 2/3 of the MFMA time.
//
// K moves in 32-deep slices through an S-slot ring (32 KiB per slot) filled by LDS-DMA S-1
// slices ahead with counted vmcnt, one barrier per slice.  Fragments of slice s+1 are read
// (inline asm, counted lgkmcnt: hipcc would drain vmcnt in front of any LDS read it can see
// while a DMA is in flight) while slice s's MFMAs run: B(s+1) before the first half of the
// MFMAs, A(s+1) before the second half (lgkmcnt counts at most 15 outstanding).  Same image
// format (img32_off / swz32), DMA sources, tile mapping and epilogue as gemm_pipe; the host
// guarantees K % 64 == 0 per split and K-major operands.
#include "gemm_kern.h"

namespace {
using namespace eag;

template <int N>
EA_DEV void wait_lgkm() {  // at most N LDS reads outstanding
  if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
}

template <int OFF>
EA_DEV bf16x8 ds_read_b128_off(uint32_t a) {  // LDS byte address a + OFF (immediate)
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}

template <int S, bool BKM>
__global__ __launch_bounds__(256, 1) void gemm_quad(GemmP p) {
  constexpr int BT = 256, BK = 32, NTT = 256, NW = 4, MI = 8, NJ = 8;
  constexpr int A_BYTES = BT * BK * 2, B_BYTES = BT * BK * 2, SLOT = A_BYTES + B_BYTES;
  constexpr int ACH = A_BYTES / (NTT * 16), BCH = B_BYTES / (NTT * 16), G = ACH + BCH;
  constexpr int EPI_BYTES = NW * 4 * 16 * EPI_LDT * 4;
  constexpr int SMEM = S * SLOT > EPI_BYTES ? S * SLOT : EPI_BYTES;
  static_assert(S >= 4 && S <= 5, "ring depth");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  probe_start(p);

  const TileIdx ti = tile_index(p);
  const int m0 = ti.tm * BT, n0 = ti.tn * BT;
  const int z = ti.z, sk = ti.sk;
  const int zb = z / p.nh, zh = z % p.nh;
  const bf16* A = (const bf16*)p.A + zb * p.sAb + zh * p.sAh;
  const bf16* B = (const bf16*)p.B + zb * p.sBb + zh * p.sBh;
  const int kbeg = sk * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nsl = max(0, (kend - kbeg) / BK);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = (w >> 1) * 128, wn = (w & 1) * 128;

  // lane-linear DMA: chunk ci = (i*NW + w)*64 + lane lands at ci*16 (64-B rows of 4 chunks);
  // its source is the global chunk whose swizzled slot that is
  auto src = [&](long ld, int mn0, int MN, bool kmaj, int ci) -> uint32_t {
    if (kmaj) {
      const int row = ci >> 2, c = (ci & 3) ^ swz32(ci >> 2);
      return (uint32_t)(((long)min(mn0 + row, MN - 1) * ld + c * 8) * 2);
    }
    // MN-major: two [32 k][128] panels per slice (gemm_pipe's image, swz_mn_bf16 chunk swizzle)
    const int pnl = ci >> 9, cj = ci & 511, k = cj >> 4, c = (cj & 15) ^ swz_mn_bf16(k);
    return (uint32_t)(((long)k * ld + min((long)(mn0 + pnl * 128 + c * 8), (long)((MN - 1) & ~7))) * 2);
  };
  const char* abase = (const char*)(A + kbeg);
  const char* bbase = (const char*)(B + (BKM ? (long)kbeg : (long)kbeg * p.ldb));
  const long bstep = (BKM ? BK : (long)BK * p.ldb) * 2;  // bytes per slice
  uint32_t aoff[ACH], boff[BCH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) aoff[i] = src(p.lda, m0, p.M, true, (i * NW + w) * 64 + lane);
#pragma unroll
  for (int i = 0; i < BCH; ++i) boff[i] = src(p.ldb, n0, p.N, BKM, (i * NW + w) * 64 + lane);

  auto issue = [&](int sl) {
    char* base = smem + (sl % S) * SLOT;
    const char* ak = abase + (long)sl * BK * 2;
    const char* bk = bbase + (long)sl * bstep;
#pragma unroll
    for (int i = 0; i < ACH; ++i)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(ak + aoff[i]),
                                       (__attribute__((address_space(3))) void*)(base + (i * NW + w) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < BCH; ++i)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(bk + boff[i]),
                                       (__attribute__((address_space(3))) void*)(base + A_BYTES + (i * NW + w) * 1024),
                                       16, 0, 0);
  };
  // Fragment reads: 16 rows (lane & 15) of a 32-deep slice, k-chunk lane >> 4.  The row
  // swizzle swz32(r0 + 16 i + (lane & 15)) depends on the lane only (r0, 16 i are multiples of
  // 16), so one lane address per operand and slot serves all 8 fragments, fragment i at the
  // immediate offset i * 1024 (a per-fragment address would hold 24 VGPRs per ring slot).
  const uint32_t lane_off = (uint32_t)((lane & 15) * 64 + (((lane >> 4) ^ swz32(lane & 15)) << 4));
  const uint32_t smem_lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  // MN-major B (16 columns wn + 16 j, k-chunk lane >> 4): frag32<false>'s two 4 x 4 transposed
  // reads; the chunk of fragment j is (2 j + (pp >> 1)) ^ swz (swz even: bit 0 untouched), so
  // the lane term and j separate as ((j ^ (swz >> 1)) << 5) | ((pp >> 1) << 4) + within
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  uint32_t trow[2], tsw[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * (lane >> 4) + 4 * h + tq;
    trow[h] = (uint32_t)(row * 256 + ((tp >> 1) << 4) + (tp & 1) * 8);
    tsw[h] = (uint32_t)(swz_mn_bf16(row) >> 1);
  }
  auto rd_bmn = [&](uint32_t pnl, int j0, bf16x8 (&f)[8]) {  // fragments j0 .. j0+3
#pragma unroll
    for (int j = j0; j < j0 + 4; ++j) {
      union { bf16x8 v; s16x4 h[2]; } o;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t a = pnl + trow[h] + ((((uint32_t)j) ^ tsw[h]) << 5);
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(o.h[h]) : "v"(a) : "memory");
      }
      f[j] = o.v;
    }
  };
  auto rd_bk = [&](uint32_t a, int j0, bf16x8 (&f)[8]) {
    if (j0 == 0) {
      f[0] = ds_read_b128_off<0>(a); f[1] = ds_read_b128_off<1024>(a);
      f[2] = ds_read_b128_off<2048>(a); f[3] = ds_read_b128_off<3072>(a);
    } else {
      f[4] = ds_read_b128_off<4096>(a); f[5] = ds_read_b128_off<5120>(a);
      f[6] = ds_read_b128_off<6144>(a); f[7] = ds_read_b128_off<7168>(a);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto mma_rows = [&](int i0, const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // one slice s: B(s+1) into the other B buffer, MFMA rows 0-3, A(s+1) rows 0-3 into the rows
  // just used, MFMA rows 4-7, A(s+1) rows 4-7 (A single-buffered, B double-buffered by call:
  // 96 fragment VGPRs beside the 256 AGPR accumulators).  lgkmcnt counts the 4-read groups in
  // issue order: A[0-3](s) | A[4-7](s) | B(s+1) | A[0-3](s+1) | ...
  auto rd4lo = [&](uint32_t a, bf16x8 (&f)[8]) {
    f[0] = ds_read_b128_off<0>(a); f[1] = ds_read_b128_off<1024>(a);
    f[2] = ds_read_b128_off<2048>(a); f[3] = ds_read_b128_off<3072>(a);
  };
  auto rd4hi = [&](uint32_t a, bf16x8 (&f)[8]) {
    f[4] = ds_read_b128_off<4096>(a); f[5] = ds_read_b128_off<5120>(a);
    f[6] = ds_read_b128_off<6144>(a); f[7] = ds_read_b128_off<7168>(a);
  };
  // lane addresses of a slot's A rows wm.. and B rows wn.. (K-major) / B panel wn >> 7 (MN-major)
  auto a_addr = [&](int sl) { return smem_lds + (uint32_t)((sl % S) * SLOT + wm * 64) + lane_off; };
  auto b_addr = [&](int sl) {
    return BKM ? smem_lds + (uint32_t)((sl % S) * SLOT + A_BYTES + wn * 64) + lane_off
               : smem_lds + (uint32_t)((sl % S) * SLOT + A_BYTES + (wn >> 7) * 8192);
  };
  auto rd_b = [&](uint32_t a, int j0, bf16x8 (&f)[8]) {
    if constexpr (BKM) rd_bk(a, j0, f);
    else rd_bmn(a, j0, f);
  };
  // reads per B half (4 fragments): 4 (K-major) or 8 (two transposed reads each); lgkmcnt order
  // per slice s: Bh0(s+1) | MFMA rows 0-3 | A[0-3](s+1) Bh1(s+1) | MFMA rows 4-7 | A[4-7](s+1)
  constexpr int NBH = BKM ? 4 : 8;
  bf16x8 fa[8], fb0[8], fb1[8];
  // the register data flow is the same every slice (the last slice re-reads its own slot
  // instead of a next one): conditional fragment reads made the compiler keep both versions
  // of the buffers live and spill
  auto step = [&](int sl, const bf16x8 (&fb)[8], bf16x8 (&nbuf)[8]) {
    const bool more = sl + 1 < nsl;
    const int nx = more ? sl + 1 : sl;
    if (more) {
      // own share of slice sl+1 landed; slices sl+2 .. sl+S-2 may stay in flight
      wait_newer<G, S - 3>(min(S - 3, nsl - 2 - sl));
      lds_barrier();  // everyone's; every wave is past its reads of slice sl-1: its slot is free
      if (sl + S - 1 < nsl) issue(sl + S - 1);
    }
    const uint32_t bad = b_addr(nx), aad = a_addr(nx);
    rd_b(bad, 0, nbuf);
    wait_lgkm<NBH>();  // every read of slice sl is in
    __builtin_amdgcn_sched_barrier(0);
    mma_rows(0, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    rd4lo(aad, fa);
    rd_b(bad, 4, nbuf);
    wait_lgkm<4 + NBH>();  // A[4-7](s) in
    __builtin_amdgcn_sched_barrier(0);
    mma_rows(4, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    rd4hi(aad, fa);
  };

  diag_stamp(p, 0);
  if (nsl > 0) {
    const int npre = min(S - 1, nsl);
    for (int sl = 0; sl < npre; ++sl) issue(sl);
    wait_newer<G, S - 2>(npre - 1);  // own share of slice 0 landed
    lds_barrier();                   // everyone's
    rd_b(b_addr(0), 0, fb0);
    rd_b(b_addr(0), 4, fb0);
    rd4lo(a_addr(0), fa);
    rd4hi(a_addr(0), fa);
    for (int sl = 0; sl < nsl; sl += 2) {  // nsl even (host: K % 64 == 0)
      step(sl, fb0, fb1);
      step(sl + 1, fb1, fb0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();  // every wave is done reading the ring: the epilogue reuses it
  diag_stamp(p, 1);
  const EpiK ek = make_epik(p);
  switch (p.splitk > 1 ? EA_EPI_STORE : p.epi.kind) {
    case EA_EPI_STORE: epi_wave<EA_EPI_STORE, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    case EA_EPI_ACT: epi_wave<EA_EPI_ACT, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    case EA_EPI_RESID: epi_wave<EA_EPI_RESID, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
    default: epi_wave<EA_EPI_DACT, MI, NJ>(p, ek, smem, z, zb, zh, m0 + wm, n0 + wn, lane, w, acc, sk); break;
  }
  if (p.diag) {
    __syncthreads();
    diag_stamp(p, 2);
  }
  probe_end(p);
}

}  // namespace

namespace eag {
int g_quad_slots = 5;
int launch_quad(GemmP& p, int b_k, dim3 grid, hipStream_t st) {
  if (b_k) {
    if (g_quad_slots == 4) hipLaunchKernelGGL((gemm_quad<4, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_quad<5, true>), grid, dim3(256), 0, st, p);
  } else {
    if (g_quad_slots == 4) hipLaunchKernelGGL((gemm_quad<4, false>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((gemm_quad<5, false>), grid, dim3(256), 0, st, p);
  }
  EA_LAUNCH_CHECK();
  return 0;
}
}  // namespace eag
