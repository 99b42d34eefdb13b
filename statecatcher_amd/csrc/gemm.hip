// Weight-gradient GEMM of the gate / output projections on gfx950 MFMA (CDNA4, wave64).
//
// dW = dYᵀ X for dY [L, I] and X [L, J] (bf16, row-major, L = B*T = 48,000 frames at the
// training shape; I = 7*D = 3584 gate rows or V = 1024 logits; J = D = 512): the backward of
// LinearSafe (lucyrnn_triton.py:20-25) / the output projection (lucyrnn_triton.py:107-109).  Both
// operands keep the reduction index L as their ROW index, so the MFMA fragments (8 consecutive
// L values per lane) are strided in memory; hipBLASLt reaches 0.86-0.9 PFLOP/s on this shape
// (split-K batched GEMM + a sum), the weakest GEMM of the step.
//
// Design (one 512-thread workgroup per CU, 8 waves as 2 (I) x 4 (J)):
//   * tile TI x 256 of dW, TI = 32 * TTI (224 at I = 3584: 16 x 2 tiles x 8 L-splits = 256
//     workgroups, and each XCD's 32 workgroups share ONE L-split, so the dY / X rows of a K-step
//     are fetched from HBM once per XCD and re-read by its 16 / 2 co-resident workgroups from L2);
//   * K-step of 64 L-rows: the dY and X row panels go HBM -> LDS by LDS-DMA (16-byte pieces,
//     saddr form, loop-invariant lane offsets), two LDS stages, the next K-step in flight
//     while this one computes;
//   * LDS images are [64 rows][512 B] with the 16-byte chunk index XOR-swizzled by
//     2 f(row), f = (row & 3) | ((row >> 3) & 1) << 2: the swizzle is applied on the DMA SOURCE
//     address (the LDS side of a DMA is lane-linear) and makes the transposed reads conflict-free;
//   * fragments come out of LDS transposed by ds_read_b64_tr_b16 (two per 16x32 operand);
//   * v_mfma_f32_16x16x32_bf16 into fp32 accumulators (per wave 16 TTI x 64 outputs);
//   * each L-split writes an fp32 partial slab; sc_colsum sums the slabs in split order
//     (deterministic) and un-permutes step-blocked gate rows in the same pass.

#include <type_traits>

#include "sc_common.h"

// SC_GEMM_ABL: ablation bitmask for tools timing only (never set in a shipped build):
//   1 no MFMAs, 2 no DMA after the prologue, 4 no LDS reads (fragments from registers),
//   8 no barrier in the main loop (wrong results)
#ifndef SC_GEMM_ABL
#define SC_GEMM_ABL 0
#endif

namespace sc {

typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));

constexpr int kTL = 64;        // L rows per K-step
constexpr int kTJ = 256;       // J columns per tile
constexpr int kRowB = 512;     // LDS image row pitch (bytes)
constexpr int kImg = kTL * kRowB;   // one operand image (32 KiB)
// LDS ring slots of 32 L-rows (32 KiB each).  5 (all of gfx950's 160 KiB) measured no faster
// than 4: with DMA alone the kernel streams L2 -> LDS at ~11 TB/s (131 us at the C2 shape)
// whatever the depth, so the ring is not latency-bound.
#ifndef SC_GEMM_SLOTS
#define SC_GEMM_SLOTS 4
#endif
constexpr int kSlots = SC_GEMM_SLOTS;
// SC_GEMM_STAGGER: the second wave of each SIMD issues its DMA after its MFMAs (measured
// 1-3% slower; kept for the record)
#ifndef SC_GEMM_STAGGER
#define SC_GEMM_STAGGER 0
#endif
// SC_GEMM_PRIO: s_setprio(1) around each half-stage's MFMAs (measured 1-2% slower).
// SC_GEMM_SGB: sched_group_barrier interleave of the transposed reads with the MFMAs, one read
// after each MFMA (measured 2-3% faster than the compiler's own order: 184-187 vs 191 us)
#ifndef SC_GEMM_PRIO
#define SC_GEMM_PRIO 0
#endif
#ifndef SC_GEMM_SGB
#define SC_GEMM_SGB 1
#endif

struct WgradArgs {
  const __bf16* A;   // dY [L][lda]
  const __bf16* B;   // X  [L][ldb]
  float* C;          // [S][I][J] fp32 partial slabs
  int L, I, J, S, ntj, tiles;
  int64_t lda, ldb;
};

__device__ __forceinline__ int swz_f(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }
// byte offset of logical 16-byte chunk c of image row `row`
__device__ __forceinline__ uint32_t img_off(int row, int c) {
  return (uint32_t)(row * kRowB + 16 * (c ^ (swz_f(row) << 1)));
}

// ds_read_b64_tr_b16 as two dwords (fragments are assembled from whole registers: composing
// them from 16-bit elements costs a v_perm / shift per element)
__device__ __forceinline__ i2v tr_read(uint32_t lds_byte) {
  return __builtin_bit_cast(i2v, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                     (s4v __attribute__((address_space(3)))*)(size_t)lds_byte));
}

// NU: 16-column fragments per wave along J (4: the 256-column tile; 2: a 128-column tile for
// layer 0's J = 80 padded to 128, whose X rows are half an image row: the lanes past them fetch
// a clamped duplicate chunk that no fragment reads)
template <int TTI, int NU = 4>
__global__ void __launch_bounds__(512) wgrad_kernel(WgradArgs a) {
  constexpr int TI = 32 * TTI;
  constexpr int TJ = 64 * NU;
  constexpr int NCA = TI / 8;   // valid 16-byte chunks per A image row
  constexpr int NCB = TJ / 8;   // ... per X image row
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];   // [2 stages][A, B]
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int wi = w >> 2, wj = w & 3;
  // XCD-aware remap: the 8 XCDs take bids round-robin; consecutive logical ids share an XCD,
  // and consecutive logical ids share an L-split.
  const int nwg = a.tiles * a.S;
  const int bid = blockIdx.x;
  const int xcd = bid % 8, qq = nwg / 8, rr = nwg % 8;   // bijective for any nwg
  const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
  const int split = lid / a.tiles, tile = lid % a.tiles;
  const int ti = tile / a.ntj, tj = tile % a.ntj;
  const int i0 = ti * TI, j0 = tj * TJ;
  const int nkb = a.L / kTL;
  const int kb0 = (int)((int64_t)split * nkb / a.S), kb1 = (int)((int64_t)(split + 1) * nkb / a.S);

  // LDS ring of kSlots half-stages (32 L-rows of dY and of X each, 32 KiB): a half-stage's DMA
  // is issued kSlots - 1 compute phases before its fragments are read.  Each wave stages rows
  // 4w .. 4w+3 of both half-images, two rows per instruction (lane >> 5 picks the row,
  // lane & 31 the physical chunk; the source chunk carries the swizzle).
  uint32_t voA[2], voB[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int row = 4 * w + 2 * q + (lane >> 5);
    const int c = (lane & 31) ^ (swz_f(row) << 1);   // logical chunk this lane fetches
    voA[q] = (uint32_t)(row * a.lda + i0 + 8 * min(c, NCA - 1)) * 2u;
    voB[q] = (uint32_t)(row * a.ldb + j0 + 8 * min(c, NCB - 1)) * 2u;
  }
  constexpr int kHalf = 32 * kRowB;   // one half-image (16 KiB)
  const uint32_t lds0 = lds_addr(lds);
  // piece q (0..3) of half-stage h: q < 2 a dY row pair, q >= 2 an X row pair
  auto stage_piece = [&](int h, int q) __attribute__((always_inline)) {
    const int64_t r = (int64_t)kb0 * kTL + 32 * h;
    const uint32_t la = lds0 + (h % kSlots) * 2 * kHalf + 4 * w * kRowB;
    if (q < 2)
      dma_to_lds_s<16>(a.A + r * a.lda, voA[q], la + q * 1024);
    else
      dma_to_lds_s<16>(a.B + r * a.ldb, voB[q - 2], la + kHalf + (q - 2) * 1024);
  };
  auto stage = [&](int h) __attribute__((always_inline)) {   // half-stage h of this split
#pragma unroll
    for (int q = 0; q < 4; ++q) stage_piece(h, q);
  };

  // transposed-read lane geometry: group g = lane >> 4 takes rows 8g .. 8g+7 of the 32-row
  // half-stage; within the group lane 4q+p addresses row q, columns 4p .. 4p+3
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  f4v acc[TTI][NU];
#pragma unroll
  for (int t = 0; t < TTI; ++t)
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[t][u] = f4v{0.f, 0.f, 0.f, 0.f};

  const int nh = 2 * (kb1 - kb0);
  // fragments of one half-stage: B (NU j-tiles) and A (TTI i-tiles), 8 bf16 each
  auto load_frags = [&](int h, i4v (&bf)[NU], i4v (&af)[TTI]) __attribute__((always_inline)) {
    const uint32_t ia = lds0 + (h % kSlots) * 2 * kHalf, ib = ia + kHalf;
    const int r0 = 8 * g + q4;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int col = wj * 16 * NU + 16 * u + 4 * p4;
      const uint32_t o = (uint32_t)((col & 7) ? 8 : 0);
      i2v lo = i2v{u, 1}, hi = lo;
      if (!(SC_GEMM_ABL & 4)) {
        lo = tr_read(ib + img_off(r0, col >> 3) + o);
        hi = tr_read(ib + img_off(r0 + 4, col >> 3) + o);
      }
      bf[u] = i4v{lo.x, lo.y, hi.x, hi.y};
    }
#pragma unroll
    for (int t = 0; t < TTI; ++t) {
      const int col = wi * (TI / 2) + 16 * t + 4 * p4;
      const uint32_t o = (uint32_t)((col & 7) ? 8 : 0);
      i2v lo = i2v{t, 1}, hi = lo;
      if (!(SC_GEMM_ABL & 4)) {
        lo = tr_read(ia + img_off(r0, col >> 3) + o);
        hi = tr_read(ia + img_off(r0 + 4, col >> 3) + o);
      }
      af[t] = i4v{lo.x, lo.y, hi.x, hi.y};
    }
  };
  // (DMA pieces interleaved between the MFMAs measured slower: 203 vs 192 us)
  auto mfmas = [&](const i4v (&bf)[NU], const i4v (&af)[TTI]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < TTI; ++t)
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (SC_GEMM_ABL & 1)
          acc[t][u][0] += (float)af[t][u] * (float)bf[u][t & 3];
        else
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(b8v, af[t]), __builtin_bit_cast(b8v, bf[u]), acc[t][u], 0, 0, 0);
      }
  };
  // Software pipeline: iteration h multiplies half-stage h (fragments already in registers)
  // while the fragments of h+1 come out of LDS.  Before its barrier a wave has retired its
  // reads of h (lgkmcnt, in lds_barrier) and its DMAs of h+1 (vmcnt: the younger h+2, h+3 stay
  // in flight); after it, h+1 is readable by all and slot h % kSlots is free for h + kSlots.
  // (4 DMA instructions per wave per half-stage: vmcnt(4 n) leaves the n youngest in flight)
  auto wait_younger = [&](int n) __attribute__((always_inline)) {
    if (n >= 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else dma_wait();
  };
  for (int h = 0; h < kSlots && h < nh; ++h) stage(h);
  i4v bfA[NU], afA[TTI], bfB[NU], afB[TTI];
  wait_younger(min(kSlots - 1, nh - 1));
  lds_barrier();
  if (nh > 0) load_frags(0, bfA, afA);
  // late: the wave issues its DMA pieces after its MFMAs instead of before.  The two waves of
  // a SIMD (w, w + 4) take opposite ends of the phase: a piece's issue blocks its wave while
  // the memory queues are full, and the other wave's MFMAs then keep the SIMD busy.  The
  // per-wave DMA counts are the same either way (vmcnt unchanged).
  const bool late = SC_GEMM_STAGGER && TTI <= 7 && w >= 4;   // (TTI = 8: no registers to spare)
  auto iter = [&](int h, i4v (&bc)[NU], i4v (&ac)[TTI], i4v (&bn)[NU], i4v (&an)[TTI])
      __attribute__((always_inline)) {
    if (h + 1 < nh) wait_younger(min(kSlots - 2, nh - 2 - h));
    if (!(SC_GEMM_ABL & 8)) lds_barrier();
    const bool st = h + kSlots < nh && !(SC_GEMM_ABL & 2);
    if (!late && st) stage(h + kSlots);
    if (h + 1 < nh) load_frags(h + 1, bn, an);
    if (SC_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
    mfmas(bc, ac);
    if (SC_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
#if SC_GEMM_SGB
    // interleave: one transposed read after each MFMA, then the remaining MFMAs (or reads)
    constexpr int NMF = NU * TTI, NRD = 2 * (NU + TTI);
#pragma unroll
    for (int q = 0; q < (NMF < NRD ? NMF : NRD); ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
    }
    if constexpr (NMF > NRD) __builtin_amdgcn_sched_group_barrier(0x008, NMF - NRD, 0);
    else if constexpr (NRD > NMF) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NMF, 0);
#endif
    if (late && st) stage(h + kSlots);
  };
  int h = 0;
  for (; h + 1 < nh; h += 2) {
    iter(h, bfA, afA, bfB, afB);
    iter(h + 1, bfB, afB, bfA, afA);
  }
  if (h < nh) iter(h, bfA, afA, bfB, afB);
  // epilogue: D row = i (4 per lane), col = j (lane & 15)
  float* cs = a.C + (int64_t)split * a.I * a.J;
#pragma unroll
  for (int t = 0; t < TTI; ++t)
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wi * (TI / 2) + 16 * t + 4 * g + r;
        const int j = j0 + wj * 16 * NU + 16 * u + (lane & 15);
        cs[(int64_t)i * a.J + j] = acc[t][u][r];
      }
}

// SC_GEMM_MF32 (A/B): the TI = 224 tile on v_mfma_f32_32x32x16_bf16.  Each wave owns one 32-column
// block of the tile (columns 32 w .. 32 w + 31) and all 7 row blocks of 32: per half-stage (two
// k-steps of 16 L-rows) 14 MFMAs of 32 cycles instead of 28 of 16 (half the matrix-instruction
// issue), from 2 x (1 + 7) fragments of two transposed reads each.  The LDS ring, its DMA and
// the images are wgrad_kernel's; the ring runs kSlots - 1 half-stages ahead (the slot a DMA
// refills was read in the previous iteration, before this iteration's barrier).
// Correct (tests/test_gpu_gemm.py on it) and measured SLOWER (tools/r5_mf32.sh, one box): 202-204
// vs 187-189 us alone, 169-173 vs 166-167 us in the C2 step -- a 224 x 32 wave tile reads 32
// fragments per half-stage where the 2 x 4 grid of 112 x 64 tiles reads 22, and halving the MFMA
// instruction count does not buy that back.  Off by default.
#ifndef SC_GEMM_MF32
#define SC_GEMM_MF32 0
#endif
typedef float f16v __attribute__((ext_vector_type(16)));
#if SC_GEMM_MF32   // (A/B builds only: tools/ab/mf32; not in the product library)

__global__ void __launch_bounds__(512) wgrad32_kernel(WgradArgs a) {
  constexpr int TTI = 7, TI = 32 * TTI, NCA = TI / 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int nwg = a.tiles * a.S;
  const int bid = blockIdx.x;
  const int xcd = bid % 8, qq = nwg / 8, rr = nwg % 8;
  const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
  const int split = lid / a.tiles, tile = lid % a.tiles;
  const int ti = tile / a.ntj, tj = tile % a.ntj;
  const int i0 = ti * TI, j0 = tj * kTJ;
  const int nkb = a.L / kTL;
  const int kb0 = (int)((int64_t)split * nkb / a.S), kb1 = (int)((int64_t)(split + 1) * nkb / a.S);

  uint32_t voA[2], voB[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int row = 4 * w + 2 * q + (lane >> 5);
    const int c = (lane & 31) ^ (swz_f(row) << 1);
    voA[q] = (uint32_t)(row * a.lda + i0 + 8 * min(c, NCA - 1)) * 2u;
    voB[q] = (uint32_t)(row * a.ldb + j0 + 8 * c) * 2u;
  }
  constexpr int kHalf = 32 * kRowB;
  const uint32_t lds0 = lds_addr(lds);
  auto stage = [&](int h) __attribute__((always_inline)) {
    const int64_t r = (int64_t)kb0 * kTL + 32 * h;
    const uint32_t la = lds0 + (h % kSlots) * 2 * kHalf + 4 * w * kRowB;
#pragma unroll
    for (int q = 0; q < 2; ++q) dma_to_lds_s<16>(a.A + r * a.lda, voA[q], la + q * 1024);
#pragma unroll
    for (int q = 0; q < 2; ++q) dma_to_lds_s<16>(a.B + r * a.ldb, voB[q], la + kHalf + q * 1024);
  };
  // 32x32x16 operand geometry: lane l holds column 32-block-base + (l & 31), k-rows
  // 8 (l >> 5) .. +7 of the k-step.  Group g = lane >> 4: columns 16 (g & 1) .., rows 8 (g >> 1) ..;
  // within the group lane 4q+p addresses row q (+4 for the second read), columns 4p .. 4p+3
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  f16v acc[TTI];
#pragma unroll
  for (int t = 0; t < TTI; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.0f;
  const int nh = 2 * (kb1 - kb0);
  auto frag = [&](uint32_t img, int r0, int col) __attribute__((always_inline)) {
    const uint32_t o = (uint32_t)((col & 7) ? 8 : 0);
    const i2v lo = tr_read(img + img_off(r0, col >> 3) + o);
    const i2v hi = tr_read(img + img_off(r0 + 4, col >> 3) + o);
    return i4v{lo.x, lo.y, hi.x, hi.y};
  };
  auto load_ks = [&](int h, int ks, i4v& bf, i4v (&af)[TTI]) __attribute__((always_inline)) {
    const uint32_t ia = lds0 + (h % kSlots) * 2 * kHalf, ib = ia + kHalf;
    const int r0 = 16 * ks + 8 * (g >> 1) + q4;
    bf = frag(ib, r0, 32 * w + 16 * (g & 1) + 4 * p4);
#pragma unroll
    for (int t = 0; t < TTI; ++t) af[t] = frag(ia, r0, 32 * t + 16 * (g & 1) + 4 * p4);
  };
  auto mfmas = [&](const i4v& bf, const i4v (&af)[TTI]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < TTI; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8v, af[t]),
                                                       __builtin_bit_cast(b8v, bf), acc[t], 0, 0, 0);
  };
  auto wait_younger = [&](int n) __attribute__((always_inline)) {
    if (n >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else dma_wait();
  };
  constexpr int kAhead = kSlots - 1;   // half-stages in flight beyond the one being read
  for (int h = 0; h < kAhead && h < nh; ++h) stage(h);
  // k-step software pipeline: iteration h multiplies k-step (h, 0) from registers while (h, 1)
  // comes out of LDS, then (h, 1) while (h + 1, 0) does -- so h + 1 must have landed before the
  // iteration's barrier, and the slot refilled there is (h - 1)'s (read during iteration h - 1)
  // (the last iteration re-reads slot h for its (h + 1, 0): unused, in bounds)
  i4v bfX, afX[TTI], bfY, afY[TTI], bfZ, afZ[TTI];
  if (nh > 0) {
    wait_younger(min(kAhead - 1, nh - 1));
    lds_barrier();
    load_ks(0, 0, bfX, afX);
  }
  auto iter = [&](int h, i4v& bc, i4v (&ac)[TTI], i4v& bn, i4v (&an)[TTI])
      __attribute__((always_inline)) {
    if (h + 1 < nh) wait_younger(min(kAhead - 2, nh - 2 - h));   // h + 1 landed
    lds_barrier();
    if (h + kAhead < nh) stage(h + kAhead);
    load_ks(h, 1, bfY, afY);
    mfmas(bc, ac);
#if SC_GEMM_SGB
#pragma unroll
    for (int q = 0; q < TTI; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS reads
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#endif
    load_ks(min(h + 1, nh - 1) == h + 1 ? h + 1 : h, 0, bn, an);
    mfmas(bfY, afY);
#if SC_GEMM_SGB
#pragma unroll
    for (int q = 0; q < TTI; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#endif
  };
  int h = 0;
  for (; h + 1 < nh; h += 2) {
    iter(h, bfX, afX, bfZ, afZ);
    iter(h + 1, bfZ, afZ, bfX, afX);
  }
  if (h < nh) iter(h, bfX, afX, bfZ, afZ);
  // epilogue: acc[t][e] = dW[i = 32 t + (e & 3) + 8 (e >> 2) + 4 (lane >> 5)][j = 32 w + (lane & 31)]
  float* cs = a.C + (int64_t)split * a.I * a.J;
#pragma unroll
  for (int t = 0; t < TTI; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int i = i0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int j = j0 + 32 * w + (lane & 31);
      cs[(int64_t)i * a.J + j] = acc[t][e];
    }
}

static void launch_wgrad32(const WgradArgs& a, hipStream_t st) {
  constexpr size_t lds = (size_t)kSlots * 2 * 32 * kRowB;
  static const bool ok = hipFuncSetAttribute((const void*)wgrad32_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  hipLaunchKernelGGL(wgrad32_kernel, dim3(a.tiles * a.S), dim3(512), lds, st, a);
}
#endif  // SC_GEMM_MF32

template <int TTI, int NU = 4>
static void launch_wgrad(const WgradArgs& a, hipStream_t st) {
  auto kern = wgrad_kernel<TTI, NU>;
  constexpr size_t lds = (size_t)kSlots * 2 * 32 * kRowB;   // kSlots x (dY, X) x 16 KiB
  static const bool ok = hipFuncSetAttribute((const void*)kern,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  hipLaunchKernelGGL(kern, dim3(a.tiles * a.S), dim3(512), lds, st, a);
}

}  // namespace sc

using namespace sc;

// J-tile of a shape: 256 columns, or 128 when J is an odd multiple of 128 (layer 0's 80 features
// zero-padded to 128)
static int wgrad_tj(int J) { return J % 256 == 0 ? 256 : 128; }
// I-tile: 224 where (I / 224) tiles x the J tiles x the splits that fill 256 CUs come out whole
static int wgrad_ti(int I, int J) {
  const int tj = wgrad_tj(J);
  const int per = tj == 256 ? 8 : 16;   // L-splits of the 224-row layout
  return I % 224 == 0 && (I / 224) * (J / tj) * per == 256 ? 224 : 256;
}

extern "C" int sc_gemm_wgrad_splits(int L, int I, int J) {
  if (L <= 0 || I <= 0 || J <= 0 || L % kTL || J % 128) return 0;
  const int tj = wgrad_tj(J);
  const int ti = wgrad_ti(I, J);
  if (I % ti) return 0;
  const int tiles = (I / ti) * (J / tj);
  // as many L-splits as fill the 256 CUs (any count: the split ranges are nkb * s / S, so they
  // may differ by one K-block), each of at least 8 K-blocks.  Powers of two left C4's shapes
  // at 56-84% of the CUs (out_proj 9 tiles x 16, FFN 48 x 4 / 24 x 8, q|k|v|o head 27 x 8).
  int S = 256 / tiles;
  S = S < (L / kTL) / 8 ? S : (L / kTL) / 8;
  return S > 1 ? S : 1;
}

extern "C" int sc_gemm_wgrad_bf16(const void* A, int64_t lda, const void* B, int64_t ldb,
                                  float* part, int L, int I, int J, int S, void* stream) {
  clear_error();
  SC_REQUIRE(A && B && part, "sc_gemm_wgrad_bf16: null pointer");
  SC_REQUIRE(L > 0 && L % kTL == 0, "sc_gemm_wgrad_bf16: L=%d must be a positive multiple of 64", L);
  SC_REQUIRE(J > 0 && J % 128 == 0, "sc_gemm_wgrad_bf16: J=%d must be a multiple of 128", J);
  SC_REQUIRE(I > 0 && I % wgrad_ti(I, J) == 0,
             "sc_gemm_wgrad_bf16: I=%d must be a multiple of 256, or of 224 at the 256-workgroup "
             "layouts (use sc_gemm_wgrad_splits to gate)", I);
  SC_REQUIRE(lda >= I && ldb >= J && lda % 8 == 0 && ldb % 8 == 0,
             "sc_gemm_wgrad_bf16: leading dimensions must cover the rows in 16-byte pieces");
  SC_REQUIRE((uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0, "sc_gemm_wgrad_bf16: unaligned operand");
  SC_REQUIRE((int64_t)kTL * lda * 2 < (1ll << 31) && (int64_t)kTL * ldb * 2 < (1ll << 31),
             "sc_gemm_wgrad_bf16: row pitch too large");
  const int ti = wgrad_ti(I, J), tj = wgrad_tj(J);
  SC_REQUIRE(I % ti == 0, "sc_gemm_wgrad_bf16: I=%d not a multiple of the %d-row tile", I, ti);
  WgradArgs a{(const __bf16*)A, (const __bf16*)B, part, L, I, J, S, J / tj,
              (I / ti) * (J / tj), lda, ldb};
  SC_REQUIRE(S >= 1 && S <= L / kTL, "sc_gemm_wgrad_bf16: S=%d outside [1, L/64]", S);
  hipStream_t st = (hipStream_t)stream;
#if SC_GEMM_MF32
  if (ti == 224) launch_wgrad32(a, st);
  else
#endif
  if (tj == 128) {
    if (ti == 224) launch_wgrad<7, 2>(a, st);
    else launch_wgrad<8, 2>(a, st);
  } else if (ti == 224) {
    launch_wgrad<7>(a, st);
  } else {
    launch_wgrad<8>(a, st);
  }
  return launch_status("sc_gemm_wgrad_bf16");
}
