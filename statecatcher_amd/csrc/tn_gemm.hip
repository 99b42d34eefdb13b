// Frame-major projection GEMMs of the LucyRNN training step on gfx950 MFMA (CDNA4, wave64).
//
//   C[M][N] = A[M][K] · B[N][K]ᵀ     bf16 in, fp32 accumulate, bf16 out
//
// with both operands K-contiguous.  The step's forward and input-gradient projections are all
// this shape (M = B*T = 48,000 frames at C2):
//   * gate forward, LinearSafe (lucyrnn_triton.py:20-25):  x [M][Din] · W [7D][Din]ᵀ, Din = 512,
//     and layer 0 with Din = 80 padded to 128 (the caller's bf16 cast writes the zero columns);
//   * gate input gradient:  dgates [M][7D] · (Wᵀ) [D][7D]ᵀ  (a 3.7 MB transposed weight copy);
//   * output-projection input gradient (lucyrnn_triton.py:107-109): dlogits [M][V] · (Woᵀ)[D][V]ᵀ.
//
// Design (one 512-thread workgroup per CU, persistent over its tiles):
//   * output tile TM x 256 (TM = 32 MF: 192 by default (256 would spill), so 48,000 rows are 250 whole panels and
//     the 3584-column forward is 3,500 tiles = 13.7 per CU; the 512-column gradients 500 tiles);
//     8 waves as 2 (rows) x 4 (columns), per wave 16 MF x 64 outputs;
//   * the MFMA A operand is the B matrix: a lane's accumulators then hold 4 consecutive output
//     columns, and the B rows of each 16-row fragment are drawn so that a lane ends the tile with
//     16 consecutive columns of one row: two 16-byte stores per row fragment;
//   * K in half-stages of 32 columns (one v_mfma_f32_16x16x32_bf16 k-step).  A ring of four LDS
//     slots ([TM + 256 rows][64 B], 28 KiB at TM = 192) is filled by LDS-DMA (16-byte pieces,
//     saddr form), three half-stages in flight;
//   * the ring runs CONTINUOUSLY over the workgroup's tiles: the DMA of the next tile's first
//     half-stages is issued while the current tile finishes, so no tile restarts the pipeline;
//   * the 16-byte chunk index of LDS row r is XOR-swizzled by F[((r >> 2) ^ (r >> 4)) & 3],
//     F = {0, 2, 3, 1}, applied on the DMA SOURCE address (the LDS side of a DMA is lane-linear);
//     with ds_read_b128's lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) every
//     fragment read of both operands is conflict-free;
//   * epilogue: the finished tile is packed to bf16 in registers and its stores are spread over
//     the next tile's half-stages (buffer stores: rows >= M fall outside the descriptor's range
//     and are dropped), so the output stream overlaps the MFMAs instead of stalling them;
//   * waits are counted: vmcnt counts LDS-DMA pieces and stores together in issue order
//     (MI355X_MICROARCH.md), and each half-stage waits for exactly the vector-memory operations
//     issued up to its own last DMA piece.
// XCD-aware: consecutive tiles (the 14 column tiles of one 192-row panel, or the two of a
// gradient panel) are taken by co-resident workgroups of one XCD, so the A panel is fetched from
// HBM once per XCD and shared through its L2.

#include "sc_common.h"

namespace sc {
namespace {

typedef __bf16 b8v __attribute__((ext_vector_type(8)));
typedef __bf16 b2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));

// SC_TN_ABL (tools timing only, never in a shipped build): 1 no MFMAs, 2 no DMA after the
// prologue, 4 no output stores (tn256) (wrong results)
#ifndef SC_TN_ABL
#define SC_TN_ABL 0
#endif
// SC_TNW_AB: also build the plain one-wave-per-SIMD kernels (tile_m 1 / 2 / 3; A/B only, measured
// slower than the library: profiles/r6_tnw.md).  The LayerNorm-fold instance tnw32_kernel<4, true>
// (sc_gemm_tn_ln_bf16, SC_LN_FOLD=2) is always built.
#ifndef SC_TNW_FENCE
#define SC_TNW_FENCE 1
#endif
#ifndef SC_TNW_IL
#define SC_TNW_IL 0
#endif
#ifndef SC_TNW_EPI
#define SC_TNW_EPI 1
#endif
#ifndef SC_TNW_AB
#define SC_TNW_AB 0
#endif

constexpr int kBK = 64;      // K columns per stage (two v_mfma_f32_16x16x32_bf16 k-steps)
constexpr int kRowB = 128;   // LDS image row pitch (bytes): whole 128-byte lines per DMA row
constexpr int kTN = 256;     // output columns per tile
constexpr int kSlots = 2;    // LDS stages

struct TnArgs {
  const __bf16* A;
  const __bf16* B;
  __bf16* C;
  int M, N, K, ntn, tiles;
  uint32_t lda, ldb, ldc;   // elements
  uint32_t cbytes;          // addressable bytes of C (M * ldc * 2)
  int gm;                   // tnw: row panels per tile group (the per-XCD raster)
};

// physical-chunk XOR of image row r (8 chunks of 16 B per 128-byte row)
__device__ __forceinline__ int swz(int r) { return (r ^ (r >> 2) ^ (r >> 4)) & 7; }

__device__ __forceinline__ i4v lds_read16(uint32_t byte) {
  return *(const __attribute__((address_space(3))) i4v*)(size_t)byte;
}

template <int MF, int SPI>
__global__ void __launch_bounds__(512) tn_kernel(TnArgs a) {
  constexpr int TM = 32 * MF;
  constexpr int NP = (TM + kTN) / 8;           // 1-KiB DMA pieces (8 rows of 128 B) per stage
  constexpr int NPW = NP / 8;                  // per wave
  static_assert(NP % 8 == 0, "pieces must split evenly over the 8 waves");
  constexpr int kSlotB = (TM + kTN) * kRowB;   // bytes per LDS stage
  constexpr int NST = 2 * MF;                  // 16-byte stores per wave per tile
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // XCD-aware logical id (bids go round-robin over the 8 XCDs): consecutive lids share an XCD
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid % 8, qq = G / 8, rr = G % 8;
  const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
  const int nks = a.K / kBK;
  const int ntw = lid < a.tiles ? (a.tiles - lid + G - 1) / G : 0;
  const int NH = ntw * nks;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA geometry: piece g = NPW w + q covers image rows 8g .. 8g+7 of [A; B] ----
  int prow[NPW];        // row within its image (A: 0..TM-1, B: 0..255)
  uint32_t pcol[NPW];   // logical element column within the stage (8 c)
#pragma unroll
  for (int q = 0; q < NPW; ++q) {
    const int R = 8 * (NPW * w + q) + (lane >> 3);
    prow[q] = R < TM ? R : R - TM;
    pcol[q] = 8u * (uint32_t)((lane & 7) ^ swz(prow[q]));
  }
  int st_h = 0, st_ks = 0, st_tile = lid;
  int st_m0 = (st_tile / a.ntn) * TM, st_n0 = (st_tile % a.ntn) * kTN;
  auto stage = [&]() __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (st_h % kSlots) * kSlotB;
    const uint32_t k0 = (uint32_t)st_ks * kBK;
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const int g = NPW * w + q;
      if (8 * g < TM) {
        const uint32_t row = (uint32_t)min(st_m0 + prow[q], a.M - 1);
        dma_to_lds_s<16>(a.A, (row * a.lda + k0 + pcol[q]) * 2u, sb + g * 1024);
      } else {
        const uint32_t row = (uint32_t)(st_n0 + prow[q]);
        dma_to_lds_s<16>(a.B, (row * a.ldb + k0 + pcol[q]) * 2u, sb + g * 1024);
      }
    }
    ++st_h;
    if (++st_ks == nks) {
      st_ks = 0;
      st_tile += G;
      st_m0 = (st_tile / a.ntn) * TM;
      st_n0 = (st_tile % a.ntn) * kTN;
    }
  };

  // ---- fragment geometry (byte offsets within a stage; k-step kk flips address bit 6) ----
  // MFMA A operand = B rows: fragment nf, lane row fr -> image row wn*64 + (fr>>2)*16 + nf*4 +
  // (fr&3), so the lane's accumulators over nf hold output columns wn*64 + fq*16 + 0..15.
  uint32_t offB[4];
#pragma unroll
  for (int nf = 0; nf < 4; ++nf) {
    const int r = wn * 64 + (fr >> 2) * 16 + nf * 4 + (fr & 3);
    offB[nf] = (uint32_t)(TM * kRowB + r * kRowB + 16 * (fq ^ swz(r)));
  }
  // MFMA B operand = A rows wm*TM/2 + mf*16 + fr
  uint32_t offA[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int r = wm * (TM / 2) + mf * 16 + fr;
    offA[mf] = (uint32_t)(r * kRowB + 16 * (fq ^ swz(r)));
  }
  auto load_frags = [&](uint32_t sb, int kk, i4v (&bf)[4], i4v (&af)[MF]) __attribute__((always_inline)) {
    const uint32_t x = 64u * kk;
#pragma unroll
    for (int nf = 0; nf < 4; ++nf) bf[nf] = lds_read16(sb + (offB[nf] ^ x));
#pragma unroll
    for (int mf = 0; mf < MF; ++mf) af[mf] = lds_read16(sb + (offA[mf] ^ x));
  };

  f4v acc[MF][4];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < 4; ++nf) acc[mf][nf] = f4v{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](const i4v (&bf)[4], const i4v (&af)[MF]) __attribute__((always_inline)) {
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < 4; ++nf)
        acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(b8v, bf[nf]), __builtin_bit_cast(b8v, af[mf]), acc[mf][nf], 0, 0, 0);
  };

  // ---- epilogue: packed bf16 rows waiting to be stored, SPI per stage over the next tile ----
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.cbytes, 0x00020000);
  i4v outv[NST];
  int st_done = NST;   // stores of the pending tile already issued
  uint32_t obase = 0;  // lane byte offset of the pending tile's first row fragment
  auto pack = [&](int tile) __attribute__((always_inline)) {
    const int m0 = (tile / a.ntn) * TM, n0 = (tile % a.ntn) * kTN;
    const uint32_t row = (uint32_t)(m0 + wm * (TM / 2) + fr);
    obase = (row * a.ldc + (uint32_t)(n0 + wn * 64 + fq * 16)) * 2u;
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        i4v v;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int nf = 2 * hlf + (d >> 1), j = 2 * (d & 1);
          const b2v p = {(__bf16)acc[mf][nf][j], (__bf16)acc[mf][nf][j + 1]};
          v[d] = __builtin_bit_cast(int, p);
        }
        outv[2 * mf + hlf] = v;
      }
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) acc[mf][nf] = f4v{0.f, 0.f, 0.f, 0.f};
    st_done = 0;
  };
  auto store_some = [&](int n) __attribute__((always_inline)) {
    const int lo = st_done, hi = min(NST, st_done + n);
#pragma unroll
    for (int s = 0; s < NST; ++s)
      if (s >= lo && s < hi) {
        const uint32_t off = obase + (uint32_t)((s >> 1) * 16) * a.ldc * 2u + (uint32_t)((s & 1) * 16);
        __builtin_amdgcn_raw_buffer_store_b128(outv[s], crs, off, 0, 0);
      }
    st_done = hi;
  };

  // ---- pipeline: stage h+1 streams in while stage h computes ----
  // Iteration h: the earlier tile's stores (issued first, so they are older than the DMA) ->
  // DMA of stage h+1 into the other slot (its last readers passed the previous barrier) ->
  // k-step 0 fragments, MFMAs with k-step 1's fragments in flight, k-step 1 MFMAs -> vmcnt(0)
  // (stage h+1 landed, this wave's stores done) -> barrier.
  if (NH > 0) {
    stage();
    dma_wait();
    lds_barrier();
  }
  int cur_ks = 0, cur_tile = lid;
  i4v bf0[4], af0[MF], bf1[4], af1[MF];
  for (int h = 0; h < NH; ++h) {
    if (st_done < NST) store_some(SPI);
    if (st_h < NH && !(SC_TN_ABL & 2)) stage();
    const uint32_t sb = lds0 + (h % kSlots) * kSlotB;
    load_frags(sb, 0, bf0, af0);
    load_frags(sb, 1, bf1, af1);
    if (SC_TN_ABL & 1) {
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
        acc[mf][0][0] += (float)(bf0[mf & 3][0] ^ af1[mf][1]) + (float)(bf1[mf & 3][2] ^ af0[mf][3]);
    } else {
      mfmas(bf0, af0);
      mfmas(bf1, af1);
    }
    if (++cur_ks == nks) {
      pack(cur_tile);
      cur_ks = 0;
      cur_tile += G;
    }
    dma_wait();
    lds_barrier();
  }
  if (st_done < NST) store_some(NST);
}

// ------------------------------------------------------------------------------------------
// 256 x 256 tiles, four-phase quadrant schedule (the default since round 3).
//
// A K-tile (64 columns) of the 256 x 256 output tile is four PHASES; in each, all 8 waves compute
// one 128 x 128 QUADRANT of the tile (per wave 64 rows x 32 columns: 4 x 2 fragments, 16
// v_mfma_f32_16x16x32_bf16) in the order (0,0) (0,1) (1,1) (1,0), so each phase needs ONE new
// operand half (A rows 0-127 / 128-255 = "A0" / "A1", B rows likewise "B0" / "B1") and reuses
// the other from registers:
//   phase 1: A0 x B0   (A0, B0 read from LDS in phase 4 of the previous K-tile)
//   phase 2: A0 x B1   (B1 read in phase 1)
//   phase 3: A1 x B1   (A1 read in phase 2)
//   phase 4: A1 x B0   (B0 read again in phase 3; A0, B0 of the next K-tile are read here)
// LDS holds two K-tiles (2 x 4 halves x 16 KiB = 128 KiB).  Each half of K-tile g + 2 is
// restaged into buffer g % 2 by LDS-DMA one phase after its last fragment read in K-tile g
// (A0 in phase 1, B1 in 2, A1 in 3, B0 in 4): three halves (6 DMA instructions per thread) stay
// in flight, and ONE counted wait per K-tile -- vmcnt(6) at the end of phase 3, which retires
// B0 of the NEXT K-tile and everything older -- orders every fragment read after its DMA.  One
// LDS-only barrier per phase; the MFMA cluster of a phase is bracketed by s_setprio so hipcc keeps
// it between its barriers (cdna_hip_programming.md T5).
// Epilogue: a quadrant's accumulators are final one phase after its last MFMAs; it is packed to
// bf16 and stored in a later phase (q00 in phase 2 and q01 in phase 4 of the tile's last K-tile,
// q11 in phase 1 and q10 in phase 2 of the next tile's first K-tile) -- the output stream runs
// beside the MFMAs and no registers are held across tiles.  Buffer stores: rows >= M fall
// outside the descriptor's range and are dropped.  Stores are never issued in phase 3 and are
// younger than the B0 DMA the phase-3 wait targets, so they only inflate that count (loads
// complete in order among themselves): the wait stays exact.
constexpr int kHalfB = 128 * kRowB;   // one operand half: 128 rows x 128 B

// Wave layout over a 128 x 128 quadrant.  SC_TN_WL = 0: 2 (rows) x 4 (columns) waves of 64 x 32,
// a lane's row fragment covers 8 consecutive columns (one 16-byte store; a 128-byte output line
// takes stores from two waves).  SC_TN_WL = 1: 4 x 2 waves of 32 x 64, 16 consecutive columns per
// lane (two 16-byte stores back to back, every output line written whole by one wave).
#ifndef SC_TN_WL
#define SC_TN_WL 0
#endif
constexpr int kTnWN = SC_TN_WL ? 2 : 4;        // waves along the columns
constexpr int kTnMF = 128 / (8 / kTnWN) / 16;  // row fragments per wave (4 or 2)
constexpr int kTnNF = 128 / kTnWN / 16;        // column fragments per wave (2 or 4)
// MFMA fragment sets of one operand half, named (static indexing only: rule 20)
struct FragA { i4v v[kTnMF][2]; };   // row fragments (x rows) x 2 k-steps
struct FragB { i4v v[kTnNF][2]; };   // column fragments (W rows) x 2 k-steps

__global__ void __launch_bounds__(512, 1) tn256_kernel(TnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int wm = w / kTnWN, wn = w % kTnWN;
  const int l15 = lane & 15, l4 = lane >> 4;

  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid % 8, qq = G / 8, rr = G % 8;
  const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
  const int nkt = a.K / kBK;
  const int ntw = lid < a.tiles ? (a.tiles - lid + G - 1) / G : 0;
  const int NG = ntw * nkt;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA: wave w stages rows 16 w .. 16 w + 15 of a half (two 1-KiB pieces of 8 rows) ----
  int drow[2];
  uint32_t dcol[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * (2 * w + q) + (lane >> 3);
    drow[q] = r;
    dcol[q] = 8u * (uint32_t)((lane & 7) ^ swz(r));
  }
  // cursor of the DMA stream: K-tile dg of this workgroup's sequence
  int dg = 0, dkt = 0, dtile = lid;
  int dm0 = (dtile / a.ntn) * 256, dn0 = (dtile % a.ntn) * 256;
  auto dma_half = [&](int h) __attribute__((always_inline)) {   // half h of K-tile dg
    const uint32_t dst = lds0 + (uint32_t)(((dg & 1) * 4 + h) * kHalfB + 2 * w * 1024);
    const uint32_t k0 = (uint32_t)dkt * kBK;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (h < 2) {
        const uint32_t row = (uint32_t)min(dm0 + h * 128 + drow[q], a.M - 1);
        dma_to_lds_s<16>(a.A, (row * a.lda + k0 + dcol[q]) * 2u, dst + q * 1024);
      } else {
        const uint32_t row = (uint32_t)(dn0 + (h - 2) * 128 + drow[q]);
        dma_to_lds_s<16>(a.B, (row * a.ldb + k0 + dcol[q]) * 2u, dst + q * 1024);
      }
    }
  };
  auto dma_next = [&]() __attribute__((always_inline)) {   // advance the cursor one K-tile
    ++dg;
    if (++dkt == nkt) {
      dkt = 0;
      dtile += G;
      dm0 = (dtile / a.ntn) * 256;
      dn0 = (dtile % a.ntn) * 256;
    }
  };

  // ---- fragment reads (byte offsets within a half; k-step kk flips address bit 6) ----
  uint32_t offA[kTnMF], offB[kTnNF];
#pragma unroll
  for (int mf = 0; mf < kTnMF; ++mf) {
    const int r = wm * 16 * kTnMF + mf * 16 + l15;
    offA[mf] = (uint32_t)(r * kRowB + 16 * (l4 ^ swz(r)));
  }
#pragma unroll
  for (int nf = 0; nf < kTnNF; ++nf) {
    // W row for MFMA row i = l15 of column fragment nf: the lane's NF x 4 accumulator values
    // then hold output columns wn*16NF + l4*4NF + 0..4NF-1 (NF/2 16-byte stores per row fragment)
    const int r = wn * 16 * kTnNF + (l15 >> 2) * 4 * kTnNF + nf * 4 + (l15 & 3);
    offB[nf] = (uint32_t)(r * kRowB + 16 * (l4 ^ swz(r)));
  }
  auto half_base = [&](int buf, int h) __attribute__((always_inline)) {
    return lds0 + (uint32_t)((buf * 4 + h) * kHalfB);
  };
  auto read_A = [&](int buf, int qm, FragA& f) __attribute__((always_inline)) {
    const uint32_t hb = half_base(buf, qm);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mf = 0; mf < kTnMF; ++mf) f.v[mf][kk] = lds_read16(hb + (offA[mf] ^ (64u * kk)));
  };
  auto read_B = [&](int buf, int qn, FragB& f) __attribute__((always_inline)) {
    const uint32_t hb = half_base(buf, 2 + qn);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nf = 0; nf < kTnNF; ++nf) f.v[nf][kk] = lds_read16(hb + (offB[nf] ^ (64u * kk)));
  };

  f4v acc[4][kTnMF][kTnNF];   // [quadrant (0,0) (0,1) (1,1) (1,0)][row frag][col frag]
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int mf = 0; mf < kTnMF; ++mf)
#pragma unroll
      for (int nf = 0; nf < kTnNF; ++nf) acc[q][mf][nf] = f4v{0.f, 0.f, 0.f, 0.f};
  auto quad = [&](f4v (&c)[kTnMF][kTnNF], const FragA& fa, const FragB& fb) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mf = 0; mf < kTnMF; ++mf)
#pragma unroll
        for (int nf = 0; nf < kTnNF; ++nf) {
          if (SC_TN_ABL & 1)
            c[mf][nf][0] += (float)(fb.v[nf][kk][0] ^ fa.v[mf][kk][1]);
          else
            c[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(b8v, fb.v[nf][kk]), __builtin_bit_cast(b8v, fa.v[mf][kk]),
                c[mf][nf], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- epilogue: one quadrant (4 row fragments x one 16-byte store), then zeroed ----
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.cbytes, 0x00020000);
  auto store_quad = [&](f4v (&c)[kTnMF][kTnNF], int m0, int n0, int qm, int qn) __attribute__((always_inline)) {
    if (SC_TN_ABL & 4) return;   // (ablation: no output stores)
    const uint32_t row = (uint32_t)(m0 + qm * 128 + wm * 16 * kTnMF + l15);
    const uint32_t col = (uint32_t)(n0 + qn * 128 + wn * 16 * kTnNF + l4 * 4 * kTnNF);
#pragma unroll
    for (int mf = 0; mf < kTnMF; ++mf) {
#pragma unroll
      for (int s2 = 0; s2 < kTnNF / 2; ++s2) {   // 8 consecutive columns per 16-byte store
        i4v v;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int nf = 2 * s2 + (d >> 1), j = 2 * (d & 1);
          const b2v p = {(__bf16)c[mf][nf][j], (__bf16)c[mf][nf][j + 1]};
          v[d] = __builtin_bit_cast(int, p);
        }
        __builtin_amdgcn_raw_buffer_store_b128(v, crs, ((row + 16u * mf) * a.ldc + col + 8u * s2) * 2u,
                                               0, 0);
      }
#pragma unroll
      for (int nf = 0; nf < kTnNF; ++nf) c[mf][nf] = f4v{0.f, 0.f, 0.f, 0.f};
    }
  };

  if (NG == 0) return;
  // ---- prologue: K-tiles 0 and 1 (halves in the steady-state issue order A0 B1 A1 B0) ----
#pragma unroll
  for (int g0 = 0; g0 < 2; ++g0)
    if (dg < NG) {
      dma_half(0); dma_half(3); dma_half(1); dma_half(2);
      dma_next();
    }
  if (NG > 1) dma_wait_younger<8>(); else dma_wait();
  lds_barrier();
  // B fragment sets X / Y alternate roles between K-tiles (static names: the K-tile loop is
  // unrolled by two): B0 is read twice per K-tile (phases 4 of the previous and 3 of this one)
  // instead of living in registers through all four phases -- 16 registers fewer, no spills
  FragA fa0, fa1;
  FragB fbX, fbY;
  read_A(0, 0, fa0);
  read_B(0, 0, fbX);
  lds_read_wait();

  int kt = 0, tile = lid, pm0 = 0, pn0 = 0;
  int m0 = (tile / a.ntn) * 256, n0 = (tile % a.ntn) * 256;
  auto ktile = [&](int g, FragB& X, FragB& Y) __attribute__((always_inline)) {
    const int buf = g & 1;
    const bool first = kt == 0, last = kt == nkt - 1;
    const bool more = dg < NG;   // K-tile g + 2 exists
    // phase 1: quadrant (0,0) = A0 x B0 (X)
    if (first && g > 0) store_quad(acc[2], pm0, pn0, 1, 1);
    if (more && !(SC_TN_ABL & 2)) dma_half(0);
    read_B(buf, 1, Y);
    quad(acc[0], fa0, X);
    lds_read_wait();
    lds_barrier();
    // phase 2: quadrant (0,1) = A0 x B1 (Y)
    if (first && g > 0) store_quad(acc[3], pm0, pn0, 1, 0);
    if (last) store_quad(acc[0], m0, n0, 0, 0);
    if (more && !(SC_TN_ABL & 2)) dma_half(3);
    read_A(buf, 1, fa1);
    quad(acc[1], fa0, Y);
    lds_read_wait();
    lds_barrier();
    // phase 3: quadrant (1,1) = A1 x B1 (Y); B0 read again into X; then retire B0 of K-tile
    // g + 1 (and all older DMA)
    if (more && !(SC_TN_ABL & 2)) dma_half(1);
    read_B(buf, 0, X);
    quad(acc[2], fa1, Y);
    lds_read_wait();
    if (more) dma_wait_younger<6>(); else dma_wait();
    lds_barrier();
    // phase 4: quadrant (1,0) = A1 x B0 (X); A0, B0 of K-tile g + 1 come out of LDS (into Y)
    if (last) store_quad(acc[1], m0, n0, 0, 1);
    if (more && !(SC_TN_ABL & 2)) dma_half(2);
    if (more) dma_next();
    if (g + 1 < NG) {
      read_A(buf ^ 1, 0, fa0);
      read_B(buf ^ 1, 0, Y);
    }
    quad(acc[3], fa1, X);
    lds_read_wait();
    lds_barrier();
    if (++kt == nkt) {
      kt = 0;
      pm0 = m0;
      pn0 = n0;
      tile += G;
      m0 = (tile / a.ntn) * 256;
      n0 = (tile % a.ntn) * 256;
    }
  };
  int g = 0;
  for (; g + 1 < NG; g += 2) {
    ktile(g, fbX, fbY);
    ktile(g + 1, fbY, fbX);
  }
  if (g < NG) ktile(g, fbX, fbY);
  store_quad(acc[2], pm0, pn0, 1, 1);
  store_quad(acc[3], pm0, pn0, 1, 0);
}

// ------------------------------------------------------------------------------------------
// 256 x 256 tiles, PING-PONG schedule (tile_m = 257 selects it; measured against tn256 above).
//
// The two waves that share a SIMD (w and w + 4) alternate roles every segment: while one runs a
// 16-MFMA compute segment, the other issues its next fragment reads (and its share of the
// LDS-DMA stream) -- the SIMD's matrix pipe is fed by one wave while the other waits on LDS.
// Waves 4-7 start one barrier late and stay offset by one segment (MI355X_MICROARCH.md "Two
// waves per SIMD", cdna_hip_programming.md §5 8-phase template).
//   * wave w: output rows 128 (w >> 2) + [0, 128) (its own A half), columns 64 (w & 3) + [0, 64);
//     per K-tile four quadrants of 64 x 32 in the order (0,0) (0,1) (1,1) (1,0): load segments
//     L1 (A rows 0-63, B cols 0-31), L2 (B cols 32-63), L3 (A rows 64-127), L4 (B cols 0-31).
//   * LDS: two K-tile buffers (4 halves x 16 KiB each).  K-tile j + 1 is staged into buffer
//     (j + 1) % 2 during K-tile j (wave w DMAs 8 of its 64 1-KiB pieces, 4 in L1 and 4 in L2);
//     its last readers (K-tile j - 1) finished a barrier earlier.  Every wave retires its own
//     pieces with vmcnt(0) at the end of its L4 -- four segments after the last one was issued
//     and one barrier before the first read of K-tile j + 1.
//   * epilogue: a finished tile's four quadrants are packed and stored in L1 of the next tile's
//     first K-tile, BEFORE that segment's DMA (so the K-tile's single vmcnt(0) also covers them,
//     six segments later); buffer stores drop rows >= M.
struct FragA1 { i4v v[4][2]; };   // one quadrant: 4 row fragments x 2 k-steps
struct FragB1 { i4v v[2][2]; };   // 2 column fragments x 2 k-steps

__global__ void __launch_bounds__(512, 1) tnpp_kernel(TnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int hf = w >> 2, wq = w & 3;
  const int l15 = lane & 15, l4 = lane >> 4;

  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid % 8, qq = G / 8, rr = G % 8;
  const int lid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
  const int nkt = a.K / kBK;
  const int ntw = lid < a.tiles ? (a.tiles - lid + G - 1) / G : 0;
  const int NG = ntw * nkt;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA: wave w stages rows 64 (w & 1) + [0, 64) of half w >> 1 (8 pieces of 8 rows) ----
  const int dh = w >> 1;                 // 0, 1: A halves; 2, 3: B halves
  uint32_t dvo[8];                       // lane byte offset within the operand, per piece
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int r = 64 * (w & 1) + 8 * q + (lane >> 3);
    dvo[q] = (uint32_t)(r) * 0u + 16u * (uint32_t)((lane & 7) ^ swz(r));   // chunk part
  }
  int dg = 0, dkt = 0, dtile = lid;
  int dm0 = (dtile / a.ntn) * 256, dn0 = (dtile % a.ntn) * 256;
  auto dma_pieces = [&](int q0) __attribute__((always_inline)) {   // pieces q0 .. q0 + 3
    const uint32_t dst = lds0 + (uint32_t)(((dg & 1) * 4 + dh) * kHalfB + 64 * (w & 1) * kRowB);
    const uint32_t kb = (uint32_t)dkt * kBK * 2u;
#pragma unroll
    for (int q = q0; q < q0 + 4; ++q) {
      const int r = 64 * (w & 1) + 8 * q + (lane >> 3);
      if (dh < 2) {
        const uint32_t row = (uint32_t)min(dm0 + dh * 128 + r, a.M - 1);
        dma_to_lds_s<16>(a.A, row * a.lda * 2u + kb + dvo[q], dst + q * 1024);
      } else {
        const uint32_t row = (uint32_t)(dn0 + (dh - 2) * 128 + r);
        dma_to_lds_s<16>(a.B, row * a.ldb * 2u + kb + dvo[q], dst + q * 1024);
      }
    }
  };
  auto dma_next = [&]() __attribute__((always_inline)) {
    ++dg;
    if (++dkt == nkt) {
      dkt = 0;
      dtile += G;
      dm0 = (dtile / a.ntn) * 256;
      dn0 = (dtile % a.ntn) * 256;
    }
  };

  // ---- fragment offsets within a half ----
  uint32_t offA[2][4], offB[2][2];
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const int r = mq * 64 + mf * 16 + l15;
      offA[mq][mf] = (uint32_t)(r * kRowB + 16 * (l4 ^ swz(r)));
    }
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const int r = (wq & 1) * 64 + nq * 32 + (l15 >> 2) * 8 + nf * 4 + (l15 & 3);
      offB[nq][nf] = (uint32_t)(r * kRowB + 16 * (l4 ^ swz(r)));
    }
  auto read_A = [&](int buf, int mq, FragA1& f) __attribute__((always_inline)) {
    const uint32_t hb = lds0 + (uint32_t)((buf * 4 + hf) * kHalfB);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mf = 0; mf < 4; ++mf) f.v[mf][kk] = lds_read16(hb + (offA[mq][mf] ^ (64u * kk)));
  };
  auto read_B = [&](int buf, int nq, FragB1& f) __attribute__((always_inline)) {
    const uint32_t hb = lds0 + (uint32_t)((buf * 4 + 2 + (wq >> 1)) * kHalfB);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) f.v[nf][kk] = lds_read16(hb + (offB[nq][nf] ^ (64u * kk)));
  };

  f4v acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int mf = 0; mf < 4; ++mf)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) acc[q][mf][nf] = f4v{0.f, 0.f, 0.f, 0.f};
  auto quad = [&](f4v (&c)[4][2], const FragA1& fa, const FragB1& fb) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
          c[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(b8v, fb.v[nf][kk]), __builtin_bit_cast(b8v, fa.v[mf][kk]),
              c[mf][nf], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.cbytes, 0x00020000);
  auto store_quad = [&](f4v (&c)[4][2], int m0, int n0, int mq, int nq) __attribute__((always_inline)) {
    const uint32_t row = (uint32_t)(m0 + hf * 128 + mq * 64 + l15);
    const uint32_t col = (uint32_t)(n0 + wq * 64 + nq * 32 + l4 * 8);
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      i4v v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int nf = d >> 1, j = 2 * (d & 1);
        const b2v p = {(__bf16)c[mf][nf][j], (__bf16)c[mf][nf][j + 1]};
        v[d] = __builtin_bit_cast(int, p);
      }
      __builtin_amdgcn_raw_buffer_store_b128(v, crs, ((row + 16u * mf) * a.ldc + col) * 2u, 0, 0);
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) c[mf][nf] = f4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_tile = [&](int m0, int n0) __attribute__((always_inline)) {
    store_quad(acc[0], m0, n0, 0, 0);
    store_quad(acc[1], m0, n0, 0, 1);
    store_quad(acc[2], m0, n0, 1, 1);
    store_quad(acc[3], m0, n0, 1, 0);
  };

  if (NG == 0) return;
  // prologue: K-tile 0 (all 8 pieces of this wave), retired before the first reads
  dma_pieces(0);
  dma_pieces(4);
  dma_next();
  dma_wait();
  lds_barrier();
  if (hf == 1) __builtin_amdgcn_s_barrier();   // waves 4-7: one segment behind

  FragA1 fa;
  FragB1 fb;
  int kt = 0, tile = lid, pm0 = 0, pn0 = 0;
  int m0 = (tile / a.ntn) * 256, n0 = (tile % a.ntn) * 256;
  for (int j = 0; j < NG; ++j) {
    const int buf = j & 1;
    const bool more = dg < NG;   // K-tile j + 1 to stage
    // L1: previous tile's stores (older than this K-tile's DMA), DMA pieces 0-3, A(mq 0), B(nq 0)
    if (kt == 0 && j > 0) store_tile(pm0, pn0);
    if (more) dma_pieces(0);
    read_A(buf, 0, fa);
    read_B(buf, 0, fb);
    lds_read_wait();
    __builtin_amdgcn_s_barrier();
    quad(acc[0], fa, fb);                              // C1: (0,0)
    __builtin_amdgcn_s_barrier();
    if (more) dma_pieces(4);                           // L2
    read_B(buf, 1, fb);
    lds_read_wait();
    __builtin_amdgcn_s_barrier();
    quad(acc[1], fa, fb);                              // C2: (0,1)
    __builtin_amdgcn_s_barrier();
    read_A(buf, 1, fa);                                // L3
    lds_read_wait();
    __builtin_amdgcn_s_barrier();
    quad(acc[2], fa, fb);                              // C3: (1,1)
    __builtin_amdgcn_s_barrier();
    read_B(buf, 0, fb);                                // L4; this wave's DMA of K-tile j + 1 lands
    lds_read_wait();
    dma_wait();
    if (more) dma_next();
    __builtin_amdgcn_s_barrier();
    quad(acc[3], fa, fb);                              // C4: (1,0)
    __builtin_amdgcn_s_barrier();
    if (++kt == nkt) {
      kt = 0;
      pm0 = m0;
      pn0 = n0;
      tile += G;
      m0 = (tile / a.ntn) * 256;
      n0 = (tile % a.ntn) * 256;
    }
  }
  store_tile(pm0, pn0);
  if (hf == 0) __builtin_amdgcn_s_barrier();   // same barrier count in both halves
}

// ------------------------------------------------------------------------------------------
// One wave per SIMD, 256 x 256 tiles (tile_m = 1): tnw_kernel.
//
// tn256 / tnpp run 8 waves (two per SIMD) of 128 x 64 outputs each; with 16x16x32 MFMAs a wave
// then reads ~0.4 fragments per MFMA, and the CU's four SIMDs together ask the LDS for ~220
// B/clk of its 256: fragment reads, not the MFMA pipe, pace their loops (0.70-0.85 PF at the
// gate shape against hipBLASLt's 1.0-1.2).  Here 4 waves each own a 128 x 128 block of the
// tile: the 256 fp32 accumulators live in the AGPR half of the 512-entry register file that one
// wave per SIMD may use (MI355X_MICROARCH.md §Register files), the two 16-fragment operand sets
// (x rows / W rows of one 32-deep k-step, 64 VGPRs each) in the VGPR half.  Per k-step a wave
// issues 16 ds_read_b128 for 64 MFMAs (1,024 cycles): ~64 B/clk/CU of LDS reads.
//   * LDS: two 64 KiB slots of one 64-deep K-tile ([256 x rows][128 B] then [256 W rows][128 B]),
//     the 16-byte chunk of image row r at physical position c ^ swz(r) (applied on the DMA source
//     address; every fragment read conflict-free under ds_read_b128's lane groups, checked by
//     script);
//   * K-tile kt: k-step 0 MFMAs on set X while set Y (k-step 1) is read; then this wave's DMA of
//     K-tile kt + 1 is retired (vmcnt(0)) and ONE barrier passed -- every wave's share of it has
//     landed and every wave has finished reading slot kt % 2 -- after which K-tile kt + 2 is DMA'd
//     into that slot and set X of K-tile kt + 1 is read while k-step 1's MFMAs run on Y.  A DMA
//     has two k-steps (2,048 MFMA cycles) to land;
//   * one tile per workgroup, no persistence: the output (32 16-byte stores per wave, each lane
//     writing 32 consecutive columns of one row) is issued after the K loop and nothing waits for
//     it, so it drains while the CU's next workgroup runs.  (A persistent workgroup would have to
//     retire those stores at its next DMA wait: gfx9's vmcnt counts both.)
//   * the MFMA A operand is the W image (lane rows drawn so that a lane's 8 x 4 accumulators of
//     one x fragment are 32 consecutive output columns), the B operand the x image;
//   * XCD-aware tile order: the tiles of an XCD are consecutive, column tiles fastest, so an x
//     panel comes from HBM once per XCD and W stays in its L2.
namespace tnw {
constexpr int kSlotB = 64 * 1024;   // one K-tile: A image 32 KiB + B image 32 KiB
// lgkmcnt(0) as the builtin (vmcnt and expcnt left at their maxima), which the compiler's waitcnt
// pass sees.  (Read in the generated code, profiles/r6_tnw.md: with either this or an inline-asm
// wait the pass still puts an lgkmcnt(0) after the first MFMA of the k-step whose next fragments
// were just issued, so each k-step exposes the LDS read latency; fragment reads issued from
// inline asm instead spill 40-48 VGPRs into the loop.)
__device__ __forceinline__ void frag_wait() {
  if (SC_TNW_FENCE) __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (SC_TNW_FENCE) __builtin_amdgcn_sched_barrier(0);
}
// SC_TNW_IL: the k-step's 16 fragment reads (+ LN's 4 statistic reads) one at a time between
// groups of 3 of the current stage's MFMAs, instead of all before the first MFMA
template <int NR>
__device__ __forceinline__ void interleave() {
  if constexpr (SC_TNW_IL) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // MFMA
    }
  }
}
struct Frag { i4v v[8]; };          // 8 fragments of one operand for one k-step
}  // namespace tnw

#if SC_TNW_AB   // (A/B builds only: measured slower than hipBLASLt, profiles/r6_tnw.md)

__global__ void __launch_bounds__(256, 1) tnw_kernel(TnArgs a) {
  using namespace tnw;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int l15 = lane & 15, l4 = lane >> 4;
  // ---- tile: XCD x (bids go round-robin over the 8 XCDs) owns row panels [p0, p0 + np); its
  // k-th workgroup takes tile k of a grouped raster: groups of gm panels, columns outer, panels
  // inner, so the ~32 tiles in flight on an XCD share gm x-panels and 32 / gm W-panels in its L2
  const int bid = blockIdx.x;
  const int npan = (a.M + 255) / 256;
  const int xcd = bid % 8, k = bid / 8;
  const int pq = npan / 8, pr = npan % 8;
  const int np = pq + (xcd < pr), p0 = xcd * pq + min(xcd, pr);
  if (k >= np * a.ntn) return;
  const int grp = k / (a.gm * a.ntn), first = grp * a.gm;
  const int gsz = min(a.gm, np - first), within = k - grp * a.gm * a.ntn;
  const int m0 = (p0 + first + within % gsz) * 256, n0 = (within / gsz) * 256;
  const int nkt = a.K / kBK;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA: wave w stages image rows 64 w .. 64 w + 63 of both operands (8 + 8 pieces) ----
  uint32_t voA[8], voB[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int r = 64 * w + 8 * q + (lane >> 3);
    const uint32_t ch = 8u * (uint32_t)((lane & 7) ^ swz(r));
    voA[q] = ((uint32_t)min(m0 + r, a.M - 1) * a.lda + ch) * 2u;
    voB[q] = ((uint32_t)(n0 + r) * a.ldb + ch) * 2u;
  }
  auto dma = [&](int kt) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((kt & 1) * kSlotB) + (uint32_t)(w * 8 * 1024);
    const __bf16* pa = a.A + kt * kBK;
    const __bf16* pb = a.B + kt * kBK;
#pragma unroll
    for (int q = 0; q < 8; ++q) dma_to_lds_s<16>(pa, voA[q], sb + q * 1024);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma_to_lds_s<16>(pb, voB[q], sb + 32 * 1024 + q * 1024);
  };

  // ---- fragment offsets within a slot (k-step kk flips address bit 6) ----
  uint32_t offX[8], offW[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    const int rx = wm * 128 + f * 16 + l15;                              // x rows
    offX[f] = (uint32_t)(rx * kRowB + 16 * (l4 ^ swz(rx)));
    const int rw = wn * 128 + (l15 >> 2) * 32 + f * 4 + (l15 & 3);       // W rows
    offW[f] = (uint32_t)(32 * 1024 + rw * kRowB + 16 * (l4 ^ swz(rw)));
  }
  auto read = [&](int kt, int kk, Frag& fx, Frag& fw) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((kt & 1) * kSlotB);
    const uint32_t x = 64u * kk;
#pragma unroll
    for (int f = 0; f < 8; ++f) fw.v[f] = lds_read16(sb + (offW[f] ^ x));
#pragma unroll
    for (int f = 0; f < 8; ++f) fx.v[f] = lds_read16(sb + (offX[f] ^ x));
  };
  f4v acc[8][8];   // [x fragment][W fragment]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](const Frag& fx, const Frag& fw) __attribute__((always_inline)) {
    if (SC_TN_ABL & 1) {   // (ablation: operands kept live, no MFMA)
#pragma unroll
      for (int f = 0; f < 8; ++f) asm volatile("" ::"v"(fx.v[f]), "v"(fw.v[f]));
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(b8v, fw.v[j]), __builtin_bit_cast(b8v, fx.v[i]), acc[i][j], 0, 0, 0);
  };

  // ---- prologue: K-tiles 0 and 1 in flight, 0 retired ----
  dma(0);
  if (nkt > 1) {
    dma(1);
    dma_wait_younger<16>();
  } else {
    dma_wait();
  }
  lds_barrier();
  Frag X, Xw, Y, Yw;
  read(0, 0, X, Xw);
  for (int kt = 0; kt < nkt; ++kt) {
    // k-step 0 on X while k-step 1's fragments come in
    read(kt, 1, Y, Yw);
    mfmas(X, Xw);
    tnw::frag_wait();
    if (kt + 1 < nkt) {
      dma_wait();      // this wave's share of K-tile kt + 1 (nothing younger is in flight)
      lds_barrier();   // ... everyone's, and every read of slot kt % 2 is done
      if (kt + 2 < nkt && !(SC_TN_ABL & 2)) dma(kt + 2);
      read(kt + 1, 0, X, Xw);
    }
    mfmas(Y, Yw);
  }

  if (SC_TN_ABL & 4) {   // (ablation: accumulators kept live, no stores)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"a"(acc[i][j]));
    return;
  }
  // ---- epilogue: per x fragment, 32 consecutive bf16 columns per lane = four 16-byte stores ----
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.cbytes, 0x00020000);
  const uint32_t col = (uint32_t)(n0 + wn * 128 + l4 * 32);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t row = (uint32_t)(m0 + wm * 128 + i * 16 + l15);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      i4v v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int j = 2 * s4 + (d >> 1), e = 2 * (d & 1);
        const b2v p = {(__bf16)acc[i][j][e], (__bf16)acc[i][j][e + 1]};
        v[d] = __builtin_bit_cast(int, p);
      }
      __builtin_amdgcn_raw_buffer_store_b128(v, crs, (row * a.ldc + col + 8u * s4) * 2u, 0, 0);
    }
  }
}

int launch_tnw(const TnArgs& a, hipStream_t st) {
  constexpr size_t lds = 2 * (size_t)tnw::kSlotB;   // 128 KiB
  static const bool ok = hipFuncSetAttribute((const void*)tnw_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  const int npan = (a.M + 255) / 256;
  const int grid = 8 * ((npan + 7) / 8) * a.ntn;
  hipLaunchKernelGGL(tnw_kernel, dim3(grid), dim3(256), lds, st, a);
  return 0;
}
#endif  // SC_TNW_AB

// ------------------------------------------------------------------------------------------
// tnw with a deeper DMA ring (tile_m = 2): tnw32_kernel<NS>.
// The same 4 waves x 128 x 128 outputs, but the K loop runs in 32-deep stages (one k-step, 64
// MFMAs per wave) held in NS slots of 32 KiB (A and W images of [256 rows][64 B]), NS - 1 of them
// in flight: with NS = 5 the whole 160 KiB of LDS, 128 KiB of operands on their way per CU and
// 4 k-steps (4,096 MFMA cycles) for each DMA to land, against one K-tile (64 KiB, 2,048 cycles)
// in tnw.  Iteration s: retire stage s (counted vmcnt: the 8 (NS - 2) younger pieces stay in
// flight) + barrier; DMA stage s + NS - 1 into the slot stage s - 1 vacated; read stage s's
// fragments while the MFMAs of stage s - 1 run.  64-byte image rows: the 16-byte chunk c of row
// r sits at c ^ f(r), f(r) = (2 (r >> 3) ^ (r >> 4)) & 3 -- conflict-free for both fragment
// patterns under ds_read_b128's lane groups (searched by script).
// LN = true: the inter-layer LayerNorm folded in (tnw32_kernel<4, true>, sc_gemm_tn_ln_bf16):
// A = the previous layer's RAW bf16 output h, B = W'' (ln_fold.hip), and
//   C = rstd (h W''^T - mean r) = LN(h) W^T - W beta   (b' = b + W beta goes into the scan's bias)
// Each thread owns one tile row: while its 32-column stages pass through LDS it reads the row's
// 4 chunks beside the fragment reads and accumulates shifted sums (shift = the row's first
// element) in VALU slots between the MFMAs; after the K loop the (rstd, mean) of the 256 rows go
// to LDS (and, from the first column tile, to stat[] for the backward) and the epilogue applies
// them with r (DMA'd into LDS in the prologue).  Every column tile of a row panel computes the
// same statistics from the same data in the same order: bitwise equal across tiles.
struct TnLn {
  const float* r;   // [N] row sums of the W'' image, image row (= output column) order
  float2* stat;     // [M] out: (rstd, mean) per row (written by the tiles of column 0)
  float eps;
};

namespace tnw32 {
constexpr int kRow = 64;                 // image row pitch (bytes): 32 bf16
constexpr int kHalf = 256 * kRow;        // one operand image (16 KiB)
constexpr int kSlot = 2 * kHalf;         // A + W (32 KiB)
__device__ __forceinline__ int f64(int r) { return ((2 * (r >> 3)) ^ (r >> 4)) & 3; }
}  // namespace tnw32

template <int NS, bool LN>
__global__ void __launch_bounds__(256, 1) tnw32_kernel(TnArgs a, TnLn ln) {
  using namespace tnw32;
  using tnw::Frag;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int l15 = lane & 15, l4 = lane >> 4;
  const int bid = blockIdx.x;
  const int npan = (a.M + 255) / 256;
  const int xcd = bid % 8, k = bid / 8;
  const int pq = npan / 8, pr = npan % 8;
  const int np = pq + (xcd < pr), p0 = xcd * pq + min(xcd, pr);
  if (k >= np * a.ntn) return;
  const int grp = k / (a.gm * a.ntn), first = grp * a.gm;
  const int gsz = min(a.gm, np - first), within = k - grp * a.gm * a.ntn;
  const int m0 = (p0 + first + within % gsz) * 256, n0 = (within / gsz) * 256;
  const int nst = a.K / 32;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA: wave w stages image rows 64 w .. 64 w + 63 of both operands (4 + 4 pieces of 16 rows) ----
  uint32_t voA[4], voB[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 64 * w + 16 * q + (lane >> 2);
    const uint32_t ch = 8u * (uint32_t)((lane & 3) ^ f64(r));
    voA[q] = ((uint32_t)min(m0 + r, a.M - 1) * a.lda + ch) * 2u;
    voB[q] = ((uint32_t)(n0 + r) * a.ldb + ch) * 2u;
  }
  auto dma = [&](int st) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((st % NS) * kSlot) + (uint32_t)(w * 4 * 1024);
    const __bf16* pa = a.A + st * 32;
    const __bf16* pb = a.B + st * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q) dma_to_lds_s<16>(pa, voA[q], sb + q * 1024);
#pragma unroll
    for (int q = 0; q < 4; ++q) dma_to_lds_s<16>(pb, voB[q], sb + kHalf + q * 1024);
  };
  uint32_t offX[8], offW[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    const int rx = wm * 128 + f * 16 + l15;
    offX[f] = (uint32_t)(rx * kRow + 16 * (l4 ^ f64(rx)));
    const int rw = wn * 128 + (l15 >> 2) * 32 + f * 4 + (l15 & 3);
    offW[f] = (uint32_t)(kHalf + rw * kRow + 16 * (l4 ^ f64(rw)));
  }
  auto read = [&](int st, Frag& fx, Frag& fw) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((st % NS) * kSlot);
#pragma unroll
    for (int f = 0; f < 8; ++f) fw.v[f] = lds_read16(sb + offW[f]);
#pragma unroll
    for (int f = 0; f < 8; ++f) fx.v[f] = lds_read16(sb + offX[f]);
  };
  f4v acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](const Frag& fx, const Frag& fw) __attribute__((always_inline)) {
    if (SC_TN_ABL & 1) {
#pragma unroll
      for (int f = 0; f < 8; ++f) asm volatile("" ::"v"(fx.v[f]), "v"(fw.v[f]));
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(b8v, fw.v[j]), __builtin_bit_cast(b8v, fx.v[i]), acc[i][j], 0, 0, 0);
  };
  // retire stage st: the pieces of the stages issued after it (up to NS - 2) may stay in flight
  auto retire = [&](int st) __attribute__((always_inline)) {
    const int younger = min(NS - 2, nst - 1 - st);
    if (younger >= NS - 2) dma_wait_younger<8 * (NS - 2)>();
    else if (younger == 2) dma_wait_younger<16>();
    else if (younger == 1) dma_wait_younger<8>();
    else dma_wait();
  };
  // ---- LN: r of the tile's 256 columns into LDS (older than every stage: the first wait
  // retires it), the row statistics of thread t's tile row ----
  constexpr uint32_t kR = (uint32_t)NS * kSlot, kStat = kR + 1024;
  const int t = threadIdx.x;
  float lsh = 0.f, ls1a = 0.f, ls1b = 0.f, ls2a = 0.f, ls2b = 0.f;
  const uint32_t statoff = (uint32_t)(t * kRow + 16 * f64(t));   // chunk c at statoff ^ 16 c
  if constexpr (LN) {
    if (w == 0) dma_to_lds_s<16>(ln.r + n0, (uint32_t)lane * 16u, lds0 + kR);
  }
  auto stat_read = [&](int st, i4v (&rv)[4]) __attribute__((always_inline)) {
    if constexpr (LN) {
      const uint32_t sb = lds0 + (uint32_t)((st % NS) * kSlot);
#pragma unroll
      for (int c = 0; c < 4; ++c) rv[c] = lds_read16(sb + (statoff ^ (16u * c)));
    }
  };
  auto stat_acc = [&](int st, const i4v (&rv)[4]) __attribute__((always_inline)) {
    if constexpr (LN) {
      if (st == 0) lsh = __uint_as_float((uint32_t)rv[0][0] << 16);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t u = (uint32_t)rv[c][d];
          const float x0 = __uint_as_float(u << 16) - lsh, x1 = __uint_as_float(u & 0xffff0000u) - lsh;
          ls1a += x0;
          ls1b += x1;
          ls2a = fmaf(x0, x0, ls2a);
          ls2b = fmaf(x1, x1, ls2b);
        }
    }
  };
  i4v sv[4];
  // ---- prologue: stages 0 .. NS - 1 in flight (every slot), stage 0 retired and read ----
#pragma unroll
  for (int st = 0; st < NS; ++st)
    if (st < nst) dma(st);
  if (nst >= NS) dma_wait_younger<8 * (NS - 1)>();
  else retire(0);
  lds_barrier();
  Frag X, Xw, Y, Yw;
  read(0, X, Xw);
  stat_read(0, sv);
  stat_acc(0, sv);
  // stage s is read after the barrier that retires it and multiplied one barrier later; at that
  // barrier every read of stage s - 1 is done, so its slot takes stage s - 1 + NS
  // LN: the reads of the next stage and the MFMAs of the current one stay in one basic block, so
  // that SC_TNW_IL can interleave them: the last pair is peeled instead of guarded.  Plain: the
  // guarded loop (the peeled form spills in the plain instances)
  if constexpr (!LN) {
    for (int st = 0; st < nst; st += 2) {
      tnw::frag_wait();
      retire(st + 1);
      lds_barrier();
      if (st + NS < nst && !(SC_TN_ABL & 2)) dma(st + NS);
      read(st + 1, Y, Yw);
      mfmas(X, Xw);
      tnw::frag_wait();
      if (st + 2 < nst) {
        retire(st + 2);
        lds_barrier();
        if (st + 1 + NS < nst && !(SC_TN_ABL & 2)) dma(st + 1 + NS);
        read(st + 2, X, Xw);
      }
      mfmas(Y, Yw);
    }
  }
  for (int st = 0; LN && st + 2 < nst; st += 2) {   // nst = K / 32 is even
    tnw::frag_wait();
    retire(st + 1);
    lds_barrier();
    if (st + NS < nst && !(SC_TN_ABL & 2)) dma(st + NS);
    read(st + 1, Y, Yw);
    stat_read(st + 1, sv);
    mfmas(X, Xw);
    tnw::interleave<LN ? 20 : 16>();
    stat_acc(st + 1, sv);
    tnw::frag_wait();
    retire(st + 2);
    lds_barrier();
    if (st + 1 + NS < nst && !(SC_TN_ABL & 2)) dma(st + 1 + NS);
    read(st + 2, X, Xw);
    stat_read(st + 2, sv);
    mfmas(Y, Yw);
    tnw::interleave<LN ? 20 : 16>();
    stat_acc(st + 2, sv);
  }
  if constexpr (LN) {   // the last pair of stages (nst - 2, nst - 1): nothing left to DMA
    tnw::frag_wait();
    retire(nst - 1);
    lds_barrier();
    read(nst - 1, Y, Yw);
    stat_read(nst - 1, sv);
    mfmas(X, Xw);
    tnw::interleave<LN ? 20 : 16>();
    stat_acc(nst - 1, sv);
    tnw::frag_wait();
    mfmas(Y, Yw);
  }
  if (SC_TN_ABL & 4) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"a"(acc[i][j]));
    return;
  }
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.cbytes, 0x00020000);
  const uint32_t col = (uint32_t)(n0 + wn * 128 + l4 * 32);
  float rr[32];   // (LN) r of the lane's 32 columns
  if constexpr (LN) {
    // row statistics (biased variance, nn.LayerNorm) -> LDS and, from column tile 0, stat[]
    const float inv = 1.0f / (float)a.K;
    const float m1 = (ls1a + ls1b) * inv;
    const float var = fmaxf((ls2a + ls2b) * inv - m1 * m1, 0.0f);
    const float2 sr = make_float2(rsq(var + ln.eps), lsh + m1);
    typedef float f2 __attribute__((ext_vector_type(2)));
    *(__attribute__((address_space(3))) f2*)(size_t)(lds0 + kStat + (uint32_t)t * 8u) = f2{sr.x, sr.y};
    if (n0 == 0 && m0 + t < a.M) ln.stat[m0 + t] = sr;
    lds_barrier();
    const uint32_t rb = lds0 + kR + (uint32_t)(wn * 128 + l4 * 32) * 4u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const i4v v = lds_read16(rb + 16u * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) rr[4 * q + e] = __int_as_float(v[e]);
    }
  }
  // SC_TNW_EPI: the wave's 128 x 128 bf16 block goes through LDS (its own 32 KiB of the ring,
  // 16-byte chunk c of block row r at c ^ (r & 15)) and leaves as 32 stores of 4 whole 256-byte
  // row segments each, instead of 32 stores of 64 scattered 16-byte pieces (a lane's 32 columns
  // of one row): the store tail is issue-bound on pieces, not bytes (MI355X_MICROARCH.md)
  const uint32_t blk = lds0 + (uint32_t)w * 32768u;
  if (SC_TNW_EPI && !LN) lds_barrier();   // every wave's last fragment reads of the ring are done
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t row = (uint32_t)(m0 + wm * 128 + i * 16 + l15);
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 sr = {1.f, 0.f};
    if constexpr (LN)
      sr = *(const __attribute__((address_space(3))) f2*)(size_t)(
          lds0 + kStat + (uint32_t)(wm * 128 + i * 16 + l15) * 8u);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      i4v v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int j = 2 * s4 + (d >> 1), e = 2 * (d & 1);
        float c0 = acc[i][j][e], c1 = acc[i][j][e + 1];
        if constexpr (LN) {   // rstd (u - mean r), column j*4 + e of the lane's 32
          c0 = (c0 - sr.y * rr[4 * j + e]) * sr.x;
          c1 = (c1 - sr.y * rr[4 * j + e + 1]) * sr.x;
        }
        const b2v p = {(__bf16)c0, (__bf16)c1};
        v[d] = __builtin_bit_cast(int, p);
      }
      if (SC_TNW_EPI) {
        const uint32_t rl = (uint32_t)(i * 16 + l15), c = (uint32_t)(l4 * 4 + s4);
        *(__attribute__((address_space(3))) i4v*)(size_t)(blk + rl * 256u + 16u * (c ^ (rl & 15u))) = v;
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(v, crs, (row * a.ldc + col + 8u * s4) * 2u, 0, 0);
      }
    }
  }
  if (SC_TNW_EPI) {
    lds_read_wait();   // (the wave reads back only its own block)
    const uint32_t ch = (uint32_t)(lane & 15);
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const uint32_t rl = (uint32_t)(4 * it + (lane >> 4));
      const i4v v = lds_read16(blk + rl * 256u + 16u * (ch ^ (rl & 15u)));
      const uint32_t row = (uint32_t)(m0 + wm * 128) + rl;
      __builtin_amdgcn_raw_buffer_store_b128(
          v, crs, (row * a.ldc + (uint32_t)(n0 + wn * 128) + 8u * ch) * 2u, 0, 0);
    }
  }
}

template <int NS, bool LN>
int launch_tnw32(const TnArgs& a, const TnLn& ln, hipStream_t st) {
  constexpr size_t lds = (size_t)NS * tnw32::kSlot + (LN ? 3072 : 0);
  static_assert(!LN || lds <= 160 * 1024, "LN needs a spare 3 KiB of LDS");
  static const bool ok = hipFuncSetAttribute((const void*)tnw32_kernel<NS, LN>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  const int npan = (a.M + 255) / 256;
  const int grid = 8 * ((npan + 7) / 8) * a.ntn;
  hipLaunchKernelGGL((tnw32_kernel<NS, LN>), dim3(grid), dim3(256), lds, st, a, ln);
  return 0;
}

// ------------------------------------------------------------------------------------------
// tnw32 with REGISTER staging instead of LDS-DMA: tnr_kernel<LN>.
// MI355X_MICROARCH.md prices one LDS-DMA piece at 100-185 issue cycles inside a phase that also
// carries 16 ds_read_b128 -- tnw32's exact phase: 8 pieces per wave per 32-deep k-step cost about
// as much issue time as the k-step's 64 MFMAs (1,024 cycles), the measured 2x.  Here each wave
// global-loads its 8 16-byte pieces of stage s + 4 into VGPRs (buffer_load_dwordx4; two staging
// sets, 64 VGPRs, two k-steps of latency cover) and ds_writes stage s + 2 from the other set into
// the LDS slot stage s vacated (two 32 KiB slots).  Per k-step s:
//   read stage s + 1's fragments (other register set) | 16 MFMAs of stage s | ds_write stage
//   s + 2, global-load stage s + 4 | 48 MFMAs | one barrier (slot s + 2 written by every wave,
//   slot s + 1 read by every wave).
// LDS images, swizzle, fragment reads, the LN statistics and the epilogue are tnw32's.
// Measured (r6r, profiles/r6_tnw.md): 321-329 us plain at the gate forward, no faster than the
// LDS-DMA tnw32, so the operand path is not what holds these kernels at 2x the library; built
// only in A/B libraries (SC_TNR=1).
#ifndef SC_TNR
#define SC_TNR 0
#endif
#if SC_TNR
template <bool LN>
__global__ void __launch_bounds__(256, 1) tnr_kernel(TnArgs a, TnLn ln) {
  using namespace tnw32;
  using tnw::Frag;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int l15 = lane & 15, l4 = lane >> 4;
  const int bid = blockIdx.x;
  const int npan = (a.M + 255) / 256;
  const int xcd = bid % 8, k = bid / 8;
  const int pq = npan / 8, pr = npan % 8;
  const int np = pq + (xcd < pr), p0 = xcd * pq + min(xcd, pr);
  if (k >= np * a.ntn) return;
  const int grp = k / (a.gm * a.ntn), first = grp * a.gm;
  const int gsz = min(a.gm, np - first), within = k - grp * a.gm * a.ntn;
  const int m0 = (p0 + first + within % gsz) * 256, n0 = (within / gsz) * 256;
  const int nst = a.K / 32;   // even, >= 2 (the host requires K % 64 == 0)
  const uint32_t lds0 = lds_addr(lds);

  // ---- staging: wave w loads image rows 64 w .. 64 w + 63 of both operands (4 + 4 pieces of 16
  // rows x 64 B), chunk (lane & 3) ^ f64(row) of its row, and ds_writes it lane-linearly ----
  // piece q's rows are 16 q further on.  A rows past M are clamped to row M - 1 (the buffer
  // range check covers the VGPR offset only, so a row offset in soffset would escape it): one
  // lane offset per piece.  B rows never pass N (N % 256 == 0): one lane offset, the row step
  // in soffset.
  const int r0 = 64 * w + (lane >> 2);
  uint32_t voA[4], chq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    chq[q] = 16u * (uint32_t)((lane & 3) ^ f64(r0 + 16 * q));
    voA[q] = (uint32_t)min(m0 + r0 + 16 * q, a.M - 1) * a.lda * 2u + chq[q];
  }
  const uint32_t voB0 = ((uint32_t)(n0 + r0) * a.ldb) * 2u;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)(a.M * a.lda * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, (int)((uint32_t)a.N * a.ldb * 2u), 0x00020000);
  struct Stg { i4v a[4], b[4]; };
  auto gload = [&](int st, Stg& g) __attribute__((always_inline)) {
    const uint32_t so = (uint32_t)st * 64u;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      g.a[q] = __builtin_amdgcn_raw_buffer_load_b128(ra, voA[q], so, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      g.b[q] = __builtin_amdgcn_raw_buffer_load_b128(rb, voB0 + chq[q], so + 32u * q * a.ldb, 0);
  };
  const uint32_t wlane = (uint32_t)(w * 4 * 1024 + lane * 16);
  auto dswrite = [&](int st, const Stg& g) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((st & 1) * kSlot) + wlane;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *(__attribute__((address_space(3))) i4v*)(size_t)(sb + q * 1024) = g.a[q];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *(__attribute__((address_space(3))) i4v*)(size_t)(sb + kHalf + q * 1024) = g.b[q];
  };
  // fragment f's offset = (base ^ 16 g(f)) + f * stride: the swizzle touches only address bits
  // 4-5, so four lane registers per operand cover the 8 fragments (the rest is the immediate)
  //   x rows wm 128 + 16 f + l15:            g(f) = f & 3,                        stride 1024
  //   W rows wn 128 + 32 (l15 >> 2) + 4 f + (l15 & 3): g(f) = 2 ((f >> 1) & 1) ^ (f >> 2), stride 256
  uint32_t ox4[4], ow4[4];
  {
    const uint32_t bx = (uint32_t)((wm * 128 + l15) * kRow + 16 * ((l4 ^ (2 * ((l15 >> 3) & 1))) & 3));
    const int rw0 = wn * 128 + (l15 >> 2) * 32 + (l15 & 3);
    const uint32_t bw = (uint32_t)(kHalf + rw0 * kRow + 16 * ((l4 ^ (2 * ((l15 >> 2) & 1))) & 3));
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      ox4[g] = bx ^ (16u * g);
      ow4[g] = bw ^ (16u * g);
    }
  }
  auto read = [&](int st, Frag& fx, Frag& fw) __attribute__((always_inline)) {
    const uint32_t sb = lds0 + (uint32_t)((st & 1) * kSlot);
#pragma unroll
    for (int f = 0; f < 8; ++f) fw.v[f] = lds_read16(sb + ow4[(2 * ((f >> 1) & 1)) ^ (f >> 2)] + 256u * f);
#pragma unroll
    for (int f = 0; f < 8; ++f) fx.v[f] = lds_read16(sb + ox4[f & 3] + 1024u * f);
  };
  f4v acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  // MFMAs of x fragments i0 .. i1 - 1 against the stage's 8 W fragments
  auto mfmas = [&](const Frag& fx, const Frag& fw, int i0, int i1) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < i0 || i >= i1) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(b8v, fw.v[j]), __builtin_bit_cast(b8v, fx.v[i]), acc[i][j], 0, 0, 0);
    }
  };
  // ---- LN: r into LDS, the row statistics of thread t's tile row (as tnw32) ----
  constexpr uint32_t kR = 2u * kSlot, kStat = kR + 1024;
  const int t = threadIdx.x;
  float lsh = 0.f, ls1a = 0.f, ls1b = 0.f, ls2a = 0.f, ls2b = 0.f;
  const uint32_t statoff = (uint32_t)(t * kRow + 16 * f64(t));
  if constexpr (LN) {
    if (w == 0) {
      const i4v rv = __builtin_amdgcn_raw_buffer_load_b128(
          __builtin_amdgcn_make_buffer_rsrc((void*)ln.r, 0, (int)(a.N * 4), 0x00020000),
          (uint32_t)(n0 + 4 * lane) * 4u, 0, 0);
      *(__attribute__((address_space(3))) i4v*)(size_t)(lds0 + kR + (uint32_t)lane * 16u) = rv;
    }
  }
  auto stat_read = [&](int st, i4v (&rv)[4]) __attribute__((always_inline)) {
    if constexpr (LN) {
      const uint32_t sb = lds0 + (uint32_t)((st & 1) * kSlot);
#pragma unroll
      for (int c = 0; c < 4; ++c) rv[c] = lds_read16(sb + (statoff ^ (16u * c)));
    }
  };
  auto stat_acc = [&](int st, const i4v (&rv)[4]) __attribute__((always_inline)) {
    if constexpr (LN) {
      if (st == 0) lsh = __uint_as_float((uint32_t)rv[0][0] << 16);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t u = (uint32_t)rv[c][d];
          const float x0 = __uint_as_float(u << 16) - lsh, x1 = __uint_as_float(u & 0xffff0000u) - lsh;
          ls1a += x0;
          ls1b += x1;
          ls2a = fmaf(x0, x0, ls2a);
          ls2b = fmaf(x1, x1, ls2b);
        }
    }
  };
  i4v sv[4];
  Stg S0, S1;
  Frag X, Xw, Y, Yw;
  // ---- prologue: stages 0 and 1 into LDS, 2 and 3 on their way ----
  gload(0, S0);
  gload(1, S1);
  dswrite(0, S0);
  if (2 < nst) gload(2, S0);
  dswrite(1, S1);
  if (3 < nst) gload(3, S1);
  lds_barrier();
  read(0, X, Xw);
  stat_read(0, sv);
  stat_acc(0, sv);
  // ---- k-step s: MFMAs on stage s (F), stage s + 1's fragments read into N, stage s + 2
  // written from staging set G (loaded two k-steps ago), stage s + 4 loaded into G ----
  auto step = [&](int s, Frag& F, Frag& Fw, Frag& N, Frag& Nw, Stg& G) __attribute__((always_inline)) {
    if (s + 1 < nst) {
      read(s + 1, N, Nw);
      stat_read(s + 1, sv);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(F, Fw, 0, 2);
    if (s + 1 < nst) stat_acc(s + 1, sv);
    __builtin_amdgcn_sched_barrier(0);
    if (s + 2 < nst) dswrite(s + 2, G);
    if (s + 4 < nst) gload(s + 4, G);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(F, Fw, 2, 8);
    lds_barrier();
  };
  for (int s = 0; s < nst; s += 2) {
    step(s, X, Xw, Y, Yw, S0);
    step(s + 1, Y, Yw, X, Xw, S1);
  }
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.cbytes, 0x00020000);
  const uint32_t col = (uint32_t)(n0 + wn * 128 + l4 * 32);
  float rr[32];
  if constexpr (LN) {
    const float inv = 1.0f / (float)a.K;
    const float m1 = (ls1a + ls1b) * inv;
    const float var = fmaxf((ls2a + ls2b) * inv - m1 * m1, 0.0f);
    const float2 sr = make_float2(rsq(var + ln.eps), lsh + m1);
    typedef float f2 __attribute__((ext_vector_type(2)));
    *(__attribute__((address_space(3))) f2*)(size_t)(lds0 + kStat + (uint32_t)t * 8u) = f2{sr.x, sr.y};
    if (n0 == 0 && m0 + t < a.M) ln.stat[m0 + t] = sr;
    lds_barrier();
    const uint32_t rb2 = lds0 + kR + (uint32_t)(wn * 128 + l4 * 32) * 4u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const i4v v = lds_read16(rb2 + 16u * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) rr[4 * q + e] = __int_as_float(v[e]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t row = (uint32_t)(m0 + wm * 128 + i * 16 + l15);
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 sr = {1.f, 0.f};
    if constexpr (LN)
      sr = *(const __attribute__((address_space(3))) f2*)(size_t)(
          lds0 + kStat + (uint32_t)(wm * 128 + i * 16 + l15) * 8u);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      i4v v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int j = 2 * s4 + (d >> 1), e = 2 * (d & 1);
        float c0 = acc[i][j][e], c1 = acc[i][j][e + 1];
        if constexpr (LN) {
          c0 = (c0 - sr.y * rr[4 * j + e]) * sr.x;
          c1 = (c1 - sr.y * rr[4 * j + e + 1]) * sr.x;
        }
        const b2v p = {(__bf16)c0, (__bf16)c1};
        v[d] = __builtin_bit_cast(int, p);
      }
      __builtin_amdgcn_raw_buffer_store_b128(v, crs, (row * a.ldc + col + 8u * s4) * 2u, 0, 0);
    }
  }
}

template <bool LN>
int launch_tnr(const TnArgs& a, const TnLn& ln, hipStream_t st) {
  constexpr size_t lds = 2 * (size_t)tnw32::kSlot + (LN ? 3072 : 0);
  static const bool ok = hipFuncSetAttribute((const void*)tnr_kernel<LN>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  const int npan = (a.M + 255) / 256;
  const int grid = 8 * ((npan + 7) / 8) * a.ntn;
  hipLaunchKernelGGL((tnr_kernel<LN>), dim3(grid), dim3(256), lds, st, a, ln);
  return 0;
}
#endif  // SC_TNR

int launch_tn256(const TnArgs& a, hipStream_t st) {
  constexpr size_t lds = 2 * 4 * (size_t)kHalfB;   // 128 KiB
  static const bool ok = hipFuncSetAttribute((const void*)tn256_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  const int grid = a.tiles < 256 ? a.tiles : 256;
  hipLaunchKernelGGL(tn256_kernel, dim3(grid), dim3(512), lds, st, a);
  return 0;
}

int launch_tnpp(const TnArgs& a, hipStream_t st) {
  constexpr size_t lds = 2 * 4 * (size_t)kHalfB;   // 128 KiB
  static const bool ok = hipFuncSetAttribute((const void*)tnpp_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  const int grid = a.tiles < 256 ? a.tiles : 256;
  hipLaunchKernelGGL(tnpp_kernel, dim3(grid), dim3(512), lds, st, a);
  return 0;
}

template <int MF, int SPI>
int launch_tn(const TnArgs& a, hipStream_t st) {
  auto kern = tn_kernel<MF, SPI>;
  constexpr size_t lds = (size_t)kSlots * (32 * MF + kTN) * kRowB;
  static const bool ok = hipFuncSetAttribute((const void*)kern,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
  (void)ok;
  const int grid = a.tiles < 256 ? a.tiles : 256;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, a);
  return 0;
}

}  // namespace
}  // namespace sc

using namespace sc;

extern "C" int sc_gemm_tn_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                               int64_t ldc, int M, int N, int K, int tile_m, void* stream) {
  clear_error();
  SC_REQUIRE(A && B && C, "sc_gemm_tn_bf16: null pointer");
  SC_REQUIRE(M > 0 && N > 0 && K > 0, "sc_gemm_tn_bf16: empty shape M=%d N=%d K=%d", M, N, K);
  SC_REQUIRE(K % kBK == 0, "sc_gemm_tn_bf16: K=%d must be a multiple of 64 (zero-pad it)", K);
  SC_REQUIRE(N % kTN == 0, "sc_gemm_tn_bf16: N=%d must be a multiple of 256", N);
  SC_REQUIRE(tile_m == 0 || (SC_TNW_AB && tile_m >= 1 && tile_m <= 3) || tile_m == 128 ||
                 tile_m == 192 || tile_m == 256 || tile_m == 257,
             "sc_gemm_tn_bf16: tile_m=%d must be 0 (default 192), 128, 192, 256 or 257 (256, "
             "ping-pong schedule); 1 / 2 / 3 (one wave per SIMD) in SC_TNW_AB builds only",
             tile_m);
  SC_REQUIRE(lda >= K && ldb >= K && ldc >= N && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0,
             "sc_gemm_tn_bf16: leading dimensions must cover the rows in 16-byte pieces");
  SC_REQUIRE((uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0 && (uintptr_t)C % 16 == 0,
             "sc_gemm_tn_bf16: operands must be 16-byte aligned");
  SC_REQUIRE((int64_t)M * lda * 2 < (1ll << 32) && (int64_t)N * ldb * 2 < (1ll << 32) &&
                 ((int64_t)M + 256) * ldc * 2 < (1ll << 32),
             "sc_gemm_tn_bf16: operands must be smaller than 4 GiB");
  const int tm = (tile_m == 257 || (tile_m >= 1 && tile_m <= 3)) ? 256 : tile_m ? tile_m : 192;
  const int ntn = N / kTN;
  const int64_t tiles = (int64_t)((M + tm - 1) / tm) * ntn;
  SC_REQUIRE(tiles < (1 << 30), "sc_gemm_tn_bf16: too many tiles");
  static const int gm = [] {
    const char* e = getenv("SC_TN_GM");
    const int v = e ? atoi(e) : 8;
    return v >= 1 ? v : 8;
  }();
  TnArgs a{(const __bf16*)A, (const __bf16*)B, (__bf16*)C, M, N, K, ntn, (int)tiles,
           (uint32_t)lda, (uint32_t)ldb, (uint32_t)ldc, (uint32_t)((int64_t)M * ldc * 2), gm};
  hipStream_t st = (hipStream_t)stream;
#if SC_TNW_AB
  if (tile_m == 1) {
    launch_tnw(a, st);
    return launch_status("sc_gemm_tn_bf16");
  }
  if (tile_m == 2 || tile_m == 3) {
#if SC_TNR
    launch_tnr<false>(a, TnLn{}, st);
#else
    if (tile_m == 2) launch_tnw32<5, false>(a, TnLn{}, st);
    else launch_tnw32<4, false>(a, TnLn{}, st);
#endif
    return launch_status("sc_gemm_tn_bf16");
  }
#endif
  if (tile_m == 257) {
    launch_tnpp(a, st);
    return launch_status("sc_gemm_tn_bf16");
  }
  if (tm == 256) {
    launch_tn256(a, st);
    return launch_status("sc_gemm_tn_bf16");
  }
  // stores per stage: a tile's 2 MF stores must be issued within the next tile's K / 64 stages
  const int nks = K / kBK, nst = 2 * (tm / 32);
  const int spi = (nst + nks - 1) / nks;
  if (tm == 128) {
    if (spi <= 1) launch_tn<4, 1>(a, st);
    else if (spi <= 2) launch_tn<4, 2>(a, st);
    else if (spi <= 4) launch_tn<4, 4>(a, st);
    else launch_tn<4, 8>(a, st);
  } else {
    if (spi <= 1) launch_tn<6, 1>(a, st);
    else if (spi <= 2) launch_tn<6, 2>(a, st);
    else if (spi <= 4) launch_tn<6, 4>(a, st);
    else if (spi <= 6) launch_tn<6, 6>(a, st);
    else launch_tn<6, 12>(a, st);
  }
  return launch_status("sc_gemm_tn_bf16");
}

extern "C" int sc_gemm_tn_ln_bf16(const void* H, int64_t ldh, const void* Wpp, int64_t ldw, void* C,
                                  int64_t ldc, int M, int N, int K, const float* r, void* stat,
                                  float eps, void* stream) {
  clear_error();
  SC_REQUIRE(H && Wpp && C && r && stat, "sc_gemm_tn_ln_bf16: null pointer");
  SC_REQUIRE(M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 256 == 0,
             "sc_gemm_tn_ln_bf16: shape M=%d N=%d K=%d (K %% 64, N %% 256)", M, N, K);
  SC_REQUIRE(ldh >= K && ldw >= K && ldc >= N && ldh % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0,
             "sc_gemm_tn_ln_bf16: leading dimensions must cover the rows in 16-byte pieces");
  SC_REQUIRE(((uintptr_t)H | (uintptr_t)Wpp | (uintptr_t)C | (uintptr_t)r) % 16 == 0 &&
                 (uintptr_t)stat % 8 == 0,
             "sc_gemm_tn_ln_bf16: misaligned operand");
  SC_REQUIRE((int64_t)M * ldh * 2 < (1ll << 32) && (int64_t)N * ldw * 2 < (1ll << 32) &&
                 ((int64_t)M + 256) * ldc * 2 < (1ll << 32),
             "sc_gemm_tn_ln_bf16: operands must be smaller than 4 GiB");
  const int ntn = N / 256;
  const int64_t tiles = (int64_t)((M + 255) / 256) * ntn;
  TnArgs a{(const __bf16*)H, (const __bf16*)Wpp, (__bf16*)C, M, N, K, ntn, (int)tiles,
           (uint32_t)ldh, (uint32_t)ldw, (uint32_t)ldc, (uint32_t)((int64_t)M * ldc * 2), 8};
#if SC_TNR
  launch_tnr<true>(a, TnLn{r, (float2*)stat, eps}, (hipStream_t)stream);
#else
  launch_tnw32<4, true>(a, TnLn{r, (float2*)stat, eps}, (hipStream_t)stream);
#endif
  return launch_status("sc_gemm_tn_ln_bf16");
}
