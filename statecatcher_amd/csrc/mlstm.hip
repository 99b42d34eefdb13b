// mLSTM (xLSTM matrix-memory) cell for gfx950: chunkwise forward and backward on MFMA.
//
// The reference's xLSTM encoder (model.py:214-229, :301-307, C4) runs the fork's mlstm_kernels
// chunkwise kernels; the math restated here is the published mLSTM recurrence in the chunkwise
// form of transformers/models/xlstm/modeling_xlstm.py:74-386 (per batch row b and head h,
// chunk length L = 64, qk scale s = DQ^-1/2):
//   b_t = sum_{r<=t in chunk} logsig(f_r),  g = b_{L-1},  stabiliser m_k of the state C~_k
//   state:  m_{k+1} = max(g + m_k, max_s a_s),  a_s = g - b_s + i_s
//           C~_{k+1} = e^{g + m_k - m_{k+1}} C~_k + sum_s e^{a_s - m_{k+1}} k_s v_s^T   (n~ same, k_s)
//   output: m_t = max(b_t + m_k, max_{s<=t} (b_t - b_s + i_s)),  W_ts = s e^{b_t - b_s + i_s - m_t}
//           num_t = sum_{s<=t} W_ts (q_t.k_s) v_s + s e^{b_t + m_k - m_t} q_t C~_k
//           den_t = sum_{s<=t} W_ts (q_t.k_s)     + s e^{b_t + m_k - m_t} q_t.n~_k
//           h_t = num_t / (max(|den_t|, e^{-m_t}) + eps)
// Kernels (16x16x32 bf16/f16 MFMA, fp32 accumulation, fp32 state):
//   mlstm_fw_walk per (b,h, 64-column block of C~), 4 waves: walks the chunks in order with the
//                state block in MFMA accumulators; per chunk S = Q K^T, causal decay mask,
//                H[:, block] = M V[:, block] + Q~ C~_k[:, block], normaliser (S and the
//                normaliser recomputed per block), then the state update.  Keeps m_t, den_t and
//                the compute-dtype image of every chunk-start state for the backward.
//   mlstm_bw_walk per (b,h), 8 waves, two roles: a walk through the chunks in reverse with dC~ in
//                MFMA accumulators, computing dk and dv on the way (intra-chunk terms through
//                A / dA = W o (dnum V^T + dden), inter-chunk terms through dC~_{k+1}), and beside
//                it a workgroup computing dq of every chunk from the forward's C~_k (no carry).
// The stabiliser m is treated as a constant in the backward (it cancels in h up to the eps
// term), as the chunkwise kernels of the mlstm_kernels family do.  Gate gradients follow from
// the pair identities  di_s = k_s.dk_s  and  dF_t = q_t.dq_t - k_t.dk_t  (F = cumulative
// logsig(f)): the kernels emit the two dot products, the host turns dF into df by a reverse
// cumulative sum times sigmoid(-f).
#include <cstdlib>
#include <initializer_list>

#include "sc_common.h"

// SC_ML_ABL: timing ablations (tools/mlstm_abl.sh; results are garbage).  Forward walk: 1 no S
// MFMAs, 2 no H MFMAs, 4 no state-update MFMAs, 8 no global stores, 16 no LDS fill.  Backward
// walk: 32 no A/dA phase, 64 no dq phase, 128 no dk/dv phase, 256 no dC update, 512 no loads,
// 1024 no dq role (its workgroups exit), 2048 no walk role; per-operand loads of the backward
// (both roles, for FETCH_SIZE differences): 4096 q, 8192 k, 16384 v, 32768 dh, 65536 h,
// 131072 the dq role's state image; 262144 no dq / dk / dv stores.
#ifndef SC_ML_ABL
#define SC_ML_ABL 0
#endif
#ifndef SC_ML_XCDH
#define SC_ML_XCDH 1
#endif
#define ML_ABL(b) ((SC_ML_ABL & (b)) != 0)

namespace sc {

namespace {

constexpr int kL = 64;    // chunk length
constexpr int kPad = 8;   // LDS row padding (elements): 16 bytes, breaks bank conflicts

typedef float f32x4 __attribute__((ext_vector_type(4)));
// 16-byte register piece (a native vector: HIP's u32x4 class defeats scalar replacement of
// register arrays, which then live in scratch)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int DT> struct MF;
template <> struct MF<SC_BF16> {
  using T = __bf16;
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MF<SC_F16> {
  using T = _Float16;
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

// 8 packed 16-bit elements of dtype IO as the compute type's fragment (a no-op when equal):
// the f16 cell reads the bf16 projection in place, rounding as a .to(float16) would
// an fp32 result stored as IO through the compute dtype's rounding first (f16 cell on bf16
// operands: the value leaves the cell as f16 and is then cast, as the split path's
// h.to(bfloat16) and autograd's gradient cast do; a no-op round trip when IO == DT)
template <int DT, int IO>
__device__ __forceinline__ typename MF<IO>::T out16(float x) {
  return (typename MF<IO>::T)(float)(typename MF<DT>::T)x;
}
template <int DT, int IO>
__device__ __forceinline__ typename MF<DT>::v8 cvt8(u32x4 x) {
  if constexpr (DT == IO) {
    return __builtin_bit_cast(typename MF<DT>::v8, x);
  } else {
    const typename MF<IO>::v8 y = __builtin_bit_cast(typename MF<IO>::v8, x);
    typename MF<DT>::v8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = (typename MF<DT>::T)(float)y[e];
    return r;
  }
}

struct MArgs {
  const void* q;   // [BH][T][DQ]
  const void* k;   // [BH][T][DQ]
  const void* v;   // [BH][T][DV]
  const float* ig;  // [BH][T] input-gate pre-activations
  const float* fg;  // [BH][T] forget-gate pre-activations
  const float* c0;  // [BH][DQ][DV] or NULL
  const float* n0;  // [BH][DQ] or NULL
  const float* m0;  // [BH] or NULL
  void* Cs;         // [BH][nc][DV][DQ] chunk-start states C~_0 .. C~_{nc-1}, transposed, in
                    // the compute dtype: the bf16 / f16 image the forward's Q~ C~_k MFMA reads
  float* c_last;    // [BH][DQ][DV] final state C~_nc (fp32: the carried segment state)
  float* ns;        // [BH][nc+1][DQ]
  float* ms;        // [BH][nc+1]
  void* h;          // [BH][T][DV]
  float* mrow;      // [BH][T] m_t
  float* den;       // [BH][T] den_t
  // backward
  const void* dh;   // [BH][T][DV]
  const float* dcT;  // [BH][DQ][DV] or NULL (gradient w.r.t. the final state)
  const float* dnT;  // [BH][DQ] or NULL
  float* dCs;       // [BH][DQ][DV]: gradient w.r.t. the initial state C~_0 (every later dC~_k
                    // stays on chip)
  float* dns;       // [BH][DQ]:     gradient w.r.t. n~_0
  void* dq;         // [BH][T][DQ]
  void* dk;
  void* dv;         // [BH][T][DV]
  float* qdq;       // [BH][T]  q_t . dq_t
  float* kdk;       // [BH][T]  k_t . dk_t
  int BH, T, nc;
  float eps, scale;
  // element offsets of q / k / dq / dk (q*) and v / dv (v*) rows: sequence bh = b NH + h, step t
  // at (bh / NH) *b + (bh % NH) *h + t *t.  Contiguous [BH][T][D]: NH = 1, b = T D, t = D; the
  // xLSTM layer reads them in place from its fused projection [B][T][N] (h = D, t = N).
  int NH;
  int64_t qb, qh, qt, vb, vh, vt;
  int xcd;   // mlstm_fw_walk on a 1-D grid with the column blocks of one bh on one XCD
};

__device__ __forceinline__ int64_t qrow(const MArgs& a, int bh, int64_t t) {
  return (int64_t)(bh / a.NH) * a.qb + (int64_t)(bh % a.NH) * a.qh + t * a.qt;
}
__device__ __forceinline__ int64_t vrow(const MArgs& a, int bh, int64_t t) {
  return (int64_t)(bh / a.NH) * a.vb + (int64_t)(bh % a.NH) * a.vh + t * a.vt;
}

__device__ __forceinline__ float logsig(float x) { return fminf(x, 0.0f) - log1pf(expf(-fabsf(x))); }

// MFMA operand fragment from an LDS tile stored [major][k] (row stride ld elements): lane l
// holds tile[r0 + (l & 15)][k0 + 8 (l >> 4) + 0..7].  A operands are stored [row][k], B
// operands [col][k] (i.e. B transposed).
template <typename V8, typename T>
__device__ __forceinline__ V8 frag(const T* tile, int ld, int r0, int k0, int lane) {
  return *(const V8*)(tile + (r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4));
}
// same, each element scaled by a per-row factor (the row is the lane's r0 + (l & 15))
template <typename V8, typename T>
__device__ __forceinline__ V8 frag_rs(const T* tile, int ld, int r0, int k0, int lane, float f) {
  V8 x = frag<V8, T>(tile, ld, r0, k0, lane);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (T)((float)x[j] * f);
  return x;
}
// same, element j scaled by fk[k0 + 8 (l >> 4) + j] (a per-k factor)
template <typename V8, typename T>
__device__ __forceinline__ V8 frag_ks(const T* tile, int ld, int r0, int k0, int lane,
                                      const float* fk) {
  V8 x = frag<V8, T>(tile, ld, r0, k0, lane);
  const float* f = fk + k0 + 8 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (T)((float)x[j] * f[j]);
  return x;
}

// ---- cross-lane helpers on DPP (VALU lane moves; __shfl_* would be an LDS permute round trip
// each, and the walks' per-chunk chains are latency-bound) ----
// lane moves within 16-lane rows; lanes whose source is out of the row keep `old`
template <int CTRL>
__device__ __forceinline__ float dppf(float old, float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                               __builtin_bit_cast(int, x), CTRL,
                                                               0xf, 0xf, false));
}
__device__ __forceinline__ float rdlane(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
constexpr int kQuadX1 = 0xB1, kQuadX2 = 0x4E, kHalfMirror = 0x141, kRowMirror = 0x140;
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
// sums over aligned groups of 4 / 8 / 16 lanes (every lane of the group gets the total)
__device__ __forceinline__ float sum4(float x) {
  x += dppf<kQuadX1>(0.0f, x);
  return x + dppf<kQuadX2>(0.0f, x);
}
__device__ __forceinline__ float sum8(float x) {
  x = sum4(x);
  return x + dppf<kHalfMirror>(0.0f, x);
}
// sum over the 16 lanes that share (lane >> 4) — the columns of one accumulator row group
__device__ __forceinline__ float sum16(float x) {
  x = sum8(x);
  return x + dppf<kRowMirror>(0.0f, x);
}
__device__ __forceinline__ float wave_max(float x) {
  x = fmaxf(x, dppf<kQuadX1>(x, x));
  x = fmaxf(x, dppf<kQuadX2>(x, x));
  x = fmaxf(x, dppf<kHalfMirror>(x, x));
  x = fmaxf(x, dppf<kRowMirror>(x, x));
  return fmaxf(fmaxf(rdlane(x, 0), rdlane(x, 16)), fmaxf(rdlane(x, 32), rdlane(x, 48)));
}
// inclusive prefix sum / max over the 64 lanes of a wave: Hillis-Steele within each 16-lane row,
// then the row totals (read as scalars) carried into the rows above
__device__ __forceinline__ float wave_prefix_sum(float x, int lane) {
  x += dppf<kRowShr1>(0.0f, x);
  x += dppf<kRowShr2>(0.0f, x);
  x += dppf<kRowShr4>(0.0f, x);
  x += dppf<kRowShr8>(0.0f, x);
  const float r1 = rdlane(x, 15), r2 = rdlane(x, 31), r3 = rdlane(x, 47);
  const int row = lane >> 4;
  const float o12 = r1 + r2;
  return x + (row == 0 ? 0.0f : row == 1 ? r1 : row == 2 ? o12 : o12 + r3);
}
__device__ __forceinline__ float wave_prefix_max(float x, int lane) {
  constexpr float ninf = -__builtin_huge_valf();
  x = fmaxf(x, dppf<kRowShr1>(ninf, x));
  x = fmaxf(x, dppf<kRowShr2>(ninf, x));
  x = fmaxf(x, dppf<kRowShr4>(ninf, x));
  x = fmaxf(x, dppf<kRowShr8>(ninf, x));
  const float r1 = rdlane(x, 15), r2 = rdlane(x, 31), r3 = rdlane(x, 47);
  const int row = lane >> 4;
  const float o12 = fmaxf(r1, r2);
  return fmaxf(x, row == 0 ? ninf : row == 1 ? r1 : row == 2 ? o12 : fmaxf(o12, r3));
}

// ---- transposed LDS fragment reads (ds_read_b64_tr_b16) ----
template <typename T>
__device__ __forceinline__ uint32_t lds_off(const T* base, int row, int ld, int col) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) T*)(base + row * ld + col);
}
__device__ __forceinline__ int2 tr_read16(uint32_t byte) {
  typedef short s4v __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(int2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                      (s4v __attribute__((address_space(3)))*)(size_t)byte));
}
// fragment (8 consecutive k for index n = n0 + (l & 15)) of an image stored [k][n] (row-major
// in k): two transposed reads of 4 k-rows x 16 n-columns per 16-lane group
template <typename V8, typename T>
__device__ __forceinline__ V8 frag_t(const T* img, int ld, int k0, int n0, int lane) {
  const int r = k0 + 8 * (lane >> 4) + ((lane & 15) >> 2), c = n0 + 4 * (lane & 3);
  const int2 lo = tr_read16(lds_off(img, r, ld, c)), hi = tr_read16(lds_off(img, r + 4, ld, c));
  return __builtin_bit_cast(V8, u32x4{(uint32_t)lo.x, (uint32_t)lo.y, (uint32_t)hi.x, (uint32_t)hi.y});
}
// same, element e scaled by fk[k0 + 8 (l >> 4) + e]
template <typename V8, typename T>
__device__ __forceinline__ V8 frag_t_ks(const T* img, int ld, int k0, int n0, int lane,
                                        const float* fk) {
  V8 x = frag_t<V8, T>(img, ld, k0, n0, lane);
  const float* f = fk + k0 + 8 * (lane >> 4);
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = (T)((float)x[e] * f[e]);
  return x;
}

// Column block of the state: C~'s columns evolve independently (C~ += K^T diag(f) V), so each
// workgroup owns kCB = 64 columns of one (b,h) -- DV/64 x BH workgroups instead of BH; n~ and m
// are recomputed by every block (they need K and the gates only) and stored by block 0.
constexpr int kCB = 64;

// ------------------------------------------------------------------------- forward: walk ----
// Gate quantities of one chunk for the lane's step s = lane, computed by every wave from the same
// 64 pre-activations (identical results in every wave: no LDS round trip for the values a lane
// needs itself, and the stabiliser m stays a per-wave register).
struct ChunkGates {
  float b;      // b_s: inclusive cumulative logsig(f) within the chunk
  float i;      // i_s
  float mt;     // m_t: the row stabiliser (t = lane)
  float rowf;   // s e^{b_t + m_k - m_t}: weight of the inter-chunk term of row t
  float fs;     // e^{g - b_s + i_s - m_{k+1}}: weight of key s in the state update
  float decay;  // e^{g + m_k - m_{k+1}}
  float mn;     // m_{k+1}
};
__device__ __forceinline__ ChunkGates chunk_gate_math(float ig, float fg, float m, float scale,
                                                      int lane) {
  ChunkGates G;
  const float b = wave_prefix_sum(logsig(fg), lane);
  G.b = b;
  G.i = ig;
  G.mt = fmaxf(b + m, b + wave_prefix_max(ig - b, lane));
  G.rowf = scale * expf(b + m - G.mt);
  const float g = rdlane(b, 63);
  const float as = g - b + ig;
  G.mn = fmaxf(g + m, wave_max(as));
  G.fs = expf(as - G.mn);
  G.decay = expf(g + m - G.mn);
  return G;
}

// One workgroup per (b,h, 64-column block of C~) walks the chunks in order and does both halves
// of the chunkwise forward for its columns: the chunk's outputs H[:, block] (S = Q K^T, causal
// decay mask, M V + Q~ C~_k, normaliser) and the state update C~_{k+1}[:, block].  The state block
// and n~ never leave the MFMA accumulators: only the state's bf16 / f16 image (what the Q~ C~_k
// MFMA consumes, kept for the backward's dq) and n~, m go to HBM.
// LDS holds every operand row-major as loaded (16-byte stores); the operands that run along a
// column (K^T in the state update, V in M V) come out through transposed reads.  Per-row weights
// scale the accumulators, per-k weights are folded into one scaled copy Kf = diag(fs) K written
// with the fill: no VALU work between a fragment read and its MFMA.
template <int DT, int IO, int DQ, int DV, int MODE>
__global__ void __launch_bounds__(256, 2) mlstm_fw_walk(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  typedef T v4t __attribute__((ext_vector_type(4)));
  constexpr int LQ = DQ + kPad, LC = kCB + kPad;
  constexpr int TJ = kCB / 16, NI = DQ / 16, NT = NI * TJ, PW = NT / 4;
  static_assert(NT % 4 == 0, "tile count must split over 4 waves");
  // MODE 0: the whole walk.  MODE 1: the state walk alone (gates, C~ / n~ / m and the state
  // image; the outputs come from mlstm_fw_out).
  static_assert(MODE == 0 || MODE == 1, "walk modes");
  constexpr bool kOut = MODE == 0;
  // XCD-aware order (a.xcd): workgroup i runs on XCD i % 8, so the DV / kCB column blocks of
  // sequence bh take i = x + 8 (NCB s + cb) for bh = 8 s + x: they read the same K / Q rows
  // chunk by chunk, and on one XCD the second and third reads hit its L2 instead of HBM
  constexpr int NCB = DV / kCB;
  int cb = blockIdx.x, bh = (int)blockIdx.y;
  if (a.xcd) {
    const int x = (int)blockIdx.x & 7, sl = (int)blockIdx.x >> 3;
    cb = sl % NCB;
    bh = (sl / NCB) * 8 + x;
  }
  const int w = threadIdx.x >> 6;
  int tid = threadIdx.x, lane = tid & 63;
  const int cj0 = cb * kCB;
  __shared__ __attribute__((aligned(16))) T Qs[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Ks[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Kf[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Vs[kL * LC];
  __shared__ __attribute__((aligned(16))) T Ms[kL * LC];   // M = S o W, then H staging
  __shared__ __attribute__((aligned(16))) T CT[kCB * LQ];  // C~_k[:, block], [j][i]
  __shared__ float sb[kL], si[kL], mts[kL], rowfs[kL], dsum[kL], qn[kL], fsv[kL], nk[DQ], np2[2 * DQ];
  const T* Q = (const T*)a.q + qrow(a, bh, 0);
  const T* K = (const T*)a.k + qrow(a, bh, 0);
  const T* V = (const T*)a.v + vrow(a, bh, 0);
  T* H = (T*)a.h + (int64_t)bh * a.T * DV;
  f32x4 acc[PW];   // C~ tiles q = w + 4 p: rows i0 = 16 (q / TJ), block columns 16 (q % TJ)
#pragma unroll
  for (int p = 0; p < PW; ++p) {
    const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = cj0 + 16 * (q % TJ);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r, j = j0 + (lane & 15);
      acc[p][r] = a.c0 ? a.c0[((int64_t)bh * DQ + i) * DV + j] : 0.0f;
    }
  }
  // n~ (fp32: the normaliser's q.n~ can cancel, and bf16 products in its sum showed) on thread
  // i < DQ; its chunk increment sum_s fs_s k_s[i] comes as two half sums from threads i, DQ + i
  float n = (tid < DQ && a.n0) ? a.n0[(int64_t)bh * DQ + tid] : 0.0f;
  float decay = 1.0f;
  float m = a.m0 ? a.m0[bh] : 0.0f;
  // chunk inputs are prefetched into registers one chunk ahead: the loads of chunk k + 1 are
  // issued right after chunk k's are written to LDS and land while chunk k computes
  constexpr int NQP = kL * DQ / 8 / 256, NVP = kL * kCB / 8 / 256;
  static_assert(NQP * 256 * 8 == kL * DQ && NVP * 256 * 8 == kL * kCB, "piece split");
  u32x4 pq[NQP], pk[NQP], pv[NVP];
  float pig, pfg;
  auto prefetch = [&](int kc) __attribute__((always_inline)) {
    const int64_t tb = (int64_t)kc * kL;
#pragma unroll
    for (int u = 0; u < NQP; ++u) {
      const int e = tid + 256 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
      if (kOut) pq[u] = *(const u32x4*)(Q + (tb + r) * a.qt + c);
      pk[u] = *(const u32x4*)(K + (tb + r) * a.qt + c);
    }
#pragma unroll
    for (int u = 0; u < NVP; ++u) {
      const int e = tid + 256 * u, r = e / (kCB / 8), c = (e % (kCB / 8)) * 8;
      pv[u] = *(const u32x4*)(V + (tb + r) * a.vt + cj0 + c);
    }
    const int64_t o = (int64_t)bh * a.T + tb + lane;
    pig = a.ig[o];
    pfg = a.fg[o];
  };
  prefetch(0);
  for (int k = 0; k < a.nc; ++k) {
    const int64_t t0 = (int64_t)k * kL;
    // re-derive the lane-dependent addresses every chunk instead of holding dozens of them in
    // VGPRs across the loop (hoisted, they pushed the prefetch registers out to scratch)
    asm volatile("" : "+v"(tid), "+v"(lane));
    const ChunkGates G = chunk_gate_math(pig, pfg, m, a.scale, lane);
    if (k > 0 && tid < DQ) n = decay * n + np2[tid] + np2[DQ + tid];   // previous chunk's update
    decay = G.decay;
    if (!ML_ABL(16)) {
#pragma unroll
      for (int u = 0; u < NQP; ++u) {
        const int e = tid + 256 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
        if (kOut) *(V8*)(Qs + r * LQ + c) = cvt8<DT, IO>(pq[u]);
        const V8 x = cvt8<DT, IO>(pk[u]);
        *(V8*)(Ks + r * LQ + c) = x;
        {
          const float f = __shfl(G.fs, r);
          V8 y;
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] = (T)((float)x[j] * f);
          *(V8*)(Kf + r * LQ + c) = y;
        }
      }
#pragma unroll
      for (int u = 0; u < NVP; ++u) {
        const int e = tid + 256 * u, r = e / (kCB / 8), c = (e % (kCB / 8)) * 8;
        *(V8*)(Vs + r * LC + c) = cvt8<DT, IO>(pv[u]);
      }
    }
    if (w == 0) {
      if constexpr (kOut) {
        sb[lane] = G.b;
        si[lane] = G.i;
        mts[lane] = G.mt;
        rowfs[lane] = G.rowf;
      }
      fsv[lane] = G.fs;
    }
    // (MODE 0: the next chunk's loads go out here, beside the whole output phase)
    if (kOut && k + 1 < a.nc) prefetch(k + 1);
    // the state at the chunk start: its MFMA image, transposed ([j][i]); a lane's four
    // accumulator rows are consecutive i, so each tile is one 8-byte LDS store
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
      v4t c;
#pragma unroll
      for (int r = 0; r < 4; ++r) c[r] = (T)acc[p][r];
      *(v4t*)(CT + (j0 + (lane & 15)) * LQ + i0 + 4 * (lane >> 4)) = c;
      // the update's decay, applied now: with the next chunk's loads in flight, a packed multiply
      // beside a register pair one of whose halves is a pending load waits for that load
      acc[p] = acc[p] * G.decay;
      asm volatile("" : "+v"(acc[p]));   // (kept here: the scheduler would sink it to its use)
    }
    if (tid < DQ) {
      nk[tid] = n;
      if (cb == 0) a.ns[((int64_t)bh * (a.nc + 1) + k) * DQ + tid] = n;
    }
    if (cb == 0 && tid == 0) a.ms[(int64_t)bh * (a.nc + 1) + k] = m;
    __syncthreads();
    // the backward's copy of the chunk-start state: CT's rows as they are, [j][i] (16-byte stores)
    {
      T* Cs = (T*)a.Cs + (((int64_t)bh * a.nc + k) * DV + cj0) * DQ;
      constexpr int NCP = kCB * DQ / 8 / 256;
      static_assert(NCP * 256 * 8 == kCB * DQ, "state image split");
#pragma unroll
      for (int u = 0; u < NCP; ++u) {
        const int e = tid + 256 * u, j = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
        if (!ML_ABL(8)) *(u32x4*)(Cs + j * DQ + c) = *(const u32x4*)(CT + j * LQ + c);
      }
    }
    // MODE 1: the next chunk's loads go out AFTER this chunk's stores.  vmcnt retires in order, so
    // a wait the compiler places for a store's source registers (reused by the state update's
    // fragments) then covers the stores alone, not loads issued a few hundred cycles earlier
    if (!kOut && k + 1 < a.nc) prefetch(k + 1);
    // From here to the state update every wave touches only its own 16 rows of Ms / qn / dsum
    // (rows 16 w ..): no barrier between the S and H phases.
    if constexpr (kOut) {
    // q_t . n~_k (4 threads per row, DQ / 4 consecutive i each)
    {
      constexpr int QP = DQ / 4;
      const int t = tid >> 2, part = tid & 3;
      float qa = 0.0f;
#pragma unroll
      for (int u = 0; u < QP / 8; ++u) {
        const V8 x = *(const V8*)(Qs + t * LQ + part * QP + 8 * u);
#pragma unroll
        for (int e = 0; e < 8; ++e) qa += (float)x[e] * nk[part * QP + 8 * u + e];
      }
      qa = sum4(qa);
      if (part == 0) qn[t] = qa;
    }
    // the row block's Q fragments (S and the inter-chunk term of H)
    V8 qa[DQ / 32];
#pragma unroll
    for (int kk = 0; kk < DQ / 32; ++kk) qa[kk] = frag<V8, T>(Qs, LQ, 16 * w, 32 * kk, lane);
    // S = Q K^T for row block w, causal column blocks; M = S o W into LDS, row sums
    {
      float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int ct = 0; ct <= w; ++ct) {
        V8 kb[DQ / 32];
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk) kb[kk] = frag<V8, T>(Ks, LQ, 16 * ct, 32 * kk, lane);
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < (ML_ABL(1) ? 0 : DQ / 32); ++kk) s4 = M::mma(qa[kk], kb[kk], s4);
        const int s = 16 * ct + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = 16 * w + 4 * (lane >> 4) + r;
          const float mv = (s <= t) ? s4[r] * a.scale * expf(sb[t] - sb[s] + si[s] - mts[t]) : 0.0f;
          rs[r] += mv;
          Ms[t * LC + s] = (T)mv;
        }
      }
      // the column blocks right of the diagonal: zero (the H MFMA reads them)
      for (int ct = w + 1; ct < 4; ++ct) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Ms[(16 * w + 4 * (lane >> 4) + r) * LC + 16 * ct + (lane & 15)] = (T)0.0f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float tot = sum16(rs[r]);
        if ((lane & 15) == 0) dsum[16 * w + 4 * (lane >> 4) + r] = tot;
      }
    }
    // H = M V + rowf (Q C~_k) for row block w, normalised; staged in the wave's own Ms rows
    // (every cj has read them first) and stored as 16-byte rows
    {
      float zi[4], rf[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * w + 4 * (lane >> 4) + r;
        rf[r] = rowfs[t];
        const float dn = dsum[t] + rf[r] * qn[t];
        zi[r] = 1.0f / (fmaxf(fabsf(dn), expf(-mts[t])) + a.eps);
      }
      f32x4 hv[TJ];
      // both k-steps of M V always (M is zero right of the diagonal block); the row block's M
      // fragments once for the TJ column blocks
      V8 ma[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ma[kk] = frag<V8, T>(Ms, LC, 16 * w, 32 * kk, lane);
#pragma unroll
      for (int cj = 0; cj < TJ; ++cj) {
        V8 vb[2], cb2[DQ / 32];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) vb[kk] = frag_t<V8, T>(Vs, LC, 32 * kk, 16 * cj, lane);
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk) cb2[kk] = frag<V8, T>(CT, LQ, 16 * cj, 32 * kk, lane);
        f32x4 h4 = {0.f, 0.f, 0.f, 0.f}, e4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < (ML_ABL(2) ? 0 : 2); ++kk) h4 = M::mma(ma[kk], vb[kk], h4);
#pragma unroll
        for (int kk = 0; kk < (ML_ABL(2) ? 0 : DQ / 32); ++kk) e4 = M::mma(qa[kk], cb2[kk], e4);
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[cj][r] = (h4[r] + rf[r] * e4[r]) * zi[r];
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int cj = 0; cj < TJ; ++cj) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Ms[(16 * w + 4 * (lane >> 4) + r) * LC + 16 * cj + (lane & 15)] = (T)hv[cj][r];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {   // 16 rows x 128 bytes = 128 pieces over 64 lanes
        const int e = lane + 64 * u, t = 16 * w + (e >> 3), c = (e & 7) * 8;
        if (!ML_ABL(8)) *(u32x4*)(H + (t0 + t) * DV + cj0 + c) = *(const u32x4*)(Ms + t * LC + c);
      }
      if (cb == 0 && lane < 16) {   // the wave's own rows
        const int t = 16 * w + lane;
        a.mrow[(int64_t)bh * a.T + t0 + t] = mts[t];
        a.den[(int64_t)bh * a.T + t0 + t] = dsum[t] + rowfs[t] * qn[t];
      }
    }
    }   // kOut
    // state update: C~ <- decay C~ + Kf^T V[:, block];  n~ <- decay n~ + Kf^T 1
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
      f32x4 c = acc[p];
#pragma unroll
      for (int kk = 0; kk < (ML_ABL(4) ? 0 : kL / 32); ++kk)
        c = M::mma(frag_t<V8, T>(Kf, LQ, 32 * kk, i0, lane),
                   frag_t<V8, T>(Vs, LC, 32 * kk, j0, lane), c);
      acc[p] = c;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (tid < 2 * DQ) {   // n~ increment: half sums over s (fp32 weights, bf16 keys)
      const int i = tid % DQ, s0 = (tid / DQ) * (kL / 2);
      float sacc = 0.0f;
#pragma unroll 8
      for (int s2 = 0; s2 < kL / 2; ++s2) sacc += fsv[s0 + s2] * (float)Ks[(s0 + s2) * LQ + i];
      np2[tid] = sacc;
    }
    m = G.mn;
    __syncthreads();
  }
  // final state: fp32 (the carried segment state) + n~, m
#pragma unroll
  for (int p = 0; p < PW; ++p) {
    const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = cj0 + 16 * (q % TJ);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      a.c_last[((int64_t)bh * DQ + i0 + 4 * (lane >> 4) + r) * DV + j0 + (lane & 15)] = acc[p][r];
  }
  if (tid < DQ) n = decay * n + np2[tid] + np2[DQ + tid];
  if (cb == 0) {
    if (tid < DQ) a.ns[((int64_t)bh * (a.nc + 1) + a.nc) * DQ + tid] = n;
    if (tid == 0) a.ms[(int64_t)bh * (a.nc + 1) + a.nc] = m;
  }
}

// Every chunk's outputs at once, after the state walk (mlstm_fw_walk MODE 1): one workgroup per
// (b,h, chunk) computes S, the decay-masked M, q.n~_k and the normaliser ONCE and then H for every
// 64-column block from the state image the walk stored (V / C~ blocks prefetched into registers
// one block ahead).  The operations and their order are the walk's H phase: bitwise the same h.
template <int DT, int IO, int DQ, int DV>
__global__ void __launch_bounds__(256, 2) mlstm_fw_out(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  constexpr int LQ = DQ + kPad, LC = kCB + kPad;
  constexpr int TJ = kCB / 16, NCB = DV / kCB;
  constexpr int NQP = kL * DQ / 8 / 256, NVP = kL * kCB / 8 / 256, NCP = kCB * DQ / 8 / 256;
  static_assert(NQP * 256 * 8 == kL * DQ && NVP * 256 * 8 == kL * kCB &&
                NCP * 256 * 8 == kCB * DQ, "piece split");
  const int bh = (int)blockIdx.x / a.nc, k = (int)blockIdx.x % a.nc, w = threadIdx.x >> 6;
  const int tid = threadIdx.x, lane = tid & 63;
  __shared__ __attribute__((aligned(16))) T Qs[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Ks[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Vs[kL * LC];
  __shared__ __attribute__((aligned(16))) T Ms[kL * LC];
  __shared__ __attribute__((aligned(16))) T Hs[kL * LC];
  __shared__ __attribute__((aligned(16))) T CT[kCB * LQ];   // C~_k[:, block], [j][i]
  __shared__ float sb[kL], si[kL], mts[kL], rowfs[kL], dsum[kL], qn[kL], nk[DQ];
  const int64_t t0 = (int64_t)k * kL;
  const T* Q = (const T*)a.q + qrow(a, bh, t0);
  const T* K = (const T*)a.k + qrow(a, bh, t0);
  const T* V = (const T*)a.v + vrow(a, bh, t0);
  T* H = (T*)a.h + ((int64_t)bh * a.T + t0) * DV;
  const T* Csb = (const T*)a.Cs + ((int64_t)bh * a.nc + k) * DV * DQ;
  u32x4 pv[NVP], pc[NCP];
  auto load_blk = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NVP; ++u) {
      const int e = tid + 256 * u, r = e / (kCB / 8), cc = (e % (kCB / 8)) * 8;
      pv[u] = *(const u32x4*)(V + r * a.vt + c * kCB + cc);
    }
#pragma unroll
    for (int u = 0; u < NCP; ++u) {
      const int e = tid + 256 * u, j = e / (DQ / 8), cc = (e % (DQ / 8)) * 8;
      pc[u] = *(const u32x4*)(Csb + (int64_t)(c * kCB + j) * DQ + cc);
    }
  };
  auto store_blk = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NVP; ++u) {
      const int e = tid + 256 * u, r = e / (kCB / 8), cc = (e % (kCB / 8)) * 8;
      *(V8*)(Vs + r * LC + cc) = cvt8<DT, IO>(pv[u]);
    }
#pragma unroll
    for (int u = 0; u < NCP; ++u) {
      const int e = tid + 256 * u, j = e / (DQ / 8), cc = (e % (DQ / 8)) * 8;
      *(u32x4*)(CT + j * LQ + cc) = pc[u];
    }
  };
  // every load of the prologue in flight at once (the small ones first: vmcnt retires in order)
  const float m = a.ms[(int64_t)bh * (a.nc + 1) + k];
  const int64_t o = (int64_t)bh * a.T + t0 + lane;
  const float igv = a.ig[o], fgv = a.fg[o];
  const float nsv = tid < DQ ? a.ns[((int64_t)bh * (a.nc + 1) + k) * DQ + tid] : 0.0f;
  u32x4 pq[NQP], pk[NQP];
#pragma unroll
  for (int u = 0; u < NQP; ++u) {
    const int e = tid + 256 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
    pq[u] = *(const u32x4*)(Q + r * a.qt + c);
    pk[u] = *(const u32x4*)(K + r * a.qt + c);
  }
  load_blk(0);
  const ChunkGates G = chunk_gate_math(igv, fgv, m, a.scale, lane);
  if (w == 0) {
    sb[lane] = G.b;
    si[lane] = G.i;
    mts[lane] = G.mt;
    rowfs[lane] = G.rowf;
  }
  if (tid < DQ) nk[tid] = nsv;
#pragma unroll
  for (int u = 0; u < NQP; ++u) {
    const int e = tid + 256 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
    *(V8*)(Qs + r * LQ + c) = cvt8<DT, IO>(pq[u]);
    *(V8*)(Ks + r * LQ + c) = cvt8<DT, IO>(pk[u]);
  }
  store_blk();
  if (NCB > 1) load_blk(1);
  __syncthreads();
  // every wave touches only its own 16 rows of Ms / Hs / qn / dsum from here on (as the walk)
  {
    constexpr int QP = DQ / 4;
    const int t = tid >> 2, part = tid & 3;
    float qa = 0.0f;
#pragma unroll
    for (int u = 0; u < QP / 8; ++u) {
      const V8 x = *(const V8*)(Qs + t * LQ + part * QP + 8 * u);
#pragma unroll
      for (int e = 0; e < 8; ++e) qa += (float)x[e] * nk[part * QP + 8 * u + e];
    }
    qa = sum4(qa);
    if (part == 0) qn[t] = qa;
  }
  V8 qa[DQ / 32];
#pragma unroll
  for (int kk = 0; kk < DQ / 32; ++kk) qa[kk] = frag<V8, T>(Qs, LQ, 16 * w, 32 * kk, lane);
  {
    float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int ct = 0; ct <= w; ++ct) {
      V8 kb[DQ / 32];
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk) kb[kk] = frag<V8, T>(Ks, LQ, 16 * ct, 32 * kk, lane);
      f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk) s4 = M::mma(qa[kk], kb[kk], s4);
      const int s = 16 * ct + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * w + 4 * (lane >> 4) + r;
        const float mv = (s <= t) ? s4[r] * a.scale * expf(sb[t] - sb[s] + si[s] - mts[t]) : 0.0f;
        rs[r] += mv;
        Ms[t * LC + s] = (T)mv;
      }
    }
    for (int ct = w + 1; ct < 4; ++ct) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Ms[(16 * w + 4 * (lane >> 4) + r) * LC + 16 * ct + (lane & 15)] = (T)0.0f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float tot = sum16(rs[r]);
      if ((lane & 15) == 0) dsum[16 * w + 4 * (lane >> 4) + r] = tot;
    }
  }
  float zi[4], rf[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = 16 * w + 4 * (lane >> 4) + r;
    rf[r] = rowfs[t];
    const float dn = dsum[t] + rf[r] * qn[t];
    zi[r] = 1.0f / (fmaxf(fabsf(dn), expf(-mts[t])) + a.eps);
  }
  V8 ma[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) ma[kk] = frag<V8, T>(Ms, LC, 16 * w, 32 * kk, lane);
#pragma unroll 1
  for (int c = 0; c < NCB; ++c) {
    f32x4 hv[TJ];
#pragma unroll
    for (int cj = 0; cj < TJ; ++cj) {
      V8 vb[2], cb2[DQ / 32];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) vb[kk] = frag_t<V8, T>(Vs, LC, 32 * kk, 16 * cj, lane);
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk) cb2[kk] = frag<V8, T>(CT, LQ, 16 * cj, 32 * kk, lane);
      f32x4 h4 = {0.f, 0.f, 0.f, 0.f}, e4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) h4 = M::mma(ma[kk], vb[kk], h4);
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk) e4 = M::mma(qa[kk], cb2[kk], e4);
#pragma unroll
      for (int r = 0; r < 4; ++r) hv[cj][r] = (h4[r] + rf[r] * e4[r]) * zi[r];
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int cj = 0; cj < TJ; ++cj) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Hs[(16 * w + 4 * (lane >> 4) + r) * LC + 16 * cj + (lane & 15)] = (T)hv[cj][r];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {   // the wave's 16 rows x 128 bytes
      const int e = lane + 64 * u, t = 16 * w + (e >> 3), cc = (e & 7) * 8;
      *(u32x4*)(H + (int64_t)t * DV + c * kCB + cc) = *(const u32x4*)(Hs + t * LC + cc);
    }
    if (c + 1 < NCB) {
      __syncthreads();   // every wave has read block c's V / C~
      store_blk();
      if (c + 2 < NCB) load_blk(c + 2);
      __syncthreads();
    }
  }
  if (lane < 16) {
    const int t = 16 * w + lane;
    a.mrow[(int64_t)bh * a.T + t0 + t] = mts[t];
    a.den[(int64_t)bh * a.T + t0 + t] = dsum[t] + rowfs[t] * qn[t];
  }
}

// ------------------------------------------------------------------------- backward: walk ----
// Two workgroup roles in one launch of 2 BH 8-wave workgroups.
// Workgroups 0 .. BH-1 walk one sequence (b,h) through the chunks in REVERSE with the state
// gradient dC~ [DQ][DV] (fp32) in MFMA accumulators and compute per chunk
//   dk_s = sum_t dA_ts q_t + es_s (v_s dC~_{k+1}^T + dn~_{k+1})
//   dv_s = sum_t A_ts dnum_t + es_s k_s dC~_{k+1}
//   dC~_k = decay dC~_{k+1} + (rowf q)^T dnum,   dn~_k = decay dn~_{k+1} + sum_t rowf_t dden_t q_t
// Workgroups BH .. 2BH-1 compute, for sequence bh - BH and each chunk independently,
//   dq_t = sum_s dA_ts k_s + rowf_t (dnum_t C~_k^T + dden_t n~_k)
// which reads the forward's states C~_k, n~_k and no carried gradient, so it leaves the serial
// walk (whose chunk then has three barriers instead of five) and runs beside it on the CUs the
// walks leave free (one workgroup per CU: 2 BH = 256 at C4).
// (dA_ts = W_ts (dnum_t . v_s + dden_t), A_ts = W_ts q_t . k_s, W_ts = s e^{b_t - b_s + i_s - m_t},
// s <= t).  Every operand lives in LDS once, row-major as loaded; MFMA fragments that run along
// a column come out through transposed reads.  The per-row weights rowf / es scale the
// accumulators (a second accumulator per job for the weighted term); the one per-k weight,
// rowf in the state update, is folded into a scaled copy Qr = diag(rowf) Q written with the fill.
// Nothing of size T x DQ x DV goes to HBM: the chunk states of the gradient stay on chip (the
// gradient w.r.t. the initial state is the only state output).
// f16 range: dh of a trained-from-scratch model sits far below f16's normal range (~1e-6 against
// 6e-5), where its images would keep 3-4 significant bits.  The f16 kernels therefore scale each
// chunk by a power of two S_k = 2^-e (max |dh / z| S_k in [0.5, 1), and in the walk the carried
// dC~ below 2^10): dnum, dden, dA and the dC~ image carry S_k, the fp32 dC~ / dn~ carry is
// rescaled exactly when S changes, and every output is divided by S_k.  bf16 has the exponent
// range of fp32 and runs unscaled.
template <int DT, int IO, int DQ, int DV>
__global__ void __launch_bounds__(512, 1) mlstm_bw_walk(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  using TI = typename MF<IO>::T;   // q / k / v / dh and the gradients in HBM (h: compute dtype)
  using V8I = typename MF<IO>::v8;
  typedef T v4t __attribute__((ext_vector_type(4)));
  constexpr bool kScale = DT == SC_F16;
  constexpr int LQ = DQ + kPad, LV = DV + kPad, LL = kL + kPad;
  constexpr int NI = DQ / 16, NJ = DV / 16;       // tile counts along DQ, DV
  constexpr int NC = NI * NJ;                     // state tiles
  static_assert(NC % 8 == 0, "state tiles must split over 8 waves");
  constexpr int PC = NC / 8;
  const int w = threadIdx.x >> 6;
  int tid = threadIdx.x, lane = tid & 63;
  __shared__ __attribute__((aligned(16))) T Qs[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Qr[kL * LQ];   // diag(rowf) Q
  __shared__ __attribute__((aligned(16))) T Ks[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Vs[kL * LV];
  __shared__ __attribute__((aligned(16))) T Dn[kL * LV];
  __shared__ __attribute__((aligned(16))) T CS[DV * LQ];   // walk: dC~_{k+1}; dq: C~_k ([j][i])
  __shared__ __attribute__((aligned(16))) T dA[kL * LL];
  __shared__ __attribute__((aligned(16))) T Am[kL * LL];
  __shared__ float sb[kL], si[kL], mt[kL], rowf[kL], es[kL], dden[kL], nk[DQ], dnk[DQ];
  __shared__ float part[NI * kL], dnp[4 * DQ], smax[16];
  constexpr int NQ8 = kL * DQ / 8, NV8 = kL * DV / 8, NC8 = DQ * DV / 8;
  constexpr int UQ = (NQ8 + 511) / 512, UV = (NV8 + 511) / 512, UC = (NC8 + 511) / 512;
  constexpr int UH = DV / 64;   // dh / h pieces per thread (8 threads per row)
  const bool walk = (int)blockIdx.x < a.BH;
  // sequence of this workgroup.  SC_ML_XCDH: the NH heads of one batch row on one XCD (bids go
  // round-robin over the 8 XCDs): in the xLSTM layer's fused gradient [B][T][N] the heads' dq /
  // dk / dv segments of a time step share cache lines (192 / 384-byte segments at a 4,624-byte
  // row pitch), and lines that heads on different XCDs write in parts reach HBM as partial lines
  // the L2s must first read (90.9 MB of FETCH per launch at C4, r6m2).  Both roles keep sharing
  // their XCD (workgroups i and BH + i, BH % 8 == 0).
  int bh = walk ? blockIdx.x : blockIdx.x - a.BH;
  if (SC_ML_XCDH && a.NH > 1 && a.BH % 8 == 0 && (a.BH / 8) % a.NH == 0) {
    const int x = bh % 8, kk = bh / 8;
    bh = (x + 8 * (kk / a.NH)) * a.NH + kk % a.NH;
  }
  const T* Qg = (const T*)a.q + qrow(a, bh, 0);
  const T* Kg = (const T*)a.k + qrow(a, bh, 0);
  const T* Vg = (const T*)a.v + vrow(a, bh, 0);
  // zero the strictly upper tiles (tc > tr) of A and dA once (they stay zero across chunks;
  // ordered before any read by the first chunk's barrier)
  for (int e = tid; e < kL * kL; e += 512) {
    const int tt = e / kL, s = e % kL;
    if ((s >> 4) > (tt >> 4)) {
      Am[tt * LL + s] = (T)0.0f;
      dA[tt * LL + s] = (T)0.0f;
    }
  }

  // ---- pieces shared by the two roles ----
  // chunk inputs in registers (issued ahead of their use)
  u32x4 rq[UQ] = {}, rk[UQ] = {}, rv[UV] = {}, rd[UH] = {}, rh[UH] = {};
  float mk = 0.f, mk1 = 0.f, g_i = 0.f, g_f = 0.f, g_m = 0.f, m_t = 0.f, dv_ = 0.f;
  auto load_rows = [&](int kc) __attribute__((always_inline)) {   // dh, h, m_t, den of the rows
    const int64_t ro = (int64_t)bh * a.T + (int64_t)kc * kL + (tid >> 3);
    const T* dh = (const T*)a.dh + ro * DV;
    const T* h = (const T*)a.h + ro * DV;
#pragma unroll
    for (int u = 0; u < UH; ++u) {
      if (!ML_ABL(512)) {
        if (!ML_ABL(32768)) rd[u] = *(const u32x4*)(dh + (tid & 7) * 8 + 64 * u);
        if (!ML_ABL(65536)) rh[u] = *(const u32x4*)(h + (tid & 7) * 8 + 64 * u);
      }
    }
    m_t = a.mrow[ro];
    dv_ = a.den[ro];
  };
  auto load_qkv = [&](int kc) __attribute__((always_inline)) {   // q, k, v and the chunk scalars
    const int64_t tb = (int64_t)kc * kL;
    const int64_t st = (int64_t)bh * (a.nc + 1) + kc;
    mk = a.ms[st];
    mk1 = a.ms[st + 1];
    const int64_t og = (int64_t)bh * a.T + tb + lane;
    g_i = a.ig[og];
    g_f = a.fg[og];
    g_m = a.mrow[og];
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int e = tid + 512 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
      if (e < NQ8 && !ML_ABL(512)) {
        if (!ML_ABL(4096)) rq[u] = *(const u32x4*)(Qg + (tb + r) * a.qt + c);
        if (!ML_ABL(8192)) rk[u] = *(const u32x4*)(Kg + (tb + r) * a.qt + c);
      }
    }
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int e = tid + 512 * u, r = e / (DV / 8), c = (e % (DV / 8)) * 8;
      if (e < NV8 && !ML_ABL(512) && !ML_ABL(16384)) rv[u] = *(const u32x4*)(Vg + (tb + r) * a.vt + c);
    }
  };
  // gate quantities (every wave, lane = step) and the Q / K (/ Qr) / V fill; returns g = b_{L-1}
  auto fill_chunk = [&](bool with_qr) __attribute__((always_inline)) {
    const float b = wave_prefix_sum(logsig(g_f), lane);
    const float rowf_l = a.scale * expf(b + mk - g_m);
    if (w == 0) {
      sb[lane] = b;
      si[lane] = g_i;
      rowf[lane] = rowf_l;
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int e = tid + 512 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
      const float f = __shfl(rowf_l, r & 63);
      if (e < NQ8) {
        const V8 x = cvt8<DT, IO>(rq[u]);
        *(V8*)(Qs + r * LQ + c) = x;
        *(V8*)(Ks + r * LQ + c) = cvt8<DT, IO>(rk[u]);
        if (with_qr) {
          V8 y;
#pragma unroll
          for (int j = 0; j < 8; ++j) y[j] = (T)((float)x[j] * f);
          *(V8*)(Qr + r * LQ + c) = y;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int e = tid + 512 * u, r = e / (DV / 8), c = (e % (DV / 8)) * 8;
      if (e < NV8) *(V8*)(Vs + r * LV + c) = cvt8<DT, IO>(rv[u]);
    }
    return b;
  };
  // the chunk's gradient scale (f16): dnum = dh / z to [0.5, 1) and the carried dC~ (largest
  // magnitude mc, in units of the previous scale S) below 2^10; z can be ~1e-6, so it is dnum,
  // not dh, that must fit.  Keeps S when nothing sets a scale.
  auto chunk_scale = [&](float z, float mc, float S) __attribute__((always_inline)) {
    float mx = 0.0f;
#pragma unroll
    for (int u = 0; u < UH; ++u) {
      const V8I xd = __builtin_bit_cast(V8I, rd[u]);
#pragma unroll
      for (int e2 = 0; e2 < 8; ++e2) mx = fmaxf(mx, fabsf((float)xd[e2]));
    }
    mx /= z;
    mx = wave_max(mx);
    mc = wave_max(mc);
    if (lane == 0) {
      smax[w] = mx;
      smax[8 + w] = mc;
    }
    __syncthreads();
    mx = smax[0];
    mc = smax[8];
#pragma unroll
    for (int v = 1; v < 8; ++v) {
      mx = fmaxf(mx, smax[v]);
      mc = fmaxf(mc, smax[8 + v]);
    }
    mc /= S;   // in true units
    float s1 = 3.0e38f, s2 = 3.0e38f;
    int ex;
    if (mx > 0.0f && mx < 3.0e38f) {
      frexpf(mx, &ex);
      s1 = ldexpf(1.0f, -ex);
    }
    if (mc > 0.0f && mc < 3.0e38f) {
      frexpf(mc, &ex);
      s2 = ldexpf(1.0f, 10 - ex);
    }
    const float Sk = fminf(s1, s2);
    return Sk < 3.0e38f ? Sk : S;
  };
  // dnum = dh S / z and dden S (8 threads per row)
  auto fill_dn = [&](float z, float Sk) __attribute__((always_inline)) {
    const int t = tid >> 3, pt = tid & 7;
    const float zs = Sk / z;
    float dot = 0.0f;
#pragma unroll
    for (int u = 0; u < UH; ++u) {
      const V8I xd = __builtin_bit_cast(V8I, rd[u]);
      const V8 xh = __builtin_bit_cast(V8, rh[u]);
      V8 o;
#pragma unroll
      for (int e2 = 0; e2 < 8; ++e2) {
        const float d = (float)xd[e2];
        dot += d * (float)xh[e2];
        o[e2] = (T)(d * zs);
      }
      *(V8*)(Dn + t * LV + pt * 8 + 64 * u) = o;
    }
    dot = sum8(dot);
    if (pt == 0) {
      const float live = fabsf(dv_) >= expf(-m_t) ? 1.0f : 0.0f;
      dden[t] = -dot * zs * (dv_ >= 0.0f ? 1.0f : -1.0f) * live;
      mt[t] = m_t;
    }
  };
  // one causal 16 x 16 tile of A = W o (Q K^T) (isA) or dA = W o (Dn V^T + dden)
  auto a_job = [&](int idx, bool isA) __attribute__((always_inline)) {
    // idx -> (tr, tc), tc <= tr: 0 (0,0) 1 (1,0) 2 (1,1) 3 (2,0) 4 (2,1) 5 (2,2) 6.. (3,*)
    const int tr = idx < 1 ? 0 : idx < 3 ? 1 : idx < 6 ? 2 : 3;
    const int tc = idx - tr * (tr + 1) / 2;
    f32x4 c4 = {0.f, 0.f, 0.f, 0.f};
    if (isA) {
      V8 fa[DQ / 32], fb[DQ / 32];
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk) {
        fa[kk] = frag<V8, T>(Qs, LQ, 16 * tr, 32 * kk, lane);
        fb[kk] = frag<V8, T>(Ks, LQ, 16 * tc, 32 * kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk) c4 = M::mma(fa[kk], fb[kk], c4);
    } else {
      V8 fa[DV / 32], fb[DV / 32];
#pragma unroll
      for (int kk = 0; kk < DV / 32; ++kk) {
        fa[kk] = frag<V8, T>(Dn, LV, 16 * tr, 32 * kk, lane);
        fb[kk] = frag<V8, T>(Vs, LV, 16 * tc, 32 * kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < DV / 32; ++kk) c4 = M::mma(fa[kk], fb[kk], c4);
    }
    const int s = 16 * tc + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tt = 16 * tr + 4 * (lane >> 4) + r;
      const float wts = (s <= tt) ? a.scale * expf(sb[tt] - sb[s] + si[s] - mt[tt]) : 0.0f;
      if (isA) Am[tt * LL + s] = (T)(c4[r] * wts);
      else dA[tt * LL + s] = (T)((c4[r] + dden[tt]) * wts);
    }
  };

  if (ML_ABL(1024) && !walk) return;
  if (ML_ABL(2048) && walk) return;
  if (!walk) {
    // ================= dq role: every chunk of sequence bh, independently =================
    TI* dQg = (TI*)a.dq + qrow(a, bh, 0);
    // (in the walk's order, last chunk first: both roles of bh run on one XCD — workgroups bh
    // and BH + bh, BH % 8 == 0 at the bench shape — and read the same q / k / v / dh / h rows,
    // so the second reader of a chunk finds them in that XCD's L2.  In forward order the two
    // met only in the middle and every row came from HBM twice.)
#pragma unroll 1
    for (int kr = 0; kr < a.nc; ++kr) {
      const int k = a.nc - 1 - kr;
      const int64_t t0 = (int64_t)k * kL;
      asm volatile("" : "+v"(tid), "+v"(lane));   // see mlstm_fw_walk
      u32x4 rc[UC] = {};
      const T* Ck = (const T*)a.Cs + ((int64_t)bh * a.nc + k) * DQ * DV;
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int e = tid + 512 * u;
        if (e < NC8 && !ML_ABL(512) && !ML_ABL(131072)) rc[u] = *(const u32x4*)(Ck + 8 * e);
      }
      const float n_k = tid < DQ ? a.ns[((int64_t)bh * (a.nc + 1) + k) * DQ + tid] : 0.0f;
      load_qkv(k);
      load_rows(k);
      fill_chunk(false);
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int e = tid + 512 * u;
        if (e < NC8) {
          const int j = (8 * e) / DQ, i = (8 * e) % DQ;
          *(u32x4*)(CS + j * LQ + i) = rc[u];
        }
      }
      if (tid < DQ) nk[tid] = n_k;
      const float z = fmaxf(fabsf(dv_), expf(-m_t)) + a.eps;
      float Sk = 1.0f;
      if constexpr (kScale) Sk = chunk_scale(z, 0.0f, 1.0f);
      fill_dn(z, Sk);
      __syncthreads();
      // ---- dA = W o (Dn V^T + dden): 10 causal tiles ----
#pragma unroll 1
      for (int jb = w; jb < (ML_ABL(32) ? 0 : 10); jb += 8) a_job(jb, false);
      __syncthreads();
      const float inv = 1.0f / Sk;
      // ---- dq = dA K + rowf (Dn C~_k^T + dden n~_k): 4 x NI tiles, wave w the row block
      // tr = w >> 1 and NI / 2 column blocks: each A fragment feeds NI / 2 MFMAs.  (The causal
      // chain always takes both k-steps: dA's tiles above the diagonal are zero.) ----
      if (!ML_ABL(64)) {
        constexpr int NC2 = NI / 2;
        const int tr = w >> 1, c0 = (w & 1) * NC2;
        f32x4 d4[NC2], e4[NC2];
#pragma unroll
        for (int c = 0; c < NC2; ++c) d4[c] = e4[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const V8 fa = frag<V8, T>(dA, LL, 16 * tr, 32 * kk, lane);
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            d4[c] = M::mma(fa, frag_t<V8, T>(Ks, LQ, 32 * kk, 16 * (c0 + c), lane), d4[c]);
        }
#pragma unroll
        for (int kk = 0; kk < DV / 32; ++kk) {
          const V8 ga = frag<V8, T>(Dn, LV, 16 * tr, 32 * kk, lane);
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            e4[c] = M::mma(ga, frag_t<V8, T>(CS, LQ, 32 * kk, 16 * (c0 + c), lane), e4[c]);
        }
#pragma unroll
        for (int c = 0; c < NC2; ++c) {
          const int ci = c0 + c, i = 16 * ci + (lane & 15);
          const float nki = nk[i];
          float qd[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int tt = 16 * tr + 4 * (lane >> 4) + r;
            const float v = d4[c][r] + rowf[tt] * (e4[c][r] + dden[tt] * nki);
            if (!ML_ABL(262144))
              dQg[(t0 + tt) * a.qt + i] = out16<DT, IO>(v * inv);
            qd[r] = sum16(v * (float)Qs[tt * LQ + i]);
          }
          if ((lane & 15) == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) part[ci * kL + 16 * tr + 4 * (lane >> 4) + r] = qd[r];
          }
        }
      }
      __syncthreads();
      if (tid < kL) {
        float sq = 0.0f;
#pragma unroll
        for (int ci = 0; ci < NI; ++ci) sq += part[ci * kL + tid];
        a.qdq[(int64_t)bh * a.T + t0 + tid] = sq * inv;
      }
    }
    return;
  }

  // ================= walk role =================
  // dC~ tiles: the waves form a 2 x 4 grid over the NI x NJ tiles, wave w owning the BI x BJ
  // block (w >> 2, w & 3); tile p = a BJ + b is at rows 16 (BI (w >> 2) + a), cols 16 (BJ (w & 3)
  // + b): per k-step the block's BI + BJ fragments feed BI BJ MFMAs
  static_assert(NI % 2 == 0 && NJ % 4 == 0, "2 x 4 wave grid");
  constexpr int BI = NI / 2, BJ = NJ / 4;
  static_assert(BI * BJ == PC, "block = the wave's tiles");
  const int ib0 = BI * (w >> 2), jb0 = BJ * (w & 3);
  f32x4 acc[PC];
#pragma unroll
  for (int p = 0; p < PC; ++p) {
    const int i0 = 16 * (ib0 + p / BJ), j0 = 16 * (jb0 + p % BJ);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r, j = j0 + (lane & 15);
      acc[p][r] = a.dcT ? a.dcT[((int64_t)bh * DQ + i) * DV + j] : 0.0f;
    }
  }
  float dn = (tid < DQ && a.dnT) ? a.dnT[(int64_t)bh * DQ + tid] : 0.0f;
  float S = 1.0f, decay = 1.0f;   // S: the current chunk's gradient scale (f16)
  TI* dKg = (TI*)a.dk + qrow(a, bh, 0);
  TI* dVg = (TI*)a.dv + vrow(a, bh, 0);
  for (int k = a.nc - 1; k >= 0; --k) {
    const int64_t t0 = (int64_t)k * kL;
    asm volatile("" : "+v"(tid), "+v"(lane));   // see mlstm_fw_walk
    // dn~_{k+1}: the previous chunk's four partial sums (after its closing barrier)
    if (k < a.nc - 1 && tid < DQ)
      dn = decay * dn + dnp[tid] + dnp[DQ + tid] + dnp[2 * DQ + tid] + dnp[3 * DQ + tid];
    // ---- chunk inputs, loaded during the previous (later) chunk: the dh and h rows are issued
    // after its first barrier, q / k / v and the chunk scalars after its A / dA phase, so both
    // land while it computes (the first chunk loads here) ----
    if (k == a.nc - 1) {
      load_rows(k);
      load_qkv(k);
    }
    const float b = fill_chunk(true);
    const float g = rdlane(b, 63);
    decay = expf(g + mk - mk1);
    if (w == 0) es[lane] = expf(g - b + g_i - mk1);
    const float z = fmaxf(fabsf(dv_), expf(-m_t)) + a.eps;
    float Sk = 1.0f;
    if constexpr (kScale) {
      float mc = 0.0f;
#pragma unroll
      for (int p = 0; p < PC; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) mc = fmaxf(mc, fabsf(acc[p][r]));
      Sk = chunk_scale(z, mc, S);
      // the carried gradients move to this chunk's scale (powers of two: exact)
      const float rs = Sk / S;
#pragma unroll
      for (int p = 0; p < PC; ++p) acc[p] *= rs;
      dn *= rs;
      S = Sk;
    }
    if (tid < DQ) dnk[tid] = dn;
    fill_dn(z, Sk);
    // ---- dC~_{k+1} image (the dk / dv operand) ----
#pragma unroll
    for (int p = 0; p < PC; ++p) {
      const int i0 = 16 * (ib0 + p / BJ), j0 = 16 * (jb0 + p % BJ);
      v4t c;
#pragma unroll
      for (int r = 0; r < 4; ++r) c[r] = (T)acc[p][r];
      *(v4t*)(CS + (j0 + (lane & 15)) * LQ + i0 + 4 * (lane >> 4)) = c;
    }
    __syncthreads();
    if (k > 0) load_rows(k - 1);   // dh / h of this chunk are consumed
    // ---- A = W o (Q K^T) and dA = W o (Dn V^T + dden): 10 causal tiles each, 20 jobs ----
#pragma unroll 1
    for (int jb = w; jb < (ML_ABL(32) ? 0 : 20); jb += 8) a_job(jb < 10 ? jb : jb - 10, jb < 10);
    __syncthreads();
    if (k > 0) load_qkv(k - 1);
    const float inv = 1.0f / S;
    // ---- dk = dA^T Q + es (V dC~^T + dn~): 4 x NI tiles; dv = A^T Dn + es (K dC~): 4 x NJ.
    // Wave w: key row block sr = w >> 1, NI / 2 dk column blocks, then NJ / 2 dv column blocks
    // in passes of NI / 2 (register-blocked: each A fragment feeds NI / 2 MFMAs) ----
    if (!ML_ABL(128)) {
      constexpr int NC2 = NI / 2;
      const int sr = w >> 1;
      {
        const int c0 = (w & 1) * NC2;
        f32x4 d4[NC2], e4[NC2];
#pragma unroll
        for (int c = 0; c < NC2; ++c) d4[c] = e4[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const V8 fa = frag_t<V8, T>(dA, LL, 32 * kk, 16 * sr, lane);
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            d4[c] = M::mma(fa, frag_t<V8, T>(Qs, LQ, 32 * kk, 16 * (c0 + c), lane), d4[c]);
        }
#pragma unroll
        for (int kk = 0; kk < DV / 32; ++kk) {
          const V8 ga = frag<V8, T>(Vs, LV, 16 * sr, 32 * kk, lane);
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            e4[c] = M::mma(ga, frag_t<V8, T>(CS, LQ, 32 * kk, 16 * (c0 + c), lane), e4[c]);
        }
#pragma unroll
        for (int c = 0; c < NC2; ++c) {
          const int ci = c0 + c, i = 16 * ci + (lane & 15);
          const float dni = dnk[i];
          float kd[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int s = 16 * sr + 4 * (lane >> 4) + r;
            const float v = d4[c][r] + es[s] * (e4[c][r] + dni);
            if (!ML_ABL(262144))
              dKg[(t0 + s) * a.qt + i] = out16<DT, IO>(v * inv);
            kd[r] = sum16(v * (float)Ks[s * LQ + i]);
          }
          if ((lane & 15) == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) part[ci * kL + 16 * sr + 4 * (lane >> 4) + r] = kd[r];
          }
        }
      }
      constexpr int NV2 = NJ / 2;
      static_assert(NV2 % NC2 == 0, "dv passes");
#pragma unroll 1
      for (int pass = 0; pass < NV2 / NC2; ++pass) {
        const int c0 = (w & 1) * NV2 + pass * NC2;
        f32x4 d4[NC2], e4[NC2];
#pragma unroll
        for (int c = 0; c < NC2; ++c) d4[c] = e4[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const V8 fa = frag_t<V8, T>(Am, LL, 32 * kk, 16 * sr, lane);
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            d4[c] = M::mma(fa, frag_t<V8, T>(Dn, LV, 32 * kk, 16 * (c0 + c), lane), d4[c]);
        }
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk) {
          const V8 ga = frag<V8, T>(Ks, LQ, 16 * sr, 32 * kk, lane);
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            e4[c] = M::mma(ga, frag<V8, T>(CS, LQ, 16 * (c0 + c), 32 * kk, lane), e4[c]);
        }
#pragma unroll
        for (int c = 0; c < NC2; ++c) {
          const int j = 16 * (c0 + c) + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int s = 16 * sr + 4 * (lane >> 4) + r;
            if (!ML_ABL(262144))
              dVg[(t0 + s) * a.vt + j] = out16<DT, IO>((d4[c][r] + es[s] * e4[c][r]) * inv);
          }
        }
      }
    }
    // ---- state gradient to the chunk start: dC~_k = decay dC~_{k+1} + Qr^T Dn ----
#pragma unroll
    for (int p = 0; p < PC; ++p) acc[p] *= decay;
#pragma unroll
    for (int kk = 0; kk < (ML_ABL(256) ? 0 : kL / 32); ++kk) {
      V8 fq[BI], fd[BJ];
#pragma unroll
      for (int x = 0; x < BI; ++x) fq[x] = frag_t<V8, T>(Qr, LQ, 32 * kk, 16 * (ib0 + x), lane);
#pragma unroll
      for (int y = 0; y < BJ; ++y) fd[y] = frag_t<V8, T>(Dn, LV, 32 * kk, 16 * (jb0 + y), lane);
#pragma unroll
      for (int p = 0; p < PC; ++p) acc[p] = M::mma(fq[p / BJ], fd[p % BJ], acc[p]);
    }
    // dn~ partial sums sum_t dden_t Qr[t][i] over four 16-step quarters (combined next chunk)
    if (tid < 4 * DQ) {
      const int i = tid % DQ, qt4 = tid / DQ;
      float sacc = 0.0f;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int tt = 16 * qt4 + u;
        sacc += dden[tt] * (float)Qr[tt * LQ + i];
      }
      dnp[qt4 * DQ + i] = sacc;
    }
    __syncthreads();
    if (tid < kL) {   // (part comes from every wave's dk jobs: after the barrier)
      float sk = 0.0f;
#pragma unroll
      for (int ci = 0; ci < NI; ++ci) sk += part[ci * kL + tid];
      a.kdk[(int64_t)bh * a.T + t0 + tid] = sk * inv;
    }
  }
  // gradient w.r.t. the initial state (unscaled)
  if (tid < DQ) dn = decay * dn + dnp[tid] + dnp[DQ + tid] + dnp[2 * DQ + tid] + dnp[3 * DQ + tid];
  const float inv = 1.0f / S;
#pragma unroll
  for (int p = 0; p < PC; ++p) {
    const int i0 = 16 * (ib0 + p / BJ), j0 = 16 * (jb0 + p % BJ);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      a.dCs[((int64_t)bh * DQ + i0 + 4 * (lane >> 4) + r) * DV + j0 + (lane & 15)] = acc[p][r] * inv;
  }
  if (tid < DQ) a.dns[(int64_t)bh * DQ + tid] = dn * inv;
}

// The forward is the state walk (mlstm_fw_walk MODE 1), then every chunk's outputs at once
// (mlstm_fw_out): 155-160 us at C4 against 180-184 us for the single walk that also computes
// the outputs (tools/mlstm_bench.py, A/B in one process).  SC_MLSTM_SPLIT=0 (environment, read
// per launch) runs the single walk: bitwise equal (tests/test_gpu_mlstm.py).
bool fwd_split() {
  const char* e = getenv("SC_MLSTM_SPLIT");
  return !(e && e[0] == '0');
}
// SC_MLSTM_XCD=0 (environment, read per launch) keeps the plain (column block, bh) grid (A/B)
bool fwd_xcd() {
  const char* e = getenv("SC_MLSTM_XCD");
  return !(e && e[0] == '0');
}
template <int DT, int IO, int DQ, int DV>
void launch_fwd(const MArgs& a0, hipStream_t st) {
  MArgs a = a0;
  a.xcd = (a.BH % 8 == 0 && fwd_xcd()) ? 1 : 0;
  const dim3 grid = a.xcd ? dim3((DV / kCB) * a.BH) : dim3(DV / kCB, a.BH);
  if (!fwd_split()) {
    hipLaunchKernelGGL((mlstm_fw_walk<DT, IO, DQ, DV, 0>), grid, dim3(256), 0, st, a);
    return;
  }
  hipLaunchKernelGGL((mlstm_fw_walk<DT, IO, DQ, DV, 1>), grid, dim3(256), 0, st, a);
  if (a.nc > 0)
    hipLaunchKernelGGL((mlstm_fw_out<DT, IO, DQ, DV>), dim3(a.BH * a.nc), dim3(256), 0, st, a);
}
template <int DT, int IO, int DQ, int DV>
void launch_bwd(const MArgs& a, hipStream_t st) {
  // workgroups 0 .. BH-1 walk, BH .. 2BH-1 take the dq terms
  hipLaunchKernelGGL((mlstm_bw_walk<DT, IO, DQ, DV>), dim3(2 * a.BH), dim3(512), 0, st, a);
}

// head dimensions compiled in (DQ, DV): the xLSTM-large defaults qk = v/2 at 64..192 wide heads
#define SC_MLSTM_DIMS(X) X(32, 64) X(64, 64) X(64, 128) X(96, 192)

template <int DT, int IO>
bool dispatch(const MArgs& a, int DQ, int DV, bool bwd, hipStream_t st) {
#define SC_CASE(q, v)                                    \
  if (DQ == q && DV == v) {                              \
    if (bwd) launch_bwd<DT, IO, q, v>(a, st);            \
    else launch_fwd<DT, IO, q, v>(a, st);                \
    return true;                                         \
  }
  SC_MLSTM_DIMS(SC_CASE)
#undef SC_CASE
  return false;
}

// (compute dtype, operand dtype) pairs: bf16 / bf16, f16 / f16, and the reference's f16 cell on
// a bf16-autocast model's projection (f16 compute, bf16 in HBM)
bool io_supported(int dtype, int io_dtype) {
  return (dtype == SC_BF16 && io_dtype == SC_BF16) || (dtype == SC_F16 && io_dtype == SC_F16) ||
         (dtype == SC_F16 && io_dtype == SC_BF16);
}
void dispatch_io(const MArgs& a, int dtype, int io_dtype, int DQ, int DV, bool bwd,
                 hipStream_t st) {
  if (dtype == SC_BF16) dispatch<SC_BF16, SC_BF16>(a, DQ, DV, bwd, st);
  else if (io_dtype == SC_F16) dispatch<SC_F16, SC_F16>(a, DQ, DV, bwd, st);
  else dispatch<SC_F16, SC_BF16>(a, DQ, DV, bwd, st);
}

bool dims_supported(int DQ, int DV) {
#define SC_CASE(q, v) if (DQ == q && DV == v) return true;
  SC_MLSTM_DIMS(SC_CASE)
#undef SC_CASE
  return false;
}

// q/k/v (and gradient) row layout: NULL = contiguous [BH][T][D]; else {NH, qb, qh, qt, vb, vh, vt}
// element strides (16-byte loads: every stride and base a multiple of 8 elements)
int set_layout(MArgs& a, const int64_t* layout, int DQ, int DV, const char* what,
               std::initializer_list<const void*> ptrs) {
  if (!layout) {
    a.NH = 1;
    a.qb = (int64_t)a.T * DQ; a.qh = 0; a.qt = DQ;
    a.vb = (int64_t)a.T * DV; a.vh = 0; a.vt = DV;
    return 0;
  }
  a.NH = (int)layout[0];
  a.qb = layout[1]; a.qh = layout[2]; a.qt = layout[3];
  a.vb = layout[4]; a.vh = layout[5]; a.vt = layout[6];
  SC_REQUIRE(a.NH > 0 && a.BH % a.NH == 0, "%s: layout NH=%d does not divide BH=%d", what, a.NH,
             a.BH);
  for (int i = 1; i < 7; ++i)
    SC_REQUIRE(layout[i] >= 0 && layout[i] % 8 == 0,
               "%s: layout stride %lld is not a multiple of 8 elements", what,
               (long long)layout[i]);
  SC_REQUIRE(a.qt >= DQ && a.vt >= DV, "%s: layout row strides overlap the rows", what);
  for (const void* p : ptrs)
    SC_REQUIRE(((uintptr_t)p & 15) == 0, "%s: strided operands must be 16-byte aligned", what);
  return 0;
}

// ----------------------------------------------------------------- gate gradients ----
// d igate = kdk, d fgate_t = sigmoid(-f_t) sum_{r>=t} (qdq_r - kdk_r) for one sequence per wave
// (lane = a contiguous T/64-step segment: segment suffix sums, then the suffix over the lanes
// above).  mode 0 writes d fgate fp32 [BH][T] (MLSTMFn); mode 1 writes both gate gradients
// through the soft cap's backward into the projection gradient at [b][t][io + h] / [b][t][fo + h]
// (MLSTMCoreFn).

// d/dx cap tanh(x / cap) = 1 - tanh(x / cap)^2, in fp32 on the fp32 gradient, one bf16 rounding
// (the torch chain it replaces rounds each of its five ops to bf16; near saturation 1 - y^2 of a
// bf16 y keeps only a few bits)
__device__ __forceinline__ float softcap_bwd(float g, float x, float cap) {
  if (!(cap > 0.0f)) return g;
  const float y = tanhf(x / cap);
  return g * (1.0f - y * y);
}

struct GateArgs {
  const float* qdq;
  const float* kdk;
  const float* fg;
  float* dfg;             // mode 0
  const __bf16* a;        // mode 1: raw pre-activations, [B][T][ld]
  __bf16* da;             // mode 1
  int BH, T, NH, io, fo;
  int64_t ld;
  float cap;
};

__global__ void __launch_bounds__(64) mlstm_gate_bwd_kernel(GateArgs g) {
  const int bh = blockIdx.x, lane = threadIdx.x;
  const int seg = g.T / 64, t0 = lane * seg;
  const int64_t base = (int64_t)bh * g.T;
  float tot = 0.0f;
  for (int t = t0 + seg - 1; t >= t0; --t) tot += g.qdq[base + t] - g.kdk[base + t];
  // suffix over the lanes above: inclusive prefix sum of the reversed lane order, minus own
  float above = 0.0f;
  {
    float x = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const float u = __shfl_down(x, d);
      if (lane + d < 64) x += u;
    }
    above = x - tot;
  }
  const int b = bh / g.NH, h = bh % g.NH;
  float run = above;
  for (int t = t0 + seg - 1; t >= t0; --t) {
    run += g.qdq[base + t] - g.kdk[base + t];
    const float dfg = run / (1.0f + expf(g.fg[base + t]));   // sigmoid(-f) R, as 1 / (1 + e^f)
    if (g.dfg) {
      g.dfg[base + t] = dfg;
    } else {
      const int64_t row = ((int64_t)b * g.T + t) * g.ld;
      const float xi = (float)g.a[row + g.io + h], xf = (float)g.a[row + g.fo + h];
      g.da[row + g.io + h] = (__bf16)softcap_bwd(g.kdk[base + t], xi, g.cap);
      g.da[row + g.fo + h] = (__bf16)softcap_bwd(dfg, xf, g.cap);
    }
  }
}

}  // namespace

}  // namespace sc

using namespace sc;

extern "C" int sc_mlstm_supported(int dtype, int DQ, int DV) {
  return (dtype == SC_BF16 || dtype == SC_F16) && dims_supported(DQ, DV);
}

extern "C" int64_t sc_mlstm_chunk_state_numel(int BH, int T, int DQ, int DV) {
  if (BH <= 0 || T <= 0 || DQ <= 0 || DV <= 0) return 0;
  return (int64_t)BH * (T / kL) * DQ * DV;
}

extern "C" int sc_mlstm_fwd_io(const void* q, const void* k, const void* v, int dtype,
                               int io_dtype,
                            const float* igate, const float* fgate, const float* c0,
                            const float* n0, const float* m0, int BH, int T, int DQ, int DV,
                            float eps, void* h, void* states_C, float* states_n,
                            float* states_m, float* c_last, float* m_rows, float* den_rows,
                            const int64_t* layout, void* stream) {
  clear_error();
  SC_REQUIRE(io_supported(dtype, io_dtype),
             "sc_mlstm_fwd: dtype %d / operand dtype %d (bf16/bf16, f16/f16, f16/bf16 only)", dtype,
             io_dtype);
  SC_REQUIRE(BH >= 0 && T >= 0, "sc_mlstm_fwd: bad shape");
  SC_REQUIRE(T % kL == 0, "sc_mlstm_fwd: T=%d is not a multiple of the chunk length %d", T, kL);
  SC_REQUIRE(dims_supported(DQ, DV), "sc_mlstm_fwd: head dims (%d, %d) not compiled in", DQ, DV);
  if (BH == 0 || T == 0) return 0;
  SC_REQUIRE(q && k && v && igate && fgate && h && states_C && states_n && states_m && c_last &&
                 m_rows && den_rows,
             "sc_mlstm_fwd: null pointer");
  MArgs a{};
  a.q = q; a.k = k; a.v = v; a.ig = igate; a.fg = fgate; a.c0 = c0; a.n0 = n0; a.m0 = m0;
  a.Cs = states_C; a.ns = states_n; a.ms = states_m; a.c_last = c_last; a.h = h; a.mrow = m_rows;
  a.den = den_rows;
  a.BH = BH; a.T = T; a.nc = T / kL; a.eps = eps; a.scale = 1.0f / sqrtf((float)DQ);
  if (int rc = set_layout(a, layout, DQ, DV, "sc_mlstm_fwd", {q, k, v})) return rc;
  hipStream_t st = (hipStream_t)stream;
  dispatch_io(a, dtype, io_dtype, DQ, DV, false, st);
  return launch_status("sc_mlstm_fwd");
}

extern "C" int sc_mlstm_fwd(const void* q, const void* k, const void* v, int dtype,
                            const float* igate, const float* fgate, const float* c0,
                            const float* n0, const float* m0, int BH, int T, int DQ, int DV,
                            float eps, void* h, void* states_C, float* states_n,
                            float* states_m, float* c_last, float* m_rows, float* den_rows,
                            const int64_t* layout, void* stream) {
  return sc_mlstm_fwd_io(q, k, v, dtype, dtype, igate, fgate, c0, n0, m0, BH, T, DQ, DV, eps, h,
                         states_C, states_n, states_m, c_last, m_rows, den_rows, layout, stream);
}

extern "C" int sc_mlstm_bwd_io(const void* q, const void* k, const void* v, int dtype,
                               int io_dtype,
                            const float* igate, const float* fgate, const void* h,
                            const void* dh, const float* dcT, const float* dnT,
                            const void* states_C, const float* states_n, const float* states_m,
                            const float* m_rows, const float* den_rows, int BH, int T, int DQ,
                            int DV, float eps, float* dstates_C, float* dstates_n, void* dq,
                            void* dk, void* dv, float* qdq, float* kdk, const int64_t* layout,
                            void* stream) {
  clear_error();
  SC_REQUIRE(io_supported(dtype, io_dtype),
             "sc_mlstm_bwd: dtype %d / operand dtype %d (bf16/bf16, f16/f16, f16/bf16 only)", dtype,
             io_dtype);
  SC_REQUIRE(T % kL == 0, "sc_mlstm_bwd: T=%d is not a multiple of the chunk length %d", T, kL);
  SC_REQUIRE(dims_supported(DQ, DV), "sc_mlstm_bwd: head dims (%d, %d) not compiled in", DQ, DV);
  if (BH == 0 || T == 0) return 0;
  SC_REQUIRE(q && k && v && igate && fgate && h && dh && states_C && states_n && states_m &&
                 m_rows && den_rows && dstates_C && dstates_n && dq && dk && dv && qdq && kdk,
             "sc_mlstm_bwd: null pointer");
  MArgs a{};
  a.q = q; a.k = k; a.v = v; a.ig = igate; a.fg = fgate; a.h = (void*)h; a.dh = dh;
  a.dcT = dcT; a.dnT = dnT; a.Cs = (void*)states_C; a.ns = (float*)states_n;
  a.ms = (float*)states_m; a.mrow = (float*)m_rows; a.den = (float*)den_rows;
  a.dCs = dstates_C; a.dns = dstates_n; a.dq = dq; a.dk = dk; a.dv = dv; a.qdq = qdq; a.kdk = kdk;
  a.BH = BH; a.T = T; a.nc = T / kL; a.eps = eps; a.scale = 1.0f / sqrtf((float)DQ);
  if (int rc = set_layout(a, layout, DQ, DV, "sc_mlstm_bwd", {q, k, v, dq, dk, dv})) return rc;
  hipStream_t st = (hipStream_t)stream;
  dispatch_io(a, dtype, io_dtype, DQ, DV, true, st);
  return launch_status("sc_mlstm_bwd");
}

extern "C" int sc_mlstm_bwd(const void* q, const void* k, const void* v, int dtype,
                            const float* igate, const float* fgate, const void* h,
                            const void* dh, const float* dcT, const float* dnT,
                            const void* states_C, const float* states_n, const float* states_m,
                            const float* m_rows, const float* den_rows, int BH, int T, int DQ,
                            int DV, float eps, float* dstates_C, float* dstates_n, void* dq,
                            void* dk, void* dv, float* qdq, float* kdk, const int64_t* layout,
                            void* stream) {
  return sc_mlstm_bwd_io(q, k, v, dtype, dtype, igate, fgate, h, dh, dcT, dnT, states_C,
                         states_n, states_m, m_rows, den_rows, BH, T, DQ, DV, eps, dstates_C,
                         dstates_n, dq, dk, dv, qdq, kdk, layout, stream);
}

extern "C" int sc_mlstm_gate_bwd(const float* qdq, const float* kdk, const float* fgate, int BH,
                                 int T, float* dfgate, const void* a, void* da, int NH,
                                 int64_t ld, int io, int fo, float cap, void* stream) {
  clear_error();
  SC_REQUIRE(BH >= 0 && T >= 0 && T % 64 == 0, "sc_mlstm_gate_bwd: T=%d (a multiple of 64)", T);
  if (BH == 0 || T == 0) return 0;
  SC_REQUIRE(qdq && kdk && fgate, "sc_mlstm_gate_bwd: null input");
  SC_REQUIRE((dfgate != nullptr) != (da != nullptr), "sc_mlstm_gate_bwd: exactly one output mode");
  if (da) {
    SC_REQUIRE(a && NH > 0 && BH % NH == 0 && io >= 0 && fo >= 0 && ld >= fo + NH && ld >= io + NH,
               "sc_mlstm_gate_bwd: projection layout");
  }
  GateArgs g{qdq, kdk, fgate, dfgate, (const __bf16*)a, (__bf16*)da, BH, T, NH > 0 ? NH : 1,
             io, fo, ld, cap};
  hipLaunchKernelGGL(mlstm_gate_bwd_kernel, dim3(BH), dim3(64), 0, (hipStream_t)stream, g);
  return launch_status("sc_mlstm_gate_bwd");
}
