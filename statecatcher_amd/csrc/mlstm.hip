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
// Kernels (one 4-wave workgroup each; 16x16x32 bf16/f16 MFMA, fp32 accumulation, fp32 state):
//   mlstm_fw_walk per (b,h, 64-column block of C~): walks the chunks in order with the state
//                block in MFMA accumulators; per chunk S = Q K^T, causal decay mask,
//                H[:, block] = M V[:, block] + Q~ C~_k[:, block], normaliser (S and the
//                normaliser recomputed per block), then the state update.  Keeps m_t, den_t and
//                the compute-dtype image of every chunk-start state for the backward.
//   mlstm_bw_dC  per (b,h): reverse walk, dC~_k = e^{g+m_k-m_{k+1}} dC~_{k+1} + Q~^T dnum
//   mlstm_bw_dQ / _dK / _dV  per (b,h,chunk): the three input gradients (intra-chunk terms
//                through dA = W o (dnum V^T + dden), inter-chunk terms through C~_k / dC~_{k+1})
// The stabiliser m is treated as a constant in the backward (it cancels in h up to the eps
// term), as the chunkwise kernels of the mlstm_kernels family do.  Gate gradients follow from
// the pair identities  di_s = k_s.dk_s  and  dF_t = q_t.dq_t - k_t.dk_t  (F = cumulative
// logsig(f)): the kernels emit the two dot products, the host turns dF into df by a reverse
// cumulative sum times sigmoid(-f).
#include <initializer_list>

#include "sc_common.h"

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
  float* dCs;       // [BH][nc+1][DQ][DV]: gradient w.r.t. C~_k (dCs[0] = dC0)
  float* dns;       // [BH][nc+1][DQ]
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

// Gate prefix quantities of one chunk, computed by wave 0 (lane = step s) into LDS:
// sb[s] = b_s (inclusive cumulative logsig f), si[s] = i_s; returns g = b_{L-1} in every lane
// of wave 0 (others get 0).
__device__ __forceinline__ void chunk_gates(const MArgs& a, int bh, int k, float* sb, float* si,
                                            int tid) {
  if (tid < 64) {
    const int64_t o = (int64_t)bh * a.T + k * kL + tid;
    const float i = a.ig[o];
    float b = logsig(a.fg[o]);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const float u = __shfl_up(b, d);
      if (tid >= d) b += u;
    }
    sb[tid] = b;
    si[tid] = i;
  }
}

// inclusive prefix max over the 64 lanes of a wave
__device__ __forceinline__ float wave_prefix_max(float x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float u = __shfl_up(x, d);
    if (lane >= d) x = fmaxf(x, u);
  }
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}
// sum over the 16 lanes that share (lane >> 4) — the columns of one accumulator row group
__device__ __forceinline__ float sum16(float x) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) x += __shfl_xor(x, o);
  return x;
}

// Column block of the state: C~'s columns evolve independently (C~ += K^T diag(f) V), so each
// workgroup owns kCB = 64 columns of one (b,h) -- DV/64 x BH workgroups instead of BH; n~ and m
// are recomputed by every block (they need K and the gates only) and stored by block 0.
constexpr int kCB = 64;

// ------------------------------------------------------------------------- forward: walk ----
// One workgroup per (b,h, 64-column block of C~) walks the chunks in order and does both halves
// of the chunkwise forward for its columns: the chunk's outputs H[:, block] (S = Q K^T, causal
// decay mask, M V + Q~ C~_k, normaliser) and the state update C~_{k+1}[:, block].  The state block
// never leaves the MFMA accumulators: only its bf16 / f16 image (what the Q~ C~_k MFMA consumes,
// kept for the backward's dq) and n~, m go to HBM -- no fp32 state stream and no re-read of it.
template <int DT, int DQ, int DV>
__global__ void __launch_bounds__(256, 2) mlstm_fw_walk(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  constexpr int TJ = kCB / 16, NT = (DQ / 16) * TJ, PW = NT / 4;
  static_assert(NT % 4 == 0, "tile count must split over 4 waves");
  const int cb = blockIdx.x, bh = blockIdx.y, w = threadIdx.x >> 6;
  int tid = threadIdx.x, lane = tid & 63;
  const int cj0 = cb * kCB;
  __shared__ __attribute__((aligned(16))) T Qs[kL * (DQ + kPad)];
  __shared__ __attribute__((aligned(16))) T Ks[kL * (DQ + kPad)];
  __shared__ __attribute__((aligned(16))) T KT[DQ * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T VT[kCB * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T Ms[kL * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T CT[kCB * (DQ + kPad)];
  __shared__ float sb[kL], si[kL], mt[kL], rowf[kL], fs[kL], dsum[kL], qn[kL], nk[DQ], scal[2];
  const T* Q = (const T*)a.q + qrow(a, bh, 0);
  const T* K = (const T*)a.k + qrow(a, bh, 0);
  const T* V = (const T*)a.v + vrow(a, bh, 0);
  T* H = (T*)a.h + (int64_t)bh * a.T * DV;
  f32x4 acc[PW];
#pragma unroll
  for (int p = 0; p < PW; ++p) {
    const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = cj0 + 16 * (q % TJ);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r, j = j0 + (lane & 15);
      acc[p][r] = a.c0 ? a.c0[((int64_t)bh * DQ + i) * DV + j] : 0.0f;
    }
  }
  float n = (tid < DQ && a.n0) ? a.n0[(int64_t)bh * DQ + tid] : 0.0f;
  float m = a.m0 ? a.m0[bh] : 0.0f;
  // chunk inputs are prefetched into registers one chunk ahead: the loads of chunk k + 1 are
  // issued right after chunk k's are written to LDS and land while chunk k computes (issued
  // and waited per loader loop they cost a full memory latency each, four times per chunk)
  constexpr int NQP = kL * DQ / 8 / 256, NVP = kL * kCB / 8 / 256;
  static_assert(NQP * 256 * 8 == kL * DQ && NVP * 256 * 8 == kL * kCB, "piece split");
  u32x4 pq[NQP], pk[NQP], pv[NVP];
  float pig = 0.0f, pfg = 0.0f;
  auto prefetch = [&](int kc) __attribute__((always_inline)) {
    const int64_t tb = (int64_t)kc * kL;
#pragma unroll
    for (int u = 0; u < NQP; ++u) {
      const int e = tid + 256 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
      pq[u] = *(const u32x4*)(Q + (tb + r) * a.qt + c);
      pk[u] = *(const u32x4*)(K + (tb + r) * a.qt + c);
    }
#pragma unroll
    for (int u = 0; u < NVP; ++u) {
      const int e = tid + 256 * u, r = e % kL, c = (e / kL) * 8;
      pv[u] = *(const u32x4*)(V + (tb + r) * a.vt + cj0 + c);
    }
    if (tid < 64) {
      const int64_t o = (int64_t)bh * a.T + tb + tid;
      pig = a.ig[o];
      pfg = a.fg[o];
    }
  };
  prefetch(0);
  for (int k = 0; k < a.nc; ++k) {
    const int64_t t0 = (int64_t)k * kL;
    // re-derive the lane-dependent addresses every chunk instead of holding dozens of them in
    // VGPRs across the loop (hoisted, they pushed the prefetch registers out to scratch)
    asm volatile("" : "+v"(tid), "+v"(lane));
#pragma unroll
    for (int u = 0; u < NQP; ++u) {
      const int e = tid + 256 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
      *(u32x4*)(Qs + r * (DQ + kPad) + c) = pq[u];
      *(u32x4*)(Ks + r * (DQ + kPad) + c) = pk[u];
      const V8 x = __builtin_bit_cast(V8, pk[u]);
#pragma unroll
      for (int j = 0; j < 8; ++j) KT[(c + j) * (kL + kPad) + r] = x[j];
    }
#pragma unroll
    for (int u = 0; u < NVP; ++u) {
      const int e = tid + 256 * u, r = e % kL, c = (e / kL) * 8;
      const V8 x = __builtin_bit_cast(V8, pv[u]);
#pragma unroll
      for (int j = 0; j < 8; ++j) VT[(c + j) * (kL + kPad) + r] = x[j];
    }
    if (tid < 64) {   // chunk_gates on the prefetched pre-activations
      float b = logsig(pfg);
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const float u = __shfl_up(b, d);
        if (tid >= d) b += u;
      }
      sb[tid] = b;
      si[tid] = pig;
    }
    if (k + 1 < a.nc) prefetch(k + 1);
    // the state at the chunk start: its MFMA image, transposed ([j][i]); a lane's four
    // accumulator rows are consecutive i, so each tile is one 8-byte LDS store
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
      typedef T v4 __attribute__((ext_vector_type(4)));
      v4 c;
#pragma unroll
      for (int r = 0; r < 4; ++r) c[r] = (T)acc[p][r];
      *(v4*)(CT + (j0 + (lane & 15)) * (DQ + kPad) + i0 + 4 * (lane >> 4)) = c;
    }
    if (tid < DQ) {
      nk[tid] = n;
      if (cb == 0) a.ns[((int64_t)bh * (a.nc + 1) + k) * DQ + tid] = n;
    }
    if (cb == 0 && tid == 0) a.ms[(int64_t)bh * (a.nc + 1) + k] = m;
    if (tid < 64) {   // wave 0: row stabilisers, output scale, state-update key weights
      const float bt = sb[tid];
      const float mi = bt + wave_prefix_max(si[tid] - bt, tid);
      const float m_t = fmaxf(bt + m, mi);
      mt[tid] = m_t;
      rowf[tid] = a.scale * expf(bt + m - m_t);
      const float g = __shfl(bt, 63);
      const float as = g - bt + si[tid];
      const float mn = fmaxf(g + m, wave_max(as));
      fs[tid] = expf(as - mn);
      if (tid == 0) {
        scal[0] = expf(g + m - mn);
        scal[1] = mn;
      }
    }
    __syncthreads();
    // the backward's copy of the chunk-start state: CT's rows as they are, [j][i] (16-byte stores)
    {
      T* Cs = (T*)a.Cs + (((int64_t)bh * a.nc + k) * DV + cj0) * DQ;
      constexpr int NCP = kCB * DQ / 8 / 256;
      static_assert(NCP * 256 * 8 == kCB * DQ, "state image split");
#pragma unroll
      for (int u = 0; u < NCP; ++u) {
        const int e = tid + 256 * u, j = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
        *(u32x4*)(Cs + j * DQ + c) = *(const u32x4*)(CT + j * (DQ + kPad) + c);
      }
    }
    // From here to the state update every wave touches only its own 16 rows of Ms / qn / dsum
    // (rows 16 w ..): no barrier between the S and H phases.
    // q_t . n~_k (4 threads per row, DQ / 4 consecutive i each)
    {
      constexpr int QP = DQ / 4;
      const int t = tid >> 2, part = tid & 3;
      float qa = 0.0f;
#pragma unroll
      for (int u = 0; u < QP / 8; ++u) {
        const V8 x = *(const V8*)(Qs + t * (DQ + kPad) + part * QP + 8 * u);
#pragma unroll
        for (int e = 0; e < 8; ++e) qa += (float)x[e] * nk[part * QP + 8 * u + e];
      }
      qa += __shfl_xor(qa, 1);
      qa += __shfl_xor(qa, 2);
      if (part == 0) qn[t] = qa;
    }
    // S = Q K^T for row block w, causal column blocks; M = S o W into LDS, row sums
    {
      float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int ct = 0; ct <= w; ++ct) {
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk)
          s4 = M::mma(frag<V8, T>(Qs, DQ + kPad, 16 * w, 32 * kk, lane),
                      frag<V8, T>(Ks, DQ + kPad, 16 * ct, 32 * kk, lane), s4);
        const int s = 16 * ct + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = 16 * w + 4 * (lane >> 4) + r;
          const float mv = (s <= t) ? s4[r] * a.scale * expf(sb[t] - sb[s] + si[s] - mt[t]) : 0.0f;
          rs[r] += mv;
          Ms[t * (kL + kPad) + s] = (T)mv;
        }
      }
      // the column blocks right of the diagonal: zero (the H MFMA reads them)
      for (int ct = w + 1; ct < 4; ++ct) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Ms[(16 * w + 4 * (lane >> 4) + r) * (kL + kPad) + 16 * ct + (lane & 15)] = (T)0.0f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float tot = sum16(rs[r]);
        if ((lane & 15) == 0) dsum[16 * w + 4 * (lane >> 4) + r] = tot;
      }
    }
    // H = M V + (rowf Q) C~_k for row block w, normalised; staged in the wave's own Ms rows
    // (every cj has read them first) and stored as 16-byte rows
    {
      const float rf = rowf[16 * w + (lane & 15)];
      const int kin = (16 * (w + 1) + 31) / 32;
      float zi[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * w + 4 * (lane >> 4) + r;
        const float dn = dsum[t] + rowf[t] * qn[t];
        zi[r] = 1.0f / (fmaxf(fabsf(dn), expf(-mt[t])) + a.eps);
      }
      f32x4 hv[TJ];
#pragma unroll
      for (int cj = 0; cj < TJ; ++cj) {
        f32x4 h4 = {0.f, 0.f, 0.f, 0.f};
        for (int kk = 0; kk < kin; ++kk)
          h4 = M::mma(frag<V8, T>(Ms, kL + kPad, 16 * w, 32 * kk, lane),
                      frag<V8, T>(VT, kL + kPad, 16 * cj, 32 * kk, lane), h4);
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk)
          h4 = M::mma(frag_rs<V8, T>(Qs, DQ + kPad, 16 * w, 32 * kk, lane, rf),
                      frag<V8, T>(CT, DQ + kPad, 16 * cj, 32 * kk, lane), h4);
        hv[cj] = h4;
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int cj = 0; cj < TJ; ++cj) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Ms[(16 * w + 4 * (lane >> 4) + r) * (kL + kPad) + 16 * cj + (lane & 15)] =
              (T)(hv[cj][r] * zi[r]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {   // 16 rows x 128 bytes = 128 pieces over 64 lanes
        const int e = lane + 64 * u, t = 16 * w + (e >> 3), c = (e & 7) * 8;
        *(u32x4*)(H + (t0 + t) * DV + cj0 + c) = *(const u32x4*)(Ms + t * (kL + kPad) + c);
      }
      if (cb == 0 && lane < 16) {   // the wave's own rows
        const int t = 16 * w + lane;
        a.mrow[(int64_t)bh * a.T + t0 + t] = mt[t];
        a.den[(int64_t)bh * a.T + t0 + t] = dsum[t] + rowf[t] * qn[t];
      }
    }
    // state update: C~ <- decay C~ + (fs K)^T V[:, block];  n~ likewise
    const float decay = scal[0];
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
      f32x4 c = acc[p] * decay;
#pragma unroll
      for (int kk = 0; kk < kL / 32; ++kk)
        c = M::mma(frag_ks<V8, T>(KT, kL + kPad, i0, 32 * kk, lane, fs),
                   frag<V8, T>(VT, kL + kPad, j0, 32 * kk, lane), c);
      acc[p] = c;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (tid < DQ) {
      float sacc = 0.0f;
#pragma unroll
      for (int u = 0; u < kL / 8; ++u) {
        const V8 x = *(const V8*)(KT + tid * (kL + kPad) + 8 * u);
#pragma unroll
        for (int e = 0; e < 8; ++e) sacc += fs[8 * u + e] * (float)x[e];
      }
      n = decay * n + sacc;
    }
    m = scal[1];
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
  if (cb == 0) {
    if (tid < DQ) a.ns[((int64_t)bh * (a.nc + 1) + a.nc) * DQ + tid] = n;
    if (tid == 0) a.ms[(int64_t)bh * (a.nc + 1) + a.nc] = m;
  }
}

// ------------------------------------------------------------------------- backward: walk ----
// One 8-wave workgroup per sequence (b,h) walks the chunks in REVERSE with the state gradient
// dC~ [DQ][DV] (fp32) in MFMA accumulators, and per chunk computes all three input gradients:
//   dq_t = sum_s dA_ts k_s + rowf_t dnum_t C~_k^T + rowf_t dden_t n~_k
//   dk_s = sum_t dA_ts q_t + es_s v_s dC~_{k+1}^T + es_s dn~_{k+1}
//   dv_s = sum_t A_ts dnum_t + es_s k_s dC~_{k+1}
//   dC~_k = decay dC~_{k+1} + (rowf q)^T dnum,   dn~_k = decay dn~_{k+1} + sum_t rowf_t dden_t q_t
// (dA_ts = W_ts (dnum_t . v_s + dden_t), A_ts = W_ts q_t . k_s, W_ts = s e^{b_t - b_s + i_s - m_t},
// s <= t).  Every operand lives in LDS once, row-major; MFMA fragments that run along a column
// come out through ds_read_b64_tr_b16 (transposed reads), so no transposed copies are stored.
// C~_k is the forward's compute-dtype image; dC~_{k+1}'s image replaces it in LDS once the dq
// terms are done.  Nothing of size T x DQ x DV goes to HBM: the chunk states of the gradient
// stay on chip (the gradient w.r.t. the initial state is the only state output).
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

template <int DT, int DQ, int DV>
__global__ void __launch_bounds__(512, 1) mlstm_bw_walk(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  constexpr int LQ = DQ + kPad, LV = DV + kPad, LL = kL + kPad;
  constexpr int NI = DQ / 16, NJ = DV / 16;       // tile counts along DQ, DV
  constexpr int NC = NI * NJ;                     // state tiles
  static_assert(NC % 8 == 0, "state tiles must split over 8 waves");
  constexpr int PC = NC / 8;
  const int bh = blockIdx.x, w = threadIdx.x >> 6;
  int tid = threadIdx.x, lane = tid & 63;
  __shared__ __attribute__((aligned(16))) T Qs[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Ks[kL * LQ];
  __shared__ __attribute__((aligned(16))) T Vs[kL * LV];
  __shared__ __attribute__((aligned(16))) T Dn[kL * LV];
  __shared__ __attribute__((aligned(16))) T CS[DV * LQ];   // C~_k, then dC~_{k+1}, [j][i]
  __shared__ __attribute__((aligned(16))) T dA[kL * LL];
  __shared__ __attribute__((aligned(16))) T Am[kL * LL];
  __shared__ float sb[kL], si[kL], mt[kL], rowf[kL], es[kL], dden[kL], nk[DQ], dnk[DQ];
  __shared__ float qpart[NI * kL], kpart[NI * kL], scal[1];
  // dC~ tiles q = w + 8 p: rows i0 = 16 (q / NJ), cols j0 = 16 (q % NJ)
  f32x4 acc[PC];
#pragma unroll
  for (int p = 0; p < PC; ++p) {
    const int q = w + 8 * p, i0 = 16 * (q / NJ), j0 = 16 * (q % NJ);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r, j = j0 + (lane & 15);
      acc[p][r] = a.dcT ? a.dcT[((int64_t)bh * DQ + i) * DV + j] : 0.0f;
    }
  }
  float dn = (tid < DQ && a.dnT) ? a.dnT[(int64_t)bh * DQ + tid] : 0.0f;
  const T* Qg = (const T*)a.q + qrow(a, bh, 0);
  const T* Kg = (const T*)a.k + qrow(a, bh, 0);
  const T* Vg = (const T*)a.v + vrow(a, bh, 0);
  T* dQg = (T*)a.dq + qrow(a, bh, 0);
  T* dKg = (T*)a.dk + qrow(a, bh, 0);
  T* dVg = (T*)a.dv + vrow(a, bh, 0);
  for (int k = a.nc - 1; k >= 0; --k) {
    const int64_t t0 = (int64_t)k * kL;
    asm volatile("" : "+v"(tid), "+v"(lane));   // see mlstm_fw_walk
    // ---- chunk inputs: every global load of the chunk issued before any LDS store (one
    // memory latency per chunk, not one per operand) ----
    {
      constexpr int NQ8 = kL * DQ / 8, NV8 = kL * DV / 8, NC8 = DQ * DV / 8;
      constexpr int UQ = (NQ8 + 511) / 512, UV = (NV8 + 511) / 512, UC = (NC8 + 511) / 512;
      constexpr int UH = DV / 64;   // dh / h pieces per thread (8 threads per row)
      u32x4 rq[UQ], rk[UQ], rv[UV], rc[UC], rd[UH], rh[UH];
      const T* Ck = (const T*)a.Cs + ((int64_t)bh * a.nc + k) * DQ * DV;
      const int t = tid >> 3, part = tid & 7;
      const int64_t ro = (int64_t)bh * a.T + t0 + t;
      const T* dh = (const T*)a.dh + ro * DV;
      const T* h = (const T*)a.h + ro * DV;
#pragma unroll
      for (int u = 0; u < UQ; ++u) {
        const int e = tid + 512 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
        if (e < NQ8) {
          rq[u] = *(const u32x4*)(Qg + (t0 + r) * a.qt + c);
          rk[u] = *(const u32x4*)(Kg + (t0 + r) * a.qt + c);
        }
      }
#pragma unroll
      for (int u = 0; u < UV; ++u) {
        const int e = tid + 512 * u, r = e / (DV / 8), c = (e % (DV / 8)) * 8;
        if (e < NV8) rv[u] = *(const u32x4*)(Vg + (t0 + r) * a.vt + c);
      }
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int e = tid + 512 * u;
        if (e < NC8) rc[u] = *(const u32x4*)(Ck + 8 * e);
      }
#pragma unroll
      for (int u = 0; u < UH; ++u) {
        rd[u] = *(const u32x4*)(dh + part * 8 + 64 * u);
        rh[u] = *(const u32x4*)(h + part * 8 + 64 * u);
      }
      const float m_t = a.mrow[ro], dv_ = a.den[ro];
#pragma unroll
      for (int u = 0; u < UQ; ++u) {
        const int e = tid + 512 * u, r = e / (DQ / 8), c = (e % (DQ / 8)) * 8;
        if (e < NQ8) {
          *(u32x4*)(Qs + r * LQ + c) = rq[u];
          *(u32x4*)(Ks + r * LQ + c) = rk[u];
        }
      }
#pragma unroll
      for (int u = 0; u < UV; ++u) {
        const int e = tid + 512 * u, r = e / (DV / 8), c = (e % (DV / 8)) * 8;
        if (e < NV8) *(u32x4*)(Vs + r * LV + c) = rv[u];
      }
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int e = tid + 512 * u;
        if (e < NC8) {
          const int j = (8 * e) / DQ, i = (8 * e) % DQ;
          *(u32x4*)(CS + j * LQ + i) = rc[u];
        }
      }
      // dnum = dh / z and dden (8 threads per row)
      const float z = fmaxf(fabsf(dv_), expf(-m_t)) + a.eps;
      float dot = 0.0f;
#pragma unroll
      for (int u = 0; u < UH; ++u) {
        const V8 xd = __builtin_bit_cast(V8, rd[u]);
        const V8 xh = __builtin_bit_cast(V8, rh[u]);
        V8 o;
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) {
          const float d = (float)xd[e2];
          dot += d * (float)xh[e2];
          o[e2] = (T)(d / z);
        }
        *(V8*)(Dn + t * LV + part * 8 + 64 * u) = o;
      }
      dot += __shfl_xor(dot, 1);
      dot += __shfl_xor(dot, 2);
      dot += __shfl_xor(dot, 4);
      if (part == 0) {
        const float live = fabsf(dv_) >= expf(-m_t) ? 1.0f : 0.0f;
        dden[t] = -dot / z * (dv_ >= 0.0f ? 1.0f : -1.0f) * live;
        mt[t] = m_t;
      }
    }
    if (tid < DQ) {
      nk[tid] = a.ns[((int64_t)bh * (a.nc + 1) + k) * DQ + tid];
      dnk[tid] = dn;
    }
    chunk_gates(a, bh, k, sb, si, tid);
    if (tid < 64) {   // wave 0 wrote sb / si; mt comes from the row threads (a barrier below)
      const int64_t st = (int64_t)bh * (a.nc + 1) + k;
      const float mk = a.ms[st], mk1 = a.ms[st + 1];
      const float g = __shfl(sb[tid], 63);
      const float m_t = a.mrow[(int64_t)bh * a.T + t0 + tid];
      rowf[tid] = a.scale * expf(sb[tid] + mk - m_t);
      es[tid] = expf(g - sb[tid] + si[tid] - mk1);
      if (tid == 0) scal[0] = expf(g + mk - mk1);
    }
    __syncthreads();
    // ---- A = W o (Q K^T) and dA = W o (Dn V^T + dden): 10 causal tiles each, 20 jobs ----
#pragma unroll 1
    for (int jb = w; jb < 20; jb += 8) {
      const bool isA = jb < 10;
      const int idx = isA ? jb : jb - 10;
      // idx -> (tr, tc), tc <= tr: 0 (0,0) 1 (1,0) 2 (1,1) 3 (2,0) 4 (2,1) 5 (2,2) 6.. (3,*)
      const int tr = idx < 1 ? 0 : idx < 3 ? 1 : idx < 6 ? 2 : 3;
      const int tc = idx - tr * (tr + 1) / 2;
      f32x4 c4 = {0.f, 0.f, 0.f, 0.f};
      if (isA) {
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk)
          c4 = M::mma(frag<V8, T>(Qs, LQ, 16 * tr, 32 * kk, lane),
                      frag<V8, T>(Ks, LQ, 16 * tc, 32 * kk, lane), c4);
      } else {
#pragma unroll
        for (int kk = 0; kk < DV / 32; ++kk)
          c4 = M::mma(frag<V8, T>(Dn, LV, 16 * tr, 32 * kk, lane),
                      frag<V8, T>(Vs, LV, 16 * tc, 32 * kk, lane), c4);
      }
      const int s = 16 * tc + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * tr + 4 * (lane >> 4) + r;
        const float wts = (s <= t) ? a.scale * expf(sb[t] - sb[s] + si[s] - mt[t]) : 0.0f;
        if (isA) Am[t * LL + s] = (T)(c4[r] * wts);
        else dA[t * LL + s] = (T)((c4[r] + dden[t]) * wts);
      }
    }
    // zero the strictly upper tiles (tc > tr) of A and dA once (they stay zero across chunks)
    if (k == a.nc - 1) {
      for (int e = tid; e < kL * kL; e += 512) {
        const int t = e / kL, s = e % kL;
        if ((s >> 4) > (t >> 4)) {
          Am[t * LL + s] = (T)0.0f;
          dA[t * LL + s] = (T)0.0f;
        }
      }
    }
    __syncthreads();
    // ---- dq = dA K + rowf (Dn C~_k^T) + rowf dden n~_k: 4 x NI tiles ----
#pragma unroll 1
    for (int jb = w; jb < 4 * NI; jb += 8) {
      const int tr = jb / NI, ci = jb % NI;
      f32x4 d4 = {0.f, 0.f, 0.f, 0.f};
      for (int kk = 0; kk <= (16 * tr + 15) / 32; ++kk)   // causal: s <= t
        d4 = M::mma(frag<V8, T>(dA, LL, 16 * tr, 32 * kk, lane),
                    frag_t<V8, T>(Ks, LQ, 32 * kk, 16 * ci, lane), d4);
      const float rf = rowf[16 * tr + (lane & 15)];
#pragma unroll
      for (int kk = 0; kk < DV / 32; ++kk)
        d4 = M::mma(frag_rs<V8, T>(Dn, LV, 16 * tr, 32 * kk, lane, rf),
                    frag_t<V8, T>(CS, LQ, 32 * kk, 16 * ci, lane), d4);
      const int i = 16 * ci + (lane & 15);
      float qd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * tr + 4 * (lane >> 4) + r;
        const float v = d4[r] + rowf[t] * dden[t] * nk[i];
        dQg[(t0 + t) * a.qt + i] = (T)v;
        qd[r] = sum16(v * (float)Qs[t * LQ + i]);
      }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) qpart[ci * kL + 16 * tr + 4 * (lane >> 4) + r] = qd[r];
      }
    }
    __syncthreads();
    // ---- dC~_{k+1} image replaces C~_k ----
#pragma unroll
    for (int p = 0; p < PC; ++p) {
      const int q = w + 8 * p, i0 = 16 * (q / NJ), j0 = 16 * (q % NJ);
      typedef T v4 __attribute__((ext_vector_type(4)));
      v4 c;
#pragma unroll
      for (int r = 0; r < 4; ++r) c[r] = (T)acc[p][r];
      *(v4*)(CS + (j0 + (lane & 15)) * LQ + i0 + 4 * (lane >> 4)) = c;
    }
    if (tid < kL) {
      float sq = 0.0f;
#pragma unroll
      for (int ci = 0; ci < NI; ++ci) sq += qpart[ci * kL + tid];
      a.qdq[(int64_t)bh * a.T + t0 + tid] = sq;
    }
    __syncthreads();
    // ---- dk = dA^T Q + es (V dC~^T) + es dn~: 4 x NI tiles; dv = A^T Dn + es (K dC~): 4 x NJ ----
#pragma unroll 1
    for (int jb = w; jb < 4 * NI + 4 * NJ; jb += 8) {
      f32x4 d4 = {0.f, 0.f, 0.f, 0.f};
      if (jb < 4 * NI) {
        const int sr = jb / NI, ci = jb % NI;
        for (int kk = (16 * sr) / 32; kk < kL / 32; ++kk)   // causal: t >= s
          d4 = M::mma(frag_t<V8, T>(dA, LL, 32 * kk, 16 * sr, lane),
                      frag_t<V8, T>(Qs, LQ, 32 * kk, 16 * ci, lane), d4);
        const float ef = es[16 * sr + (lane & 15)];
#pragma unroll
        for (int kk = 0; kk < DV / 32; ++kk)
          d4 = M::mma(frag_rs<V8, T>(Vs, LV, 16 * sr, 32 * kk, lane, ef),
                      frag_t<V8, T>(CS, LQ, 32 * kk, 16 * ci, lane), d4);
        const int i = 16 * ci + (lane & 15);
        float kd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = 16 * sr + 4 * (lane >> 4) + r;
          const float v = d4[r] + es[s] * dnk[i];
          dKg[(t0 + s) * a.qt + i] = (T)v;
          kd[r] = sum16(v * (float)Ks[s * LQ + i]);
        }
        if ((lane & 15) == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) kpart[ci * kL + 16 * sr + 4 * (lane >> 4) + r] = kd[r];
        }
      } else {
        const int jv = jb - 4 * NI, sr = jv / NJ, cj = jv % NJ;
        for (int kk = (16 * sr) / 32; kk < kL / 32; ++kk)
          d4 = M::mma(frag_t<V8, T>(Am, LL, 32 * kk, 16 * sr, lane),
                      frag_t<V8, T>(Dn, LV, 32 * kk, 16 * cj, lane), d4);
        const float ef = es[16 * sr + (lane & 15)];
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk)
          d4 = M::mma(frag_rs<V8, T>(Ks, LQ, 16 * sr, 32 * kk, lane, ef),
                      frag<V8, T>(CS, LQ, 16 * cj, 32 * kk, lane), d4);
        const int j = 16 * cj + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) dVg[(t0 + 16 * sr + 4 * (lane >> 4) + r) * a.vt + j] = (T)d4[r];
      }
    }
    // ---- state gradient to the chunk start: dC~_k = decay dC~_{k+1} + (rowf Q)^T Dn ----
    const float decay = scal[0];
#pragma unroll
    for (int p = 0; p < PC; ++p) {
      const int q = w + 8 * p, i0 = 16 * (q / NJ), j0 = 16 * (q % NJ);
      f32x4 c = acc[p] * decay;
#pragma unroll
      for (int kk = 0; kk < kL / 32; ++kk)
        c = M::mma(frag_t_ks<V8, T>(Qs, LQ, 32 * kk, i0, lane, rowf),
                   frag_t<V8, T>(Dn, LV, 32 * kk, j0, lane), c);
      acc[p] = c;
    }
    if (tid < DQ) {
      float sacc = 0.0f;
      for (int t = 0; t < kL; ++t) sacc += rowf[t] * dden[t] * (float)Qs[t * LQ + tid];
      dn = decay * dn + sacc;
    }
    __syncthreads();
    if (tid < kL) {
      float sk = 0.0f;
#pragma unroll
      for (int ci = 0; ci < NI; ++ci) sk += kpart[ci * kL + tid];
      a.kdk[(int64_t)bh * a.T + t0 + tid] = sk;
    }
  }
  // gradient w.r.t. the initial state
#pragma unroll
  for (int p = 0; p < PC; ++p) {
    const int q = w + 8 * p, i0 = 16 * (q / NJ), j0 = 16 * (q % NJ);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      a.dCs[((int64_t)bh * DQ + i0 + 4 * (lane >> 4) + r) * DV + j0 + (lane & 15)] = acc[p][r];
  }
  if (tid < DQ) a.dns[(int64_t)bh * DQ + tid] = dn;
}

template <int DT, int DQ, int DV>
void launch_fwd(const MArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((mlstm_fw_walk<DT, DQ, DV>), dim3(DV / kCB, a.BH), dim3(256), 0, st, a);
}
template <int DT, int DQ, int DV>
void launch_bwd(const MArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((mlstm_bw_walk<DT, DQ, DV>), dim3(a.BH), dim3(512), 0, st, a);
}

// head dimensions compiled in (DQ, DV): the xLSTM-large defaults qk = v/2 at 64..192 wide heads
#define SC_MLSTM_DIMS(X) X(32, 64) X(64, 64) X(64, 128) X(96, 192)

template <int DT>
bool dispatch(const MArgs& a, int DQ, int DV, bool bwd, hipStream_t st) {
#define SC_CASE(q, v)                                    \
  if (DQ == q && DV == v) {                              \
    if (bwd) launch_bwd<DT, q, v>(a, st);                \
    else launch_fwd<DT, q, v>(a, st);                    \
    return true;                                         \
  }
  SC_MLSTM_DIMS(SC_CASE)
#undef SC_CASE
  return false;
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

}  // namespace

}  // namespace sc

using namespace sc;

extern "C" int sc_mlstm_supported(int dtype, int DQ, int DV) {
  return (dtype == SC_BF16 || dtype == SC_F16) && dims_supported(DQ, DV);
}

extern "C" int64_t sc_mlstm_state_numel(int BH, int T, int DQ, int DV) {
  if (BH <= 0 || T <= 0 || DQ <= 0 || DV <= 0) return 0;
  return (int64_t)BH * (T / kL + 1) * DQ * DV;
}

extern "C" int64_t sc_mlstm_chunk_state_numel(int BH, int T, int DQ, int DV) {
  if (BH <= 0 || T <= 0 || DQ <= 0 || DV <= 0) return 0;
  return (int64_t)BH * (T / kL) * DQ * DV;
}

extern "C" int sc_mlstm_fwd(const void* q, const void* k, const void* v, int dtype,
                            const float* igate, const float* fgate, const float* c0,
                            const float* n0, const float* m0, int BH, int T, int DQ, int DV,
                            float eps, void* h, void* states_C, float* states_n,
                            float* states_m, float* c_last, float* m_rows, float* den_rows,
                            const int64_t* layout, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_BF16 || dtype == SC_F16, "sc_mlstm_fwd: dtype %d (bf16/f16 only)", dtype);
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
  if (dtype == SC_BF16) dispatch<SC_BF16>(a, DQ, DV, false, st);
  else dispatch<SC_F16>(a, DQ, DV, false, st);
  return launch_status("sc_mlstm_fwd");
}

extern "C" int sc_mlstm_bwd(const void* q, const void* k, const void* v, int dtype,
                            const float* igate, const float* fgate, const void* h,
                            const void* dh, const float* dcT, const float* dnT,
                            const void* states_C, const float* states_n, const float* states_m,
                            const float* m_rows, const float* den_rows, int BH, int T, int DQ,
                            int DV, float eps, float* dstates_C, float* dstates_n, void* dq,
                            void* dk, void* dv, float* qdq, float* kdk, const int64_t* layout,
                            void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_BF16 || dtype == SC_F16, "sc_mlstm_bwd: dtype %d (bf16/f16 only)", dtype);
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
  if (dtype == SC_BF16) dispatch<SC_BF16>(a, DQ, DV, true, st);
  else dispatch<SC_F16>(a, DQ, DV, true, st);
  return launch_status("sc_mlstm_bwd");
}
