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
  void* Cs;         // [BH][nc][DQ][DV] chunk-start states C~_0 .. C~_{nc-1} in the compute
                    // dtype: the bf16 / f16 image the forward's Q~ C~_k MFMA consumes
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

// Chunk rows [t0, t0+64) of a [T][D] matrix into LDS, row-major [64][D+kPad] or transposed
// [D][64+kPad], 16-byte global loads (D % 8 == 0).
template <typename T, int D>
__device__ __forceinline__ void load_rows(T* dst, const T* src, int64_t ld, int tid) {
  for (int e = tid; e < kL * D / 8; e += 256) {
    const int r = e / (D / 8), c = (e % (D / 8)) * 8;
    *(uint4*)(dst + r * (D + kPad) + c) = *(const uint4*)(src + (int64_t)r * ld + c);
  }
}
// (transposing loaders: consecutive lanes take consecutive ROWS of one 8-column piece, so each
// of the eight 2-byte LDS stores per piece hits consecutive addresses across the wave; with
// lanes along the columns every store of a wave landed in one bank, 32-way)
template <typename T, int D>
__device__ __forceinline__ void load_rows_t(T* dst, const T* src, int64_t ld, int tid) {
  for (int e = tid; e < kL * D / 8; e += 256) {
    const int r = e % kL, c = (e / kL) * 8;
    const uint4 raw = *(const uint4*)(src + (int64_t)r * ld + c);
    const T* x = (const T*)&raw;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[(c + j) * (kL + kPad) + r] = x[j];
  }
}

// columns [c0, c0 + W) of chunk rows [t0, t0+64) of a [T][D] matrix, transposed into LDS
// [W][64+kPad] (16-byte global loads; W % 8 == 0)
template <typename T, int D, int W>
__device__ __forceinline__ void load_cols_t(T* dst, const T* src, int64_t ld, int c0, int tid) {
  for (int e = tid; e < kL * W / 8; e += 256) {
    const int r = e % kL, c = (e / kL) * 8;
    const uint4 raw = *(const uint4*)(src + (int64_t)r * ld + c0 + c);
    const T* x = (const T*)&raw;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[(c + j) * (kL + kPad) + r] = x[j];
  }
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
  const int cb = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
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
  for (int k = 0; k < a.nc; ++k) {
    const int64_t t0 = (int64_t)k * kL;
    load_rows<T, DQ>(Qs, Q + t0 * a.qt, a.qt, tid);
    load_rows<T, DQ>(Ks, K + t0 * a.qt, a.qt, tid);
    load_rows_t<T, DQ>(KT, K + t0 * a.qt, a.qt, tid);
    load_cols_t<T, DV, kCB>(VT, V + t0 * a.vt, a.vt, cj0, tid);
    chunk_gates(a, bh, k, sb, si, tid);
    // the state at the chunk start: its MFMA image (transposed, [j][i]) and the backward's copy
    T* Cs = (T*)a.Cs + ((int64_t)bh * a.nc + k) * DQ * DV;
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + 4 * (lane >> 4) + r, j = j0 + (lane & 15);
        const T c = (T)acc[p][r];
        CT[j * (DQ + kPad) + i] = c;
        Cs[(int64_t)i * DV + cj0 + j] = c;
      }
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
    // q_t . n~_k (4 threads per row)
    {
      const int t = tid >> 2, part = tid & 3;
      float qa = 0.0f;
      for (int i = part; i < DQ; i += 4) qa += (float)Qs[t * (DQ + kPad) + i] * nk[i];
      qa += __shfl_xor(qa, 1);
      qa += __shfl_xor(qa, 2);
      if (part == 0) qn[t] = qa;
    }
    // S = Q K^T for row block w, causal column blocks; M = S o W into LDS, row sums
    {
      float rs[4] = {0.f, 0.f, 0.f, 0.f};
      for (int ct = 0; ct < 4; ++ct) {
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
        if (ct <= w) {
#pragma unroll
          for (int kk = 0; kk < DQ / 32; ++kk)
            s4 = M::mma(frag<V8, T>(Qs, DQ + kPad, 16 * w, 32 * kk, lane),
                        frag<V8, T>(Ks, DQ + kPad, 16 * ct, 32 * kk, lane), s4);
        }
        const int s = 16 * ct + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = 16 * w + 4 * (lane >> 4) + r;
          const float mv = (s <= t) ? s4[r] * a.scale * expf(sb[t] - sb[s] + si[s] - mt[t]) : 0.0f;
          rs[r] += mv;
          Ms[t * (kL + kPad) + s] = (T)mv;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float tot = sum16(rs[r]);
        if ((lane & 15) == 0) dsum[16 * w + 4 * (lane >> 4) + r] = tot;
      }
    }
    __syncthreads();
    // H = M V + (rowf Q) C~_k for row block w; normalise and store
    {
      const float rf = rowf[16 * w + (lane & 15)];
      const int kin = (16 * (w + 1) + 31) / 32;
      for (int cj = 0; cj < TJ; ++cj) {
        f32x4 h4 = {0.f, 0.f, 0.f, 0.f};
        for (int kk = 0; kk < kin; ++kk)
          h4 = M::mma(frag<V8, T>(Ms, kL + kPad, 16 * w, 32 * kk, lane),
                      frag<V8, T>(VT, kL + kPad, 16 * cj, 32 * kk, lane), h4);
#pragma unroll
        for (int kk = 0; kk < DQ / 32; ++kk)
          h4 = M::mma(frag_rs<V8, T>(Qs, DQ + kPad, 16 * w, 32 * kk, lane, rf),
                      frag<V8, T>(CT, DQ + kPad, 16 * cj, 32 * kk, lane), h4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = 16 * w + 4 * (lane >> 4) + r;
          const float dn = dsum[t] + rowf[t] * qn[t];
          const float z = fmaxf(fabsf(dn), expf(-mt[t])) + a.eps;
          H[(t0 + t) * DV + cj0 + 16 * cj + (lane & 15)] = (T)(h4[r] / z);
        }
      }
      if (cb == 0 && tid < kL) {
        const float dn = dsum[tid] + rowf[tid] * qn[tid];
        a.mrow[(int64_t)bh * a.T + t0 + tid] = mt[tid];
        a.den[(int64_t)bh * a.T + t0 + tid] = dn;
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
    }
    if (tid < DQ) {
      float sacc = 0.0f;
      for (int s = 0; s < kL; ++s) sacc += fs[s] * (float)KT[tid * (kL + kPad) + s];
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

// dnum_t = dh_t / Z_t and dden_t for the 64 rows of a chunk (4 threads per row): dnum rows go
// to LDS row-major ([t][j]) and/or transposed ([j][t]); dden, Z into LDS arrays.
template <typename T, int DV>
__device__ __forceinline__ void chunk_dnum(const MArgs& a, int bh, int64_t t0, T* dn_rm, T* dn_t,
                                           float* dden, int tid) {
  const int t = tid >> 2, part = tid & 3;
  const T* dh = (const T*)a.dh + ((int64_t)bh * a.T + t0 + t) * DV;
  const T* h = (const T*)a.h + ((int64_t)bh * a.T + t0 + t) * DV;
  const float m_t = a.mrow[(int64_t)bh * a.T + t0 + t];
  const float dn = a.den[(int64_t)bh * a.T + t0 + t];
  const float z = fmaxf(fabsf(dn), expf(-m_t)) + a.eps;
  float dot = 0.0f;
  for (int j = part * 8; j < DV; j += 32) {
    const uint4 rd = *(const uint4*)(dh + j), rh = *(const uint4*)(h + j);
    const T* xd = (const T*)&rd;
    const T* xh = (const T*)&rh;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = (float)xd[e];
      dot += d * (float)xh[e];
      const T v = (T)(d / z);
      if (dn_rm) dn_rm[t * (DV + kPad) + j + e] = v;
      if (dn_t) dn_t[(j + e) * (kL + kPad) + t] = v;
    }
  }
  dot += __shfl_xor(dot, 1);
  dot += __shfl_xor(dot, 2);
  if (part == 0) {
    // den enters through max(|den|, e^{-m}): only the |den| branch carries a gradient
    const float live = fabsf(dn) >= expf(-m_t) ? 1.0f : 0.0f;
    dden[t] = -dot / z * (dn >= 0.0f ? 1.0f : -1.0f) * live;
  }
}

// ------------------------------------------------------------------------- backward: dC~ ----
template <int DT, int DQ, int DV>
__global__ void __launch_bounds__(256) mlstm_bw_dC(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  constexpr int TJ = DV / 16, NT = (DQ / 16) * TJ, PW = NT / 4;
  const int bh = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ __attribute__((aligned(16))) T QT[DQ * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T DnT[DV * (kL + kPad)];
  __shared__ float sb[kL], si[kL], rowf[kL], dden[kL], scal[1];
  f32x4 acc[PW];
#pragma unroll
  for (int p = 0; p < PW; ++p) {
    const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r, j = j0 + (lane & 15);
      acc[p][r] = a.dcT ? a.dcT[((int64_t)bh * DQ + i) * DV + j] : 0.0f;
    }
  }
  float dn = (tid < DQ && a.dnT) ? a.dnT[(int64_t)bh * DQ + tid] : 0.0f;
  auto store = [&](int k) {
    float* C = a.dCs + ((int64_t)bh * (a.nc + 1) + k) * DQ * DV;
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(i0 + 4 * (lane >> 4) + r) * DV + j0 + (lane & 15)] = acc[p][r];
    }
    if (tid < DQ) a.dns[((int64_t)bh * (a.nc + 1) + k) * DQ + tid] = dn;
  };
  for (int k = a.nc - 1; k >= 0; --k) {
    store(k + 1);
    const int64_t t0 = (int64_t)k * kL;
    load_rows_t<T, DQ>(QT, (const T*)a.q + qrow(a, bh, t0), a.qt, tid);
    chunk_dnum<T, DV>(a, bh, t0, (T*)nullptr, DnT, dden, tid);
    chunk_gates(a, bh, k, sb, si, tid);
    if (tid < 64) {
      const int64_t st = (int64_t)bh * (a.nc + 1) + k;
      const float mk = a.ms[st], mk1 = a.ms[st + 1];
      const float m_t = a.mrow[(int64_t)bh * a.T + t0 + tid];
      rowf[tid] = a.scale * expf(sb[tid] + mk - m_t);
      if (tid == 0) scal[0] = expf(sb[63] + mk - mk1);
    }
    __syncthreads();
    const float decay = scal[0];
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int q = w + 4 * p, i0 = 16 * (q / TJ), j0 = 16 * (q % TJ);
      f32x4 c = acc[p] * decay;
#pragma unroll
      for (int kk = 0; kk < kL / 32; ++kk)
        c = M::mma(frag_ks<V8, T>(QT, kL + kPad, i0, 32 * kk, lane, rowf),
                   frag<V8, T>(DnT, kL + kPad, j0, 32 * kk, lane), c);
      acc[p] = c;
    }
    if (tid < DQ) {
      float sacc = 0.0f;
      for (int t = 0; t < kL; ++t) sacc += rowf[t] * dden[t] * (float)QT[tid * (kL + kPad) + t];
      dn = decay * dn + sacc;
    }
    __syncthreads();
  }
  store(0);
}

// Shared by the dQ and dK kernels: dA_ts = W_ts (dnum_t . v_s + dden_t) for row block w
// (t), causal column blocks, from LDS dnum [t][j] and V [s][j]; written to LDS row-major
// (dQ) or transposed (dK).
template <typename M, int DV, bool TRANS>
__device__ __forceinline__ void chunk_dA(const typename M::T* Dn, const typename M::T* Vs,
                                         typename M::T* out, const float* sb, const float* si,
                                         const float* mt, const float* dden, float scale, int w,
                                         int lane) {
  using T = typename M::T;
  using V8 = typename M::v8;
  for (int ct = 0; ct < 4; ++ct) {
    f32x4 p4 = {0.f, 0.f, 0.f, 0.f};
    if (ct <= w) {
#pragma unroll
      for (int kk = 0; kk < DV / 32; ++kk)
        p4 = M::mma(frag<V8, T>(Dn, DV + kPad, 16 * w, 32 * kk, lane),
                    frag<V8, T>(Vs, DV + kPad, 16 * ct, 32 * kk, lane), p4);
    }
    const int s = 16 * ct + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 16 * w + 4 * (lane >> 4) + r;
      const float v = (s <= t) ? (p4[r] + dden[t]) * scale * expf(sb[t] - sb[s] + si[s] - mt[t]) : 0.0f;
      if (TRANS) out[s * (kL + kPad) + t] = (T)v;
      else out[t * (kL + kPad) + s] = (T)v;
    }
  }
}

// gate prefix + per-row m_t, rowf_t (= s e^{b_t + m_k - m_t}) and per-key es_s (= e^{a_s - m_{k+1}})
__device__ __forceinline__ void chunk_rows(const MArgs& a, int bh, int k, float* sb, float* si,
                                           float* mt, float* rowf, float* es, int tid) {
  chunk_gates(a, bh, k, sb, si, tid);
  if (tid < 64) {
    const int64_t st = (int64_t)bh * (a.nc + 1) + k;
    const float mk = a.ms[st], mk1 = a.ms[st + 1];
    const float m_t = a.mrow[(int64_t)bh * a.T + (int64_t)k * kL + tid];
    const float g = __shfl(sb[63], 0);
    mt[tid] = m_t;
    if (rowf) rowf[tid] = a.scale * expf(sb[tid] + mk - m_t);
    if (es) es[tid] = expf(g - sb[tid] + si[tid] - mk1);
  }
}

// ------------------------------------------------------------------------- backward: dQ -----
template <int DT, int DQ, int DV>
__global__ void __launch_bounds__(256) mlstm_bw_dQ(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  const int k = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ __attribute__((aligned(16))) T Dn[kL * (DV + kPad)];
  __shared__ __attribute__((aligned(16))) T Vs[kL * (DV + kPad)];
  __shared__ __attribute__((aligned(16))) T dA[kL * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T KT[DQ * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T Cm[DQ * (DV + kPad)];
  __shared__ float sb[kL], si[kL], mt[kL], rowf[kL], dden[kL], nk[DQ];
  const int64_t t0 = (int64_t)k * kL;
  load_rows<T, DV>(Vs, (const T*)a.v + vrow(a, bh, t0), a.vt, tid);
  load_rows_t<T, DQ>(KT, (const T*)a.k + qrow(a, bh, t0), a.qt, tid);
  const int64_t st = (int64_t)bh * (a.nc + 1) + k;
  const T* Ck = (const T*)a.Cs + ((int64_t)bh * a.nc + k) * DQ * DV;
  for (int e = tid; e < DQ * DV / 8; e += 256) {   // 16-byte pieces of the [DQ][DV] image
    const int i = (8 * e) / DV, j = (8 * e) % DV;
    *(uint4*)(Cm + i * (DV + kPad) + j) = *(const uint4*)(Ck + 8 * e);
  }
  if (tid < DQ) nk[tid] = a.ns[st * DQ + tid];
  chunk_dnum<T, DV>(a, bh, t0, Dn, (T*)nullptr, dden, tid);
  chunk_rows(a, bh, k, sb, si, mt, rowf, nullptr, tid);
  __syncthreads();
  chunk_dA<M, DV, false>(Dn, Vs, dA, sb, si, mt, dden, a.scale, w, lane);
  __syncthreads();
  const float rf = rowf[16 * w + (lane & 15)];
  const int kin = (16 * (w + 1) + 31) / 32;
  const T* Q = (const T*)a.q + qrow(a, bh, t0);
  T* dQ = (T*)a.dq + qrow(a, bh, t0);
  float qd[4] = {0.f, 0.f, 0.f, 0.f};
  for (int ci = 0; ci < DQ / 16; ++ci) {
    f32x4 d4 = {0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < kin; ++kk)
      d4 = M::mma(frag<V8, T>(dA, kL + kPad, 16 * w, 32 * kk, lane),
                  frag<V8, T>(KT, kL + kPad, 16 * ci, 32 * kk, lane), d4);
#pragma unroll
    for (int kk = 0; kk < DV / 32; ++kk)
      d4 = M::mma(frag_rs<V8, T>(Dn, DV + kPad, 16 * w, 32 * kk, lane, rf),
                  frag<V8, T>(Cm, DV + kPad, 16 * ci, 32 * kk, lane), d4);
    const int i = 16 * ci + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 16 * w + 4 * (lane >> 4) + r;
      const float v = d4[r] + rowf[t] * dden[t] * nk[i];
      dQ[t * a.qt + i] = (T)v;
      qd[r] += v * (float)Q[t * a.qt + i];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float tot = sum16(qd[r]);
    if ((lane & 15) == 0) a.qdq[(int64_t)bh * a.T + t0 + 16 * w + 4 * (lane >> 4) + r] = tot;
  }
}

// ------------------------------------------------------------------------- backward: dK -----
template <int DT, int DQ, int DV>
__global__ void __launch_bounds__(256) mlstm_bw_dK(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  const int k = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ __attribute__((aligned(16))) T Dn[kL * (DV + kPad)];
  __shared__ __attribute__((aligned(16))) T Vs[kL * (DV + kPad)];
  __shared__ __attribute__((aligned(16))) T dAT[kL * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T QT[DQ * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T dCm[DQ * (DV + kPad)];
  __shared__ float sb[kL], si[kL], mt[kL], es[kL], dden[kL], dnk[DQ];
  const int64_t t0 = (int64_t)k * kL;
  load_rows<T, DV>(Vs, (const T*)a.v + vrow(a, bh, t0), a.vt, tid);
  load_rows_t<T, DQ>(QT, (const T*)a.q + qrow(a, bh, t0), a.qt, tid);
  const int64_t st1 = (int64_t)bh * (a.nc + 1) + k + 1;
  const float* dC = a.dCs + st1 * DQ * DV;
  for (int e = tid; e < DQ * DV; e += 256) dCm[(e / DV) * (DV + kPad) + e % DV] = (T)dC[e];
  if (tid < DQ) dnk[tid] = a.dns[st1 * DQ + tid];
  chunk_dnum<T, DV>(a, bh, t0, Dn, (T*)nullptr, dden, tid);
  chunk_rows(a, bh, k, sb, si, mt, nullptr, es, tid);
  __syncthreads();
  chunk_dA<M, DV, true>(Dn, Vs, dAT, sb, si, mt, dden, a.scale, w, lane);
  __syncthreads();
  // row block w holds keys s in [16w, 16w+16): intra sums over t >= s
  const float ef = es[16 * w + (lane & 15)];
  const int k0 = (16 * w) / 32;
  const T* K = (const T*)a.k + qrow(a, bh, t0);
  T* dK = (T*)a.dk + qrow(a, bh, t0);
  float kd[4] = {0.f, 0.f, 0.f, 0.f};
  for (int ci = 0; ci < DQ / 16; ++ci) {
    f32x4 d4 = {0.f, 0.f, 0.f, 0.f};
    for (int kk = k0; kk < kL / 32; ++kk)
      d4 = M::mma(frag<V8, T>(dAT, kL + kPad, 16 * w, 32 * kk, lane),
                  frag<V8, T>(QT, kL + kPad, 16 * ci, 32 * kk, lane), d4);
#pragma unroll
    for (int kk = 0; kk < DV / 32; ++kk)
      d4 = M::mma(frag_rs<V8, T>(Vs, DV + kPad, 16 * w, 32 * kk, lane, ef),
                  frag<V8, T>(dCm, DV + kPad, 16 * ci, 32 * kk, lane), d4);
    const int i = 16 * ci + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 16 * w + 4 * (lane >> 4) + r;
      const float v = d4[r] + es[s] * dnk[i];
      dK[s * a.qt + i] = (T)v;
      kd[r] += v * (float)K[s * a.qt + i];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float tot = sum16(kd[r]);
    if ((lane & 15) == 0) a.kdk[(int64_t)bh * a.T + t0 + 16 * w + 4 * (lane >> 4) + r] = tot;
  }
}

// ------------------------------------------------------------------------- backward: dV -----
template <int DT, int DQ, int DV>
__global__ void __launch_bounds__(256) mlstm_bw_dV(MArgs a) {
  using M = MF<DT>;
  using T = typename M::T;
  using V8 = typename M::v8;
  const int k = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ __attribute__((aligned(16))) T Qs[kL * (DQ + kPad)];
  __shared__ __attribute__((aligned(16))) T Ks[kL * (DQ + kPad)];
  __shared__ __attribute__((aligned(16))) T AT[kL * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T DnT[DV * (kL + kPad)];
  __shared__ __attribute__((aligned(16))) T dCT[DV * (DQ + kPad)];
  __shared__ float sb[kL], si[kL], mt[kL], es[kL], dden[kL];
  const int64_t t0 = (int64_t)k * kL;
  load_rows<T, DQ>(Qs, (const T*)a.q + qrow(a, bh, t0), a.qt, tid);
  load_rows<T, DQ>(Ks, (const T*)a.k + qrow(a, bh, t0), a.qt, tid);
  const int64_t st1 = (int64_t)bh * (a.nc + 1) + k + 1;
  const float* dC = a.dCs + st1 * DQ * DV;
  for (int e = tid; e < DQ * DV; e += 256) {
    const int i = e / DV, j = e % DV;
    dCT[j * (DQ + kPad) + i] = (T)dC[e];
  }
  chunk_dnum<T, DV>(a, bh, t0, (T*)nullptr, DnT, dden, tid);
  chunk_rows(a, bh, k, sb, si, mt, nullptr, es, tid);
  __syncthreads();
  // A_ts = W_ts S_ts, transposed into LDS [s][t]
  for (int ct = 0; ct < 4; ++ct) {
    f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
    if (ct <= w) {
#pragma unroll
      for (int kk = 0; kk < DQ / 32; ++kk)
        s4 = M::mma(frag<V8, T>(Qs, DQ + kPad, 16 * w, 32 * kk, lane),
                    frag<V8, T>(Ks, DQ + kPad, 16 * ct, 32 * kk, lane), s4);
    }
    const int s = 16 * ct + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 16 * w + 4 * (lane >> 4) + r;
      const float v = (s <= t) ? s4[r] * a.scale * expf(sb[t] - sb[s] + si[s] - mt[t]) : 0.0f;
      AT[s * (kL + kPad) + t] = (T)v;
    }
  }
  __syncthreads();
  const float ef = es[16 * w + (lane & 15)];
  const int k0 = (16 * w) / 32;
  T* dV = (T*)a.dv + vrow(a, bh, t0);
  for (int cj = 0; cj < DV / 16; ++cj) {
    f32x4 d4 = {0.f, 0.f, 0.f, 0.f};
    for (int kk = k0; kk < kL / 32; ++kk)
      d4 = M::mma(frag<V8, T>(AT, kL + kPad, 16 * w, 32 * kk, lane),
                  frag<V8, T>(DnT, kL + kPad, 16 * cj, 32 * kk, lane), d4);
#pragma unroll
    for (int kk = 0; kk < DQ / 32; ++kk)
      d4 = M::mma(frag_rs<V8, T>(Ks, DQ + kPad, 16 * w, 32 * kk, lane, ef),
                  frag<V8, T>(dCT, DQ + kPad, 16 * cj, 32 * kk, lane), d4);
    const int j = 16 * cj + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) dV[(16 * w + 4 * (lane >> 4) + r) * a.vt + j] = (T)d4[r];
  }
}

template <int DT, int DQ, int DV>
void launch_fwd(const MArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((mlstm_fw_walk<DT, DQ, DV>), dim3(DV / kCB, a.BH), dim3(256), 0, st, a);
}
template <int DT, int DQ, int DV>
void launch_bwd(const MArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((mlstm_bw_dC<DT, DQ, DV>), dim3(a.BH), dim3(256), 0, st, a);
  hipLaunchKernelGGL((mlstm_bw_dQ<DT, DQ, DV>), dim3(a.nc, a.BH), dim3(256), 0, st, a);
  hipLaunchKernelGGL((mlstm_bw_dK<DT, DQ, DV>), dim3(a.nc, a.BH), dim3(256), 0, st, a);
  hipLaunchKernelGGL((mlstm_bw_dV<DT, DQ, DV>), dim3(a.nc, a.BH), dim3(256), 0, st, a);
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
