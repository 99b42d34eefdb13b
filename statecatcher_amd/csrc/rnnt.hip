// RNN-T (transducer) loss for gfx950: the lattice the reference gets from warp_rnnt
// (model.py:73-105, train.py:38-42, :144; gather=True semantics: only the blank and the next
// label of every (t, u) node enter the loss).
//
//   rnnt_emit_kernel   one wave per lattice node (b,t,u): row log-sum-exp over V (when fed
//                      logits: the log_softmax of model.py:93 is fused), then the node's blank
//                      and label log-probs in base 2, stored DIAGONAL-MAJOR ([b][t+u][u]) so
//                      that the wavefront below reads one coalesced row per step.
//   rnnt_shift_kernel  one wave per diagonal row: subtracts from every blank log-prob of frame t
//                      the frame's largest, cb[t], and from every label-u log-prob the largest
//                      over t, cy[u] (both gathered by the emission producers with order-mapped
//                      integer atomicMax, so they are exact and independent of order).  Every
//                      path takes exactly one blank per frame and one emission of each label, so
//                      the shift moves every path by the same sum cb + sum cy: exact, and it keeps
//                      the fp32 lattice values near 0.  Unshifted, nodes of one diagonal lie
//                      hundreds of bits apart and their rounding put ~1e-2 of relative error into
//                      the arc occupancies at T=1500, U=150 (tools/ctc_precision.py --rnnt).
//   rnnt_ab_kernel     one workgroup per (sequence, direction): alpha forward and beta backward
//                      run concurrently.  Lane = label position u; the lattice is swept by
//                      anti-diagonals n = t + u (all nodes of a diagonal are independent), the
//                      neighbour (t, u-1) / (t, u+1) value crosses lanes by a DPP lane shift;
//                      waves carry a K-lane halo and exchange through LDS every K diagonals.
//                      Values are base-2 logs with a finite "dead" sentinel and are re-centred
//                      on the workgroup max every 2K diagonals; the running offset is fp64
//                      (|alpha| reaches ~1e4 at T=1500, U=150), stored once per re-centring.
//   rnnt_grad_kernel   one wave per node: occupancies of the two gathered arcs from alpha, beta
//                      and log P (offsets recombined in fp64), then the full gradient row
//                      (softmax-corrected when fed logits, sparse when fed log-probs).
#include "sc_common.h"

namespace sc {

namespace {

constexpr float kDeadR = -1e30f;

struct RnntWs {
  float* lse;      // [B][T][U1]      natural-log row normaliser per node (logits input)
  float* lpb;      // [B][ND][U1p]    base-2 blank log-prob of node (t,u) at [t+u][u]
  float* lpy;      // [B][ND][U1p]    base-2 log-prob of label y[u] at node (t,u)
  float* alpha;    // [B][ND][U1p]    base-2, relative to offA[b][t+u]
  float* beta;     // [B][ND][U1p]    base-2, relative to offB[b][t+u]
  double* offA;    // [B][ND]
  double* offB;    // [B][ND]
  double* logp2;   // [B]             base-2 log P(y|x) of the SHIFTED lattice (log2 P - shifts)
  unsigned* cmb;   // [B][T]          order-mapped max over u of the frame's blank log-probs
  unsigned* cmy;   // [B][U1]         order-mapped max over t of label u's log-probs (follows cmb)
};

// float <-> unsigned key with the same order (0 is below every key: "no value")
__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// the shift a key stands for: 0 when nothing live was seen (the sentinel must stay dead)
__device__ __forceinline__ float kshift(unsigned k) {
  const float f = __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
  return (k != 0u && f > -1e29f) ? f : 0.0f;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
int u1p_of(int Umax) { return 64 * ((Umax + 1 + 63) / 64); }

size_t ws_layout(int B, int T, int Umax, RnntWs* w, void* base) {
  const int U1 = Umax + 1, U1p = u1p_of(Umax), ND = T + Umax;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p + off;
    off += align256(bytes);
    return (void*)r;
  };
  RnntWs t;
  t.lse = (float*)take((size_t)B * T * U1 * 4);
  t.lpb = (float*)take((size_t)B * ND * U1p * 4);
  t.lpy = (float*)take((size_t)B * ND * U1p * 4);
  t.alpha = (float*)take((size_t)B * ND * U1p * 4);
  t.beta = (float*)take((size_t)B * ND * U1p * 4);
  t.offA = (double*)take((size_t)B * ND * 8);
  t.offB = (double*)take((size_t)B * ND * 8);
  t.logp2 = (double*)take((size_t)B * 8);
  t.cmb = (unsigned*)take((size_t)B * (T + U1) * 4);
  t.cmy = t.cmb + (size_t)B * T;
  if (w) *w = t;
  return off;
}

struct RnntArgs {
  const void* x;
  int is_logits, B, T, Umax, V, blank, U1, U1p, ND;
  int64_t sb, st, su;
  const int64_t* row_off;   // compact layout: first row of sequence b (NULL: dense strides)
  const int64_t* lab;
  int64_t labs;
  const int64_t* flen;
  const int64_t* llen;
  float* nll;
  RnntWs ws;
  const float* scale;
  void* grad;
  int vec, nvec;   // rows read/written as 16-byte vectors: nvec per lane (V = 64 * N * nvec)
  int kh;          // diagonals between halo exchanges of rnnt_ab_kernel (re-centring: 2 kh)
};

__device__ __forceinline__ int clampr(int64_t v, int lo, int hi) {
  return (int)(v < lo ? lo : (v > hi ? hi : v));
}

// element offset of node (b, t, u)'s row
__device__ __forceinline__ int64_t node_row(const RnntArgs& a, int b, int t, int u, int Ub) {
  if (a.row_off) return (a.row_off[b] + (int64_t)t * (Ub + 1) + u) * a.su;
  return (int64_t)b * a.sb + (int64_t)t * a.st + (int64_t)u * a.su;
}

__device__ __forceinline__ int label_at(const RnntArgs& a, int b, int u) {
  const int lab = (int)a.lab[(int64_t)b * a.labs + u];
  return lab < 0 ? 0 : (lab >= a.V ? a.V - 1 : lab);
}

// ---------------------------------------------------------------------------- emissions -----
constexpr int kNvMax = 4;   // 16-byte vectors per lane held in registers (V <= 64 * N * 4)

template <int DT>
__global__ void __launch_bounds__(256) rnnt_emit_kernel(RnntArgs a) {
  using E = Elem<DT>;
  using T = typename E::T;
  using VL = Vec16<DT>;
  const int lane = threadIdx.x & 63;
  const int64_t node = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (node >= (int64_t)a.B * a.T * a.U1) return;
  const int b = (int)(node / ((int64_t)a.T * a.U1));
  const int t = (int)((node / a.U1) % a.T), u = (int)(node % a.U1);
  const int Tb = clampr(a.flen[b], 0, a.T), Ub = clampr(a.llen[b], 0, a.Umax);
  if (t >= Tb || u > Ub) return;
  const T* p = (const T*)a.x + node_row(a, b, t, u, Ub);
  float lse = 0.0f;
  if (a.is_logits && a.vec) {   // whole row in registers: max pass, then one exp per element
    float f[kNvMax][VL::N];
    float m = -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < kNvMax; ++j) {
      if (j < a.nvec) {
        VL::ld(p + (j * 64 + lane) * VL::N, f[j]);
#pragma unroll
        for (int k = 0; k < VL::N; ++k) m = fmaxf(m, f[j][k]);
      }
    }
    m = wave_max_dpp(m);
    float l = 0.0f;
#pragma unroll
    for (int j = 0; j < kNvMax; ++j)
      if (j < a.nvec) {
#pragma unroll
        for (int k = 0; k < VL::N; ++k) l += fexp(f[j][k] - m);
      }
    l = wave_sum_dpp(l);
    lse = m + flog(l);
  } else if (a.is_logits) {      // any V / alignment: online max-rescaled sum
    float m = -__builtin_huge_valf(), l = 0.0f;
    for (int v = lane; v < a.V; v += 64) {
      const float xv = E::ld(p[v]);
      const float mn = fmaxf(m, xv);
      l = l * fexp(m - mn) + fexp(xv - mn);
      m = mn;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float mo = __shfl_xor(m, o);
      const float lo = __shfl_xor(l, o);
      const float mn = fmaxf(m, mo);
      l = (mn == -__builtin_huge_valf()) ? 0.0f : l * fexp(m - mn) + lo * fexp(mo - mn);
      m = mn;
    }
    lse = m + flog(l);
  }
  if (lane == 0) {
    const int64_t d = ((int64_t)b * a.ND + t + u) * a.U1p + u;
    a.ws.lse[node] = lse;
    const float lb = fmaxf((E::ld(p[a.blank]) - lse) * kLog2e, kDeadR);
    a.ws.lpb[d] = lb;
    atomicMax(a.ws.cmb + (int64_t)b * a.T + t, fkey(lb));
    if (u < Ub) {
      const float ly = fmaxf((E::ld(p[label_at(a, b, u)]) - lse) * kLog2e, kDeadR);
      a.ws.lpy[d] = ly;
      atomicMax(a.ws.cmy + (int64_t)b * a.U1 + u, fkey(ly));
    } else {
      a.ws.lpy[d] = kDeadR;
    }
  }
}

// the emission shift (see the file header), in place, one wave per diagonal row (b, n)
__global__ void __launch_bounds__(256) rnnt_shift_kernel(RnntArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)a.B * a.ND) return;
  const int b = (int)(row / a.ND), n = (int)(row % a.ND);
  const int Tb = clampr(a.flen[b], 0, a.T), Ub = clampr(a.llen[b], 0, a.Umax);
  if (n >= Tb + Ub) return;
  float* pb = a.ws.lpb + row * a.U1p;
  float* py = a.ws.lpy + row * a.U1p;
  for (int u = lane; u <= Ub; u += 64) {
    const int t = n - u;
    if (t < 0 || t >= Tb) continue;
    const float vb = pb[u];
    if (vb > -1e29f) pb[u] = fmaxf(vb - kshift(a.ws.cmb[(int64_t)b * a.T + t]), kDeadR);
    if (u < Ub) {
      const float vy = py[u];
      if (vy > -1e29f) py[u] = fmaxf(vy - kshift(a.ws.cmy[(int64_t)b * a.U1 + u]), kDeadR);
    }
  }
}

// ---------------------------------------------------------------------------- alpha / beta --
__device__ __forceinline__ float lse2_live(float x, float y) {
  const float m = fmaxf(x, y);
  return m + log2_(exp2_(x - m) + exp2_(y - m));
}

__device__ __forceinline__ float dpp_shr1(float v) {   // value of lane-1 (lane 0: dead)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(kDeadR), __float_as_int(v),
                                                     0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_shl1(float v) {   // value of lane+1 (lane 63: dead)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(kDeadR), __float_as_int(v),
                                                     0x130, 0xf, 0xf, false));
}

// K (diagonals between halo exchanges) so that ceil((Umax + 1) / (64 - K)) waves fit a
// 1024-thread group; 0 if none does
int ab_halo_k(int Umax) {
  for (int K : {16, 8, 4, 2, 1})
    if ((Umax + 1 + (64 - K) - 1) / (64 - K) <= 16) return K;
  return 0;
}

// Lane = label position u; the lattice is swept by anti-diagonals n = t + u.  On diagonal n the
// value of node (t, u) needs (t-1, u) — the same lane on the previous diagonal — and (t, u-1)
// (alpha) or (t, u+1) (beta) — the neighbouring lane — so a wave advances K diagonals with one
// DPP lane shift each and no LDS.  Each wave owns 64 - K consecutive u and carries a K-lane
// halo of its neighbour's (left for alpha, right for beta), which a missing neighbour corrupts
// one lane per diagonal; every K diagonals the owned values are published to LDS, one barrier,
// and the halo lanes re-read theirs.  Every second exchange re-centres on the workgroup max
// (fp64 offset, stored once per re-centring).  Alpha/beta rows go out through buffer stores
// whose out-of-range offset drops invalid and halo lanes (no exec-mask branches in the loop).
template <int K, bool BETA>
__device__ __forceinline__ void ab_run(const RnntArgs& a, int b, int Tb, int Ub) {
  constexpr int OW = 64 - K;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = uniform(tid >> 6);
  const int nw = blockDim.x >> 6;
  const int u = BETA ? w * OW + lane : w * OW + lane - K;
  const bool own = BETA ? (lane < OW) : (lane >= K);
  const int nd = Tb + Ub;          // diagonals 0 .. nd-1
  const int64_t base = (int64_t)b * a.ND * a.U1p;
  const int uc = u < 0 ? 0 : (u >= a.U1p ? a.U1p - 1 : u);   // clamped, for addressing only
  const int uy = BETA ? uc : (u > 0 ? min(u - 1, a.U1p - 1) : 0);
  const float* lpb = a.ws.lpb + base;
  const float* lpy = a.ws.lpy + base;
  constexpr uint32_t kDrop = 0x80000000u;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (BETA ? a.ws.beta : a.ws.alpha) + base, 0, (int)(4u * (uint32_t)a.ND * (uint32_t)a.U1p),
      0x00020000);
  double* offn = (BETA ? a.ws.offB : a.ws.offA) + (int64_t)b * a.ND;
  if (tid == 0) offn[0] = 0.0;
  extern __shared__ __attribute__((aligned(16))) float pub[];   // [2][nw*OW] published values
  __shared__ float wmax[16];
  const int nst = nw * OW;
  // emissions of diagonal step i come from workspace row r(i): alpha reads the arcs entering
  // diagonal n = i from row n-1 ((t-1,u) blank, (t,u-1) label), beta the arcs leaving row n
  auto row_of = [&](int i) {
    const int r = BETA ? nd - 1 - min(i, nd - 1) : min(i, nd - 1) - 1;
    return r < 0 ? 0 : r;
  };
  constexpr int kPf = 16;
  float ebA[kPf], eyA[kPf], ebB[kPf], eyB[kPf];
  auto load = [&](float (&eb)[kPf], float (&ey)[kPf], int i0) {
#pragma unroll
    for (int j = 0; j < kPf; ++j) {
      const int64_t r = (int64_t)row_of(i0 + j) * a.U1p;
      eb[j] = lpb[r + uc];
      ey[j] = lpy[r + uy];
    }
  };
  double off = 0.0;
  float v = kDeadR;
  int exch = 0;
  auto body = [&](const float (&eb)[kPf], const float (&ey)[kPf], int i0)
      __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kPf; ++j) {
      const int i = i0 + j;
      if (i >= nd) break;
      const int n = BETA ? nd - 1 - i : i;
      const int t = n - u;
      const bool valid = u >= 0 && u <= Ub && t >= 0 && t < Tb;
      float nv;
      if (!BETA) {
        const float vn = dpp_shr1(v);                      // (t, u-1) on diagonal n-1
        nv = i == 0 ? (u == 0 ? 0.0f : kDeadR)
                    : lse2_live(t >= 1 ? v + eb[j] : kDeadR, u >= 1 ? vn + ey[j] : kDeadR);
      } else {
        const float vn = dpp_shl1(v);                      // (t, u+1) on diagonal n+1
        nv = i == 0 ? (u == Ub ? eb[j] : kDeadR)           // terminal blank of (Tb-1, Ub)
                    : lse2_live(t + 1 < Tb ? v + eb[j] : kDeadR, u < Ub ? vn + ey[j] : kDeadR);
      }
      v = valid ? fmaxf(nv, kDeadR) : kDeadR;
      if (j % K == K - 1) {   // halo exchange (+ re-centre every second one)
        const int par = exch & 1;
        const bool norm = par == 1;
        if (own && u < nst) pub[par * nst + u] = v;
        if (norm) {
          const float m = wave_max_dpp(own ? v : kDeadR);
          if (lane == 0) wmax[w] = m;
        }
        lds_barrier();
        if (!own) v = (u >= 0 && u < nst) ? pub[par * nst + u] : kDeadR;
        if (norm) {
          float m = kDeadR;
          for (int q = 0; q < nw; ++q) m = fmaxf(m, wmax[q]);
          if (m > 0.5f * kDeadR) {   // all dead: keep the sentinel
            v -= m;
            off += (double)m;
          }
          if (tid == 0) offn[(exch + 1) >> 1] = off;
        }
        ++exch;
      }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ors,
                                            (own && valid) ? (uint32_t)(4 * u) : kDrop,
                                            (uint32_t)n * 4u * (uint32_t)a.U1p, 0);
    }
  };
  load(ebA, eyA, 0);
  for (int i0 = 0; i0 < nd; i0 += 2 * kPf) {
    load(ebB, eyB, i0 + kPf);
    body(ebA, eyA, i0);
    if (i0 + kPf >= nd) break;
    load(ebA, eyA, i0 + 2 * kPf);
    body(ebB, eyB, i0 + kPf);
  }
  if (!BETA) {
    // the emission shift of every path, sum_t cb[t] + sum_{u<Ub} cy[u], fp64 in a fixed order
    __shared__ double csum[16];
    double cs = 0.0;
    for (int i = tid; i < Tb + Ub; i += blockDim.x)
      cs += (double)kshift(i < Tb ? a.ws.cmb[(int64_t)b * a.T + i] : a.ws.cmy[(int64_t)b * a.U1 + i - Tb]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o);
    if (lane == 0) csum[w] = cs;
    lds_barrier();
    if (own && u == Ub) {   // log P = alpha(Tb-1, Ub) + its terminal blank (+ the shift)
      double ctot = 0.0;
      for (int q = 0; q < nw; ++q) ctot += csum[q];
      const double lp = (double)v + (double)lpb[(int64_t)(nd - 1) * a.U1p + Ub] + off;
      a.ws.logp2[b] = lp;
      a.nll[b] = (float)(-(lp + ctot) * 0.6931471805599453);
    }
  }
}

// ONE WAVE per (sequence, direction) when U + 1 <= 64 PPL label positions (PPL <= 4; C5's U = 150
// takes PPL = 3): lane l holds u = l PPL .. l PPL + PPL - 1, so a diagonal needs one DPP lane shift
// (alpha: the previous lane's last u; beta: the next lane's first) and PPL independent
// log-sum-exps -- no halo lanes, no LDS, no barrier (the multi-wave kernel above exchanges halos
// through LDS with a workgroup barrier every K diagonals).  Re-centred on the wave max every
// kAb1R diagonals (fp64 offsets, stored per re-centring; the gradient indexes them with kh =
// kAb1R / 2).
constexpr int kAb1R = 32;
constexpr int kAb1P = 16;   // emission prefetch depth (diagonals)

template <int PPL, bool BETA>
__device__ __forceinline__ void ab1_run(const RnntArgs& a, int b, int Tb, int Ub) {
  const int lane = threadIdx.x;
  const int nd = Tb + Ub;
  const int64_t base = (int64_t)b * a.ND * a.U1p;
  constexpr uint32_t kDrop = 0x80000000u;
  // byte offsets in a row: the node's own column (blank arc, stores) and its label arc's
  // column (alpha: the arc from u - 1; beta: the arc from u itself)
  uint32_t vb[PPL], vy[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int u = lane * PPL + j;
    vb[j] = u <= Ub ? (uint32_t)(4 * u) : kDrop;
    const int uy = BETA ? u : u - 1;
    vy[j] = (uy >= 0 && uy < Ub && u <= Ub) ? (uint32_t)(4 * uy) : kDrop;
  }
  const uint32_t rowb = 4u * (uint32_t)a.U1p;
  const int nbytes = (int)(rowb * (uint32_t)a.ND);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(a.ws.lpb + base, 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(a.ws.lpy + base, 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (BETA ? a.ws.beta : a.ws.alpha) + base, 0, nbytes, 0x00020000);
  double* offn = (BETA ? a.ws.offB : a.ws.offA) + (int64_t)b * a.ND;
  if (lane == 0) offn[0] = 0.0;
  // emissions of diagonal step i: alpha reads the arcs entering diagonal n = i from row n - 1,
  // beta the arcs leaving row n = nd - 1 - i
  auto row_of = [&](int i) {
    const int r = BETA ? nd - 1 - min(i, nd - 1) : min(i, nd - 1) - 1;
    return r < 0 ? 0 : r;
  };
  float ebA[kAb1P][PPL], eyA[kAb1P][PPL], ebB[kAb1P][PPL], eyB[kAb1P][PPL];
  auto load = [&](float (&eb)[kAb1P][PPL], float (&ey)[kAb1P][PPL], int i0) {
#pragma unroll
    for (int s = 0; s < kAb1P; ++s) {
      const uint32_t so = (uint32_t)row_of(i0 + s) * rowb;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        eb[s][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, vb[j], so, 0));
        ey[s][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(yrs, vy[j], so, 0));
      }
    }
  };
  float v[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) v[j] = kDeadR;
  double off = 0.0;
  auto body = [&](const float (&eb)[kAb1P][PPL], const float (&ey)[kAb1P][PPL], int i0)
      __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < kAb1P; ++s) {
      const int i = i0 + s;
      if (i >= nd) break;
      const int n = BETA ? nd - 1 - i : i;
      float nb[PPL];   // the neighbour u -/+ 1 on the previous diagonal
      if (!BETA) {
        nb[0] = dpp_shr1(v[PPL - 1]);
#pragma unroll
        for (int j = 1; j < PPL; ++j) nb[j] = v[j - 1];
      } else {
        nb[PPL - 1] = dpp_shl1(v[0]);
#pragma unroll
        for (int j = 0; j + 1 < PPL; ++j) nb[j] = v[j + 1];
      }
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const int u = lane * PPL + j;
        const int t = n - u;
        const bool valid = u <= Ub && t >= 0 && t < Tb;
        float nv;
        if (!BETA) {
          nv = i == 0 ? (u == 0 ? 0.0f : kDeadR)
                      : lse2_live(t >= 1 ? v[j] + eb[s][j] : kDeadR, u >= 1 ? nb[j] + ey[s][j] : kDeadR);
        } else {
          nv = i == 0 ? (u == Ub ? eb[s][j] : kDeadR)   // terminal blank of (Tb-1, Ub)
                      : lse2_live(t + 1 < Tb ? v[j] + eb[s][j] : kDeadR, u < Ub ? nb[j] + ey[s][j] : kDeadR);
        }
        v[j] = valid ? fmaxf(nv, kDeadR) : kDeadR;
      }
      if ((i + 1) % kAb1R == 0) {   // re-centre on the wave max
        float m = kDeadR;
#pragma unroll
        for (int j = 0; j < PPL; ++j) m = fmaxf(m, v[j]);
        m = wave_max_dpp(m);
        if (m > 0.5f * kDeadR) {   // all dead: keep the sentinel
#pragma unroll
          for (int j = 0; j < PPL; ++j) v[j] -= m;
          off += (double)m;
        }
        if (lane == 0) offn[(i + 1) / kAb1R] = off;
      }
      const uint32_t so = (uint32_t)n * rowb;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const int u = lane * PPL + j;
        const int t = n - u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[j]), ors,
                                              (u <= Ub && t >= 0 && t < Tb) ? vb[j] : kDrop, so, 0);
      }
    }
  };
  load(ebA, eyA, 0);
  for (int i0 = 0; i0 < nd; i0 += 2 * kAb1P) {
    load(ebB, eyB, i0 + kAb1P);
    body(ebA, eyA, i0);
    if (i0 + kAb1P >= nd) break;
    load(ebA, eyA, i0 + 2 * kAb1P);
    body(ebB, eyB, i0 + kAb1P);
  }
  if (!BETA) {
    // the emission shift of every path, sum_t cb[t] + sum_{u<Ub} cy[u], fp64 in a fixed order
    double cs = 0.0;
    for (int i = lane; i < Tb + Ub; i += 64)
      cs += (double)kshift(i < Tb ? a.ws.cmb[(int64_t)b * a.T + i] : a.ws.cmy[(int64_t)b * a.U1 + i - Tb]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o);
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      if (lane * PPL + j == Ub) {   // log P = alpha(Tb-1, Ub) + its terminal blank (+ the shift)
        const double lp = (double)v[j] + (double)a.ws.lpb[base + (int64_t)(nd - 1) * a.U1p + Ub] + off;
        a.ws.logp2[b] = lp;
        a.nll[b] = (float)(-(lp + cs) * 0.6931471805599453);
      }
    }
  }
}

template <int PPL>
__global__ void __launch_bounds__(64) rnnt_ab1_kernel(RnntArgs a) {
  const bool is_beta = blockIdx.x >= a.B;
  const int b = is_beta ? blockIdx.x - a.B : blockIdx.x;
  const int Tb = clampr(a.flen[b], 0, a.T), Ub = clampr(a.llen[b], 0, a.Umax);
  if (Tb == 0) {   // no frames: no alignment exists
    if (!is_beta && threadIdx.x == 0) {
      a.nll[b] = __builtin_huge_valf();
      a.ws.logp2[b] = -__builtin_huge_val();
    }
    return;
  }
  if (is_beta) ab1_run<PPL, true>(a, b, Tb, Ub);
  else ab1_run<PPL, false>(a, b, Tb, Ub);
}

// label positions per lane of the one-wave lattice (0: the multi-wave kernel).  Off unless
// SC_RNNT_AB1=1 in the environment: measured at C5 (B=32, T=1500, U=150; profiles/
// r4_lattice_ab.md) the one-wave kernel took 411 us against the multi-wave kernel's 205 us —
// with PPL = 3 label positions per lane, one wave issues three log-sum-exps (6 quarter-rate
// exp2 / log2) per diagonal, where three waves of the multi-wave kernel issue one each.
int ab1_ppl(int Umax) {
  static const bool on = [] {
    const char* e = getenv("SC_RNNT_AB1");
    return e && e[0] == '1';
  }();
  const int ppl = (Umax + 1 + 63) / 64;
  return (on && ppl <= 4) ? ppl : 0;
}

template <int K>
__global__ void __launch_bounds__(1024) rnnt_ab_kernel(RnntArgs a) {
  const bool is_beta = blockIdx.x >= a.B;
  const int b = is_beta ? blockIdx.x - a.B : blockIdx.x;
  const int Tb = clampr(a.flen[b], 0, a.T), Ub = clampr(a.llen[b], 0, a.Umax);
  if (Tb == 0) {   // no frames: no alignment exists
    if (!is_beta && threadIdx.x == 0) {
      a.nll[b] = __builtin_huge_valf();
      a.ws.logp2[b] = -__builtin_huge_val();
    }
    return;
  }
  if (is_beta) ab_run<K, true>(a, b, Tb, Ub);
  else ab_run<K, false>(a, b, Tb, Ub);
}

// ---------------------------------------------------------------------------- gradient ------
// N consecutive gradient values (N = elements per 16 bytes of the INPUT type) as 16-byte stores
// of the gradient type (two stores for an fp32 gradient of 16-bit logits).
template <int GT, int N>
__device__ __forceinline__ void store_row_vec(typename Elem<GT>::T* g, const float (&f)[N]) {
  constexpr int NG = Vec16<GT>::N;
#pragma unroll
  for (int h = 0; h < N / NG; ++h) {
    float q[NG];
#pragma unroll
    for (int k = 0; k < NG; ++k) q[k] = f[h * NG + k];
    Vec16<GT>::st(g + h * NG, q);
  }
}

template <int DT, int GT>
__global__ void __launch_bounds__(256) rnnt_grad_kernel(RnntArgs a) {
  using E = Elem<DT>;
  using G = Elem<GT>;
  const int lane = threadIdx.x & 63;
  const int64_t node = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (node >= (int64_t)a.B * a.T * a.U1) return;
  const int b = (int)(node / ((int64_t)a.T * a.U1));
  const int t = (int)((node / a.U1) % a.T), u = (int)(node % a.U1);
  const int Tb = clampr(a.flen[b], 0, a.T), Ub = clampr(a.llen[b], 0, a.Umax);
  const bool valid = t < Tb && u <= Ub;
  if (!valid && a.row_off) return;   // compact rows exist only for valid nodes
  const int64_t row = valid ? node_row(a, b, t, u, Ub)
                            : (int64_t)b * a.sb + (int64_t)t * a.st + (int64_t)u * a.su;
  typename G::T* g = (typename G::T*)a.grad + row;
  if (!valid) {   // dense padding rows carry no loss
    if (a.vec) {
      constexpr int N = Vec16<DT>::N;
      float z[N];
#pragma unroll
      for (int k = 0; k < N; ++k) z[k] = 0.0f;
      for (int j = 0; j < a.nvec; ++j) store_row_vec<GT, N>(g + (j * 64 + lane) * N, z);
    } else {
      for (int v = lane; v < a.V; v += 64) g[v] = G::st(0.0f);
    }
    return;
  }
  const double lp2 = a.ws.logp2[b];
  const float sc = a.scale[b];
  float gb = 0.0f, gy = 0.0f;
  if (lp2 > -1e300 && sc != 0.0f) {
    const int n = t + u;
    const int64_t base = (int64_t)b * a.ND * a.U1p;
    // offsets: one per re-centring (every 2 kh diagonals); alpha's step index is n, beta's
    // nd - 1 - n' for diagonal n' = n + 1
    const int per = 2 * a.kh, nd = Tb + Ub;
    const double oA = a.ws.offA[(int64_t)b * a.ND + (n + 1) / per];
    const double oB = a.ws.offB[(int64_t)b * a.ND + (nd - n - 1) / per];
    const double al = (double)a.ws.alpha[base + (int64_t)n * a.U1p + u] + oA;
    const float eb = a.ws.lpb[base + (int64_t)n * a.U1p + u];
    if (t + 1 < Tb) {
      const double be = (double)a.ws.beta[base + (int64_t)(n + 1) * a.U1p + u] + oB;
      gb = -exp2_((float)(al + eb + be - lp2));
    } else if (u == Ub) {
      gb = -exp2_((float)(al + eb - lp2));
    }
    if (u < Ub) {
      const float ey = a.ws.lpy[base + (int64_t)n * a.U1p + u];
      const double be = (double)a.ws.beta[base + (int64_t)(n + 1) * a.U1p + u + 1] + oB;
      gy = -exp2_((float)(al + ey + be - lp2));
    }
    gb *= sc;
    gy *= sc;
  }
  const int yl = u < Ub ? label_at(a, b, u) : -1;
  const typename E::T* x = (const typename E::T*)a.x + row;
  const float lse = a.ws.lse[node];
  const float tot = gb + gy;
  if (a.vec) {
    using VX = Vec16<DT>;
    for (int j = 0; j < a.nvec; ++j) {
      const int v0 = (j * 64 + lane) * VX::N;
      float f[VX::N];
      if (a.is_logits) {
        VX::ld(x + v0, f);
      }
#pragma unroll
      for (int k = 0; k < VX::N; ++k) {
        float o = a.is_logits ? -fexp(f[k] - lse) * tot : 0.0f;
        if (v0 + k == a.blank) o += gb;
        if (v0 + k == yl) o += gy;
        f[k] = o;
      }
      store_row_vec<GT, VX::N>(g + v0, f);
    }
    return;
  }
  for (int v = lane; v < a.V; v += 64) {
    float o = a.is_logits ? -fexp(E::ld(x[v]) - lse) * tot : 0.0f;
    if (v == a.blank) o += gb;
    if (v == yl) o += gy;
    g[v] = G::st(o);
  }
}

void launch_ab(const RnntArgs& a, hipStream_t st) {
  switch (ab1_ppl(a.Umax)) {
    case 1: hipLaunchKernelGGL((rnnt_ab1_kernel<1>), dim3(2 * a.B), dim3(64), 0, st, a); return;
    case 2: hipLaunchKernelGGL((rnnt_ab1_kernel<2>), dim3(2 * a.B), dim3(64), 0, st, a); return;
    case 3: hipLaunchKernelGGL((rnnt_ab1_kernel<3>), dim3(2 * a.B), dim3(64), 0, st, a); return;
    case 4: hipLaunchKernelGGL((rnnt_ab1_kernel<4>), dim3(2 * a.B), dim3(64), 0, st, a); return;
    default: break;
  }
  const int K = a.kh;
  const int nw = (a.U1 + (64 - K) - 1) / (64 - K);
  const size_t sh = 2 * (size_t)nw * (64 - K) * sizeof(float);
  switch (K) {
    case 16: hipLaunchKernelGGL((rnnt_ab_kernel<16>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    case 8: hipLaunchKernelGGL((rnnt_ab_kernel<8>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    case 4: hipLaunchKernelGGL((rnnt_ab_kernel<4>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    case 2: hipLaunchKernelGGL((rnnt_ab_kernel<2>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    default: hipLaunchKernelGGL((rnnt_ab_kernel<1>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
  }
}

// the shift maxima start at key 0 ("nothing seen"); the emission producers raise them
void clear_shift(const RnntArgs& a, hipStream_t st) {
  zero_async(a.ws.cmb, (size_t)a.B * (a.T + a.U1) * 4, st);
}
// shift the emissions, then alpha / beta
void launch_lattice(const RnntArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.ND;
  hipLaunchKernelGGL(rnnt_shift_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a);
  launch_ab(a, st);
}

template <int DT>
void launch_fwd(const RnntArgs& a, hipStream_t st) {
  const int64_t nodes = (int64_t)a.B * a.T * a.U1;
  clear_shift(a, st);
  hipLaunchKernelGGL((rnnt_emit_kernel<DT>), dim3((unsigned)((nodes + 3) / 4)), dim3(256), 0, st, a);
  launch_lattice(a, st);
}

template <int DT, int GT>
void launch_bwd(const RnntArgs& a, hipStream_t st) {
  const int64_t nodes = (int64_t)a.B * a.T * a.U1;
  hipLaunchKernelGGL((rnnt_grad_kernel<DT, GT>), dim3((unsigned)((nodes + 3) / 4)), dim3(256), 0,
                     st, a);
}

int rnnt_check(const void* x, int dt, int B, int T, int Umax, int V, const int64_t* labels,
               const int64_t* fl, const int64_t* ll, int blank, const void* ws, size_t wsb,
               const char* who) {
  SC_REQUIRE(dt == SC_F32 || dt == SC_BF16 || dt == SC_F16, "%s: unsupported dtype %d", who, dt);
  SC_REQUIRE(B >= 0 && T >= 0 && V > 0 && Umax >= 0, "%s: bad shape", who);
  SC_REQUIRE(ab_halo_k(Umax) > 0, "%s: max label count %d exceeds %d", who, Umax, 16 * 63 - 1);
  SC_REQUIRE(blank >= 0 && blank < V, "%s: blank %d outside [0, %d)", who, blank, V);
  SC_REQUIRE((int64_t)B * T * (Umax + 1) < (1ll << 40), "%s: lattice too large", who);
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(x && fl && ll && ws, "%s: null pointer", who);
  SC_REQUIRE(Umax == 0 || labels, "%s: null labels", who);
  const size_t need = ws_layout(B, T, Umax, nullptr, nullptr);
  SC_REQUIRE(wsb >= need, "%s: workspace %zu < %zu bytes", who, wsb, need);
  return 0;
}

RnntArgs make_args(const void* x, int is_logits, int B, int T, int Umax, int V, int64_t sb,
                   int64_t st, int64_t su, const int64_t* row_off, const int64_t* labels,
                   int64_t labs, const int64_t* fl, const int64_t* ll, int blank, float* nll,
                   const void* ws, const float* scale, void* grad) {
  RnntArgs a;
  a.x = x;
  a.is_logits = is_logits;
  a.B = B;
  a.T = T;
  a.Umax = Umax;
  a.V = V;
  a.blank = blank;
  a.U1 = Umax + 1;
  a.U1p = u1p_of(Umax);
  a.ND = T + Umax;
  a.sb = sb;
  a.st = st;
  a.su = su;
  a.row_off = row_off;
  a.lab = labels;
  a.labs = labs;
  a.flen = fl;
  a.llen = ll;
  a.nll = nll;
  ws_layout(B, T, Umax, &a.ws, const_cast<void*>(ws));
  a.scale = scale;
  a.grad = grad;
  a.vec = 0;
  a.nvec = 0;
  // diagonals per re-centring / 2 (the gradients' offset index)
  a.kh = ab1_ppl(Umax) ? kAb1R / 2 : ab_halo_k(Umax);
  return a;
}

// rows as 16-byte vectors when every row start is 16-byte aligned and V fills whole vectors
void set_vec(RnntArgs& a, int esize) {
  const int n = 16 / esize;
  const bool al = ((uintptr_t)a.x % 16 == 0) && (!a.grad || (uintptr_t)a.grad % 16 == 0) &&
                  a.su % n == 0 && (a.row_off || (a.sb % n == 0 && a.st % n == 0));
  if (al && a.V % (64 * n) == 0 && a.V / (64 * n) <= kNvMax) {
    a.vec = 1;
    a.nvec = a.V / (64 * n);
  }
}

int esize_of(int dt) { return dt == SC_F32 ? 4 : 2; }

// ------------------------------------------------------------------ fused joiner (C5) -----
// RNNTPredictorJoiner (model.py:112-145) + the fp32 log_softmax of model.py:93 + the gathered
// lattice, WITHOUT the (B, T, U+1, V) logits (928 MB per utterance in fp32 at T=1500, U=150,
// V=1024).  Node n = (b, t, u): z_n = tanh(enc[b,t] + pred[b,u]) (J = 64), logits_n = W z_n + bias.
//
//   joint_fwd_kernel  logits on MFMA (v_mfma_f32_32x32x16_bf16, W resident in LDS, z as the B
//                     operand computed in registers), online log-sum-exp over V with the node on the
//                     lane (the 32x32 accumulator holds one node's 16 logits per lane), blank and
//                     label logits as direct dot products -> lse, lpb, lpy in rnnt_ab's layout.
//   joint_bwd_kernel  backward in one pass: logits recomputed once, dense dlogits = a_n softmax_n
//                     (a_n = occupancy of the node's two arcs x scale) feed both dW (accumulator
//                     as the next MFMA's operand, dW resident in registers) and dZ (p transposed
//                     through LDS); d pre = dZ (1 - z^2) -> d enc / d pred partials (see below).
// Each kernel evaluates exp once per logit; the logits themselves never leave registers.
constexpr int kJ = 64;
constexpr int kVmaxJ = 1024;   // W image [V][64] bf16 = 128 KB of LDS
typedef __bf16 jbf8 __attribute__((ext_vector_type(8)));
typedef float jf16 __attribute__((ext_vector_type(16)));
typedef short js4 __attribute__((ext_vector_type(4)));

struct JointArgs {
  RnntArgs r;
  const float* enc;    // [B][T][64]   enc_proj(enc_out), contiguous
  const float* pred;   // [B][U1][64]  pred_proj(embedding(blank-prefixed labels)), contiguous
  const __bf16* W;     // [V][64]      joiner.weight
  const float* bias;   // [V]          joiner.bias
  int ntb, nus, S, vs;   // t-blocks, u-splits, dW slices, vocab splits of the backward
  float* d_enc;        // [vs * nus][B][T][64]
  float* d_pred;       // [B][vs * ntb][U1][64]   (vocab split vh at t-block row vh * ntb + tb)
  float* dW;           // [S][V][64]       partials of sum_n dlogits_n z_n^T
  float* db;           // [S][V]
};

// [row][8 x 16 B] images, the chunk XOR-swizzled by s(row) = ((row >> 1) & 1) << 2 | (row >> 2) & 3.
// A 256-B bank row holds two image rows, so a slot is (row & 1) 8 + (chunk ^ s(row)): the 16 rows
// of a ds_read_b128 lane group (distinct row & 15, one chunk) and the 4 aligned rows x 4 aligned
// chunks of a ds_read_b64_tr_b16 half both land on 16 distinct slots (row & 7 as the swizzle left
// both 2-way: rows r and r + 2 of a transposed read, r and r + 8 of a row read shared a slot)
__device__ __forceinline__ uint32_t wswz(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ uint32_t wimg(int row, int chunk) {
  return (uint32_t)(row * 128 + 16 * (chunk ^ wswz(row)));
}
// the joint backward's p image: as wimg, and the two 8-byte halves of a chunk swapped on odd rows,
// so that the 16 rows of a ds_write_b64 lane group (one chunk, one half) take the 16 distinct
// 8-byte places of a 128-B write bank window; col is an element index, a multiple of 4
__device__ __forceinline__ uint32_t pimg_off(int row, int col) {
  return wimg(row, col >> 3) + 8 * (((col >> 2) & 1) ^ (row & 1));
}

__device__ __forceinline__ jbf8 lds_b128(const unsigned char* lds, uint32_t off) {
  return *(const jbf8*)(lds + off);
}

// ds_read_b64_tr_b16: group lane 4q+p addresses row R0+q, columns C0+4p..+3 of the image; lane i
// of the group receives column C0+i of rows R0..R0+3
template <bool P = false>
__device__ __forceinline__ js4 tr_rd(const unsigned char* lds, int R0, int C0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int row = R0 + q, col = C0 + 4 * p;
  const uint32_t off = P ? pimg_off(row, col) : wimg(row, col >> 3) + 8 * ((col >> 2) & 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (js4 __attribute__((address_space(3)))*)(size_t)(lds_addr(lds) + off));
}

__device__ __forceinline__ jbf8 cat8(js4 lo, js4 hi) {
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(jbf8, r);
}

__device__ __forceinline__ jf16 mfma32(jbf8 a, jbf8 b, jf16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float tanh_(float x) {
  return 1.0f - 2.0f * rcp(exp2_(2.0f * kLog2e * x) + 1.0f);
}

// registers 8s..8s+7 of an accumulator as a bf16 fragment (k-step s of a following MFMA that
// sums over the accumulator's row index)
__device__ __forceinline__ jbf8 pack8(const float* p) {
  jbf8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)p[e];
  return r;
}

// cooperative copy of W (bf16 [V][64]) and bias into the LDS images
__device__ __forceinline__ void load_w(const JointArgs& a, unsigned char* lds) {
  const int V = a.r.V;
  for (int i = threadIdx.x; i < V * 8; i += blockDim.x) {
    const int v = i >> 3, c = i & 7;
    *(uint4*)(lds + wimg(v, c)) = *(const uint4*)(a.W + (int64_t)v * kJ + 8 * c);
  }
  float* bias = (float*)(lds + kVmaxJ * 128);
  for (int i = threadIdx.x; i < V; i += blockDim.x) bias[i] = a.bias[i];
}

// z of (b, t, u) at j = 16 s + 8 h + e (the B operand of the node-on-lane logits MFMA), bf16, for
// the task's two columns u0, u0 + 1 (nc of them valid).  Every load is issued before the first
// tanh: one exposed memory latency per task (per-s loads and uses had the compiler wait vmcnt(0)
// eight times).
__device__ __forceinline__ void z_frags2(const JointArgs& a, int b, int t, int u0, int nc, bool ok,
                                         int h, jbf8 (&zb)[2][4]) {
  const float* ep = a.enc + ((int64_t)b * a.r.T + t) * kJ + 8 * h;
  const float* pp0 = a.pred + ((int64_t)b * a.r.U1 + u0) * kJ + 8 * h;
  const float* pp1 = nc > 1 ? pp0 + kJ : pp0;
  float4 e[8], p0[8], p1[8];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    e[2 * s] = *(const float4*)(ep + 16 * s);
    e[2 * s + 1] = *(const float4*)(ep + 16 * s + 4);
    p0[2 * s] = *(const float4*)(pp0 + 16 * s);
    p0[2 * s + 1] = *(const float4*)(pp0 + 16 * s + 4);
    p1[2 * s] = *(const float4*)(pp1 + 16 * s);
    p1[2 * s + 1] = *(const float4*)(pp1 + 16 * s + 4);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float4* p = c ? p1 : p0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float4 e0 = e[2 * s], e1 = e[2 * s + 1], q0 = p[2 * s], q1 = p[2 * s + 1];
      const float x[8] = {e0.x + q0.x, e0.y + q0.y, e0.z + q0.z, e0.w + q0.w,
                          e1.x + q1.x, e1.y + q1.y, e1.z + q1.z, e1.w + q1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) zb[c][s][k] = (__bf16)(ok ? tanh_(x[k]) : 0.0f);
    }
  }
}

// logits of one 32-row vocab block for the lane's node (node-on-lane orientation):
// acc[r] = bias[v] + sum_j W[v][j] z[j], v = v0 + (r&3) + 8(r>>2) + 4h
__device__ __forceinline__ jf16 logits_vblock(const unsigned char* lds, int v0, int lane,
                                              const jbf8 (&zb)[4]) {
  const int h = lane >> 5;
  const float* bias = (const float*)(lds + kVmaxJ * 128);
  jf16 acc;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 bb = *(const float4*)(bias + v0 + 8 * q + 4 * h);
    acc[4 * q + 0] = bb.x;
    acc[4 * q + 1] = bb.y;
    acc[4 * q + 2] = bb.z;
    acc[4 * q + 3] = bb.w;
  }
  const int row = v0 + (lane & 31);
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = mfma32(lds_b128(lds, wimg(row, 2 * s + h)), zb[s], acc);
  return acc;
}

// sum over the lane's half (32 lanes) of 32 values per lane; lane l ends with the total of value
// index (l & 31) in v[0]
__device__ __forceinline__ void half_reduce32(float (&v)[32], int lane) {
#pragma unroll
  for (int st = 16; st >= 1; st >>= 1) {
    const bool up = (lane & st) != 0;
#pragma unroll
    for (int i = 0; i < st; ++i) {
      const float keep = up ? v[i + st] : v[i];
      const float send = up ? v[i] : v[i + st];
      v[i] = keep + __shfl_xor(send, st);
    }
  }
}

__device__ __forceinline__ float half_sum(float x) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// SC_JOINT_FWD_TREE: 1 = the vocab block's max and exponential sum as pairwise trees.  Measured
// slower (tools/j_ab.sh, C5 B=32: 2.28-2.29 ms vs 2.12-2.17 ms for the chains): the two columns
// and two waves per SIMD already cover the chains' latency, and the trees cost registers.
#ifndef SC_JOINT_FWD_TREE
#define SC_JOINT_FWD_TREE 0
#endif
__global__ void __launch_bounds__(512) joint_fwd_kernel(JointArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  load_w(a, lds);
  __syncthreads();
  const RnntArgs& r = a.r;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int nup = (r.U1 + 1) / 2;
  const int64_t ntask = (int64_t)r.B * a.ntb * nup;
  // (wave-uniform in an SGPR: the per-task lengths and labels become scalar loads)
  const int64_t wid = (int64_t)blockIdx.x * 8 + uniform(threadIdx.x >> 6), nwv = (int64_t)gridDim.x * 8;
  for (int64_t task = wid; task < ntask; task += nwv) {
    const int b = (int)(task / ((int64_t)a.ntb * nup));
    const int tb = (int)((task / nup) % a.ntb), up = (int)(task % nup);
    const int Tb = clampr(r.flen[b], 0, r.T), Ub = clampr(r.llen[b], 0, r.Umax);
    const int t = tb * 32 + (lane & 31);
    if (uniform(tb * 32) >= Tb || 2 * up > Ub) continue;
    const bool tok = t < Tb;
    const int tc = tok ? t : Tb - 1;
    const int nc = (2 * up + 1 <= Ub) ? 2 : 1;
    jbf8 zb[2][4];
    float m[2], s[2];
    // the two columns' labels, loaded beside z (used after the vocab loop)
    int ylab[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) ylab[c] = 2 * up + c < Ub ? label_at(r, b, 2 * up + c) : r.blank;
    z_frags2(a, b, tc, 2 * up, nc, tok, h, zb);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      m[c] = -__builtin_huge_valf();
      s[c] = 0.0f;
    }
    for (int v0 = 0; v0 < r.V; v0 += 32) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (c >= nc) break;
        const jf16 x = logits_vblock(lds, v0, lane, zb[c]);
#if SC_JOINT_FWD_TREE
        // the block's max and exponential sum as pairwise trees (depth 4, not chains of 15 / 16
        // dependent operations: the loop is one latency chain per column and wave)
        float t8[8], e[16];
#pragma unroll
        for (int q = 0; q < 8; ++q) t8[q] = fmaxf(x[2 * q], x[2 * q + 1]);
#pragma unroll
        for (int w2 = 4; w2 >= 1; w2 >>= 1)
#pragma unroll
          for (int q = 0; q < w2; ++q) t8[q] = fmaxf(t8[2 * q], t8[2 * q + 1]);
        const float bm = t8[0];
        const float mn = fmaxf(m[c], bm), ml = mn * kLog2e;
#pragma unroll
        for (int q = 0; q < 16; ++q) e[q] = exp2_(fmaf(x[q], kLog2e, -ml));
#pragma unroll
        for (int w2 = 8; w2 >= 1; w2 >>= 1)
#pragma unroll
          for (int q = 0; q < w2; ++q) e[q] = e[2 * q] + e[2 * q + 1];
        s[c] = fmaf(s[c], exp2_(m[c] * kLog2e - ml), e[0]);
        m[c] = mn;
#else
        float bm = x[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) bm = fmaxf(bm, x[q]);
        const float mn = fmaxf(m[c], bm), ml = mn * kLog2e;
        float acc = s[c] * exp2_(m[c] * kLog2e - ml);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += exp2_(fmaf(x[q], kLog2e, -ml));
        s[c] = acc;
        m[c] = mn;
#endif
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (c >= nc) break;
      const int u = 2 * up + c;
      const float mo = __shfl_xor(m[c], 32), so = __shfl_xor(s[c], 32);
      const float M = fmaxf(m[c], mo);
      const float lse = M + flog(s[c] * exp2_((m[c] - M) * kLog2e) + so * exp2_((mo - M) * kLog2e));
      // blank and label logits: dot products over the lane's 32 j, halves combined
      const int yl = ylab[c];
      float lb = 0.0f, ly = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const jbf8 wb = lds_b128(lds, wimg(r.blank, 2 * q + h));
        const jbf8 wy = lds_b128(lds, wimg(yl, 2 * q + h));
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float zf = (float)zb[c][q][e];
          lb = fmaf((float)wb[e], zf, lb);
          ly = fmaf((float)wy[e], zf, ly);
        }
      }
      lb += __shfl_xor(lb, 32);
      ly += __shfl_xor(ly, 32);
      const float* bias = (const float*)(lds + kVmaxJ * 128);
      lb += bias[r.blank];
      ly += bias[yl];
      const float lb2 = fmaxf((lb - lse) * kLog2e, kDeadR);
      const float ly2 = u < Ub ? fmaxf((ly - lse) * kLog2e, kDeadR) : kDeadR;
      if (h == 0 && tok) {
        const int64_t node = ((int64_t)b * r.T + t) * r.U1 + u;
        const int64_t d = ((int64_t)b * r.ND + t + u) * r.U1p + u;
        r.ws.lse[node] = lse;
        r.ws.lpb[d] = lb2;
        r.ws.lpy[d] = ly2;
        atomicMax(r.ws.cmb + (int64_t)b * r.T + t, fkey(lb2));
      }
      // label u's max over the column's 32 frames first: one atomic per column
      unsigned ky = (h == 0 && tok && u < Ub) ? fkey(ly2) : 0u;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) ky = max(ky, (unsigned)__shfl_xor((int)ky, o));
      if (lane == 0 && u < Ub) atomicMax(r.ws.cmy + (int64_t)b * r.U1 + u, ky);
    }
  }
}

// Backward in ONE pass over the logits (joint_bwd_kernel).  A workgroup of 4 waves (one per
// SIMD, up to 512 registers each) owns half of the vocabulary (16 blocks of 32 rows of W, 64 KB of
// LDS) and walks node columns (b, 32-frame t-block, u); every wave takes 4 of the vocab blocks of
// every column:
//   x[n][v] = z_n . W_v          (v_mfma_f32_32x32x16_bf16: node on the row, v on the lane)
//   p[n][v] = a_n exp(x + b_v - lse_n)                 (dense dlogits, once per logit)
//   dW[v][j] += sum_n p[n][v] z[n][j]   (p's registers are the A operand: the sum runs over the
//                                        accumulator's row index; dW stays in registers)
//   dZ[n][j] += sum_v p[n][v] W[v][j]   (p transposed through a 4 KB per-wave LDS image and read
//                                        back by ds_read_b64_tr_b16)
// The gathered lattice's sparse arcs enter p itself (p[n][blank] -= wb_n, p[n][y_u] -= wy_n in
// the one or two blocks holding those rows), so dW, d bias and dZ need no separate terms.
// dZ is a partial over the wave's vocab blocks; everything downstream of it is linear, so each
// wave folds its partial straight into d pre = dZ (1 - z^2), d enc (accumulated over u in a
// per-wave LDS partial) and d pred (summed over the t-block), and the partials meet only in small
// LDS reductions (d pred per column, d enc per task) and in the host's fixed-order sums over the
// vocab halves.  Node occupancies (alpha, beta, lse: fp64 offsets) of the next column are loaded
// while the current one computes.
// SC_JOINT_SB: a scheduling barrier between the vocab blocks of a column (A/B in tools only)
#ifndef SC_JOINT_SB
#define SC_JOINT_SB 1
#endif
#ifndef SC_JOINT_BF
#define SC_JOINT_BF 0
#endif
// SC_JOINT_ABL: ablation bits for tools timing only (never set in a shipped build; wrong results):
//   1 the column epilogue without the 1 - z^2 factor, 2 no column epilogue, 4 no exponentials,
//   8 no p transpose / dZ MFMAs
#ifndef SC_JOINT_ABL
#define SC_JOINT_ABL 0
#endif
// SC_JOINT_PRIO: s_setprio 1 on waves 4-7 for the whole kernel (MI355X_MICROARCH.md, "Two waves
// per SIMD", item 4: the second-dispatched half loses every arbitration to its older partner).
// Measured (tools/joint_probe.py, C5 B=32, A/B in one process): 6.80-6.87 -> 6.20-6.26 ms.
#ifndef SC_JOINT_PRIO
#define SC_JOINT_PRIO 1
#endif
#ifndef SC_JOINT_ST8   // 1: column staging on all 8 waves (0: waves 0-3, A/B in tools only)
#define SC_JOINT_ST8 1
#endif
// SC_JOINT_SKEW: the two waves of a SIMD run the column's phases in different orders -- waves
// 0-3 stage column u + 1 first and then compute column u, waves 4-7 (s_setprio 1) compute
// column u first and stage afterwards -- so that one wave's staging VALU / LDS work sits beside
// the other's MFMA blocks instead of both waves of a SIMD doing the same phase at once.  The
// DMA-issuing and node roles move to waves 0-3 (they issue early in the column).
#ifndef SC_JOINT_SKEW
#define SC_JOINT_SKEW 0
#endif
// SC_JOINT_DEPTH: LDS-DMA landing buffers of the column operands from HBM (pred row, node fields):
// 2 = the DMA of column u + 2 is issued while column u computes and retired at its end (one
// column of latency cover), 3 = column u + 3, retired at the end of column u + 1 (two columns).
// Measured equal (tools/j_ab.sh, C5 B=32: 6.24-6.44 ms either way): the column loop does not wait
// on these loads, so the shorter ring stays.
#ifndef SC_JOINT_DEPTH
#define SC_JOINT_DEPTH 2
#endif
constexpr int kVbWg = 16;   // vocab blocks (of 32) per workgroup
constexpr int kJW = 8;      // waves per workgroup: two per SIMD, so one wave's exp / pack /
                            // transpose work runs beside the other's MFMAs (<= 256 registers each)
constexpr int kVbW = kVbWg / kJW;   // vocab blocks per wave

// Node scalars of a column (the arcs' occupancies need alpha, beta, the emissions, lse and the
// fp64 offsets) and its pred row come into LDS by LDS-DMA one column ahead (wave 0; lanes 0..31 =
// the column's 32 nodes), not into VGPRs: a register prefetch held 24 registers across the
// column (the kernel spilled at 256) and was drained by the first scratch reload's or label
// load's vmcnt(0), one column early.  Field f of node i sits at [f][i].
constexpr int kNF = 11;   // alpha, lpb, lpy, beta(t+1), beta(u+1), lse, offA lo/hi, offB lo/hi, label
__device__ __forceinline__ void node_dma(const RnntArgs& a, int b, int t, int u, int Tb, int Ub,
                                         uint32_t dst) {
  const bool ok = t < Tb && u <= Ub;
  const int tc = ok ? t : 0, uc = ok ? u : 0;
  const int n = tc + uc;
  const int64_t base = (int64_t)b * a.ND * a.U1p;
  const int per = 2 * a.kh, nd = Tb + Ub;
  dma_to_lds<4>(a.ws.alpha + base + (int64_t)n * a.U1p + uc, dst);
  dma_to_lds<4>(a.ws.lpb + base + (int64_t)n * a.U1p + uc, dst + 128);
  dma_to_lds<4>(a.ws.lpy + base + (int64_t)n * a.U1p + uc, dst + 2 * 128);
  // (row n + 1 = ND for the lattice's last node of the last sequence: the workspace's next
  // region, read and never used)
  dma_to_lds<4>(a.ws.beta + base + (int64_t)(n + 1) * a.U1p + uc, dst + 3 * 128);
  dma_to_lds<4>(a.ws.beta + base + (int64_t)(n + 1) * a.U1p + min(uc + 1, a.U1p - 1), dst + 4 * 128);
  dma_to_lds<4>(a.ws.lse + ((int64_t)b * a.T + tc) * a.U1 + uc, dst + 5 * 128);
  const double* oa = a.ws.offA + (int64_t)b * a.ND + (n + 1) / per;
  const double* ob = a.ws.offB + (int64_t)b * a.ND + max(nd - n - 1, 0) / per;
  dma_to_lds<4>(oa, dst + 6 * 128);
  dma_to_lds<4>((const char*)oa + 4, dst + 7 * 128);
  dma_to_lds<4>(ob, dst + 8 * 128);
  dma_to_lds<4>((const char*)ob + 4, dst + 9 * 128);
  // the column's label (low dword of the int64; every lane the same address)
  if (Ub > 0) dma_to_lds<4>(a.lab + (int64_t)b * a.labs + min(u, Ub - 1), dst + 10 * 128);
}

__device__ __forceinline__ float f_at(const uint32_t* f, int k, int i) {
  return __uint_as_float(f[k * 32 + i]);
}
__device__ __forceinline__ double d_at(const uint32_t* f, int k, int i) {
  return __hiloint2double((int)f[(k + 1) * 32 + i], (int)f[k * 32 + i]);
}

// (wb, wy, lse2) of node i of a column whose fields landed at f: the two arcs' occupancies x the
// sequence's loss scale (as rnnt_grad_kernel; both <= 0 there, returned here as positive weights)
__device__ __forceinline__ void node_finish(const uint32_t* f, int i, double lp2, float sc, int t,
                                            int u, int Tb, int Ub, float& wb, float& wy, float& l2) {
  const bool ok = t < Tb && u <= Ub;
  wb = 0.0f;
  wy = 0.0f;
  const double al = (double)f_at(f, 0, i) + d_at(f, 6, i);
  const double oB = d_at(f, 8, i);
  if (t + 1 < Tb) wb = exp2_((float)(al + f_at(f, 1, i) + ((double)f_at(f, 3, i) + oB) - lp2));
  else if (u == Ub) wb = exp2_((float)(al + f_at(f, 1, i) - lp2));
  if (u < Ub) wy = exp2_((float)(al + f_at(f, 2, i) + ((double)f_at(f, 4, i) + oB) - lp2));
  const bool live = ok && lp2 > -1e300 && sc != 0.0f;
  wb = live ? wb * sc : 0.0f;
  wy = live ? wy * sc : 0.0f;
  l2 = ok ? f_at(f, 5, i) * kLog2e : 1e30f;
}

struct BwdLds {   // byte offsets of the LDS regions
  static constexpr int kDeP = 36;                       // d enc partial row pitch (floats)
  static constexpr int kW = 0;                          // W half image [512][128 B]
  static constexpr int kBias = kW + kVbWg * 32 * 128;   // [512] fp32, x log2(e)
  // column operands, two buffers (column u + 1 is staged while u computes):
  static constexpr int kZ = kBias + kVbWg * 32 * 4;     // z bf16 image [2][32][128 B]
  static constexpr int kZP = 36;                        // 1 - z^2 row pitch (floats)
  static constexpr int kZ32 = kZ + 2 * 32 * 128;        // 1 - z^2 fp32 [2][64 j][kZP], node fastest
  static constexpr int kNs = kZ32 + 2 * 64 * kZP * 4;   // node scalars: c, wb, wy, label [2][4][32]
  static constexpr int kRed = kNs + 2 * 4 * 32 * 4;     // d pred partials [2][8][64]
  static constexpr int kEnc = kRed + 2 * kJW * 64 * 4;  // the task's enc rows fp32 [32][64]
  static constexpr int kP = kEnc + 32 * 64 * 4;         // per-wave p image [8][32][128 B]
  static constexpr int kDe = kP;                        // d enc partials [4][64 j][36], at the
                                                        // task's end: over the p images
  static constexpr int kPr = kP + (kJW * 32 * 128 > 4 * 64 * kDeP * 4 ? kJW * 32 * 128
                                                                       : 4 * 64 * kDeP * 4);
  // LDS-DMA landing zones, SC_JOINT_DEPTH - 1 columns ahead: pred rows [depth][64] fp32, node
  // fields [depth][kNF][32]
  static constexpr int kNd = kPr + SC_JOINT_DEPTH * 64 * 4;
  static constexpr int kEnd = kNd + SC_JOINT_DEPTH * kNF * 32 * 4;
};

__global__ void __launch_bounds__(64 * kJW) joint_bwd_kernel(JointArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const RnntArgs& r = a.r;
  const int nvb = r.V / 32, VS = a.vs;
  const int vh = blockIdx.x % VS, slot = blockIdx.x / VS, nslot = gridDim.x / VS;
  const int vb0 = vh * kVbWg, nvw = min(kVbWg, nvb - vb0);   // this workgroup's vocab blocks
  const int w = uniform(threadIdx.x >> 6);
  int th = threadIdx.x, lane = th & 63, h = lane >> 5;
  int g1 = (lane >> 4) & 1;
  unsigned char* wl = lds + BwdLds::kW;
  float* bias_l = (float*)(lds + BwdLds::kBias);
  unsigned char* const zimg0 = lds + BwdLds::kZ;
  float* const z320 = (float*)(lds + BwdLds::kZ32);   // 1 - z^2
  float* encl = (float*)(lds + BwdLds::kEnc);
  float* const ns0 = (float*)(lds + BwdLds::kNs);   // [2][c | wb | wy][32]
  unsigned char* pimg = lds + BwdLds::kP + w * 32 * 128;
  float* const red0 = (float*)(lds + BwdLds::kRed);   // [2][8][64]
  float* dep = (float*)(lds + BwdLds::kDe);              // [4][64][kDeP]: waves w, w + 4
  // this half of W and its bias (x log2 e)
  for (int i = th; i < nvw * 32 * 8; i += 64 * kJW) {
    const int v = i >> 3, c = i & 7;
    *(uint4*)(wl + wimg(v, c)) = *(const uint4*)(a.W + (int64_t)(vb0 * 32 + v) * kJ + 8 * c);
  }
  for (int i = th; i < nvw * 32; i += 64 * kJW) bias_l[i] = a.bias[vb0 * 32 + i] * kLog2e;

  jf16 acc[kVbW][2];
  float dbs[kVbW];
#pragma unroll
  for (int k = 0; k < kVbW; ++k) {
    dbs[k] = 0.0f;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[k][jb][q] = 0.0f;
  }
  const int ntbp = VS * a.ntb;   // t-block rows of the d pred / g partial layouts
  const int64_t ntask = (int64_t)r.B * a.ntb * a.nus;
#if SC_JOINT_ST8
  // staging spread over all 8 waves (node zn, j = 4 jq ..): each wave's share of the column's
  // serial work (tanh, node scalars, DMA issue, d pred) stays small, so the barrier does not wait
  // on one loaded wave; the roles: node DMA wave 6, pred DMA wave 5, node_finish wave 7, d pred
  // wave 4
  const int zn = th >> 4, jg = th & 15;
  constexpr bool stager = true;
  constexpr int kWn = SC_JOINT_SKEW ? 2 : 6, kWp = SC_JOINT_SKEW ? 1 : 5,
                kWf = SC_JOINT_SKEW ? 3 : 7, kWd = SC_JOINT_SKEW ? 0 : 4;
#else
  const int zn = (th >> 3) & 31, jg = th & 7;   // staging (threads < 256): node zn, j = 8 jg ..
  const bool stager = th < 256;
  constexpr int kWn = 0, kWp = 0, kWf = 0, kWd = 0;
#endif
  constexpr int kSE = SC_JOINT_ST8 ? 4 : 8;   // staged elements per thread
  if (SC_JOINT_PRIO && w >= 4) __builtin_amdgcn_s_setprio(1);
  for (int64_t task = slot; task < ntask; task += nslot) {
    const int b = (int)(task / ((int64_t)a.ntb * a.nus));
    const int tb = (int)((task / a.nus) % a.ntb), us = (int)(task % a.nus);
    const int Tb = clampr(r.flen[b], 0, r.T), Ub = clampr(r.llen[b], 0, r.Umax);
    // columns of this task (none when the t-block or the u-range lies outside the lattice: the
    // task still writes its zero d enc partial)
    const int ua = (int)((int64_t)us * r.U1 / a.nus);
    const int ue = tb * 32 < Tb ? min((int)((int64_t)(us + 1) * r.U1 / a.nus), Ub + 1) : ua;
    const bool zok = tb * 32 + zn < Tb;
    lds_barrier();   // the previous task's reads of encl / d enc partials are done
    // d enc of the task: this wave's partial over its vocab blocks, in registers across u
    // (Y's layout: [jb][q] = node (q & 3) + 8 (q >> 2) + 4 h, j = jb 32 + (lane & 31))
    float dacc[2][16];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < 16; ++q) dacc[jb][q] = 0.0f;
    if (ua < ue && stager) {
      const float* ep = a.enc + ((int64_t)b * r.T + (zok ? tb * 32 + zn : Tb - 1)) * kJ + kSE * jg;
#pragma unroll
      for (int e = 0; e < kSE; e += 4)
        *(float4*)(encl + zn * 64 + kSE * jg + e) = *(const float4*)(ep + e);
    }
    // the column operands that come from HBM (pred row, node scalars, label) land in LDS one
    // column ahead by LDS-DMA from wave 0 (node_dma), retired by wave 0's dma_wait() before the
    // column's barrier; no VGPR holds them and no compiler-visible load sits in the column loop
    uint32_t* const ndl0 = (uint32_t*)(lds + BwdLds::kNd);   // [depth][kNF][32]
    float* const prl0 = (float*)(lds + BwdLds::kPr);          // [depth][64]
    const double lp2 = r.ws.logp2[b];
    const float lsc = r.scale[b];
    auto col_dma = [&](int uu, int bf) __attribute__((always_inline)) {
      if (w == kWp)
        dma_to_lds<4>(a.pred + ((int64_t)b * r.U1 + uu) * kJ + lane, lds_addr(prl0 + bf * 64));
      if (w == kWn && lane < 32)
        node_dma(r, b, tb * 32 + lane, uu, Tb, Ub, lds_addr(ndl0 + bf * kNF * 32));
    };
    auto col_dma_wait = [&]() __attribute__((always_inline)) {
      if (w == kWp || w == kWn) dma_wait();
    };
    // retire every column DMA but the youngest column's (this wave's pieces per column: the pred
    // row 1, the node fields 10 + the label)
    auto col_dma_wait_older = [&]() __attribute__((always_inline)) {
      if (w == kWp) dma_wait_younger<1>();
      if (w == kWn) {
        if (Ub > 0) dma_wait_younger<kNF>();
        else dma_wait_younger<kNF - 1>();
      }
    };
    // DMA buffer of column uu (its landing zone)
    auto dbuf = [&](int uu) __attribute__((always_inline)) {
      return SC_JOINT_DEPTH == 2 ? (uu - ua) & 1 : (uu - ua) % SC_JOINT_DEPTH;
    };
    // stage column uu into buffer bf: z (bf16 image + fp32 1 - z^2), node scalars, label; the
    // DMA of the column after it is issued here and lands while this one computes
    auto stage = [&](int uu, int bf) __attribute__((always_inline)) {
      if (!stager) return;
      const int db = dbuf(uu);
      const float* pr = prl0 + db * 64 + kSE * jg;
      const float* el = encl + zn * 64 + kSE * jg;
      float xs[kSE];
#pragma unroll
      for (int e = 0; e < kSE; e += 4) {
        const float4 pv = *(const float4*)(pr + e), ev = *(const float4*)(el + e);
        xs[e] = ev.x + pv.x;
        xs[e + 1] = ev.y + pv.y;
        xs[e + 2] = ev.z + pv.z;
        xs[e + 3] = ev.w + pv.w;
      }
      float zf[kSE];
      __bf16 zb[kSE];
#pragma unroll
      for (int e = 0; e < kSE; ++e) {
        zf[e] = zok ? tanh_(xs[e]) : 0.0f;
        zb[e] = (__bf16)zf[e];
      }
      if constexpr (kSE == 8) {
        jbf8 z8;
#pragma unroll
        for (int e = 0; e < 8; ++e) z8[e] = zb[e];
        *(jbf8*)(zimg0 + bf * 32 * 128 + wimg(zn, jg)) = z8;
      } else {
        typedef __bf16 jbf4 __attribute__((ext_vector_type(4)));
        *(jbf4*)(zimg0 + bf * 32 * 128 + wimg(zn, jg >> 1) + 8 * (jg & 1)) =
            jbf4{zb[0], zb[1], zb[2], zb[3]};
      }
      // tanh' = 1 - z^2, once per element (every wave scales its dZ partial by it)
      // ([j][n]: the epilogue reads a lane's four consecutive nodes as one 16-byte piece)
      float* zz = z320 + bf * 64 * BwdLds::kZP + kSE * jg * BwdLds::kZP + zn;
#pragma unroll
      for (int e = 0; e < kSE; ++e) zz[e * BwdLds::kZP] = 1.0f - zf[e] * zf[e];
      if (w == kWf && lane < 32) {
        const int th = lane;
        const uint32_t* nf = ndl0 + db * kNF * 32;
        float wb, wy, l2;
        node_finish(nf, th, lp2, lsc, tb * 32 + th, uu, Tb, Ub, wb, wy, l2);
        const float an = wb + wy;
        // p = a exp2(x log2e + b log2e - l2) = exp2(x log2e + b log2e + c), c = log2 a - l2
        float* ns = ns0 + bf * 128;
        ns[th] = an > 0.0f ? log2_(an) - l2 : -1e30f;
        ns[32 + th] = wb;
        ns[64 + th] = wy;
        if (th == 0) {
          const int lab = (int)nf[10 * 32];
          ((int*)ns)[96] = uu < Ub ? (lab < 0 ? 0 : (lab >= r.V ? r.V - 1 : lab)) : r.blank;
        }
      }
      // (DMA buffer dbuf(uu + depth - 1) = dbuf(uu - 1) was read by stage(uu - 1), before the
      // barrier that ended column uu - 2)
      if (uu + SC_JOINT_DEPTH - 1 < ue) col_dma(uu + SC_JOINT_DEPTH - 1, dbuf(uu + SC_JOINT_DEPTH - 1));
    };
    if (ua < ue) {
#pragma unroll
      for (int d = 0; d < SC_JOINT_DEPTH - 1; ++d)
        if (ua + d < ue) col_dma(ua + d, d);
      col_dma_wait();
      lds_barrier();   // the first columns' DMA has landed
      stage(ua, 0);
    }
    if (SC_JOINT_DEPTH == 2) col_dma_wait();
    lds_barrier();
    for (int u = ua; u < ue; ++u) {
      // lane-dependent addresses re-derived per column, not held across it (register budget of
      // two waves per SIMD)
      asm volatile("" : "+v"(th), "+v"(lane), "+v"(h), "+v"(g1));
      const int cb = (u - ua) & 1;
      const unsigned char* zimg = zimg0 + cb * 32 * 128;
      const float* z32 = z320 + cb * 64 * BwdLds::kZP;
      const float* ns_c = ns0 + cb * 128;
      const float* ns_wb = ns_c + 32;
      const float* ns_wy = ns_c + 64;
      float* red = red0 + cb * kJW * 64;
      const bool stage_late = SC_JOINT_SKEW && w >= 4;
      if (u + 1 < ue && !stage_late) stage(u + 1, cb ^ 1);   // into the other buffer (read two columns ago)
      // column operands: z rows (logits A operand), z^T (dW B operand), node terms per register
      jbf8 zA[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) zA[s] = lds_b128(zimg, wimg(lane & 31, 2 * s + h));

      jf16 Y[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 16; ++q) Y[jb][q] = 0.0f;
      const int yl = uniform(((const int*)ns_c)[96]);
      // logits of vocab block k (W rows of a block past the vocabulary: block 0, p forced to 0)
      auto logits_blk = [&](int k) __attribute__((always_inline)) {
        const int lvb = w + kJW * k;
        const int vl = (lvb < nvw ? lvb : 0) * 32 + (lane & 31);
        jf16 x;
#pragma unroll
        for (int q = 0; q < 16; ++q) x[q] = 0.0f;
#pragma unroll
        for (int s = 0; s < 4; ++s) x = mfma32(zA[s], lds_b128(wl, wimg(vl, 2 * s + h)), x);
        return x;
      };
      // (no software pipeline across the wave's blocks: the other wave on the SIMD covers the
      // logits' latency, and its registers are the two-waves-per-SIMD budget)
#pragma unroll
      for (int k = 0; k < kVbW; ++k) {
        // every wave runs all kVbW blocks (no early exit: its PHIs cost a copy of Y)
        const int lvb = w + kJW * k;
        const bool vok = lvb < nvw;
        const int lvc = vok ? lvb : 0;   // (the W rows read for a block past the vocabulary)
        const int vl = lvc * 32 + (lane & 31);
        const jf16 x = logits_blk(k);
        const float bl = vok ? bias_l[vl] : -1e30f;
        float p[16], ps = 0.0f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // node terms c_n (re-read per block: registers)
          const float4 cv = *(const float4*)(ns_c + 8 * g + 4 * h);
          if (SC_JOINT_ABL & 4) {
            p[4 * g] = fmaf(x[4 * g], kLog2e, bl + cv.x);
            p[4 * g + 1] = fmaf(x[4 * g + 1], kLog2e, bl + cv.y);
            p[4 * g + 2] = fmaf(x[4 * g + 2], kLog2e, bl + cv.z);
            p[4 * g + 3] = fmaf(x[4 * g + 3], kLog2e, bl + cv.w);
          } else {
            p[4 * g] = exp2_(fmaf(x[4 * g], kLog2e, bl + cv.x));
            p[4 * g + 1] = exp2_(fmaf(x[4 * g + 1], kLog2e, bl + cv.y));
            p[4 * g + 2] = exp2_(fmaf(x[4 * g + 2], kLog2e, bl + cv.z));
            p[4 * g + 3] = exp2_(fmaf(x[4 * g + 3], kLog2e, bl + cv.w));
          }
        }
        // the sparse arcs of the gathered lattice: dlogits[n][blank] -= wb_n, dlogits[n][y_u] -=
        // wy_n (one or two blocks per column), so dW, d bias and dZ all take them from p
        const int vg0 = (vb0 + lvb) * 32;
#if SC_JOINT_BF
        {   // branch-free (A/B: one scheduling region per column)
#else
        if (vok && ((unsigned)(r.blank - vg0) < 32u || (unsigned)(yl - vg0) < 32u)) {
#endif
          const int v = vg0 + (lane & 31);
          const float mb = v == r.blank ? 1.0f : 0.0f, my = v == yl ? 1.0f : 0.0f;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 bw = *(const float4*)(ns_wb + 8 * g + 4 * h);
            const float4 yw = *(const float4*)(ns_wy + 8 * g + 4 * h);
            p[4 * g] -= mb * bw.x + my * yw.x;
            p[4 * g + 1] -= mb * bw.y + my * yw.y;
            p[4 * g + 2] -= mb * bw.z + my * yw.z;
            p[4 * g + 3] -= mb * bw.w + my * yw.w;
          }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) ps += p[q];
        dbs[k] += ps;
        jbf8 pf[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          pf[s2] = pack8(p + 8 * s2);
#pragma unroll
          for (int jb = 0; jb < 2; ++jb)   // z^T fragments re-read per block (registers)
            acc[k][jb] = mfma32(pf[s2],
                                cat8(tr_rd(zimg, 16 * s2 + 4 * h, jb * 32 + 16 * g1, lane),
                                     tr_rd(zimg, 16 * s2 + 8 + 4 * h, jb * 32 + 16 * g1, lane)),
                                acc[k][jb]);
        }
        // p^T through the wave's image: registers 4g..4g+3 are rows n = 8g + 4h .. +3 of column
        // v = lane & 31 -> 8 bytes at [v][8g + 4h] (whole packed dwords: element-wise bf16
        // extraction from the vector miscompiles into a broadcast of one element)
        typedef int ji2 __attribute__((ext_vector_type(2)));
        typedef int ji4 __attribute__((ext_vector_type(4)));
        if (SC_JOINT_ABL & 8) {
          asm volatile("" :: "v"(pf[0]), "v"(pf[1]));
          continue;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const ji4 d = __builtin_bit_cast(ji4, pf[g >> 1]);
          *(ji2*)(pimg + pimg_off(lane & 31, 8 * g + 4 * h)) = ji2{d[2 * (g & 1)], d[2 * (g & 1) + 1]};
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const jbf8 pt = cat8(tr_rd<true>(pimg, 16 * s2 + 4 * h, 16 * g1, lane),
                               tr_rd<true>(pimg, 16 * s2 + 8 + 4 * h, 16 * g1, lane));
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) {
            const jbf8 wt = cat8(tr_rd(wl, lvc * 32 + 16 * s2 + 4 * h, jb * 32 + 16 * g1, lane),
                                 tr_rd(wl, lvc * 32 + 16 * s2 + 8 + 4 * h, jb * 32 + 16 * g1, lane));
            Y[jb] = mfma32(pt, wt, Y[jb]);
          }
        }
#if SC_JOINT_SB
        __builtin_amdgcn_sched_barrier(0);   // one vocab block's live state at a time
#endif
      }
      // Y[jb][q] = this wave's part of dZ[node n_q][j = jb*32 + (lane & 31)],
      // n_q = (q & 3) + 8 (q >> 2) + 4 h: d pre = dZ (1 - z^2) into the wave's d enc partial
      // (LDS, [j][n]) and d pred (over n)
      // (registers 4g .. 4g+3 are the consecutive nodes 8g + 4h .. +3: one conflict-free 16-byte
      // read of [j][n] per g, and packed fp32 products / sums over register pairs)
      typedef float jf2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int jb = 0; jb < ((SC_JOINT_ABL & 2) ? 0 : 2); ++jb) {
        const int j = jb * 32 + (lane & 31);
        jf2 sp2 = {0.0f, 0.0f};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 zz = (SC_JOINT_ABL & 1) ? make_float4(1.f, 1.f, 1.f, 1.f)
                                               : *(const float4*)(z32 + j * BwdLds::kZP + 8 * g + 4 * h);
          const jf2 o0 = jf2{Y[jb][4 * g], Y[jb][4 * g + 1]} * jf2{zz.x, zz.y};
          const jf2 o1 = jf2{Y[jb][4 * g + 2], Y[jb][4 * g + 3]} * jf2{zz.z, zz.w};
          const jf2 a0 = jf2{dacc[jb][4 * g], dacc[jb][4 * g + 1]} + o0;
          const jf2 a1 = jf2{dacc[jb][4 * g + 2], dacc[jb][4 * g + 3]} + o1;
          dacc[jb][4 * g] = a0.x;
          dacc[jb][4 * g + 1] = a0.y;
          dacc[jb][4 * g + 2] = a1.x;
          dacc[jb][4 * g + 3] = a1.y;
          sp2 += o0 + o1;
        }
        float sp = sp2.x + sp2.y;
        sp += __shfl_xor(sp, 32);
        if (h == 0) red[w * 64 + j] = sp;
      }
      if (SC_JOINT_ABL & 2) asm volatile("" :: "v"(Y[0]), "v"(Y[1]));
      if (u + 1 < ue && stage_late) stage(u + 1, cb ^ 1);   // (SC_JOINT_SKEW: waves 4-7 stage last)
      // the column's one barrier: its d pred partials and the next column's operands are
      // complete (the DMA of column u + 2 included: at depth 3 issued one column earlier, the
      // younger one of column u + 3 stays in flight), and this column's buffer is free for
      // column u + 2
      if (SC_JOINT_DEPTH == 2 || u + SC_JOINT_DEPTH >= ue) col_dma_wait();   // (none younger)
      else col_dma_wait_older();
      lds_barrier();
      if (w == kWd) {   // d pred of this column: the wave partials (red buffers alternate)
        float s = 0.0f;
#pragma unroll
        for (int ww = 0; ww < kJW; ++ww) s += red[ww * 64 + lane];
        a.d_pred[(((int64_t)b * ntbp + vh * a.ntb + tb) * r.U1 + u) * kJ + lane] = s;
      }
    }
    // d enc of the task: the 8 waves' register partials meet in 4 LDS slots (waves w and w + 4
    // share slot w & 3, in two rounds), then 8 values per thread, j fastest (coalesced)
    float* slotp = dep + (w & 3) * 64 * BwdLds::kDeP;
#pragma unroll
    for (int rnd = 0; rnd < 2; ++rnd) {
      if ((w >> 2) == rnd) {
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          const int j = jb * 32 + (lane & 31);
#pragma unroll
          for (int g = 0; g < 4; ++g) {   // nodes 8g + 4h .. +3 = registers 4g .. 4g+3
            float4* de4 = (float4*)(slotp + j * BwdLds::kDeP + 8 * g + 4 * h);
            float4 v = make_float4(dacc[jb][4 * g], dacc[jb][4 * g + 1], dacc[jb][4 * g + 2],
                                   dacc[jb][4 * g + 3]);
            if (rnd) {
              const float4 o = *de4;
              v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            *de4 = v;
          }
        }
      }
      lds_barrier();
    }
    float* dst = a.d_enc + ((int64_t)(vh * a.nus + us) * r.B + b) * r.T * kJ;
#pragma unroll
    for (int i = 0; i < 32 * 64 / (64 * kJW); ++i) {
      const int e = th + 64 * kJW * i, n = e >> 6, j = e & 63;
      const int tq = tb * 32 + n;
      float s = 0.0f;
      if (ua < ue) {
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) s += dep[(ww * 64 + j) * BwdLds::kDeP + n];
      }
      if (tq < r.T) dst[(int64_t)tq * kJ + j] = s;
    }
  }
  // acc[k][jb][q] = dW[v = (vb0 + w + 4k) * 32 + (q&3) + 8(q>>2) + 4h][j = jb*32 + (lane&31)]
  float* dw = a.dW + (int64_t)slot * r.V * kJ;
#pragma unroll
  for (int k = 0; k < kVbW; ++k) {
    const int lvb = w + kJW * k;
    if (lvb >= nvw) continue;
    const int vbg = vb0 + lvb;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int v = vbg * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        dw[(int64_t)v * kJ + jb * 32 + (lane & 31)] = acc[k][jb][q];
      }
    const float tot = dbs[k] + __shfl_xor(dbs[k], 32);
    if (h == 0) a.db[(int64_t)slot * r.V + vbg * 32 + (lane & 31)] = tot;
  }
}

// ---------------------------------------------------------------------------------------------
// joint_bwd_pc_kernel: the same backward with the two waves of each SIMD in PRODUCER / CONSUMER
// roles (SC_JOINT_PC=1).  joint_bwd_kernel's column loop is one dependency chain per wave and
// vocab block (logits MFMA -> exp -> pack -> dW MFMA -> p image -> transposed reads -> dZ MFMA),
// ~3 k cycles per block against 384 MFMA cycles (profiles/r3c_joint_stamps.txt).  Here the chain
// is cut at the p image:
//   producer (waves 4-7, s_setprio 1), pair i = w - 4, vocab blocks i, i + 4, i + 8, i + 12:
//     per step one block of the current column: logits (4 MFMAs), p = exp(...) with the sparse
//     arcs, d bias, dW += p z (4 MFMAs, dW of the 4 blocks in registers), p image -> the pair's
//     LDS slot of this step;
//   consumer (waves 0-3), pair i: per step the block its producer finished one step earlier:
//     dZ += p^T W (the slot's transposed p, 4 MFMAs); after a column's last block the epilogue
//     (d pre = dZ (1 - z^2) into the d enc partial and the d pred partial) and, one step later,
//     the column staging (tanh of z, 1 - z^2, node scalars, the DMA of the column after next).
// One barrier per step (4 per column); the p slots alternate by step parity.  Staging runs one
// column ahead of the producer, so 1 - z^2 is triple-buffered (the consumer's epilogue of column
// u, column u + 1 waiting, u + 2 being staged).
// Measured (tools/r5_pc.sh, C5 B=32, alternated): 8.72-8.80 ms against 6.21-6.24 ms for
// joint_bwd_kernel, every joiner test passing on it.  The producer's per-block chain (logits ->
// exp -> dW -> p image, ~2 k cycles) is now the only chain in flight on its SIMD, where the
// one-pass kernel keeps two (one per wave); two chains per producer need ~270 registers with the
// consumer's dW / dZ / d enc state live across the same loop.  Kept off.
#ifndef SC_JOINT_PC
#define SC_JOINT_PC 0
#endif
#if SC_JOINT_PC   // (A/B builds only: tools/ab/jpc; not in the product library)
constexpr int kPcBlk = 4;   // vocab blocks per producer

struct PcLds {   // byte offsets
  static constexpr int kDeP = 36;
  static constexpr int kZP = 36;
  static constexpr int kW = 0;                            // W half image [512][128 B]
  static constexpr int kBias = kW + kVbWg * 32 * 128;     // [512] fp32, x log2(e)
  static constexpr int kZ = kBias + kVbWg * 32 * 4;       // z bf16 image [2][32][128 B]
  static constexpr int kZ32 = kZ + 2 * 32 * 128;          // 1 - z^2 [3][64 j][kZP], node fastest
  static constexpr int kNs = kZ32 + 3 * 64 * kZP * 4;     // node scalars c, wb, wy, label [2][128]
  static constexpr int kRed = kNs + 2 * 128 * 4;          // d pred partials [2][4][64]
  static constexpr int kEnc = kRed + 2 * 4 * 64 * 4;      // the task's enc rows fp32 [32][64]
  static constexpr int kP = kEnc + 32 * 64 * 4;           // p slots [2][4 pairs][32][128 B]
  static constexpr int kDe = kP;                          // d enc partials [4][64 j][kDeP]: at
                                                          // the task's end, over the p slots
  static constexpr int kPr = kP + (2 * 4 * 32 * 128 > 4 * 64 * kDeP * 4 ? 2 * 4 * 32 * 128
                                                                       : 4 * 64 * kDeP * 4);
  static constexpr int kNd = kPr + 2 * 64 * 4;            // LDS-DMA landing: pred [2][64]
  static constexpr int kEnd = kNd + 2 * kNF * 32 * 4;     // node fields [2][kNF][32]
};
static_assert(PcLds::kEnd <= 160 * 1024, "joint_bwd_pc LDS");

__global__ void __launch_bounds__(512) joint_bwd_pc_kernel(JointArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const RnntArgs& r = a.r;
  const int nvb = r.V / 32, VS = a.vs;
  const int vh = blockIdx.x % VS, slot = blockIdx.x / VS, nslot = gridDim.x / VS;
  const int vb0 = vh * kVbWg, nvw = min(kVbWg, nvb - vb0);
  const int w = uniform(threadIdx.x >> 6);
  const bool prod = w >= 4;
  const int pi = w & 3;   // pair
  int th = threadIdx.x, lane = th & 63, h = lane >> 5;
  int g1 = (lane >> 4) & 1;
  unsigned char* wl = lds + PcLds::kW;
  float* bias_l = (float*)(lds + PcLds::kBias);
  unsigned char* const zimg0 = lds + PcLds::kZ;
  float* const z320 = (float*)(lds + PcLds::kZ32);
  float* encl = (float*)(lds + PcLds::kEnc);
  float* const ns0 = (float*)(lds + PcLds::kNs);
  float* const red0 = (float*)(lds + PcLds::kRed);
  float* dep = (float*)(lds + PcLds::kDe);
  for (int i = th; i < nvw * 32 * 8; i += 512) {
    const int v = i >> 3, c = i & 7;
    *(uint4*)(wl + wimg(v, c)) = *(const uint4*)(a.W + (int64_t)(vb0 * 32 + v) * kJ + 8 * c);
  }
  for (int i = th; i < nvw * 32; i += 512) bias_l[i] = a.bias[vb0 * 32 + i] * kLog2e;

  // producer state: dW of its 4 blocks and their bias-gradient partial sums.  The consumers keep
  // their dZ (Y) in acc[0] and their d enc partial in acc[1]: one register set for both roles
  // (the compiler would otherwise keep both live across the step loop)
  jf16 acc[kPcBlk][2];
  float dbs[kPcBlk];
#pragma unroll
  for (int k = 0; k < kPcBlk; ++k) {
    dbs[k] = 0.0f;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[k][jb][q] = 0.0f;
  }
  const int ntbp = VS * a.ntb;
  const int64_t ntask = (int64_t)r.B * a.ntb * a.nus;
  // staging on the consumers (threads < 256): node zn, j = 8 jg .. 8 jg + 7; roles: node DMA
  // wave 1, pred DMA wave 2, node_finish wave 3, d pred sum wave 0
  const bool stager = th < 256;
  const int zn = (th >> 3) & 31, jg = th & 7;
  constexpr int kWn = 1, kWp = 2, kWf = 3, kWd = 0;
  if (prod) __builtin_amdgcn_s_setprio(1);
  for (int64_t task = slot; task < ntask; task += nslot) {
    const int b = (int)(task / ((int64_t)a.ntb * a.nus));
    const int tb = (int)((task / a.nus) % a.ntb), us = (int)(task % a.nus);
    const int Tb = clampr(r.flen[b], 0, r.T), Ub = clampr(r.llen[b], 0, r.Umax);
    const int ua = (int)((int64_t)us * r.U1 / a.nus);
    const int ue = tb * 32 < Tb ? min((int)((int64_t)(us + 1) * r.U1 / a.nus), Ub + 1) : ua;
    const bool zok = tb * 32 + zn < Tb;
    lds_barrier();   // the previous task's reads of encl / d enc partials are done
    jf16 (&Y)[2] = acc[0];      // consumer: dZ of the column it is draining
    jf16 (&dacc)[2] = acc[1];   // consumer: this task's d enc partial (Y's layout)
    if (!prod) {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          dacc[jb][q] = 0.0f;
          Y[jb][q] = 0.0f;
        }
    }
    if (ua < ue && stager) {
      const float* ep = a.enc + ((int64_t)b * r.T + (zok ? tb * 32 + zn : Tb - 1)) * kJ + 8 * jg;
      *(float4*)(encl + zn * 64 + 8 * jg) = *(const float4*)ep;
      *(float4*)(encl + zn * 64 + 8 * jg + 4) = *(const float4*)(ep + 4);
    }
    uint32_t* const ndl0 = (uint32_t*)(lds + PcLds::kNd);
    float* const prl0 = (float*)(lds + PcLds::kPr);
    const double lp2 = r.ws.logp2[b];
    const float lsc = r.scale[b];
    auto col_dma = [&](int uu, int bf) __attribute__((always_inline)) {
      if (w == kWp)
        dma_to_lds<4>(a.pred + ((int64_t)b * r.U1 + uu) * kJ + lane, lds_addr(prl0 + bf * 64));
      if (w == kWn && lane < 32)
        node_dma(r, b, tb * 32 + lane, uu, Tb, Ub, lds_addr(ndl0 + bf * kNF * 32));
    };
    auto col_dma_wait = [&]() __attribute__((always_inline)) {
      if (w == kWp || w == kWn) dma_wait();
    };
    // stage column uu (consumers): z image (buffer uu - ua & 1), 1 - z^2 ((uu - ua) % 3), node
    // scalars (& 1); the DMA of column uu + 1 is issued at its end (landing buffer (uu+1-ua) & 1)
    auto stage = [&](int uu) __attribute__((always_inline)) {
      if (!stager) return;
      const int cu = uu - ua, bf = cu & 1, b3 = cu % 3;
      const float* pr = prl0 + bf * 64 + 8 * jg;
      const float* el = encl + zn * 64 + 8 * jg;
      float zf[8];
      jbf8 z8;
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const float4 pv = *(const float4*)(pr + e), ev = *(const float4*)(el + e);
        const float xs[4] = {ev.x + pv.x, ev.y + pv.y, ev.z + pv.z, ev.w + pv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          zf[e + q] = zok ? tanh_(xs[q]) : 0.0f;
          z8[e + q] = (__bf16)zf[e + q];
        }
      }
      *(jbf8*)(zimg0 + bf * 32 * 128 + wimg(zn, jg)) = z8;
      float* zz = z320 + b3 * 64 * PcLds::kZP + 8 * jg * PcLds::kZP + zn;
#pragma unroll
      for (int e = 0; e < 8; ++e) zz[e * PcLds::kZP] = 1.0f - zf[e] * zf[e];
      if (w == kWf && lane < 32) {
        const uint32_t* nf = ndl0 + bf * kNF * 32;
        float wb, wy, l2;
        node_finish(nf, lane, lp2, lsc, tb * 32 + lane, uu, Tb, Ub, wb, wy, l2);
        const float an = wb + wy;
        float* ns = ns0 + bf * 128;
        ns[lane] = an > 0.0f ? log2_(an) - l2 : -1e30f;
        ns[32 + lane] = wb;
        ns[64 + lane] = wy;
        if (lane == 0) {
          const int lab = (int)nf[10 * 32];
          ((int*)ns)[96] = uu < Ub ? (lab < 0 ? 0 : (lab >= r.V ? r.V - 1 : lab)) : r.blank;
        }
      }
      if (uu + 1 < ue) col_dma(uu + 1, (cu + 1) & 1);
    };
    const int ncol = ue - ua;
    if (ncol > 0) {
      col_dma(ua, 0);
      col_dma_wait();
      lds_barrier();
      stage(ua);   // (issues the DMA of column ua + 1)
    }
    col_dma_wait();
    lds_barrier();
    jbf8 zA[4];   // producer: the current column's z rows (logits A operand)
    const int nstep = ncol > 0 ? 4 * ncol + 1 : 0;
    for (int g = 0; g < nstep; ++g) {
      asm volatile("" : "+v"(th), "+v"(lane), "+v"(h), "+v"(g1));
      const int up = g >> 2, kp = g & 3;   // producer: column ua + up, block kp
      if (prod) {
        if (up < ncol) {
          const int cb = up & 1;
          const unsigned char* zimg = zimg0 + cb * 32 * 128;
          const float* ns_c = ns0 + cb * 128;
          if (kp == 0) {
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) zA[s2] = lds_b128(zimg, wimg(lane & 31, 2 * s2 + h));
          }
          const int yl = uniform(((const int*)ns_c)[96]);
          unsigned char* pslot = lds + PcLds::kP + ((g & 1) * 4 + pi) * 32 * 128;
#pragma unroll
          for (int k = 0; k < kPcBlk; ++k) {   // (static register index: one block per step)
            if (k != kp) continue;
            const int lvb = pi + 4 * k;
            const bool vok = lvb < nvw;
            const int vl = (vok ? lvb : 0) * 32 + (lane & 31);
            jf16 x;
#pragma unroll
            for (int q = 0; q < 16; ++q) x[q] = 0.0f;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) x = mfma32(zA[s2], lds_b128(wl, wimg(vl, 2 * s2 + h)), x);
            const float bl = vok ? bias_l[vl] : -1e30f;
            float p[16], ps = 0.0f;
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
              const float4 cv = *(const float4*)(ns_c + 8 * gq + 4 * h);
              p[4 * gq] = exp2_(fmaf(x[4 * gq], kLog2e, bl + cv.x));
              p[4 * gq + 1] = exp2_(fmaf(x[4 * gq + 1], kLog2e, bl + cv.y));
              p[4 * gq + 2] = exp2_(fmaf(x[4 * gq + 2], kLog2e, bl + cv.z));
              p[4 * gq + 3] = exp2_(fmaf(x[4 * gq + 3], kLog2e, bl + cv.w));
            }
            const int vg0 = (vb0 + lvb) * 32;
            if (vok && ((unsigned)(r.blank - vg0) < 32u || (unsigned)(yl - vg0) < 32u)) {
              const int v = vg0 + (lane & 31);
              const float mb = v == r.blank ? 1.0f : 0.0f, my = v == yl ? 1.0f : 0.0f;
#pragma unroll
              for (int gq = 0; gq < 4; ++gq) {
                const float4 bw = *(const float4*)(ns_c + 32 + 8 * gq + 4 * h);
                const float4 yw = *(const float4*)(ns_c + 64 + 8 * gq + 4 * h);
                p[4 * gq] -= mb * bw.x + my * yw.x;
                p[4 * gq + 1] -= mb * bw.y + my * yw.y;
                p[4 * gq + 2] -= mb * bw.z + my * yw.z;
                p[4 * gq + 3] -= mb * bw.w + my * yw.w;
              }
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) ps += p[q];
            dbs[k] += ps;
            jbf8 pf[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              pf[s2] = pack8(p + 8 * s2);
#pragma unroll
              for (int jb = 0; jb < 2; ++jb)
                acc[k][jb] = mfma32(pf[s2],
                                    cat8(tr_rd(zimg, 16 * s2 + 4 * h, jb * 32 + 16 * g1, lane),
                                         tr_rd(zimg, 16 * s2 + 8 + 4 * h, jb * 32 + 16 * g1, lane)),
                                    acc[k][jb]);
            }
            typedef int ji2 __attribute__((ext_vector_type(2)));
            typedef int ji4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
              const ji4 d = __builtin_bit_cast(ji4, pf[gq >> 1]);
              *(ji2*)(pslot + pimg_off(lane & 31, 8 * gq + 4 * h)) =
                  ji2{d[2 * (gq & 1)], d[2 * (gq & 1) + 1]};
            }
          }
        }
      } else {
        // consumer: the block its producer wrote one step ago (step g - 1)
        const int gc = g - 1;
        if (gc >= 0) {
          const int kc = gc & 3;
          const int lvb = pi + 4 * kc;
          const int lvc = lvb < nvw ? lvb : 0;   // (a block past the vocabulary has p = 0)
          const unsigned char* pslot = lds + PcLds::kP + ((gc & 1) * 4 + pi) * 32 * 128;
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const jbf8 pt = cat8(tr_rd<true>(pslot, 16 * s2 + 4 * h, 16 * g1, lane),
                                 tr_rd<true>(pslot, 16 * s2 + 8 + 4 * h, 16 * g1, lane));
#pragma unroll
            for (int jb = 0; jb < 2; ++jb) {
              const jbf8 wt = cat8(tr_rd(wl, lvc * 32 + 16 * s2 + 4 * h, jb * 32 + 16 * g1, lane),
                                   tr_rd(wl, lvc * 32 + 16 * s2 + 8 + 4 * h, jb * 32 + 16 * g1, lane));
              Y[jb] = mfma32(pt, wt, Y[jb]);
            }
          }
          if (kc == 3) {
            // the column's epilogue: d pre = dZ (1 - z^2) into the d enc partial and the d pred
            // partial (red, buffer by column parity), then Y starts the next column at 0
            const int cc = gc >> 2;
            const float* z32 = z320 + (cc % 3) * 64 * PcLds::kZP;
            float* red = red0 + (cc & 1) * 4 * 64;
            typedef float jf2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int jb = 0; jb < 2; ++jb) {
              const int j = jb * 32 + (lane & 31);
              jf2 sp2 = {0.0f, 0.0f};
#pragma unroll
              for (int gq = 0; gq < 4; ++gq) {
                const float4 zz = *(const float4*)(z32 + j * PcLds::kZP + 8 * gq + 4 * h);
                const jf2 o0 = jf2{Y[jb][4 * gq], Y[jb][4 * gq + 1]} * jf2{zz.x, zz.y};
                const jf2 o1 = jf2{Y[jb][4 * gq + 2], Y[jb][4 * gq + 3]} * jf2{zz.z, zz.w};
                const jf2 a0 = jf2{dacc[jb][4 * gq], dacc[jb][4 * gq + 1]} + o0;
                const jf2 a1 = jf2{dacc[jb][4 * gq + 2], dacc[jb][4 * gq + 3]} + o1;
                dacc[jb][4 * gq] = a0.x;
                dacc[jb][4 * gq + 1] = a0.y;
                dacc[jb][4 * gq + 2] = a1.x;
                dacc[jb][4 * gq + 3] = a1.y;
                sp2 += o0 + o1;
              }
              float sp = sp2.x + sp2.y;
              sp += __shfl_xor(sp, 32);
              if (h == 0) red[pi * 64 + j] = sp;
#pragma unroll
              for (int q = 0; q < 16; ++q) Y[jb][q] = 0.0f;
            }
          }
        }
        // one step into producer column up (>= 1): the d pred of column up - 1 (its epilogue
        // wrote red one barrier ago); and the staging of column up + 1
        if (kp == 1 && up >= 1 && up - 1 < ncol && w == kWd) {
          const int cc = up - 1;
          const float* red = red0 + (cc & 1) * 4 * 64;
          const float s4 = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
          a.d_pred[(((int64_t)b * ntbp + vh * a.ntb + tb) * r.U1 + ua + cc) * kJ + lane] = s4;
        }
        if (kp == 1 && up + 1 < ncol) stage(ua + up + 1);
      }
      // the DMA of the column staged next (issued one column ago) lands before that staging
      if (kp == 0) col_dma_wait();
      lds_barrier();
    }
    // the last column's d pred (its epilogue ran in the final step)
    if (ncol > 0 && w == kWd) {
      const int cc = ncol - 1;
      const float* red = red0 + (cc & 1) * 4 * 64;
      const float s4 = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
      a.d_pred[(((int64_t)b * ntbp + vh * a.ntb + tb) * r.U1 + ua + cc) * kJ + lane] = s4;
    }
    lds_barrier();   // (the p slots are free: the d enc partials go over them)
    // d enc of the task: the 4 consumers' register partials in 4 LDS slots, then 4 values per
    // thread (j fastest)
    if (!prod) {
      float* slotp = dep + pi * 64 * PcLds::kDeP;
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const int j = jb * 32 + (lane & 31);
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *(float4*)(slotp + j * PcLds::kDeP + 8 * gq + 4 * h) =
              make_float4(dacc[jb][4 * gq], dacc[jb][4 * gq + 1], dacc[jb][4 * gq + 2], dacc[jb][4 * gq + 3]);
      }
    }
    lds_barrier();
    float* dst = a.d_enc + ((int64_t)(vh * a.nus + us) * r.B + b) * r.T * kJ;
#pragma unroll
    for (int i = 0; i < 32 * 64 / 512; ++i) {
      const int e = th + 512 * i, n = e >> 6, j = e & 63;
      const int tq = tb * 32 + n;
      float sum = 0.0f;
      if (ua < ue) {
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) sum += dep[(ww * 64 + j) * PcLds::kDeP + n];
      }
      if (tq < r.T) dst[(int64_t)tq * kJ + j] = sum;
    }
  }
  // acc[k][jb][q] = dW[v = (vb0 + pi + 4k) * 32 + (q&3) + 8(q>>2) + 4h][j = jb*32 + (lane&31)]
  if (prod) {
    float* dw = a.dW + (int64_t)slot * r.V * kJ;
#pragma unroll
    for (int k = 0; k < kPcBlk; ++k) {
      const int lvb = pi + 4 * k;
      if (lvb >= nvw) continue;
      const int vbg = vb0 + lvb;
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int v = vbg * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
          dw[(int64_t)v * kJ + jb * 32 + (lane & 31)] = acc[k][jb][q];
        }
      const float tot = dbs[k] + __shfl_xor(dbs[k], 32);
      if (h == 0) a.db[(int64_t)slot * r.V + vbg * 32 + (lane & 31)] = tot;
    }
  }
}
#endif  // SC_JOINT_PC

size_t joint_lds_fwd() { return (size_t)kVmaxJ * 128 + kVmaxJ * 4; }

template <typename K>
bool joint_lds_attr(K kern, size_t bytes) {
  return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes) == hipSuccess;
}
size_t joint_lds_bwd() { return (size_t)BwdLds::kEnd; }

// real t-blocks / u-splits of the task decomposition (the exported geometry multiplies both by
// the vocab split, the leading partial dimension of d enc and the t-block rows of d pred)
void joint_geometry(int B, int T, int Umax, int* ntb, int* nus, int* S) {
  *ntb = (T + 31) / 32;
  // d enc is accumulated over u in registers; split u only as far as needed to give every SIMD
  // about three (b, t-block) tasks
  const int64_t base = (int64_t)B * *ntb;
  int n = 1;
  while (n < 8 && base * n < 3 * 2048 && n < Umax + 1) n *= 2;
  *nus = n;
  *S = 256;
}
int joint_vsplit(int V) { return (V / 32 + kVbWg - 1) / kVbWg; }

}  // namespace

}  // namespace sc

using namespace sc;

extern "C" size_t sc_rnnt_workspace_bytes(int B, int T, int max_labels) {
  if (B <= 0 || T <= 0 || max_labels < 0) return 256;
  return ws_layout(B, T, max_labels, nullptr, nullptr);
}

extern "C" int sc_rnnt_fwd(const void* x, int x_dtype, int is_logits, int B, int T, int max_labels,
                           int V, int64_t stride_b, int64_t stride_t, int64_t stride_u,
                           const int64_t* row_offsets, const int64_t* labels,
                           int64_t label_stride, const int64_t* frames_lengths,
                           const int64_t* labels_lengths, int blank, float* nll, void* workspace,
                           size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = rnnt_check(x, x_dtype, B, T, max_labels, V, labels, frames_lengths, labels_lengths,
                      blank, workspace, workspace_bytes, "sc_rnnt_fwd");
  if (rc) return rc;
  if (B == 0) return 0;
  SC_REQUIRE(nll, "sc_rnnt_fwd: null nll");
  SC_REQUIRE(T > 0, "sc_rnnt_fwd: T == 0 is handled by the caller");
  RnntArgs a = make_args(x, is_logits, B, T, max_labels, V, stride_b, stride_t, stride_u,
                         row_offsets, labels, label_stride, frames_lengths, labels_lengths, blank,
                         nll, workspace, nullptr, nullptr);
  set_vec(a, esize_of(x_dtype));
  hipStream_t st = (hipStream_t)stream;
  switch (x_dtype) {
    case SC_F32: launch_fwd<SC_F32>(a, st); break;
    case SC_BF16: launch_fwd<SC_BF16>(a, st); break;
    default: launch_fwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_rnnt_fwd");
}

extern "C" int sc_rnnt_bwd(const void* x, int x_dtype, int is_logits, int B, int T, int max_labels,
                           int V, int64_t stride_b, int64_t stride_t, int64_t stride_u,
                           const int64_t* row_offsets, const int64_t* labels,
                           int64_t label_stride, const int64_t* frames_lengths,
                           const int64_t* labels_lengths, int blank, const float* scale,
                           void* grad, int grad_dtype, const void* workspace,
                           size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = rnnt_check(x, x_dtype, B, T, max_labels, V, labels, frames_lengths, labels_lengths,
                      blank, workspace, workspace_bytes, "sc_rnnt_bwd");
  if (rc) return rc;
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(scale && grad, "sc_rnnt_bwd: null scale/grad");
  SC_REQUIRE(grad_dtype == SC_F32 || grad_dtype == x_dtype,
             "sc_rnnt_bwd: grad dtype must be fp32 or the input dtype");
  RnntArgs a = make_args(x, is_logits, B, T, max_labels, V, stride_b, stride_t, stride_u,
                         row_offsets, labels, label_stride, frames_lengths, labels_lengths, blank,
                         nullptr, workspace, scale, grad);
  set_vec(a, esize_of(x_dtype));
  hipStream_t st = (hipStream_t)stream;
  if (grad_dtype == SC_F32) {
    switch (x_dtype) {
      case SC_F32: launch_bwd<SC_F32, SC_F32>(a, st); break;
      case SC_BF16: launch_bwd<SC_BF16, SC_F32>(a, st); break;
      default: launch_bwd<SC_F16, SC_F32>(a, st); break;
    }
  } else {
    switch (x_dtype) {
      case SC_BF16: launch_bwd<SC_BF16, SC_BF16>(a, st); break;
      default: launch_bwd<SC_F16, SC_F16>(a, st); break;
    }
  }
  return launch_status("sc_rnnt_bwd");
}

// ------------------------------------------------------------------ fused joiner entry points --

namespace sc {
namespace {
int joint_check(const float* enc, const float* pred, const void* W, const float* bias, int B, int T,
                int Umax, int V, int J, const int64_t* labels, const int64_t* fl,
                const int64_t* ll, int blank, const void* ws, size_t wsb, const char* who) {
  SC_REQUIRE(J == kJ, "%s: join_dim %d (only 64, train.py:639's default, is compiled)", who, J);
  SC_REQUIRE(V > 0 && V % 32 == 0 && V <= kVmaxJ, "%s: V=%d must be a multiple of 32 <= %d", who, V,
             kVmaxJ);
  SC_REQUIRE(B >= 0 && T >= 0 && Umax >= 0, "%s: bad shape", who);
  SC_REQUIRE(ab_halo_k(Umax) > 0, "%s: max label count %d exceeds %d", who, Umax, 16 * 63 - 1);
  SC_REQUIRE(blank >= 0 && blank < V, "%s: blank %d outside [0, %d)", who, blank, V);
  SC_REQUIRE((int64_t)B * T * (Umax + 1) < (1ll << 40), "%s: lattice too large", who);
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(enc && pred && W && bias && fl && ll && ws, "%s: null pointer", who);
  SC_REQUIRE(Umax == 0 || labels, "%s: null labels", who);
  SC_REQUIRE(((uintptr_t)enc | (uintptr_t)pred | (uintptr_t)W) % 16 == 0, "%s: unaligned operand", who);
  SC_REQUIRE(wsb >= ws_layout(B, T, Umax, nullptr, nullptr), "%s: workspace too small", who);
  return 0;
}

JointArgs joint_args(const float* enc, const float* pred, const void* W, const float* bias, int B,
                     int T, int Umax, int V, const int64_t* labels, int64_t labs,
                     const int64_t* fl, const int64_t* ll, int blank, float* nll, const void* ws,
                     const float* scale) {
  JointArgs j;
  j.r = make_args(enc, 1, B, T, Umax, V, 0, 0, 0, nullptr, labels, labs, fl, ll, blank, nll, ws,
                  scale, nullptr);
  j.enc = enc;
  j.pred = pred;
  j.W = (const __bf16*)W;
  j.bias = bias;
  joint_geometry(B, T, Umax, &j.ntb, &j.nus, &j.S);
  j.vs = joint_vsplit(V);
  j.S /= j.vs;
  j.d_enc = j.d_pred = j.dW = j.db = nullptr;
  return j;
}
}  // namespace
}  // namespace sc

extern "C" int sc_rnnt_joint_geometry(int B, int T, int max_labels, int V, int* t_blocks,
                                      int* u_splits, int* slices) {
  clear_error();
  SC_REQUIRE(t_blocks && u_splits && slices, "sc_rnnt_joint_geometry: null pointer");
  joint_geometry(B, T, max_labels, t_blocks, u_splits, slices);
  const int vs = joint_vsplit(V);
  *t_blocks *= vs;
  *u_splits *= vs;
  *slices /= vs;
  return 0;
}

extern "C" int sc_rnnt_joint_fwd(const float* enc, const float* pred, const void* W, const float* bias,
                                 int B, int T, int max_labels, int V, int J, const int64_t* labels,
                                 int64_t label_stride, const int64_t* frames_lengths,
                                 const int64_t* labels_lengths, int blank, float* nll,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = joint_check(enc, pred, W, bias, B, T, max_labels, V, J, labels, frames_lengths,
                       labels_lengths, blank, workspace, workspace_bytes, "sc_rnnt_joint_fwd");
  if (rc) return rc;
  if (B == 0) return 0;
  SC_REQUIRE(nll && T > 0, "sc_rnnt_joint_fwd: null nll / T == 0 is handled by the caller");
  JointArgs j = joint_args(enc, pred, W, bias, B, T, max_labels, V, labels, label_stride,
                           frames_lengths, labels_lengths, blank, nll, workspace, nullptr);
  static const bool ok = joint_lds_attr(joint_fwd_kernel, joint_lds_fwd());
  SC_REQUIRE(ok, "sc_rnnt_joint_fwd: LDS attribute");
  hipStream_t st = (hipStream_t)stream;
  clear_shift(j.r, st);
  hipLaunchKernelGGL(joint_fwd_kernel, dim3(256), dim3(512), joint_lds_fwd(), st, j);
  launch_lattice(j.r, st);
  return launch_status("sc_rnnt_joint_fwd");
}

extern "C" int sc_rnnt_joint_bwd(const float* enc, const float* pred, const void* W, const float* bias,
                                 int B, int T, int max_labels, int V, int J, const int64_t* labels,
                                 int64_t label_stride, const int64_t* frames_lengths,
                                 const int64_t* labels_lengths, int blank, const float* scale,
                                 float* d_enc, float* d_pred, float* dW, float* db,
                                 const void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = joint_check(enc, pred, W, bias, B, T, max_labels, V, J, labels, frames_lengths,
                       labels_lengths, blank, workspace, workspace_bytes, "sc_rnnt_joint_bwd");
  if (rc) return rc;
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(scale && d_enc && d_pred && dW && db, "sc_rnnt_joint_bwd: null output");
  JointArgs j = joint_args(enc, pred, W, bias, B, T, max_labels, V, labels, label_stride,
                           frames_lengths, labels_lengths, blank, nullptr, workspace, scale);
  j.d_enc = d_enc;
  j.d_pred = d_pred;
  j.dW = dW;
  j.db = db;
  hipStream_t st = (hipStream_t)stream;
#if SC_JOINT_PC
  {
    static const bool okpc = joint_lds_attr(joint_bwd_pc_kernel, (size_t)PcLds::kEnd);
    SC_REQUIRE(okpc, "sc_rnnt_joint_bwd: LDS attribute");
    hipLaunchKernelGGL(joint_bwd_pc_kernel, dim3(j.S * j.vs), dim3(512), (size_t)PcLds::kEnd, st, j);
    return launch_status("sc_rnnt_joint_bwd");
  }
#endif
  static const bool ok = joint_lds_attr(joint_bwd_kernel, joint_lds_bwd());
  SC_REQUIRE(ok, "sc_rnnt_joint_bwd: LDS attribute");
  hipLaunchKernelGGL(joint_bwd_kernel, dim3(j.S * j.vs), dim3(64 * kJW), joint_lds_bwd(), st, j);
  return launch_status("sc_rnnt_joint_bwd");
}
