// RNN-T (transducer) loss for gfx950: the lattice the reference gets from warp_rnnt
// (model.py:73-105, train.py:38-42, :144; gather=True semantics: only the blank and the next
// label of every (t, u) node enter the loss).
//
//   rnnt_emit_kernel   one wave per lattice node (b,t,u): row log-sum-exp over V (when fed
//                      logits: the log_softmax of model.py:93 is fused), then the node's blank
//                      and label log-probs in base 2, stored DIAGONAL-MAJOR ([b][t+u][u]) so
//                      that the wavefront below reads one coalesced row per step.
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
  double* logp2;   // [B]             base-2 log P(y|x)
};

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
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float l = 0.0f;
#pragma unroll
    for (int j = 0; j < kNvMax; ++j)
      if (j < a.nvec) {
#pragma unroll
        for (int k = 0; k < VL::N; ++k) l += fexp(f[j][k] - m);
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
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
    a.ws.lpb[d] = fmaxf((E::ld(p[a.blank]) - lse) * kLog2e, kDeadR);
    a.ws.lpy[d] = u < Ub ? fmaxf((E::ld(p[label_at(a, b, u)]) - lse) * kLog2e, kDeadR) : kDeadR;
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
          float m = own ? v : kDeadR;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
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
  if (!BETA && own && u == Ub) {   // log P = alpha(Tb-1, Ub) + its terminal blank
    const double lp = (double)v + (double)lpb[(int64_t)(nd - 1) * a.U1p + Ub] + off;
    a.ws.logp2[b] = lp;
    a.nll[b] = (float)(-lp * (double)kLn2);
  }
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

template <int DT>
void launch_fwd(const RnntArgs& a, hipStream_t st) {
  const int64_t nodes = (int64_t)a.B * a.T * a.U1;
  hipLaunchKernelGGL((rnnt_emit_kernel<DT>), dim3((unsigned)((nodes + 3) / 4)), dim3(256), 0, st, a);
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
  a.kh = ab_halo_k(Umax);
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
