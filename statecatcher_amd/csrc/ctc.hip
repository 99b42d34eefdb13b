// CTC loss forward (alpha, beta, nll) and gradient for gfx950, with log_softmax fused.
//
// Replaces the reference's loss layer `enc_out.log_softmax(-1).transpose(0,1)` +
// nn.CTCLoss(blank=0, zero_infinity=True) (model.py:68-71, train.py:142), i.e. ATen's
// ctc_loss/_ctc_loss_backward.  Semantics kept: blank-extended label sequence of 2U+1 states,
// log-space recursions, nll = -log p(l|x) (+inf when infeasible), gradient
//   grad[t,v] = scale_b * (exp(lp[t,v]) - exp(lcab[t,v] + nll - lp[t,v]))   (t < in_len)
// which ATen returns for log-prob inputs and which equals d nll / d logits when the
// log_softmax is fused (is_logits=1).  The time axis is never transposed: x stays [B,T,V].
//
// Kernels (all on the caller's stream):
//   ctc_lse_kernel      one wave per (b,t) row: log-sum-exp over V (skipped for log-probs)
//   ctc_chain_kernel    per b: for every target position the next position with the same
//                       label, so label occupancies are summed in a fixed order (bitwise
//                       deterministic, no atomics)
//   ctc_ab_kernel       2B workgroups, one state per lane: B run alpha forward in time, B run
//                       beta backward, concurrently; emissions x[b,t,label(s)] for the next 8
//                       steps are gathered into registers while the current 8 steps compute
//   ctc_grad_kernel     one workgroup per (b,t) row: label occupancies into an LDS row of V
//                       log-sums, then one coalesced pass writing the gradient row
#include "sc_common.h"

namespace sc {

constexpr int kCtcP = 8;           // emission prefetch depth (steps)
constexpr int kCtcMaxStates = 1024;
constexpr float kNegInf = -__builtin_huge_valf();

// alpha/beta are stored NORMALISED: stored_t(s) = alpha_t(s) - offA_t where offA_t (fp64) is
// the running sum of the per-step maxima.  At T=1500 |alpha| reaches ~1e4, where an fp32 ulp is
// ~1e-3: un-normalised fp32 lattices put ~0.5% error into exp(alpha+beta+nll-lp).  With the
// offsets in fp64 the posterior exponent is formed from O(10) fp32 terms.
struct CtcWs {
  float* lse;
  float* alpha;
  float* beta;
  double* offA;   // [B,T]
  double* offB;   // [B,T]
  double* nll64;  // [B]
  int* chain;
  int* first;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static CtcWs carve(void* ws, int B, int T, int S, int Um) {
  char* p = (char*)ws;
  CtcWs w;
  w.lse = (float*)p; p += align256((size_t)B * T * 4);
  w.alpha = (float*)p; p += align256((size_t)B * T * S * 4);
  w.beta = (float*)p; p += align256((size_t)B * T * S * 4);
  w.offA = (double*)p; p += align256((size_t)B * T * 8);
  w.offB = (double*)p; p += align256((size_t)B * T * 8);
  w.nll64 = (double*)p; p += align256((size_t)B * 8);
  w.chain = (int*)p; p += align256((size_t)B * Um * 4);
  w.first = (int*)p;
  return w;
}

static size_t ws_bytes(int B, int T, int Umax) {
  const int S = 2 * Umax + 1;
  const int Um = Umax > 0 ? Umax : 1;
  return align256((size_t)B * T * 4) + 2 * align256((size_t)B * T * S * 4) +
         2 * align256((size_t)B * T * 8) + align256((size_t)B * 8) + 2 * align256((size_t)B * Um * 4);
}

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == kNegInf) return kNegInf;
  return m + flog(fexp(a - m) + fexp(b - m));
}

__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(fmaxf(a, b), c);
  if (m == kNegInf) return kNegInf;
  return m + flog(fexp(a - m) + fexp(b - m) + fexp(c - m));
}

struct CtcArgs {
  const void* x;
  int is_logits, B, T, V, S, Umax, blank;
  int64_t sb, stt;
  const int64_t* tg;
  int64_t tgs;
  const int64_t* in_lens;
  const int64_t* tgt_lens;
  float* nll;
  CtcWs ws;
  const float* scale;
  void* grad;
};

__device__ __forceinline__ int clampi(int64_t v, int lo, int hi) {
  return (int)(v < lo ? lo : (v > hi ? hi : v));
}

// ---------------------------------------------------------------------------- lse -----------
template <int DT>
__global__ void __launch_bounds__(256) ctc_lse_kernel(CtcArgs a) {
  using E = Elem<DT>;
  using T = typename E::T;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)a.B * a.T) return;
  const int b = (int)(row / a.T), t = (int)(row % a.T);
  const T* p = (const T*)a.x + (int64_t)b * a.sb + (int64_t)t * a.stt;
  float m = kNegInf, l = 0.0f;
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
    l = (mn == kNegInf) ? 0.0f : l * fexp(m - mn) + lo * fexp(mo - mn);
    m = mn;
  }
  if (lane == 0) a.ws.lse[row] = m + flog(l);
}

// ---------------------------------------------------------------------------- chains --------
__global__ void __launch_bounds__(256) ctc_chain_kernel(CtcArgs a) {
  const int b = blockIdx.x;
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  const int Um = a.Umax > 0 ? a.Umax : 1;
  for (int u = threadIdx.x; u < Um; u += blockDim.x) {
    int nxt = -1, first = 0;
    if (u < Ub) {
      const int64_t lab = tg[u];
      for (int q = u + 1; q < Ub; ++q)
        if (tg[q] == lab) { nxt = q; break; }
      first = 1;
      for (int q = 0; q < u; ++q)
        if (tg[q] == lab) { first = 0; break; }
    }
    a.ws.chain[(int64_t)b * Um + u] = nxt;
    a.ws.first[(int64_t)b * Um + u] = first;
  }
}

// ---------------------------------------------------------------------------- alpha / beta --
template <int DT>
__global__ void __launch_bounds__(1024) ctc_ab_kernel(CtcArgs a) {
  using E = Elem<DT>;
  using T = typename E::T;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const bool is_beta = blockIdx.x >= a.B;
  const int b = is_beta ? blockIdx.x - a.B : blockIdx.x;
  const int s = threadIdx.x;
  const int Tb = clampi(a.in_lens[b], 0, a.T);
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  const int Sb = 2 * Ub + 1;
  const bool act = s < Sb;
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  int lab = a.blank;
  bool skip = false;   // alpha: transition s-2 -> s;  beta: transition s+2 -> s
  if (act && (s & 1)) lab = (int)tg[(s - 1) >> 1];
  // out-of-range labels are undefined input (as in ATen); clamp so no load leaves the row
  const int labc = lab < 0 ? 0 : (lab >= a.V ? a.V - 1 : lab);
  if (act) {
    if (!is_beta) {
      skip = (s & 1) && s >= 3 && lab != a.blank && lab != (int)tg[(s - 3) >> 1];
    } else if (s + 2 < Sb && !(s & 1)) {
      skip = false;
    } else if (s + 2 < Sb) {
      const int l2 = (int)tg[(s + 1) >> 1];
      skip = l2 != a.blank && l2 != lab;
    }
  }
  float* buf0 = sm;
  float* buf1 = sm + blockDim.x;
  float* outp = (is_beta ? a.ws.beta : a.ws.alpha) + (int64_t)b * a.T * a.S;
  if (Tb == 0) {
    if (!is_beta && s == 0) a.nll[b] = (Ub == 0) ? 0.0f : __builtin_huge_valf();
    return;
  }
  const T* xb = (const T*)a.x + (int64_t)b * a.sb + (act ? labc : 0);
  const float* lse = a.ws.lse + (int64_t)b * a.T;
  // time index of the i-th processed step
  auto tstep = [&](int i) { return is_beta ? Tb - 1 - i : i; };
  T cx[kCtcP], nx[kCtcP];
  float cl[kCtcP], nl[kCtcP];
  auto load = [&](T (&xr)[kCtcP], float (&lr)[kCtcP], int i0) {
#pragma unroll
    for (int j = 0; j < kCtcP; ++j) {
      const int i = min(i0 + j, Tb - 1);
      const int t = tstep(i);
      xr[j] = xb[(int64_t)t * a.stt];
      lr[j] = a.is_logits ? lse[t] : 0.0f;
    }
  };
  load(cx, cl, 0);
  float* prev = buf0;
  float* cur = buf1;
  __shared__ float wmax[2][16];
  const int lane = s & 63, wv = s >> 6, nwv = blockDim.x >> 6;
  double* offp = (is_beta ? a.ws.offB : a.ws.offA) + (int64_t)b * a.T;
  double off = 0.0;   // log-offset of the values in `prev` (all threads hold the same value)
  float mprev = 0.0f; // max of the previous step, already folded into `off`
  for (int i0 = 0; i0 < Tb; i0 += kCtcP) {
    if (i0 + kCtcP < Tb) load(nx, nl, i0 + kCtcP);
#pragma unroll
    for (int j = 0; j < kCtcP; ++j) {
      const int i = i0 + j;
      if (i >= Tb) break;
      const int t = tstep(i);
      const float lp = E::ld(cx[j]) - cl[j];
      float v;
      if (i == 0) {
        v = (act && (is_beta ? (s >= Sb - 2) : (s <= 1))) ? lp : kNegInf;
      } else if (!act) {
        v = kNegInf;
      } else if (!is_beta) {
        const float a1 = s > 0 ? prev[s - 1] : kNegInf;
        const float a2 = skip ? prev[s - 2] : kNegInf;
        v = lse3(prev[s], a1, a2) - mprev + lp;
      } else {
        const float b1 = s + 1 < Sb ? prev[s + 1] : kNegInf;
        const float b2 = skip ? prev[s + 2] : kNegInf;
        v = lse3(prev[s], b1, b2) - mprev + lp;
      }
      cur[s] = v;
      if (act) outp[(int64_t)t * a.S + s] = v;
      if (s == 0) offp[t] = off;
      float mx = v;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      if (lane == 0) wmax[i & 1][wv] = mx;
      lds_barrier();
      float m = kNegInf;
      for (int q = 0; q < nwv; ++q) m = fmaxf(m, wmax[i & 1][q]);
      mprev = (m == kNegInf) ? 0.0f : m;
      off += (double)mprev;
      float* tmp = prev; prev = cur; cur = tmp;
    }
#pragma unroll
    for (int j = 0; j < kCtcP; ++j) {
      cx[j] = nx[j];
      cl[j] = nl[j];
    }
  }
  if (!is_beta && s == 0) {
    // prev holds the last step relative to off - mprev
    const float ll = Sb > 1 ? lse2(prev[Sb - 1], prev[Sb - 2]) : prev[0];
    const double nll = (ll == kNegInf) ? __builtin_huge_val() : -((double)ll + (off - (double)mprev));
    a.ws.nll64[b] = nll;
    a.nll[b] = (float)nll;
  }
}

// ---------------------------------------------------------------------------- gradient ------
template <int DT, int GT>
__global__ void __launch_bounds__(256) ctc_grad_kernel(CtcArgs a) {
  using E = Elem<DT>;
  using G = Elem<GT>;
  extern __shared__ __attribute__((aligned(16))) float lcab[];   // V log-sums + 8 (m,l) pairs
  const int b = blockIdx.x / a.T, t = blockIdx.x % a.T;
  const int tid = threadIdx.x;
  const int Tb = clampi(a.in_lens[b], 0, a.T);
  typename G::T* g = (typename G::T*)a.grad + ((int64_t)b * a.T + t) * a.V;
  const float sc = a.scale[b];
  if (t >= Tb || sc == 0.0f) {
    for (int v = tid; v < a.V; v += 256) g[v] = G::st(0.0f);
    return;
  }
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  const int Sb = 2 * Ub + 1;
  const int Um = a.Umax > 0 ? a.Umax : 1;
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  for (int v = tid; v < a.V; v += 256) lcab[v] = kNegInf;
  __syncthreads();
  const float* al = a.ws.alpha + ((int64_t)b * a.T + t) * a.S;
  const float* be = a.ws.beta + ((int64_t)b * a.T + t) * a.S;
  // exp(lcab + nll - lp) with lcab = lse(stored) + offA + offB: fold the fp64 offsets first
  const float koff = (float)(a.ws.offA[(int64_t)b * a.T + t] + a.ws.offB[(int64_t)b * a.T + t] +
                             a.ws.nll64[b]);
  const int* chain = a.ws.chain + (int64_t)b * Um;
  const int* first = a.ws.first + (int64_t)b * Um;
  float m = kNegInf, l = 0.0f;   // blank-label occupancy, per thread
  for (int s = tid; s < Sb; s += 256) {
    const int lab = (s & 1) ? (int)tg[(s - 1) >> 1] : a.blank;
    const float val = al[s] + be[s];
    if (lab == a.blank) {
      const float mn = fmaxf(m, val);
      if (mn != kNegInf) {
        l = l * fexp(m - mn) + fexp(val - mn);
        m = mn;
      }
    } else {
      const int u = (s - 1) >> 1;
      if (first[u]) {
        float acc = val;
        for (int q = chain[u]; q >= 0; q = chain[q]) acc = lse2(acc, al[2 * q + 1] + be[2 * q + 1]);
        if (lab >= 0 && lab < a.V) lcab[lab] = acc;
      }
    }
  }
  // block reduce of the blank (m, l)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o);
    const float lo = __shfl_xor(l, o);
    const float mn = fmaxf(m, mo);
    l = (mn == kNegInf) ? 0.0f : l * fexp(m - mn) + lo * fexp(mo - mn);
    m = mn;
  }
  float* red = lcab + a.V;
  const int wv = tid >> 6;
  if ((tid & 63) == 0) {
    red[2 * wv] = m;
    red[2 * wv + 1] = l;
  }
  __syncthreads();
  if (tid == 0) {
    float M = kNegInf, L = 0.0f;
    for (int q = 0; q < 4; ++q) {
      const float mo = red[2 * q], lo = red[2 * q + 1];
      const float mn = fmaxf(M, mo);
      L = (mn == kNegInf) ? 0.0f : L * fexp(M - mn) + lo * fexp(mo - mn);
      M = mn;
    }
    if (a.blank >= 0 && a.blank < a.V) lcab[a.blank] = (M == kNegInf) ? kNegInf : M + flog(L);
  }
  __syncthreads();
  const typename E::T* xr = (const typename E::T*)a.x + (int64_t)b * a.sb + (int64_t)t * a.stt;
  const float lse = a.is_logits ? a.ws.lse[(int64_t)b * a.T + t] : 0.0f;
  for (int v = tid; v < a.V; v += 256) {
    const float lp = E::ld(xr[v]) - lse;
    const float gv = fexp(lp) - fexp(lcab[v] + koff - lp);
    g[v] = G::st(gv * sc);
  }
}

template <int DT>
static void launch_fwd(const CtcArgs& a, hipStream_t st) {
  if (a.is_logits) {
    const int64_t rows = (int64_t)a.B * a.T;
    hipLaunchKernelGGL((ctc_lse_kernel<DT>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a);
  }
  hipLaunchKernelGGL(ctc_chain_kernel, dim3(a.B), dim3(256), 0, st, a);
  const int nthr = ((a.S + 63) / 64) * 64;
  hipLaunchKernelGGL((ctc_ab_kernel<DT>), dim3(2 * a.B), dim3(nthr), 2 * nthr * sizeof(float), st, a);
}

template <int DT, int GT>
static void launch_bwd(const CtcArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((ctc_grad_kernel<DT, GT>), dim3((unsigned)((int64_t)a.B * a.T)), dim3(256),
                     (a.V + 8) * sizeof(float), st, a);
}

}  // namespace sc

using namespace sc;

extern "C" size_t sc_ctc_workspace_bytes(int B, int T, int max_target_len) {
  if (B <= 0 || T <= 0 || max_target_len < 0) return 256;
  return ws_bytes(B, T, max_target_len);
}

static int ctc_check(const void* x, int x_dtype, int B, int T, int V, int max_target_len,
                     const int64_t* targets, const int64_t* in_lens, const int64_t* tgt_lens,
                     int blank, void* ws, size_t wsb, const char* who) {
  SC_REQUIRE(x_dtype == SC_F32 || x_dtype == SC_BF16 || x_dtype == SC_F16,
             "%s: unsupported dtype %d", who, x_dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && V > 0 && max_target_len >= 0, "%s: bad shape", who);
  SC_REQUIRE(2 * max_target_len + 1 <= kCtcMaxStates,
             "%s: max target length %d exceeds %d", who, max_target_len, (kCtcMaxStates - 1) / 2);
  SC_REQUIRE(blank >= 0 && blank < V, "%s: blank %d outside [0, %d)", who, blank, V);
  SC_REQUIRE((int64_t)B * T <= 0x7fffffff, "%s: B*T too large", who);
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(x && in_lens && tgt_lens && ws, "%s: null pointer", who);
  SC_REQUIRE(max_target_len == 0 || targets, "%s: null targets", who);
  SC_REQUIRE(wsb >= ws_bytes(B, T, max_target_len), "%s: workspace %zu < %zu bytes", who, wsb,
             ws_bytes(B, T, max_target_len));
  return 0;
}

extern "C" int sc_ctc_fwd(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                          int64_t stride_b, int64_t stride_t, const int64_t* targets,
                          int64_t target_stride, int max_target_len, const int64_t* in_lens,
                          const int64_t* tgt_lens, int blank, float* nll, void* workspace,
                          size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = ctc_check(x, x_dtype, B, T, V, max_target_len, targets, in_lens, tgt_lens, blank,
                     workspace, workspace_bytes, "sc_ctc_fwd");
  if (rc) return rc;
  if (B == 0) return 0;
  SC_REQUIRE(nll, "sc_ctc_fwd: null nll");
  if (T == 0) {
    SC_REQUIRE(false, "sc_ctc_fwd: T == 0 is handled by the caller");
  }
  const int S = 2 * max_target_len + 1;
  CtcArgs a{x, is_logits, B, T, V, S, max_target_len, blank, stride_b, stride_t, targets,
            target_stride, in_lens, tgt_lens, nll, carve(workspace, B, T, S, max_target_len > 0 ? max_target_len : 1),
            nullptr, nullptr};
  hipStream_t st = (hipStream_t)stream;
  switch (x_dtype) {
    case SC_F32: launch_fwd<SC_F32>(a, st); break;
    case SC_BF16: launch_fwd<SC_BF16>(a, st); break;
    default: launch_fwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_ctc_fwd");
}

extern "C" int sc_ctc_bwd(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                          int64_t stride_b, int64_t stride_t, const int64_t* targets,
                          int64_t target_stride, int max_target_len, const int64_t* in_lens,
                          const int64_t* tgt_lens, int blank, const float* nll,
                          const float* scale, void* grad, int grad_dtype, const void* workspace,
                          size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = ctc_check(x, x_dtype, B, T, V, max_target_len, targets, in_lens, tgt_lens, blank,
                     (void*)workspace, workspace_bytes, "sc_ctc_bwd");
  if (rc) return rc;
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(grad_dtype == SC_F32 || grad_dtype == SC_BF16 || grad_dtype == SC_F16,
             "sc_ctc_bwd: unsupported grad dtype %d", grad_dtype);
  SC_REQUIRE(nll && scale && grad, "sc_ctc_bwd: null pointer");
  const int S = 2 * max_target_len + 1;
  CtcArgs a{x, is_logits, B, T, V, S, max_target_len, blank, stride_b, stride_t, targets,
            target_stride, in_lens, tgt_lens, (float*)nll,
            carve((void*)workspace, B, T, S, max_target_len > 0 ? max_target_len : 1), scale, grad};
  hipStream_t st = (hipStream_t)stream;
#define SC_CTC_BWD(DT)                                               \
  switch (grad_dtype) {                                              \
    case SC_F32: launch_bwd<DT, SC_F32>(a, st); break;               \
    case SC_BF16: launch_bwd<DT, SC_BF16>(a, st); break;             \
    default: launch_bwd<DT, SC_F16>(a, st); break;                   \
  }
  switch (x_dtype) {
    case SC_F32: SC_CTC_BWD(SC_F32) break;
    case SC_BF16: SC_CTC_BWD(SC_BF16) break;
    default: SC_CTC_BWD(SC_F16) break;
  }
#undef SC_CTC_BWD
  return launch_status("sc_ctc_bwd");
}
