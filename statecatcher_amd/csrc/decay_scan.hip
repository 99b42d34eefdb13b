// First-order decay scan s_t = decay_t * s_{t-1} + kv_t (forward and adjoint), gfx950.
//
// Replaces the reference Triton kernel fused_decay_scan (lucyrnn_triton.py:158-177, launched by
// the native LucyRNN train mode at lucyrnn.py:143-151), which runs one scalar program per
// (b, d) stepping serially over T.  Generalised with an optional initial state so the native
// LucyRNN's carried state and its gated h recurrence (h_t = a_t h_{t-1} + b_t) use it too.
//
// Same decomposition as lucy_scan.hip: workgroup = (b, 64 columns) x NW waves splitting each
// 64-step super-chunk in time; per super-chunk every wave publishes its segment's affine map
// (prod decay, local scan) in LDS, one LDS-only barrier, composes the maps of earlier waves.
// Next super-chunk's inputs are in flight during the compute.  Bytes per (b,t,d): fwd 2e in +
// e out; bwd 3e in (decay, s_{t-1}, dout) + 2e out.

#include "sc_common.h"

namespace sc {

constexpr int kDChunk = 64;

struct DecayArgs {
  const void* kv;       // fwd: kv           bwd: s_all
  const void* decay;
  const void* dout;     // bwd only
  void* out;            // fwd: s_all        bwd: dkv
  void* out2;           // bwd: ddecay
  const float* init;
  float* dinit;
  int B, T, D, nsc;
  int64_t sb, st;
};

template <int DT, int NW, int LC>
__global__ void __launch_bounds__(NW * 64) decay_scan_fwd_kernel(DecayArgs a) {
  static_assert(NW * LC == kDChunk, "super-chunk must be 64 steps");
  using E = Elem<DT>;
  using T = typename E::T;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int d = blockIdx.x * 64 + lane;
  const bool dok = d < a.D;
  const int dc = dok ? d : a.D - 1;
  __shared__ float2 agg[NW][64];
  __shared__ float car[2][64];
  const T* kp = (const T*)a.kv + (int64_t)b * a.sb + dc;
  const T* ap = (const T*)a.decay + (int64_t)b * a.sb + dc;
  T* op = (T*)a.out + (int64_t)b * a.sb + d;
  if (w == 0) car[0][lane] = (a.init && dok) ? a.init[(int64_t)b * a.D + d] : 0.0f;
  T ck[LC], ca[LC], nk[LC], na[LC];
  const int Tm1 = a.T - 1;
  auto load = [&](T (&kb)[LC], T (&ab)[LC], int k) {
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const int64_t t = min(k * kDChunk + w * LC + j, Tm1);
      kb[j] = kp[t * a.st];
      ab[j] = ap[t * a.st];
    }
  };
  if (a.nsc > 0) load(ck, ca, 0);
  lds_barrier();
  for (int k = 0; k < a.nsc; ++k) {
    if (k + 1 < a.nsc) load(nk, na, k + 1);
    const int t0 = k * kDChunk + w * LC;
    float dec[LC], u[LC];
    float A = 1.0f, Bv = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const bool ok = t0 + j < a.T;
      dec[j] = ok ? E::ld(ca[j]) : 1.0f;
      u[j] = ok ? E::ld(ck[j]) : 0.0f;
      A *= dec[j];
      Bv = dec[j] * Bv + u[j];
    }
    agg[w][lane] = make_float2(A, Bv);
    lds_barrier();
    float s = car[k & 1][lane];
    for (int q = 0; q < w; ++q) {
      const float2 m = agg[q][lane];
      s = m.x * s + m.y;
    }
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      s = dec[j] * s + u[j];
      if (dok && t0 + j < a.T) op[(int64_t)(t0 + j) * a.st] = E::st(s);
    }
    if (w == NW - 1) car[(k + 1) & 1][lane] = s;
    lds_barrier();   // agg reuse + carry visibility
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      ck[j] = nk[j];
      ca[j] = na[j];
    }
  }
}

template <int DT, int NW, int LC>
__global__ void __launch_bounds__(NW * 64) decay_scan_bwd_kernel(DecayArgs a) {
  static_assert(NW * LC == kDChunk, "super-chunk must be 64 steps");
  using E = Elem<DT>;
  using T = typename E::T;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int d = blockIdx.x * 64 + lane;
  const bool dok = d < a.D;
  const int dc = dok ? d : a.D - 1;
  __shared__ float2 agg[NW][64];
  __shared__ float car[2][64];
  const T* sp = (const T*)a.kv + (int64_t)b * a.sb + dc;      // s_all
  const T* ap = (const T*)a.decay + (int64_t)b * a.sb + dc;
  const T* gp = (const T*)a.dout + (int64_t)b * a.sb + dc;
  T* dkp = (T*)a.out + (int64_t)b * a.sb + d;
  T* ddp = (T*)a.out2 + (int64_t)b * a.sb + d;
  const float s_init = (a.init && dok) ? a.init[(int64_t)b * a.D + d] : 0.0f;
  if (w == 0) car[0][lane] = 0.0f;
  // c*: current super-chunk; n*: prefetch.  sprev = s_{t-1}, decay at t+1 comes from the carry.
  T cs[LC], ca[LC], cg[LC], ns[LC], na[LC], ng[LC];
  const int Tm1 = a.T - 1;
  auto load = [&](T (&sb)[LC], T (&ab)[LC], T (&gb)[LC], int k) {
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const int t = k * kDChunk + w * LC + j;
      const int64_t tc = min(t, Tm1);
      sb[j] = sp[(int64_t)max(min(t - 1, Tm1), 0) * a.st];
      ab[j] = ap[tc * a.st];
      gb[j] = gp[tc * a.st];
    }
  };
  if (a.nsc > 0) load(cs, ca, cg, a.nsc - 1);
  lds_barrier();
  for (int it = 0; it < a.nsc; ++it) {
    const int k = a.nsc - 1 - it;
    if (k > 0) load(ns, na, ng, k - 1);
    const int t0 = k * kDChunk + w * LC;
    float dec[LC], gv[LC];
    float P = 1.0f, Q = 0.0f;
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      const bool ok = t0 + j < a.T;
      dec[j] = ok ? E::ld(ca[j]) : 1.0f;
      gv[j] = ok ? E::ld(cg[j]) : 0.0f;
      Q = dec[j] * (gv[j] + Q);
      P *= dec[j];
    }
    agg[w][lane] = make_float2(P, Q);
    lds_barrier();
    float C = car[it & 1][lane];
    for (int q = NW - 1; q > w; --q) {
      const float2 m = agg[q][lane];
      C = m.x * C + m.y;
    }
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      const float g = gv[j] + C;
      C = dec[j] * g;
      const int t = t0 + j;
      if (dok && t < a.T) {
        const float sprev = t > 0 ? E::ld(cs[j]) : s_init;
        dkp[(int64_t)t * a.st] = E::st(g);
        ddp[(int64_t)t * a.st] = E::st(g * sprev);
      }
    }
    if (w == 0) car[(it + 1) & 1][lane] = C;
    lds_barrier();
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      cs[j] = ns[j];
      ca[j] = na[j];
      cg[j] = ng[j];
    }
  }
  if (a.dinit && w == 0 && dok) a.dinit[(int64_t)b * a.D + d] = car[a.nsc & 1][lane];
}

template <int DT>
static void launch_decay(const DecayArgs& a, bool bwd, hipStream_t st) {
  dim3 grid((a.D + 63) / 64, a.B);
  if (bwd)
    hipLaunchKernelGGL((decay_scan_bwd_kernel<DT, 8, 8>), grid, dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((decay_scan_fwd_kernel<DT, 8, 8>), grid, dim3(512), 0, st, a);
}

static int run_decay(const DecayArgs& a, int dtype, bool bwd, void* stream, const char* what) {
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case SC_F32: launch_decay<SC_F32>(a, bwd, st); break;
    case SC_BF16: launch_decay<SC_BF16>(a, bwd, st); break;
    default: launch_decay<SC_F16>(a, bwd, st); break;
  }
  return launch_status(what);
}

}  // namespace sc

using namespace sc;

extern "C" int sc_decay_scan_fwd(const void* kv, const void* decay, void* out, int dtype,
                                 const float* init, int B, int T, int D, int64_t stride_b,
                                 int64_t stride_t, int64_t stride_d, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16,
             "sc_decay_scan_fwd: unsupported dtype %d", dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && D >= 0 && B <= 65535, "sc_decay_scan_fwd: bad shape");
  SC_REQUIRE(stride_d == 1, "sc_decay_scan_fwd: stride_d must be 1 (got %lld)", (long long)stride_d);
  if (B == 0 || D == 0 || T == 0) return 0;
  SC_REQUIRE(kv && decay && out, "sc_decay_scan_fwd: null pointer");
  DecayArgs a{kv, decay, nullptr, out, nullptr, init, nullptr, B, T, D,
              (T + kDChunk - 1) / kDChunk, stride_b, stride_t};
  return run_decay(a, dtype, false, stream, "sc_decay_scan_fwd");
}

extern "C" int sc_decay_scan_bwd(const void* decay, const void* s_all, const void* dout, void* dkv,
                                 void* ddecay, int dtype, const float* init, float* dinit, int B,
                                 int T, int D, int64_t stride_b, int64_t stride_t,
                                 int64_t stride_d, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16,
             "sc_decay_scan_bwd: unsupported dtype %d", dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && D >= 0 && B <= 65535, "sc_decay_scan_bwd: bad shape");
  SC_REQUIRE(stride_d == 1, "sc_decay_scan_bwd: stride_d must be 1 (got %lld)", (long long)stride_d);
  if (B == 0 || D == 0) return 0;
  if (T == 0) {
    SC_REQUIRE(!dinit, "sc_decay_scan_bwd: T == 0 with dinit: caller must zero dinit");
    return 0;
  }
  SC_REQUIRE(decay && s_all && dout && dkv && ddecay, "sc_decay_scan_bwd: null pointer");
  DecayArgs a{s_all, decay, dout, dkv, ddecay, init, dinit, B, T, D,
              (T + kDChunk - 1) / kDChunk, stride_b, stride_t};
  return run_decay(a, dtype, true, stream, "sc_decay_scan_bwd");
}
