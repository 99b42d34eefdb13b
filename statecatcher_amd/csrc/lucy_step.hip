// Streaming (one frame per call) step of the native LucyRNN, infer mode.
//
// Replaces the body of the reference's per-frame loop, lucyrnn.py:172-184, i.e.
// LucyRNNCell.forward (lucyrnn.py:44-70) for T = 1, with the state kept resident in HBM in fp32
// between calls.  Per layer the host runs two library GEMMs (input_proj, then the gate
// projection) and the two kernels below; the whole frame (all layers + output projection +
// greedy step, decode.hip) is captured once in a hipGraph and replayed per frame or per block of
// frames (statecatcher_amd/streaming.py).
//
//   lucy_step_ln_kernel    u = LayerNorm_in(a)                                 (:45)
//   lucy_step_cell_kernel  MODE_FUSED   (:47-54, :64-68)  g = [z k v h_pre dl] (r dropped: the
//                                        reference computes sigmoid(LN_r(r)) and never uses it)
//                          MODE_UNFUSED_A (:55-60)        g = [z k v dl]; s' = dec s + k v;
//                                        writes y = u + s' (the input of W_h) and the masked s
//                          MODE_UNFUSED_B (:61-68)        hp = W_h(u + s'); c = tanh(LN_h(hp))
//
// One wave per batch row; each lane holds NPL = ceil(D/64) elements (d = lane + 64 i < D) in
// registers, so every LayerNorm is two wave reductions and every access is a coalesced run.
#include "sc_common.h"

namespace sc {

enum { MODE_FUSED = 0, MODE_UNFUSED_A = 1, MODE_UNFUSED_B = 2 };

struct StepArgs {
  const void* g;   // gate GEMM output rows (dtype DT), row stride g_stride
  int64_t g_stride;
  const void* u;   // MODE_UNFUSED_A: LN_in output [B,D]; ln kernel: its input
  const void* hp;  // MODE_UNFUSED_B: W_h output [B,D]
  const float *lnz_w, *lnz_b, *lnh_w, *lnh_b;   // null when layer_norm=False
  float eps;
  float* h;        // fp32 state [B,D], in place
  float* s;        // fp32 state [B,D], in place
  void* out;       // [B,D] dtype DT: next-layer input h (FUSED / B), u + s' (A), LN output (ln)
  const float* mask;   // [B] frame mask or null
  int B, D;
};

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// LayerNorm of the NPL-per-lane row in place (nn.LayerNorm: biased variance, eps inside rsqrt);
// elements past D hold 0 and stay out of the sums
template <int NPL>
__device__ __forceinline__ void ln_row(float (&x)[NPL], const float* w, const float* b, float eps,
                                       int D, int lane) {
  if (!w) return;
  float sm = 0.0f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) sm += x[i];
  const float mu = wave_sum(sm) / (float)D;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    x[i] = lane + 64 * i < D ? x[i] - mu : 0.0f;
    q += x[i] * x[i];
  }
  const float rs = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int d = lane + 64 * i;
    if (d < D) x[i] = x[i] * rs * w[d] + b[d];
  }
}

template <int DT, int NPL>
__device__ __forceinline__ void load_row(float (&x)[NPL], const void* base, int64_t off, int D,
                                         int lane) {
  using E = Elem<DT>;
  const typename E::T* p = (const typename E::T*)base + off;
#pragma unroll
  for (int i = 0; i < NPL; ++i) x[i] = lane + 64 * i < D ? E::ld(p[lane + 64 * i]) : 0.0f;
}

template <int DT, int NPL>
__device__ __forceinline__ void store_row(const float (&x)[NPL], void* base, int64_t off, int D,
                                          int lane) {
  using E = Elem<DT>;
  typename E::T* p = (typename E::T*)base + off;
#pragma unroll
  for (int i = 0; i < NPL; ++i)
    if (lane + 64 * i < D) p[lane + 64 * i] = E::st(x[i]);
}

__device__ __forceinline__ float sig_exact(float x) { return 1.0f / (1.0f + expf(-x)); }

template <int DT, int NPL>
__global__ void __launch_bounds__(256) lucy_step_ln_kernel(StepArgs a) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.B) return;
  float x[NPL];
  load_row<DT, NPL>(x, a.u, (int64_t)b * a.D, a.D, lane);
  ln_row<NPL>(x, a.lnz_w, a.lnz_b, a.eps, a.D, lane);
  store_row<DT, NPL>(x, a.out, (int64_t)b * a.D, a.D, lane);
}

template <int DT, int NPL, int MODE>
__global__ void __launch_bounds__(256) lucy_step_cell_kernel(StepArgs a) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.B) return;
  const int D = a.D;
  const int64_t gr = (int64_t)b * a.g_stride, row = (int64_t)b * D;
  const float m = a.mask ? a.mask[b] : 1.0f;
  float z[NPL];
  load_row<DT, NPL>(z, a.g, gr, D, lane);
  if constexpr (MODE != MODE_UNFUSED_A) {   // the h update: z gate and the candidate
    ln_row<NPL>(z, a.lnz_w, a.lnz_b, a.eps, D, lane);
    float c[NPL];
    if constexpr (MODE == MODE_FUSED) {
      // s' = sigmoid(dl) s + k v, then c = tanh(LN_h(h_pre + s'))
      float k[NPL], v[NPL], dl[NPL];
      load_row<DT, NPL>(k, a.g, gr + D, D, lane);
      load_row<DT, NPL>(v, a.g, gr + 2 * D, D, lane);
      load_row<DT, NPL>(c, a.g, gr + 3 * D, D, lane);
      load_row<DT, NPL>(dl, a.g, gr + 4 * D, D, lane);
#pragma unroll
      for (int i = 0; i < NPL; ++i) {
        const int d = lane + 64 * i;
        if (d >= D) break;
        const float sp = a.s[row + d];
        const float sn = sig_exact(dl[i]) * sp + k[i] * v[i];
        c[i] += sn;
        a.s[row + d] = m * sn + (1.0f - m) * sp;
      }
    } else {
      load_row<DT, NPL>(c, a.hp, row, D, lane);
    }
    ln_row<NPL>(c, a.lnh_w, a.lnh_b, a.eps, D, lane);
    float hn[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int d = lane + 64 * i;
      if (d >= D) break;
      const float zg = sig_exact(z[i]);
      const float hp = a.h[row + d];
      const float hv = (1.0f - zg) * tanhf(c[i]) + zg * hp;
      hn[i] = m * hv + (1.0f - m) * hp;
      a.h[row + d] = hn[i];
    }
    store_row<DT, NPL>(hn, a.out, row, D, lane);
  } else {
    // unfused stage A: s' = sigmoid(W_decay u) s + (W_k u)(W_v u); y = u + s'
    float k[NPL], v[NPL], dl[NPL], y[NPL];
    load_row<DT, NPL>(k, a.g, gr + D, D, lane);
    load_row<DT, NPL>(v, a.g, gr + 2 * D, D, lane);
    load_row<DT, NPL>(dl, a.g, gr + 3 * D, D, lane);
    load_row<DT, NPL>(y, a.u, row, D, lane);
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int d = lane + 64 * i;
      if (d >= D) break;
      const float sp = a.s[row + d];
      const float sn = sig_exact(dl[i]) * sp + k[i] * v[i];
      y[i] += sn;
      a.s[row + d] = m * sn + (1.0f - m) * sp;
    }
    store_row<DT, NPL>(y, a.out, row, D, lane);
  }
}

template <int DT, int NPL>
static void launch_npl(int mode, const StepArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.B + 3) / 4)), blk(256);
  switch (mode) {
    case MODE_FUSED:
      hipLaunchKernelGGL((lucy_step_cell_kernel<DT, NPL, MODE_FUSED>), grid, blk, 0, st, a); break;
    case MODE_UNFUSED_A:
      hipLaunchKernelGGL((lucy_step_cell_kernel<DT, NPL, MODE_UNFUSED_A>), grid, blk, 0, st, a); break;
    case MODE_UNFUSED_B:
      hipLaunchKernelGGL((lucy_step_cell_kernel<DT, NPL, MODE_UNFUSED_B>), grid, blk, 0, st, a); break;
    default:   // the LayerNorm
      hipLaunchKernelGGL((lucy_step_ln_kernel<DT, NPL>), grid, blk, 0, st, a); break;
  }
}

template <int DT>
static void launch_dt(int mode, const StepArgs& a, hipStream_t st) {
  const int n = (a.D + 63) / 64;
  if (n <= 1) launch_npl<DT, 1>(mode, a, st);
  else if (n <= 2) launch_npl<DT, 2>(mode, a, st);
  else if (n <= 4) launch_npl<DT, 4>(mode, a, st);
  else if (n <= 8) launch_npl<DT, 8>(mode, a, st);
  else if (n <= 12) launch_npl<DT, 12>(mode, a, st);
  else launch_npl<DT, 16>(mode, a, st);
}

static bool npl_ok(int D) { return D > 0 && D <= 16 * 64; }

}  // namespace sc

using namespace sc;

extern "C" int sc_lucy_step_supported(int dtype, int D) {
  return (dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16) && npl_ok(D);
}

extern "C" int sc_lucy_step_ln(const void* x, int dtype, const float* w, const float* b, float eps,
                               void* y, int B, int D, void* stream) {
  clear_error();
  SC_REQUIRE(sc_lucy_step_supported(dtype, D), "sc_lucy_step_ln: unsupported dtype %d / D %d",
             dtype, D);
  SC_REQUIRE(B >= 0, "sc_lucy_step_ln: bad B %d", B);
  if (B == 0) return 0;
  SC_REQUIRE(x && w && b && y, "sc_lucy_step_ln: null pointer");
  StepArgs a{};
  a.u = x; a.lnz_w = w; a.lnz_b = b; a.eps = eps; a.out = y; a.B = B; a.D = D;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case SC_F32: launch_dt<SC_F32>(-1, a, st); break;
    case SC_BF16: launch_dt<SC_BF16>(-1, a, st); break;
    default: launch_dt<SC_F16>(-1, a, st); break;
  }
  return launch_status("sc_lucy_step_ln");
}

extern "C" int sc_lucy_step_cell(int mode, const void* g, int dtype, int64_t g_stride,
                                 const void* u, const void* hp, const float* lnz_w,
                                 const float* lnz_b, const float* lnh_w, const float* lnh_b,
                                 float eps, float* h, float* s, void* out, const float* mask, int B,
                                 int D, void* stream) {
  clear_error();
  SC_REQUIRE(sc_lucy_step_supported(dtype, D), "sc_lucy_step_cell: unsupported dtype %d / D %d",
             dtype, D);
  SC_REQUIRE(mode >= MODE_FUSED && mode <= MODE_UNFUSED_B, "sc_lucy_step_cell: bad mode %d", mode);
  SC_REQUIRE(B >= 0, "sc_lucy_step_cell: bad B %d", B);
  if (B == 0) return 0;
  const int ngate = mode == MODE_FUSED ? 5 : 4;
  SC_REQUIRE(g && out, "sc_lucy_step_cell: null pointer");
  SC_REQUIRE(g_stride >= (int64_t)ngate * D, "sc_lucy_step_cell: g row stride %lld < %d*D",
             (long long)g_stride, ngate);
  SC_REQUIRE(mode == MODE_UNFUSED_B ? (h != nullptr && hp != nullptr) : (s != nullptr),
             "sc_lucy_step_cell: null state");
  SC_REQUIRE(mode != MODE_FUSED || h, "sc_lucy_step_cell: null h");
  SC_REQUIRE(mode != MODE_UNFUSED_A || u, "sc_lucy_step_cell: null u");
  SC_REQUIRE((lnz_w == nullptr) == (lnz_b == nullptr) && (lnh_w == nullptr) == (lnh_b == nullptr),
             "sc_lucy_step_cell: LayerNorm weight and bias must both be given or both null");
  StepArgs a{g, g_stride, u, hp, lnz_w, lnz_b, lnh_w, lnh_b, eps, h, s, out, mask, B, D};
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case SC_F32: launch_dt<SC_F32>(mode, a, st); break;
    case SC_BF16: launch_dt<SC_BF16>(mode, a, st); break;
    default: launch_dt<SC_F16>(mode, a, st); break;
  }
  return launch_status("sc_lucy_step_cell");
}
