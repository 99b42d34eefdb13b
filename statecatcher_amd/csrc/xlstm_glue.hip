// Elementwise / row-norm glue of the xLSTM-large block (config C4: the encoder the reference
// builds at model.py:214-229 from its xlstm fork; structure as transformers'
// modeling_xlstm.py:870-1205) fused into single HBM passes, forward and backward.  Under bf16
// autocast each of these is 5-10 torch kernels with fp32 intermediates (RMSNorm: float, pow,
// mean, add, rsqrt, mul, cast, mul; the gated head norm: mean, sub, var, rsqrt, mul, cast, mul,
// sigmoid, mul) -- >60% of the C4 step.  Each kernel here reads its operands once and writes
// once, reproducing the module's roundings: values the module rounds to bf16 in the middle of
// the chain are rounded at the same points, the rest is fp32.
//
//   rms_fwd / rms_bwd     RMSNorm (force_float32_reductions): n = bf16(x rsqrt(mean x^2 + eps)),
//                         y = bf16(n w); one wave per row, 8-byte loads.  dW as per-workgroup
//                         fp32 partial rows (fixed-order sum by sc_colsum: deterministic).
//   mhln_fwd / mhln_bwd   out = bf16(bf16(sigmoid(o)) * bf16(LN_head(h)) * w): the mLSTM layer's
//                         MultiHeadLayerNorm of the cell output (h in the cell's [B][NH][T][DH]
//                         layout, no transpose copy) gated by sigmoid(o) (o a strided view of the
//                         fused projection); 16 lanes per head.  Backward writes dh in the cell
//                         layout and do into the projection-gradient layout.
//   swiglu_fwd / _bwd     y = bf16(bf16(silu(g)) * u) for [g | u] = the fused up-projection;
//                         the backward writes [dg | du] as ONE row, the up-projection's gradient.
// All bytes: one read of each operand, one write of each result -- HBM-bound.
#include "sc_common.h"

namespace sc {
namespace {

typedef uint16_t u16;

__device__ __forceinline__ float bf(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ u16 tobf(float f) {
  return __builtin_bit_cast(u16, (__bf16)f);
}
__device__ __forceinline__ float rbf(float f) { return bf(tobf(f)); }   // round through bf16

// 4 bf16 as one 8-byte load / store
__device__ __forceinline__ void ld4(const u16* p, float (&v)[4]) {
  const uint2 q = *(const uint2*)p;
  v[0] = __uint_as_float(q.x << 16);
  v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16);
  v[3] = __uint_as_float(q.y & 0xffff0000u);
}
// 4 f16 rounded to bf16 (an f16 mLSTM cell's h as the split path's h.to(bfloat16) sees it)
__device__ __forceinline__ void ld4_h16(const u16* p, float (&v)[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 q = *(const h4*)p;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = rbf((float)q[k]);
}
// the same conversions from an 8-byte piece already in registers (loads issued a row ahead)
__device__ __forceinline__ void cvt4(uint2 q, float (&v)[4]) {
  v[0] = __uint_as_float(q.x << 16);
  v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16);
  v[3] = __uint_as_float(q.y & 0xffff0000u);
}
__device__ __forceinline__ void cvt4_h16(uint2 q, float (&v)[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 x = __builtin_bit_cast(h4, q);
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = rbf((float)x[k]);
}
__device__ __forceinline__ void st4(u16* p, const float (&v)[4]) {
  uint2 q;
  q.x = (uint32_t)tobf(v[0]) | ((uint32_t)tobf(v[1]) << 16);
  q.y = (uint32_t)tobf(v[2]) | ((uint32_t)tobf(v[3]) << 16);
  *(uint2*)p = q;
}

template <int W>
__device__ __forceinline__ float group_sum(float x) {   // sum over aligned groups of W lanes
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

constexpr int kPartWg = 512;   // workgroups (and partial rows) of the weight-gradient passes

// ------------------------------------------------------------------------------ RMSNorm ------
// CH = D / 256 chunks of 4 per lane
// ADD: the block's residual add folded in -- s = bf16(x + r) is written and normalised (the
// torch chain's bf16 add, then RMSNorm of its result)
template <int CH, bool ADD>
__global__ void __launch_bounds__(256) rms_fwd_kernel(const u16* x, const u16* r, u16* s,
                                                      const float* w, u16* y, float* rstd,
                                                      int64_t rows, float eps) {
  constexpr int D = 256 * CH;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[CH][4];
  float ss = 0.0f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    ld4(x + row * D + (c * 64 + lane) * 4, v[c]);
    if constexpr (ADD) {
      float rv[4];
      ld4(r + row * D + (c * 64 + lane) * 4, rv);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] = rbf(v[c][k] + rv[k]);
      st4(s + row * D + (c * 64 + lane) * 4, v[c]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) ss = fmaf(v[c][k], v[c][k], ss);
  }
  ss = group_sum<64>(ss);
  const float rs = rsq(ss / (float)D + eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int e0 = (c * 64 + lane) * 4;
    const float4 wv = *(const float4*)(w + e0);
    const float o[4] = {rbf(v[c][0] * rs) * wv.x, rbf(v[c][1] * rs) * wv.y,
                        rbf(v[c][2] * rs) * wv.z, rbf(v[c][3] * rs) * wv.w};
    st4(y + row * D + e0, o);
  }
  if (lane == 0) rstd[row] = rs;
}

// dx = rstd (g - xh mean(g xh)), g = dy w, xh = x rstd;  dW partial = sum_rows dy bf16(xh)
// ADD: dx = bf16(bf16(dx) + dres), the residual branch's gradient accumulated as autograd
// accumulates the two bf16 gradients of the block's sum
template <int CH, bool ADD>
__global__ void __launch_bounds__(256) rms_bwd_kernel(const u16* x, const u16* dy, const u16* dres,
                                                      const float* w, const float* rstd, u16* dx,
                                                      float* part, int64_t rows) {
  constexpr int D = 256 * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ float red[4][D];
  float dwp[CH][4];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) dwp[c][k] = 0.0f;
  float wr[CH][4];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const float4 q = *(const float4*)(w + (c * 64 + lane) * 4);
    wr[c][0] = q.x; wr[c][1] = q.y; wr[c][2] = q.z; wr[c][3] = q.w;
  }
  // grid-stride rows with the next row's inputs loaded while this one computes (each wave
  // walks ~rows / 2048 rows; a load-then-use loop paid a memory latency per row)
  const int64_t rstep = (int64_t)gridDim.x * 4;
  uint2 px[CH], pd[CH], pr[CH];
  float prs = 0.0f;
  auto load_row = [&](int64_t row) __attribute__((always_inline)) {
    prs = rstd[row];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      px[c] = *(const uint2*)(x + row * D + (c * 64 + lane) * 4);
      pd[c] = *(const uint2*)(dy + row * D + (c * 64 + lane) * 4);
      if constexpr (ADD) pr[c] = *(const uint2*)(dres + row * D + (c * 64 + lane) * 4);
    }
  };
  if ((int64_t)blockIdx.x * 4 + wv < rows) load_row((int64_t)blockIdx.x * 4 + wv);
  for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < rows; row += rstep) {
    const float rs = prs;
    uint2 cx[CH], cd[CH], cr[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      cx[c] = px[c];
      cd[c] = pd[c];
      cr[c] = pr[c];
    }
    if (row + rstep < rows) load_row(row + rstep);
    float xv[CH][4], gv[CH][4];
    float dot = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float dv[4];
      cvt4(cx[c], xv[c]);
      cvt4(cd[c], dv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float xh = xv[c][k] * rs;
        gv[c][k] = dv[k] * wr[c][k];
        dot = fmaf(gv[c][k], xh, dot);
        dwp[c][k] = fmaf(dv[k], rbf(xh), dwp[c][k]);
        xv[c][k] = xh;
      }
    }
    dot = group_sum<64>(dot) / (float)D;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = rs * (gv[c][k] - xv[c][k] * dot);
      if constexpr (ADD) {
        float rv[4];
        cvt4(cr[c], rv);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = rbf(o[k]) + rv[k];
      }
      st4(dx + row * D + (c * 64 + lane) * 4, o);
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wv][(c * 64 + lane) * 4 + k] = dwp[c][k];
  __syncthreads();
  for (int e = threadIdx.x; e < D; e += 256)
    part[(int64_t)blockIdx.x * D + e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
}

// ------------------------------------------------------------------ gated head LayerNorm ------
// Row m = (b, t); head n of the row is h[b][n][t][0..DH), 16 lanes per head (NH <= 4), CH = DH / 64
// chunks of 4 per lane.  o / out / do rows: [M][ld] with columns n * DH + e.
struct MhArgs {
  const u16* h;
  const u16* o;
  const float* w;
  u16* out;
  float* mean;
  float* rstd;
  const u16* dy;
  u16* dh;
  u16* dgo;
  float* part;
  int B, T, NH;
  int64_t ldo, ldy, lddo;
  float eps;
  int h16;   // h is f16 (read rounded to bf16), else bf16
};

template <int CH>
__global__ void __launch_bounds__(256) mhln_fwd_kernel(MhArgs a) {
  constexpr int DH = 64 * CH;
  const int lane = threadIdx.x & 63, n = lane >> 4, sub = lane & 15;
  const int64_t M = (int64_t)a.B * a.T;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M || n >= a.NH) return;   // (whole lane groups: the group sums stay within a head)
  const int b = (int)(m / a.T), t = (int)(m % a.T);
  const u16* hp = a.h + (((int64_t)b * a.NH + n) * a.T + t) * DH;
  float v[CH][4];
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    if (a.h16) ld4_h16(hp + (c * 16 + sub) * 4, v[c]);
    else ld4(hp + (c * 16 + sub) * 4, v[c]);
#pragma unroll
    for (int k = 0; k < 4; ++k) s += v[c][k];
  }
  const float mu = group_sum<16>(s) / (float)DH;
  float q = 0.0f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) q = fmaf(v[c][k] - mu, v[c][k] - mu, q);
  const float rs = rsq(group_sum<16>(q) / (float)DH + a.eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = n * DH + (c * 16 + sub) * 4;
    float ov[4], r[4];
    ld4(a.o + m * a.ldo + col, ov);
    const float4 wv = *(const float4*)(a.w + col);
    const float wk[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      r[k] = rbf(sigm(ov[k])) * (rbf((v[c][k] - mu) * rs) * wk[k]);
    st4(a.out + m * (int64_t)(a.NH * DH) + col, r);
  }
  if (sub == 0) {
    a.mean[m * a.NH + n] = mu;
    a.rstd[m * a.NH + n] = rs;
  }
}

// z = bf16(xh) w, s = bf16(sigmoid(o)):  do = dy z s (1 - s);  dxh = dy s w;
// dh = rstd (dxh - mean(dxh) - xh mean(dxh xh));  dW partial = sum_rows dy s bf16(xh)
template <int CH>
__global__ void __launch_bounds__(256) mhln_bwd_kernel(MhArgs a) {
  constexpr int DH = 64 * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, n = lane >> 4, sub = lane & 15;
  const int64_t M = (int64_t)a.B * a.T;
  const int DV = a.NH * DH;
  extern __shared__ float red[];   // [4][DV]
  float dwp[CH][4];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) dwp[c][k] = 0.0f;
  const bool hok = n < a.NH;
  // grid-stride rows with the next row's h / o / dy / statistics loaded while this one computes
  // (a load-then-use loop paid one memory latency per row: 122 us at C4 for 375 MB)
  const int64_t mstep = (int64_t)gridDim.x * 4;
  uint2 ph[CH], po[CH], pd[CH];
  float pmu = 0.0f, prs = 0.0f;
  auto load_row = [&](int64_t m) __attribute__((always_inline)) {
    const int b = (int)(m / a.T), t = (int)(m % a.T);
    const int64_t hrow = (((int64_t)b * a.NH + n) * a.T + t) * DH;
    pmu = a.mean[m * a.NH + n];
    prs = a.rstd[m * a.NH + n];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = n * DH + (c * 16 + sub) * 4;
      ph[c] = *(const uint2*)(a.h + hrow + (c * 16 + sub) * 4);
      po[c] = *(const uint2*)(a.o + m * a.ldo + col);
      pd[c] = *(const uint2*)(a.dy + m * a.ldy + col);
    }
  };
  if (hok && (int64_t)blockIdx.x * 4 + wv < M) load_row((int64_t)blockIdx.x * 4 + wv);
  for (int64_t m = (int64_t)blockIdx.x * 4 + wv; m < M; m += mstep) {
    if (!hok) continue;
    const int b = (int)(m / a.T), t = (int)(m % a.T);
    const int64_t hrow = (((int64_t)b * a.NH + n) * a.T + t) * DH;
    const float mu = pmu, rs = prs;
    uint2 ch[CH], co[CH], cd[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      ch[c] = ph[c];
      co[c] = po[c];
      cd[c] = pd[c];
    }
    if (m + mstep < M) load_row(m + mstep);
    float xh[CH][4], g[CH][4];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int col = n * DH + (c * 16 + sub) * 4;
      float hv[4], ov[4], dv[4], dov[4];
      if (a.h16) cvt4_h16(ch[c], hv);
      else cvt4(ch[c], hv);
      cvt4(co[c], ov);
      cvt4(cd[c], dv);
      const float4 wq = *(const float4*)(a.w + col);
      const float wk[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x = (hv[k] - mu) * rs;
        const float nb = rbf(x);
        const float sg = rbf(sigm(ov[k]));
        dov[k] = dv[k] * nb * wk[k] * sg * (1.0f - sg);
        const float dz = dv[k] * sg;
        dwp[c][k] = fmaf(dz, nb, dwp[c][k]);
        g[c][k] = dz * wk[k];
        xh[c][k] = x;
        s1 += g[c][k];
        s2 = fmaf(g[c][k], x, s2);
      }
      st4(a.dgo + m * a.lddo + col, dov);
    }
    s1 = group_sum<16>(s1) / (float)DH;
    s2 = group_sum<16>(s2) / (float)DH;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = rs * (g[c][k] - s1 - xh[c][k] * s2);
      st4(a.dh + hrow + (c * 16 + sub) * 4, o);
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (hok) red[wv * DV + n * DH + (c * 16 + sub) * 4 + k] = dwp[c][k];
  __syncthreads();
  for (int e = threadIdx.x; e < DV; e += 256)
    a.part[(int64_t)blockIdx.x * DV + e] = red[e] + red[DV + e] + red[2 * DV + e] + red[3 * DV + e];
}

// ------------------------------------------------------------------------------ SwiGLU -------
// a [rows][2F] = [g | u]; y [rows][F].  One thread per 4 columns.
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const u16* a, u16* y, int64_t rows, int F) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;   // index of a 4-column group
  const int F4 = F / 4;
  if (q >= rows * F4) return;
  const int64_t r = q / F4;
  const int c = (int)(q % F4) * 4;
  float g[4], u[4], o[4];
  ld4(a + r * 2 * F + c, g);
  ld4(a + r * 2 * F + F + c, u);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = rbf(g[k] * sigm(g[k])) * u[k];
  st4(y + r * F + c, o);
}

// silu'(g) = s (1 + g (1 - s)), s = sigmoid(g):  dg = bf16(dy u) silu'(g),  du = dy bf16(silu(g))
__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const u16* a, const u16* dy, u16* da,
                                                         int64_t rows, int F) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int F4 = F / 4;
  if (q >= rows * F4) return;
  const int64_t r = q / F4;
  const int c = (int)(q % F4) * 4;
  float g[4], u[4], d[4], dg[4], du[4];
  ld4(a + r * 2 * F + c, g);
  ld4(a + r * 2 * F + F + c, u);
  ld4(dy + r * F + c, d);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float s = sigm(g[k]);
    dg[k] = rbf(d[k] * u[k]) * (s * (1.0f + g[k] * (1.0f - s)));
    du[k] = d[k] * rbf(g[k] * s);
  }
  st4(da + r * 2 * F + c, dg);
  st4(da + r * 2 * F + F + c, du);
}

int part_rows(int64_t rows) { return (int)(rows < (int64_t)kPartWg * 4 ? (rows + 3) / 4 : kPartWg); }

}  // namespace
}  // namespace sc

using namespace sc;

extern "C" int sc_xlstm_part_rows(int64_t rows) { return rows > 0 ? part_rows(rows) : 1; }

template <bool ADD>
static int rms_fwd_launch(const void* x, const void* r, void* s, const float* w, void* y,
                          float* rstd, int64_t rows, int D, float eps, void* stream) {
  if (rows == 0) return 0;
  const dim3 g((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const u16 *xp = (const u16*)x, *rp = (const u16*)r;
  u16 *sp = (u16*)s, *yp = (u16*)y;
  switch (D / 256) {
    case 1: hipLaunchKernelGGL((rms_fwd_kernel<1, ADD>), g, dim3(256), 0, st, xp, rp, sp, w, yp, rstd, rows, eps); break;
    case 2: hipLaunchKernelGGL((rms_fwd_kernel<2, ADD>), g, dim3(256), 0, st, xp, rp, sp, w, yp, rstd, rows, eps); break;
    case 3: hipLaunchKernelGGL((rms_fwd_kernel<3, ADD>), g, dim3(256), 0, st, xp, rp, sp, w, yp, rstd, rows, eps); break;
    default: hipLaunchKernelGGL((rms_fwd_kernel<4, ADD>), g, dim3(256), 0, st, xp, rp, sp, w, yp, rstd, rows, eps); break;
  }
  return 0;
}

template <bool ADD>
static void rms_bwd_launch(const void* x, const void* dy, const void* dres, const float* w,
                           const float* rstd, void* dx, float* part, int64_t rows, int D,
                           void* stream) {
  const dim3 g((unsigned)part_rows(rows));
  hipStream_t st = (hipStream_t)stream;
  const u16 *xp = (const u16*)x, *dyp = (const u16*)dy, *rp = (const u16*)dres;
  u16* dxp = (u16*)dx;
  switch (D / 256) {
    case 1: hipLaunchKernelGGL((rms_bwd_kernel<1, ADD>), g, dim3(256), 0, st, xp, dyp, rp, w, rstd, dxp, part, rows); break;
    case 2: hipLaunchKernelGGL((rms_bwd_kernel<2, ADD>), g, dim3(256), 0, st, xp, dyp, rp, w, rstd, dxp, part, rows); break;
    case 3: hipLaunchKernelGGL((rms_bwd_kernel<3, ADD>), g, dim3(256), 0, st, xp, dyp, rp, w, rstd, dxp, part, rows); break;
    default: hipLaunchKernelGGL((rms_bwd_kernel<4, ADD>), g, dim3(256), 0, st, xp, dyp, rp, w, rstd, dxp, part, rows); break;
  }
}

extern "C" int sc_rmsnorm_fwd(const void* x, const float* w, void* y, float* rstd, int64_t rows,
                              int D, float eps, void* stream) {
  clear_error();
  SC_REQUIRE(x && w && y && rstd, "sc_rmsnorm_fwd: null pointer");
  SC_REQUIRE(D == 256 || D == 512 || D == 768 || D == 1024,
             "sc_rmsnorm_fwd: D=%d (256, 512, 768 or 1024)", D);
  SC_REQUIRE(rows >= 0, "sc_rmsnorm_fwd: rows < 0");
  rms_fwd_launch<false>(x, nullptr, nullptr, w, y, rstd, rows, D, eps, stream);
  return launch_status("sc_rmsnorm_fwd");
}

extern "C" int sc_rmsnorm_add_fwd(const void* x, const void* r, void* s, const float* w, void* y,
                                  float* rstd, int64_t rows, int D, float eps, void* stream) {
  clear_error();
  SC_REQUIRE(x && r && s && w && y && rstd, "sc_rmsnorm_add_fwd: null pointer");
  SC_REQUIRE(D == 256 || D == 512 || D == 768 || D == 1024,
             "sc_rmsnorm_add_fwd: D=%d (256, 512, 768 or 1024)", D);
  SC_REQUIRE(rows >= 0, "sc_rmsnorm_add_fwd: rows < 0");
  rms_fwd_launch<true>(x, r, s, w, y, rstd, rows, D, eps, stream);
  return launch_status("sc_rmsnorm_add_fwd");
}

extern "C" int sc_rmsnorm_bwd(const void* x, const void* dy, const float* w, const float* rstd,
                              void* dx, float* part, int64_t rows, int D, void* stream) {
  clear_error();
  SC_REQUIRE(x && dy && w && rstd && dx && part, "sc_rmsnorm_bwd: null pointer");
  SC_REQUIRE(D == 256 || D == 512 || D == 768 || D == 1024, "sc_rmsnorm_bwd: D=%d", D);
  if (rows <= 0) return 0;
  rms_bwd_launch<false>(x, dy, nullptr, w, rstd, dx, part, rows, D, stream);
  return launch_status("sc_rmsnorm_bwd");
}

extern "C" int sc_rmsnorm_add_bwd(const void* s, const void* dy, const void* dres, const float* w,
                                  const float* rstd, void* dx, float* part, int64_t rows, int D,
                                  void* stream) {
  clear_error();
  SC_REQUIRE(s && dy && dres && w && rstd && dx && part, "sc_rmsnorm_add_bwd: null pointer");
  SC_REQUIRE(D == 256 || D == 512 || D == 768 || D == 1024, "sc_rmsnorm_add_bwd: D=%d", D);
  if (rows <= 0) return 0;
  rms_bwd_launch<true>(s, dy, dres, w, rstd, dx, part, rows, D, stream);
  return launch_status("sc_rmsnorm_add_bwd");
}

static int mh_check(int B, int T, int NH, int DH, const char* who) {
  SC_REQUIRE(B >= 0 && T >= 0, "%s: bad shape", who);
  SC_REQUIRE(NH >= 1 && NH <= 4 && (DH == 64 || DH == 128 || DH == 192 || DH == 256),
             "%s: NH=%d DH=%d (NH <= 4, DH in 64..256 by 64)", who, NH, DH);
  return 0;
}

static int mhln_fwd(const void* h, int h16, const void* o, int64_t ldo, const float* w,
                    void* out, float* mean, float* rstd, int B, int T, int NH, int DH, float eps,
                    void* stream) {
  clear_error();
  if (int rc = mh_check(B, T, NH, DH, "sc_mhln_gate_fwd")) return rc;
  SC_REQUIRE(h && o && w && out && mean && rstd, "sc_mhln_gate_fwd: null pointer");
  SC_REQUIRE(ldo >= NH * DH && ldo % 4 == 0, "sc_mhln_gate_fwd: ldo");
  const int64_t M = (int64_t)B * T;
  if (M == 0) return 0;
  MhArgs a{(const u16*)h, (const u16*)o, w, (u16*)out, mean, rstd, nullptr, nullptr, nullptr,
           nullptr, B, T, NH, ldo, 0, 0, eps, h16};
  const dim3 g((unsigned)((M + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  switch (DH / 64) {
    case 1: hipLaunchKernelGGL(mhln_fwd_kernel<1>, g, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(mhln_fwd_kernel<2>, g, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL(mhln_fwd_kernel<3>, g, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(mhln_fwd_kernel<4>, g, dim3(256), 0, st, a); break;
  }
  return launch_status("sc_mhln_gate_fwd");
}
extern "C" int sc_mhln_gate_fwd(const void* h, const void* o, int64_t ldo, const float* w, void* out,
                                float* mean, float* rstd, int B, int T, int NH, int DH, float eps,
                                void* stream) {
  return mhln_fwd(h, 0, o, ldo, w, out, mean, rstd, B, T, NH, DH, eps, stream);
}
extern "C" int sc_mhln_gate_fwd_h16(const void* h, const void* o, int64_t ldo, const float* w,
                                    void* out, float* mean, float* rstd, int B, int T, int NH,
                                    int DH, float eps, void* stream) {
  return mhln_fwd(h, 1, o, ldo, w, out, mean, rstd, B, T, NH, DH, eps, stream);
}

static int mhln_bwd(const void* h, int h16, const void* o, int64_t ldo, const float* w,
                    const float* mean, const float* rstd, const void* dy, int64_t ldy, void* dh,
                    void* dgo, int64_t lddo, float* part, int B, int T, int NH, int DH,
                    void* stream) {
  clear_error();
  if (int rc = mh_check(B, T, NH, DH, "sc_mhln_gate_bwd")) return rc;
  SC_REQUIRE(h && o && w && mean && rstd && dy && dh && dgo && part, "sc_mhln_gate_bwd: null pointer");
  SC_REQUIRE(ldo % 4 == 0 && ldy % 4 == 0 && lddo % 4 == 0, "sc_mhln_gate_bwd: strides");
  const int64_t M = (int64_t)B * T;
  if (M == 0) return 0;
  MhArgs a{(const u16*)h, (const u16*)o, w, nullptr, const_cast<float*>(mean),
           const_cast<float*>(rstd), (const u16*)dy, (u16*)dh, (u16*)dgo, part, B, T, NH, ldo,
           ldy, lddo, 0.0f, h16};
  const dim3 g((unsigned)part_rows(M));
  const size_t lds = (size_t)4 * NH * DH * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  switch (DH / 64) {
    case 1: hipLaunchKernelGGL(mhln_bwd_kernel<1>, g, dim3(256), lds, st, a); break;
    case 2: hipLaunchKernelGGL(mhln_bwd_kernel<2>, g, dim3(256), lds, st, a); break;
    case 3: hipLaunchKernelGGL(mhln_bwd_kernel<3>, g, dim3(256), lds, st, a); break;
    default: hipLaunchKernelGGL(mhln_bwd_kernel<4>, g, dim3(256), lds, st, a); break;
  }
  return launch_status("sc_mhln_gate_bwd");
}
extern "C" int sc_mhln_gate_bwd(const void* h, const void* o, int64_t ldo, const float* w,
                                const float* mean, const float* rstd, const void* dy, int64_t ldy,
                                void* dh, void* dgo, int64_t lddo, float* part, int B, int T,
                                int NH, int DH, void* stream) {
  return mhln_bwd(h, 0, o, ldo, w, mean, rstd, dy, ldy, dh, dgo, lddo, part, B, T, NH, DH, stream);
}
extern "C" int sc_mhln_gate_bwd_h16(const void* h, const void* o, int64_t ldo, const float* w,
                                    const float* mean, const float* rstd, const void* dy,
                                    int64_t ldy, void* dh, void* dgo, int64_t lddo, float* part,
                                    int B, int T, int NH, int DH, void* stream) {
  return mhln_bwd(h, 1, o, ldo, w, mean, rstd, dy, ldy, dh, dgo, lddo, part, B, T, NH, DH, stream);
}

extern "C" int sc_swiglu_fwd(const void* a, void* y, int64_t rows, int F, void* stream) {
  clear_error();
  SC_REQUIRE(a && y, "sc_swiglu_fwd: null pointer");
  SC_REQUIRE(F > 0 && F % 4 == 0 && rows >= 0, "sc_swiglu_fwd: F=%d must be a multiple of 4", F);
  const int64_t n = rows * (F / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const u16*)a, (u16*)y, rows, F);
  return launch_status("sc_swiglu_fwd");
}

extern "C" int sc_swiglu_bwd(const void* a, const void* dy, void* da, int64_t rows, int F,
                             void* stream) {
  clear_error();
  SC_REQUIRE(a && dy && da, "sc_swiglu_bwd: null pointer");
  SC_REQUIRE(F > 0 && F % 4 == 0 && rows >= 0, "sc_swiglu_bwd: F=%d must be a multiple of 4", F);
  const int64_t n = rows * (F / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const u16*)a, (const u16*)dy, (u16*)da, rows, F);
  return launch_status("sc_swiglu_bwd");
}
