// Inter-layer LayerNorm of the LucyRNN stack (lucyrnn_triton.py:96-97, :136-137: nn.LayerNorm(D),
// eps 1e-5, biased variance, affine) for gfx950: forward and backward in the activation dtype
// with fp32 statistics, so the bf16 scan output feeds the next bf16 GEMM without the fp32
// round trip (and its cast kernels) that autocast's LayerNorm costs.
//
//   fwd: one wave per row (rows = B*T), 16-byte loads, two-pass mean/variance in registers;
//        writes y (same dtype as x) and per-row mean / rstd (fp32) for the backward.
//   bwd: one wave per row for dx; dgamma/dbeta are accumulated per lane across the rows a
//        workgroup walks (grid-stride) and written as per-workgroup partial rows [P,2,D],
//        reduced by a fixed-order second pass (deterministic, no atomics).
// Bytes per row: fwd 2*D*e (+8), bwd 3*D*e (+8) — HBM-bound.
#include "sc_common.h"

namespace sc {

struct LnArgs {
  const void* x;
  const void* dy;
  const float* gamma;
  const float* beta;
  void* y;     // fwd output / bwd dx
  float* mean;
  float* rstd;
  float* part;  // bwd: [P, 2, D] partial (dgamma, dbeta)
  int64_t rows;
  int D;
  float eps;
};

template <typename T, int VEC>
struct Vec {
  T v[VEC];
};

// CH = 16-byte chunks per lane per row; VEC elements per chunk; D == 64 * CH * VEC
template <int DT, int CH>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnArgs a) {
  using E = Elem<DT>;
  using T = typename E::T;
  constexpr int VEC = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const Vec<T, VEC>* xr = (const Vec<T, VEC>*)((const T*)a.x + row * a.D);
  float xv[CH][VEC];
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const Vec<T, VEC> q = xr[c * 64 + lane];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      xv[c][k] = E::ld(q.v[k]);
      s += xv[c][k];
    }
  }
  s = wave_sum_dpp(s);
  const float mu = s / (float)a.D;
  float q2 = 0.0f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const float dv = xv[c][k] - mu;
      q2 += dv * dv;
    }
  q2 = wave_sum_dpp(q2);
  const float rs = rsq(q2 / (float)a.D + a.eps);
  Vec<T, VEC>* yr = (Vec<T, VEC>*)((T*)a.y + row * a.D);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int e0 = (c * 64 + lane) * VEC;
    Vec<T, VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      o.v[k] = E::st((xv[c][k] - mu) * rs * a.gamma[e0 + k] + a.beta[e0 + k]);
    yr[c * 64 + lane] = o;
  }
  if (lane == 0) {
    a.mean[row] = mu;
    a.rstd[row] = rs;
  }
}

template <int DT, int CH>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnArgs a) {
  using E = Elem<DT>;
  using T = typename E::T;
  constexpr int VEC = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  float g[CH][VEC], dgs[CH][VEC], dbs[CH][VEC];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      g[c][k] = a.gamma[(c * 64 + lane) * VEC + k];
      dgs[c][k] = 0.0f;
      dbs[c][k] = 0.0f;
    }
  const float invD = 1.0f / (float)a.D;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < a.rows; row += (int64_t)gridDim.x * 4) {
    const Vec<T, VEC>* xr = (const Vec<T, VEC>*)((const T*)a.x + row * a.D);
    const Vec<T, VEC>* dr = (const Vec<T, VEC>*)((const T*)a.dy + row * a.D);
    const float mu = a.mean[row], rs = a.rstd[row];
    float xh[CH][VEC], dxh[CH][VEC];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const Vec<T, VEC> qx = xr[c * 64 + lane];
      const Vec<T, VEC> qd = dr[c * 64 + lane];
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const float dyv = E::ld(qd.v[k]);
        xh[c][k] = (E::ld(qx.v[k]) - mu) * rs;
        dxh[c][k] = dyv * g[c][k];
        dgs[c][k] += dyv * xh[c][k];
        dbs[c][k] += dyv;
        s1 += dxh[c][k];
        s2 += dxh[c][k] * xh[c][k];
      }
    }
    s1 = wave_sum_dpp(s1);
    s2 = wave_sum_dpp(s2);
    s1 *= invD;
    s2 *= invD;
    Vec<T, VEC>* outr = (Vec<T, VEC>*)((T*)a.y + row * a.D);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      Vec<T, VEC> o;
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = E::st(rs * (dxh[c][k] - s1 - xh[c][k] * s2));
      outr[c * 64 + lane] = o;
    }
  }
  // per-workgroup partials: waves 0..3 summed in a fixed order through LDS
  extern __shared__ __attribute__((aligned(16))) float red[];   // [4][2][D]
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int e = (c * 64 + lane) * VEC + k;
      red[(wv * 2 + 0) * a.D + e] = dgs[c][k];
      red[(wv * 2 + 1) * a.D + e] = dbs[c][k];
    }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * a.D; e += 256) {
    const float v = red[e] + red[2 * a.D + e] + red[4 * a.D + e] + red[6 * a.D + e];
    a.part[(int64_t)blockIdx.x * 2 * a.D + e] = v;
  }
}

// fixed-order sum of the P partial rows: out[n] = sum_p part[p][n].  A workgroup owns 64
// columns; its 16 waves each sum a contiguous block of rows (coalesced 256-B row segments) into
// 8 interleaved accumulators (8 independent loads in flight), then a fixed-order LDS sum.
__global__ void __launch_bounds__(1024) ln_part_sum_kernel(const float* part, int P, int n, float* out) {
  __shared__ float accw[16][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int per = (P + 15) / 16;
  const int p0 = q * per, p1 = min(P, p0 + per);
  float acc = 0.0f;
  if (e < n) {
    float r[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    int p = p0;
    for (; p + 8 <= p1; p += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += part[(int64_t)(p + j) * n + e];
    }
    for (int j = 0; p < p1; ++p, ++j) r[j] += part[(int64_t)p * n + e];
    acc = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  }
  accw[q][lane] = acc;
  __syncthreads();
  if (q == 0 && e < n) {
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += accw[w][lane];
    out[e] = t;
  }
}

constexpr int kLnBwdBlocks = 1024;   // 4 per CU: 16 waves/CU keep x and dy loads in flight

template <int DT>
static int ln_chunks(int D) {
  using T = typename Elem<DT>::T;
  constexpr int VEC = 16 / sizeof(T);
  if (D % (64 * VEC)) return 0;
  const int ch = D / (64 * VEC);
  return (ch == 1 || ch == 2 || ch == 4 || ch == 8) ? ch : 0;
}

template <int DT>
static void launch_ln_fwd(const LnArgs& a, int ch, hipStream_t st) {
  dim3 grid((unsigned)((a.rows + 3) / 4));
  switch (ch) {
    case 1: hipLaunchKernelGGL((ln_fwd_kernel<DT, 1>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((ln_fwd_kernel<DT, 2>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((ln_fwd_kernel<DT, 4>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((ln_fwd_kernel<DT, 8>), grid, dim3(256), 0, st, a); break;
  }
}

template <int DT>
static void launch_ln_bwd(const LnArgs& a, int ch, int P, hipStream_t st) {
  const size_t sh = 8 * (size_t)a.D * sizeof(float);
  switch (ch) {
    case 1: hipLaunchKernelGGL((ln_bwd_kernel<DT, 1>), dim3(P), dim3(256), sh, st, a); break;
    case 2: hipLaunchKernelGGL((ln_bwd_kernel<DT, 2>), dim3(P), dim3(256), sh, st, a); break;
    case 4: hipLaunchKernelGGL((ln_bwd_kernel<DT, 4>), dim3(P), dim3(256), sh, st, a); break;
    default: hipLaunchKernelGGL((ln_bwd_kernel<DT, 8>), dim3(P), dim3(256), sh, st, a); break;
  }
}

static int ln_ch(int dtype, int D) {
  switch (dtype) {
    case SC_F32: return ln_chunks<SC_F32>(D);
    case SC_BF16: return ln_chunks<SC_BF16>(D);
    default: return ln_chunks<SC_F16>(D);
  }
}

}  // namespace sc

using namespace sc;

extern "C" int sc_layernorm_supported(int dtype, int D) {
  if (dtype != SC_F32 && dtype != SC_BF16 && dtype != SC_F16) return 0;
  return ln_ch(dtype, D) != 0;
}

extern "C" int64_t sc_layernorm_bwd_workspace_numel(int64_t rows, int D) {
  const int64_t P = rows < kLnBwdBlocks * 4 ? (rows + 3) / 4 : kLnBwdBlocks;
  return (P > 0 ? P : 1) * 2 * (int64_t)D;
}

extern "C" int sc_layernorm_fwd(const void* x, int dtype, const float* gamma, const float* beta,
                                void* y, float* mean, float* rstd, int64_t rows, int D, float eps,
                                void* stream) {
  clear_error();
  SC_REQUIRE(rows >= 0 && D > 0, "sc_layernorm_fwd: bad shape rows=%lld D=%d", (long long)rows, D);
  const int ch = ln_ch(dtype, D);
  SC_REQUIRE(ch, "sc_layernorm_fwd: unsupported (dtype %d, D %d): D must be 64*16B/elem * {1,2,4,8}",
             dtype, D);
  if (rows == 0) return 0;
  SC_REQUIRE(x && gamma && beta && y && mean && rstd, "sc_layernorm_fwd: null pointer");
  SC_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0,
             "sc_layernorm_fwd: x and y must be 16-byte aligned");
  LnArgs a{x, nullptr, gamma, beta, y, mean, rstd, nullptr, rows, D, eps};
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case SC_F32: launch_ln_fwd<SC_F32>(a, ch, st); break;
    case SC_BF16: launch_ln_fwd<SC_BF16>(a, ch, st); break;
    default: launch_ln_fwd<SC_F16>(a, ch, st); break;
  }
  return launch_status("sc_layernorm_fwd");
}

extern "C" int sc_layernorm_bwd(const void* x, const void* dy, int dtype, const float* gamma,
                                const float* mean, const float* rstd, void* dx, float* dgamma,
                                float* workspace, int64_t rows, int D, void* stream) {
  clear_error();
  SC_REQUIRE(rows >= 0 && D > 0, "sc_layernorm_bwd: bad shape");
  const int ch = ln_ch(dtype, D);
  SC_REQUIRE(ch, "sc_layernorm_bwd: unsupported (dtype %d, D %d)", dtype, D);
  hipStream_t st = (hipStream_t)stream;
  if (rows == 0) {
    zero_async(dgamma, 2 * sizeof(float) * D, st);
    return launch_status("sc_layernorm_bwd");
  }
  SC_REQUIRE(x && dy && gamma && mean && rstd && dx && dgamma && workspace,
             "sc_layernorm_bwd: null pointer");
  SC_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0,
             "sc_layernorm_bwd: x, dy, dx must be 16-byte aligned");
  const int P = (int)(sc_layernorm_bwd_workspace_numel(rows, D) / (2 * D));
  LnArgs a{x, dy, gamma, nullptr, dx, (float*)mean, (float*)rstd, workspace, rows, D, 0.0f};
  switch (dtype) {
    case SC_F32: launch_ln_bwd<SC_F32>(a, ch, P, st); break;
    case SC_BF16: launch_ln_bwd<SC_BF16>(a, ch, P, st); break;
    default: launch_ln_bwd<SC_F16>(a, ch, P, st); break;
  }
  hipLaunchKernelGGL(ln_part_sum_kernel, dim3((2 * D + 63) / 64), dim3(1024), 0, st,
                     (const float*)workspace, P, 2 * D, dgamma);
  return launch_status("sc_layernorm_bwd");
}
