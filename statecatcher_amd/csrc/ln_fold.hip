// The inter-layer LayerNorm of the LucyRNN stack (lucyrnn_triton.py:96-97, :136-137; nn.LayerNorm
// eps 1e-5, biased variance) folded into the next layer's gate projection, for gfx950.
//
// LN(h) W^T + b = rstd (h W''^T - mean r) + b' with
//   W'' = (W diag gamma)(I - 1 1^T / D)     rows centred, so h W''^T = (h - mean) (W diag gamma)^T
//   b'  = b + W beta
//   r   = row sums of W'' as rounded to bf16 (0 in exact arithmetic; the bf16 image's residual,
//         taken back out on load so the centring stays exact to the GEMM's own rounding)
// The projection GEMM then reads the previous layer's RAW output h, and the LayerNorm costs no
// pass of its own: the previous scan writes per-(row, 64-unit block) (mean, M2) records of its
// output, the next scan combines them and applies rstd / mean where it already added the bias
// (lucy_scan.hip, sc_lucy_scan_fwd_ln / _bwd_ln).  The kernels here are the pieces around it:
//   ln_fold_prep_kernel   per weight row: mean_k gamma_k W_nk (the centring shift), b', r
//   ln_fold_bwd_kernel    dL/dh from dL/du W'' (the input-gradient GEMM's output), which already
//                         carries rstd: dh = g - mean(g) - xhat mean(xhat g), xhat = (h - mean) rstd
//   ln_fold_wgrad_kernel  dL/dW, dL/dgamma, dL/dbeta from M = dL/dW'' and dL/db':
//                         dW = gamma (M - rowmean M) + db' beta^T, dgamma = sum_n W (M - rowmean M),
//                         dbeta = sum_n W db'  (fixed-order partial rows + ln_fold_sum_kernel)
#include "sc_common.h"

namespace sc {

// ------------------------------------------------------------------------ prep --------------
struct FoldPrepJob {
  const float* w;       // [rows][ld] fp32
  const float* gamma;   // [D]
  const float* beta;    // [D]
  const float* bias;    // [rows] or NULL
  float* shift;         // [rows] out: mean_k gamma_k W_nk
  float* bias_out;      // [rows] out: b + W beta
  float* rowsum;        // [rows] out: sum_k bf16(gamma_k W_nk - shift_n)
  int64_t ld;
  int rows, D;
};
constexpr int kMaxFoldJobs = 16;
struct FoldPrepTable {
  FoldPrepJob j[kMaxFoldJobs];
  int32_t first[kMaxFoldJobs + 1];   // prefix of the jobs' workgroups (4 rows each)
  int32_t nj;
};

// gamma_k W_nk - shift_n rounded as the weight image rounds it (optim.hip images_kernel): both
// sides use this one expression, unfused (sc_common.h mul_sub_rn)
__device__ __forceinline__ float fold_elem(float g, float w, float m) { return mul_sub_rn(g, w, m); }

__global__ void __launch_bounds__(256) ln_fold_prep_kernel(FoldPrepTable t) {
  const int wg = blockIdx.x;
  int i = 0;
  while (i + 1 < t.nj && wg >= t.first[i + 1]) ++i;
  const FoldPrepJob& j = t.j[i];
  const int lane = threadIdx.x & 63;
  const int n = (wg - t.first[i]) * 4 + (threadIdx.x >> 6);
  if (n >= j.rows) return;
  const float* wr = j.w + (int64_t)n * j.ld;
  float gw = 0.0f, wb = 0.0f;
  // the row in registers (D <= 1024: up to 4 pieces of 4 per lane), 16-byte loads when aligned
  constexpr int kMaxP = 4;
  float4 wv[kMaxP], gv[kMaxP];
  const bool vec = (j.D % 256) == 0 && j.D <= 1024 && (j.ld % 4) == 0 &&
                   (((uintptr_t)wr | (uintptr_t)j.gamma | (uintptr_t)j.beta) & 15) == 0;
  if (vec) {
    const int np = j.D / 256;
#pragma unroll
    for (int c = 0; c < kMaxP; ++c) {
      if (c < np) {
        wv[c] = *(const float4*)(wr + 4 * (lane + 64 * c));
        gv[c] = *(const float4*)(j.gamma + 4 * (lane + 64 * c));
        const float4 be = *(const float4*)(j.beta + 4 * (lane + 64 * c));
        gw += mul_sub_rn(gv[c].x, wv[c].x, 0.0f) + mul_sub_rn(gv[c].y, wv[c].y, 0.0f) +
              mul_sub_rn(gv[c].z, wv[c].z, 0.0f) + mul_sub_rn(gv[c].w, wv[c].w, 0.0f);
        wb = fmaf(wv[c].x, be.x, fmaf(wv[c].y, be.y, fmaf(wv[c].z, be.z, fmaf(wv[c].w, be.w, wb))));
      }
    }
  } else {
    for (int k = lane; k < j.D; k += 64) {
      gw += mul_sub_rn(j.gamma[k], wr[k], 0.0f);
      wb = fmaf(wr[k], j.beta[k], wb);
    }
  }
  const float m = wave_sum_dpp(gw) / (float)j.D;
  wb = wave_sum_dpp(wb);
  float r = 0.0f;
  if (vec) {
    const int np = j.D / 256;
#pragma unroll
    for (int c = 0; c < kMaxP; ++c)
      if (c < np)
        r += ((float)(__bf16)fold_elem(gv[c].x, wv[c].x, m) + (float)(__bf16)fold_elem(gv[c].y, wv[c].y, m)) +
             ((float)(__bf16)fold_elem(gv[c].z, wv[c].z, m) + (float)(__bf16)fold_elem(gv[c].w, wv[c].w, m));
  } else {
    for (int k = lane; k < j.D; k += 64) r += (float)(__bf16)fold_elem(j.gamma[k], wr[k], m);
  }
  r = wave_sum_dpp(r);
  if (lane == 0) {
    j.shift[n] = m;
    j.bias_out[n] = (j.bias ? j.bias[n] : 0.0f) + wb;
    j.rowsum[n] = r;
  }
}

// ------------------------------------------------------------------------ input gradient ----
// One wave per row, D = 64 VPL elements: VPL per lane as 16-byte pieces (VPL = 8: bf16 D = 512)
template <int VPL>
__global__ void __launch_bounds__(256) ln_fold_bwd_kernel(const __bf16* __restrict__ g,
                                                          const __bf16* __restrict__ h,
                                                          const float2* __restrict__ stat,
                                                          __bf16* __restrict__ dh, int64_t rows) {
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  static_assert(VPL % 8 == 0, "16-byte pieces of bf16");
  constexpr int NP = VPL / 8;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = 64 * VPL;
  const b8* gr = (const b8*)(g + row * D);
  const b8* hr = (const b8*)(h + row * D);
  b8 gv[NP], hv[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    gv[p] = gr[p * 64 + lane];
    hv[p] = hr[p * 64 + lane];
  }
  const float2 st = stat[row];   // (rstd, mean)
  float s1 = 0.0f, s2 = 0.0f;
  float xh[VPL], gf[VPL];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gf[8 * p + e] = (float)gv[p][e];
      xh[8 * p + e] = ((float)hv[p][e] - st.y) * st.x;
      s1 += gf[8 * p + e];
      s2 = fmaf(xh[8 * p + e], gf[8 * p + e], s2);
    }
  const float m1 = wave_sum_dpp(s1) * (1.0f / D);
  const float m2 = wave_sum_dpp(s2) * (1.0f / D);
  b8* out = (b8*)(dh + row * D);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    b8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (__bf16)(gf[8 * p + e] - m1 - xh[8 * p + e] * m2);
    out[p * 64 + lane] = o;
  }
}

// ------------------------------------------------------------------------ weight gradient ---
// Workgroup = 4 waves over a contiguous run of kRowsPerWg rows; lane holds columns
// lane + 64 c (c < VPL).  Partial rows of dgamma / dbeta per workgroup in a fixed order.
constexpr int kRowsPerWg = 16;
template <int VPL>
__global__ void __launch_bounds__(256) ln_fold_wgrad_kernel(
    const float* __restrict__ M, const float* __restrict__ w, int64_t ld,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ dbias, int rows, float* __restrict__ dw, float* __restrict__ part) {
  constexpr int D = 64 * VPL;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ float red[4][2][D];
  float gk[VPL], bk[VPL], dg[VPL], db[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    gk[c] = gamma[lane + 64 * c];
    bk[c] = beta[lane + 64 * c];
    dg[c] = db[c] = 0.0f;
  }
  const int n0 = blockIdx.x * kRowsPerWg;
  for (int n = n0 + wv; n < min(rows, n0 + kRowsPerWg); n += 4) {
    const float* mr = M + (int64_t)n * D;
    const float* wr = w + (int64_t)n * ld;
    float mv[VPL], s = 0.0f;
#pragma unroll
    for (int c = 0; c < VPL; ++c) {
      mv[c] = mr[lane + 64 * c];
      s += mv[c];
    }
    const float mean = wave_sum_dpp(s) * (1.0f / D);
    const float dbn = dbias[n];
#pragma unroll
    for (int c = 0; c < VPL; ++c) {
      const float cm = mv[c] - mean;
      const float wn = wr[lane + 64 * c];
      dw[(int64_t)n * D + lane + 64 * c] = fmaf(dbn, bk[c], gk[c] * cm);
      dg[c] = fmaf(wn, cm, dg[c]);
      db[c] = fmaf(wn, dbn, db[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < VPL; ++c) {
    red[wv][0][lane + 64 * c] = dg[c];
    red[wv][1][lane + 64 * c] = db[c];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * D; k += 256) {
    const int q = k / D, col = k % D;
    part[((int64_t)blockIdx.x * 2 + q) * D + col] =
        ((red[0][q][col] + red[1][q][col]) + red[2][q][col]) + red[3][q][col];
  }
}

// dgamma_dbeta [2][D] = sum over the P partial rows in a fixed order: a workgroup per 64 columns,
// wave q sums rows q, q + 4, ... (loads unrolled by 4), then the 4 wave sums in order
__global__ void __launch_bounds__(256) ln_fold_sum_kernel(const float* __restrict__ part, int P,
                                                         int D2, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int kc = k < D2 ? k : D2 - 1;
  float s = 0.0f;
  int p = q;
  for (; p + 12 < P; p += 16) {
    const float a0 = part[(int64_t)p * D2 + kc], a1 = part[(int64_t)(p + 4) * D2 + kc];
    const float a2 = part[(int64_t)(p + 8) * D2 + kc], a3 = part[(int64_t)(p + 12) * D2 + kc];
    s = (((s + a0) + a1) + a2) + a3;
  }
  for (; p < P; p += 4) s += part[(int64_t)p * D2 + kc];
  red[q][lane] = s;
  __syncthreads();
  if (q == 0 && k < D2) out[k] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

}  // namespace sc

using namespace sc;

static bool fold_d_ok(int D) { return D == 512 || D == 1024; }

extern "C" int sc_ln_fold_prep(const sc_ln_fold_job* jobs, int njobs, void* stream) {
  clear_error();
  SC_REQUIRE(njobs >= 0 && njobs <= kMaxFoldJobs && (njobs == 0 || jobs),
             "sc_ln_fold_prep: 0..%d jobs per call", kMaxFoldJobs);
  FoldPrepTable tb{};
  int64_t wgs = 0;
  for (int i = 0; i < njobs; ++i) {
    const sc_ln_fold_job& j = jobs[i];
    SC_REQUIRE(j.rows >= 0 && j.D > 0 && j.ld >= j.D, "sc_ln_fold_prep: job %d has a bad shape", i);
    SC_REQUIRE(j.rows == 0 || (j.w && j.gamma && j.beta && j.shift && j.bias_out && j.rowsum),
               "sc_ln_fold_prep: job %d has a null pointer", i);
    tb.j[tb.nj] = FoldPrepJob{j.w, j.gamma, j.beta, j.bias, j.shift, j.bias_out, j.rowsum, j.ld,
                              (int)j.rows, (int)j.D};
    tb.first[tb.nj] = (int32_t)wgs;
    wgs += (j.rows + 3) / 4;
    ++tb.nj;
  }
  if (wgs == 0) return 0;
  tb.first[tb.nj] = (int32_t)wgs;
  hipLaunchKernelGGL(ln_fold_prep_kernel, dim3((unsigned)wgs), dim3(256), 0, (hipStream_t)stream, tb);
  return launch_status("sc_ln_fold_prep");
}

extern "C" int sc_ln_fold_bwd(const void* g, const void* h, int dtype, const float* stat, void* dh,
                              int64_t rows, int D, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_BF16, "sc_ln_fold_bwd: bf16 only (dtype %d)", dtype);
  SC_REQUIRE(fold_d_ok(D), "sc_ln_fold_bwd: D=%d must be 512 or 1024", D);
  SC_REQUIRE(rows >= 0, "sc_ln_fold_bwd: negative rows");
  if (rows == 0) return 0;
  SC_REQUIRE(g && h && stat && dh, "sc_ln_fold_bwd: null pointer");
  SC_REQUIRE(((uintptr_t)g | (uintptr_t)h | (uintptr_t)dh) % 16 == 0,
             "sc_ln_fold_bwd: rows must be 16-byte aligned");
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const __bf16 *gp = (const __bf16*)g, *hp = (const __bf16*)h;
  const float2* sp = (const float2*)stat;
  __bf16* op = (__bf16*)dh;
  if (D == 512) hipLaunchKernelGGL(ln_fold_bwd_kernel<8>, grid, dim3(256), 0, st, gp, hp, sp, op, rows);
  else hipLaunchKernelGGL(ln_fold_bwd_kernel<16>, grid, dim3(256), 0, st, gp, hp, sp, op, rows);
  return launch_status("sc_ln_fold_bwd");
}

extern "C" int64_t sc_ln_fold_wgrad_workspace_numel(int rows, int D) {
  if (rows <= 0 || D <= 0) return 1;
  return (int64_t)((rows + kRowsPerWg - 1) / kRowsPerWg) * 2 * D;
}

extern "C" int sc_ln_fold_wgrad(const float* M, const float* w, int64_t ld, const float* gamma,
                                const float* beta, const float* dbias, int rows, int D, float* dw,
                                float* dgamma_dbeta, float* workspace, void* stream) {
  clear_error();
  SC_REQUIRE(fold_d_ok(D), "sc_ln_fold_wgrad: D=%d must be 512 or 1024", D);
  SC_REQUIRE(rows > 0 && ld >= D, "sc_ln_fold_wgrad: bad shape rows=%d ld=%lld", rows, (long long)ld);
  SC_REQUIRE(M && w && gamma && beta && dbias && dw && dgamma_dbeta && workspace,
             "sc_ln_fold_wgrad: null pointer");
  const int P = (rows + kRowsPerWg - 1) / kRowsPerWg;
  hipStream_t st = (hipStream_t)stream;
  if (D == 512)
    hipLaunchKernelGGL(ln_fold_wgrad_kernel<8>, dim3(P), dim3(256), 0, st, M, w, ld, gamma, beta,
                       dbias, rows, dw, workspace);
  else
    hipLaunchKernelGGL(ln_fold_wgrad_kernel<16>, dim3(P), dim3(256), 0, st, M, w, ld, gamma, beta,
                       dbias, rows, dw, workspace);
  hipLaunchKernelGGL(ln_fold_sum_kernel, dim3((2 * D + 63) / 64), dim3(256), 0, st, workspace, P,
                     2 * D, dgamma_dbeta);
  return launch_status("sc_ln_fold_wgrad");
}
