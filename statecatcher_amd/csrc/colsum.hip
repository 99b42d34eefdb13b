// Deterministic column sums of a row-major matrix into fp32: out[n] = sum_m x[m][n].
//
// The training step's reductions over rows — the bias gradient of the output projection
// (dy.sum(0) over B*T = 48,000 rows of V = 1,024 bf16 logit gradients, lucyrnn_triton.py:8-25's
// Linear), the split-K partial sums of the weight gradients, and the per-row gate-bias partials —
// were torch reduce kernels at 2-3 TB/s.  Two passes, fixed summation order:
//   colsum_part_kernel   workgroup (column slab of 64 lanes x 8 columns, row chunk): each lane
//                        accumulates 8 columns over its wave's rows with 16-byte loads (fp32:
//                        2 x 16 B), then the 4 waves are summed in a fixed order -> part[chunk][n]
//   colsum_final_kernel  out[n] = sum over chunks, in chunk order (8 independent accumulators);
//                        skipped when one chunk covers all rows (the first pass writes out)
// An optional block transpose of the output index serves the step-blocked gate layout
// (ops.step_blocked_rows): input column (a, b, c) of an (A, Bf, C) factorisation lands at
// output (b, a, c).
#include <algorithm>

#include "sc_common.h"

namespace sc {

struct ColsumArgs {
  const void* x;
  int64_t M, N, ld;
  float* part;      // [chunks][N]
  int chunks;
  float* out;
  int64_t A, Bf, C; // output block transpose (A = 1: identity)
};

__device__ __forceinline__ int64_t out_index(const ColsumArgs& a, int64_t n) {
  if (a.A == 1) return n;
  const int64_t ci = n % a.C, bi = (n / a.C) % a.Bf, ai = n / (a.C * a.Bf);   // (a, b, c)
  return (bi * a.A + ai) * a.C + ci;                                           // -> (b, a, c)
}

template <int DT>
__global__ void __launch_bounds__(256) colsum_part_kernel(ColsumArgs a) {
  using T = typename Elem<DT>::T;
  __shared__ float red[4][64 * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n0 = ((int64_t)blockIdx.x * 64 + lane) * 8;
  const int chunk = blockIdx.y;
  const int64_t rows = (a.M + a.chunks - 1) / a.chunks;
  const int64_t r0 = chunk * rows, r1 = std::min<int64_t>(a.M, r0 + rows);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n0 + 8 <= a.N) {
    auto ld8 = [&](int64_t r, float (&f)[8]) {
      const T* p = (const T*)a.x + r * a.ld + n0;
      if constexpr (Vec16<DT>::N == 8) {
        Vec16<DT>::ld(p, f);
      } else {
        Vec16<DT>::ld(p, *(float(*)[4])&f[0]);
        Vec16<DT>::ld(p + 4, *(float(*)[4])&f[4]);
      }
    };
    int64_t r = r0 + w;
    for (; r + 12 < r1; r += 16) {   // four rows' loads in flight per lane
      float f0[8], f1[8], f2[8], f3[8];
      ld8(r, f0);
      ld8(r + 4, f1);
      ld8(r + 8, f2);
      ld8(r + 12, f3);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ((f0[k] + f1[k]) + f2[k]) + f3[k];
    }
    for (; r < r1; r += 4) {
      float f[8];
      ld8(r, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
    }
  } else if (n0 < a.N) {   // ragged last slab
    for (int64_t r = r0 + w; r < r1; r += 4) {
      const T* p = (const T*)a.x + r * a.ld + n0;
      for (int k = 0; k < 8 && n0 + k < a.N; ++k) acc[k] += Elem<DT>::ld(p[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[w][lane * 8 + k] = acc[k];
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 8; i += 256) {
    const int64_t n = (int64_t)blockIdx.x * 512 + i;
    if (n >= a.N) continue;
    const float v = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    if (a.chunks > 1) a.part[(int64_t)chunk * a.N + n] = v;
    else a.out[out_index(a, n)] = v;   // one chunk: no second pass
  }
}

__global__ void __launch_bounds__(256) colsum_final_kernel(ColsumArgs a) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= a.N) return;
  float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int c = 0;
  for (; c + 8 <= a.chunks; c += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a.part[(int64_t)(c + j) * a.N + n];
  }
  for (int j = 0; c < a.chunks; ++c, ++j) r[j] += a.part[(int64_t)c * a.N + n];
  a.out[out_index(a, n)] = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

// zero_async: see sc_common.h.  Words when dst and bytes allow it, else bytes.
__global__ void __launch_bounds__(256) zero_words_kernel(uint32_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = 0u;
}
__global__ void __launch_bounds__(256) zero_bytes_kernel(unsigned char* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = 0;
}

void zero_async(void* dst, size_t bytes, hipStream_t st) {
  if (!dst || bytes == 0) return;
  const bool words = ((uintptr_t)dst % 4) == 0 && bytes % 4 == 0;
  const int64_t n = words ? (int64_t)(bytes / 4) : (int64_t)bytes;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
  if (words)
    hipLaunchKernelGGL(zero_words_kernel, dim3(g), dim3(256), 0, st, (uint32_t*)dst, n);
  else
    hipLaunchKernelGGL(zero_bytes_kernel, dim3(g), dim3(256), 0, st, (unsigned char*)dst, n);
}

static int colsum_chunks(int64_t M, int64_t N) {
  // enough workgroups to fill the chip (slabs x chunks >= ~512), each chunk >= 128 rows, and
  // at most 128 chunks so the second pass stays short
  const int64_t slabs = (N + 511) / 512;
  int64_t c = (512 + slabs - 1) / slabs;
  c = std::min<int64_t>(c, std::max<int64_t>(1, M / 128));
  return (int)std::max<int64_t>(1, std::min<int64_t>(c, 128));
}

}  // namespace sc

using namespace sc;

extern "C" size_t sc_colsum_workspace_bytes(int64_t M, int64_t N) {
  const int c = colsum_chunks(M, N);
  return c > 1 ? (size_t)c * (size_t)N * sizeof(float) : 16;
}

extern "C" int sc_colsum(const void* x, int dtype, int64_t M, int64_t N, int64_t ld,
                         int64_t perm_a, int64_t perm_b, float* out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16,
             "sc_colsum: unsupported dtype %d", dtype);
  SC_REQUIRE(M >= 0 && N >= 0 && ld >= N, "sc_colsum: bad shape");
  SC_REQUIRE(perm_a >= 1 && perm_b >= 1 && N % (perm_a * perm_b) == 0,
             "sc_colsum: block transpose %lld x %lld does not divide N = %lld", (long long)perm_a,
             (long long)perm_b, (long long)N);
  if (N == 0) return 0;
  SC_REQUIRE(out, "sc_colsum: null output");
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {
    zero_async(out, N * sizeof(float), st);
    return launch_status("sc_colsum");
  }
  SC_REQUIRE(x, "sc_colsum: null pointer");
  const int elem = dtype == SC_F32 ? 4 : 2;
  SC_REQUIRE(((uintptr_t)x % 16) == 0 && (ld * elem) % 16 == 0,
             "sc_colsum: x and its row stride must be 16-byte aligned");
  const int chunks = colsum_chunks(M, N);
  SC_REQUIRE(chunks == 1 || (workspace && workspace_bytes >= (size_t)chunks * N * sizeof(float)),
             "sc_colsum: workspace too small");
  ColsumArgs a{x, M, N, ld, (float*)workspace, chunks, out, perm_a, perm_b, N / (perm_a * perm_b)};
  const dim3 g1((unsigned)((N + 511) / 512), (unsigned)chunks);
  switch (dtype) {
    case SC_F32: hipLaunchKernelGGL(colsum_part_kernel<SC_F32>, g1, dim3(256), 0, st, a); break;
    case SC_BF16: hipLaunchKernelGGL(colsum_part_kernel<SC_BF16>, g1, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(colsum_part_kernel<SC_F16>, g1, dim3(256), 0, st, a); break;
  }
  if (chunks > 1)
    hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, a);
  return launch_status("sc_colsum");
}
