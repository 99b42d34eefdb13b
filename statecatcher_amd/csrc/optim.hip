// Optimizer side of the training step on gfx950: the gradient-norm clip + Adam/AdamW update,
// and the per-step bf16 weight images the projections consume.
//
// Replaces (train.py:543-552, under the autocast of train.py:517-535):
//   torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)   -> adam_sumsq + the clip
//   optimizer.step()  (torch.optim.Adam / AdamW)                   -> adam_step_kernel
//   w.to(bf16) [+ row permutation, + w^T copy] per projection      -> images_kernel
// torch runs these as ~10 launches (foreach norm, its cleanup, stack, norm of norms, add, div,
// clamp, step-count increment, fused Adam) plus 2-3 cast/transpose copies per weight; here the
// optimizer is two launches and the weight images one launch for the whole model.
//
//   adam_sumsq_kernel  one workgroup per gradient chunk: fp32 sum of squares -> part[chunk]
//   adam_step_kernel   one workgroup per chunk: every workgroup sums part[] in the same fixed
//                      order (fp64), so all see the same clip coefficient with no atomics and no
//                      extra launch; then one 16-byte-vector pass p, g, m, v -> p, m, v
//   images_kernel      64 x 64 tiles: fp32 rows (step-blocked row permutation on the source
//                      index) -> bf16 rows with zero pad columns, and the transposed tile through
//                      LDS so the w^T image is written as whole 32-byte row pieces
#include "sc_common.h"

namespace sc {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxAdamT = 24;     // tensors per launch (kernel-argument table)
constexpr int kMaxParts = 2048;   // partial sums the step kernel re-reduces per workgroup
constexpr int64_t kStepChunk = 8192;

struct AdamTable {
  float* p[kMaxAdamT];
  const float* g[kMaxAdamT];
  float* m[kMaxAdamT];
  float* v[kMaxAdamT];
  int64_t n[kMaxAdamT];
  int32_t first[kMaxAdamT + 1];   // prefix of the tensors' chunk counts within this launch
  int32_t nt;
  int32_t part_base;              // first partial slot of this launch (sumsq)
  int64_t chunk;                  // elements per workgroup
};

// fp32 scalars as torch's kernels see them: each one a Python double (1 - beta1, lr / bc1, ...)
// computed in double and rounded once to float at the launch
struct StepScalars {
  const float* part;
  int64_t nparts;
  float max_norm, b1c, b2, b2c, eps, wd, dmul, step_size, bc2_sqrt;
  int decoupled;
  float* norm_out;
};

// tensor of workgroup `wg` (wave-uniform: kernel arguments and blockIdx only)
__device__ __forceinline__ int table_slot(const AdamTable& t, int wg) {
  int i = 0;
  while (i + 1 < t.nt && wg >= t.first[i + 1]) ++i;
  return i;
}

__device__ __forceinline__ float block_sum(float x, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = x;
  __syncthreads();
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < kThreads / 64; ++k) s += red[k];
  return s;
}

__global__ void __launch_bounds__(kThreads) adam_sumsq_kernel(AdamTable t, float* part) {
  __shared__ float red[kThreads / 64];
  const int wg = blockIdx.x;
  const int i = table_slot(t, wg);
  const int64_t c0 = (int64_t)(wg - t.first[i]) * t.chunk;
  const int64_t c1 = min(c0 + t.chunk, t.n[i]);
  const float* g = t.g[i];
  float acc0 = 0.0f, acc1 = 0.0f;
  int64_t k = c0;
  if (((uintptr_t)g & 15) == 0) {   // chunk starts are multiples of 4 elements
    const int64_t v1 = c0 + ((c1 - c0) & ~(int64_t)3);
    for (int64_t e = c0 + 4 * threadIdx.x; e < v1; e += 4 * kThreads) {
      const float4 x = *(const float4*)(g + e);
      acc0 = fmaf(x.x, x.x, acc0);
      acc1 = fmaf(x.y, x.y, acc1);
      acc0 = fmaf(x.z, x.z, acc0);
      acc1 = fmaf(x.w, x.w, acc1);
    }
    k = v1;
  }
  for (int64_t e = k + threadIdx.x; e < c1; e += kThreads) acc0 = fmaf(g[e], g[e], acc0);
  const float s = block_sum(acc0 + acc1, red);
  if (threadIdx.x == 0) part[t.part_base + wg] = s;
}

// clip coefficient of clip_grad_norm_: max_norm / (total + 1e-6), clamped to at most 1 (NaN
// propagates, as torch.clamp does)
__device__ float clip_coef(const StepScalars& s, double* red) {
  double a = 0.0;
  for (int64_t k = threadIdx.x; k < s.nparts; k += kThreads) a += (double)s.part[k];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {   // fixed tree: identical in every workgroup
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float total = (float)sqrt(red[0]);
  if (s.norm_out && blockIdx.x == 0 && threadIdx.x == 0) s.norm_out[0] = total;
  const float c = s.max_norm / (total + 1e-6f);
  return (c < 1.0f || c != c) ? c : 1.0f;
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float coef,
                                          const StepScalars& s) {
  g = g * coef;
  if (s.wd != 0.0f) {
    if (s.decoupled) p = p * s.dmul;                  // AdamW: param.mul_(1 - lr * wd)
    else g = g + s.wd * p;                            // Adam: grad.add(param, alpha=wd)
  }
  m = m + s.b1c * (g - m);                            // exp_avg.lerp_(grad, 1 - beta1)
  v = v * s.b2 + s.b2c * g * g;                       // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
  p = p - s.step_size * (m / denom);                  // param.addcdiv_(exp_avg, denom, -step_size)
}

__global__ void __launch_bounds__(kThreads) adam_step_kernel(AdamTable t, StepScalars s) {
  __shared__ double red[kThreads];
  const float coef = s.part ? clip_coef(s, red) : 1.0f;
  const int wg = blockIdx.x;
  const int i = table_slot(t, wg);
  const int64_t c0 = (int64_t)(wg - t.first[i]) * t.chunk;
  const int64_t c1 = min(c0 + t.chunk, t.n[i]);
  float* p = t.p[i];
  const float* g = t.g[i];
  float* m = t.m[i];
  float* v = t.v[i];
  int64_t k = c0;
  if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) {
    const int64_t v1 = c0 + ((c1 - c0) & ~(int64_t)3);
    for (int64_t e = c0 + 4 * threadIdx.x; e < v1; e += 4 * kThreads) {
      float4 pp = *(float4*)(p + e);
      const float4 gg = *(const float4*)(g + e);
      float4 mm = *(float4*)(m + e);
      float4 vv = *(float4*)(v + e);
      adam_elem(pp.x, gg.x, mm.x, vv.x, coef, s);
      adam_elem(pp.y, gg.y, mm.y, vv.y, coef, s);
      adam_elem(pp.z, gg.z, mm.z, vv.z, coef, s);
      adam_elem(pp.w, gg.w, mm.w, vv.w, coef, s);
      *(float4*)(p + e) = pp;
      *(float4*)(m + e) = mm;
      *(float4*)(v + e) = vv;
    }
    k = v1;
  }
  for (int64_t e = k + threadIdx.x; e < c1; e += kThreads) {
    float pp = p[e], mm = m[e], vv = v[e];
    adam_elem(pp, g[e], mm, vv, coef, s);
    p[e] = pp;
    m[e] = mm;
    v[e] = vv;
  }
}

// ------------------------------------------------------------------------ weight images ----
constexpr int kMaxJobs = 16;
constexpr int kTile = 64;

struct ImageTable {
  sc_image_job j[kMaxJobs];
  int32_t first[kMaxJobs + 1];   // prefix of the jobs' tile counts
  int32_t tiles_c[kMaxJobs];     // column tiles per job (over cols_pad)
  int32_t nj;
};

__device__ __forceinline__ uint16_t bf16_bits(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__global__ void __launch_bounds__(kThreads) images_kernel(ImageTable t) {
  __shared__ uint16_t tile[kTile][kTile + 2];
  const int wg = blockIdx.x;
  int i = 0;
  while (i + 1 < t.nj && wg >= t.first[i + 1]) ++i;
  const sc_image_job& j = t.j[i];
  const int local = wg - t.first[i];
  const int64_t r0 = (int64_t)(local / t.tiles_c[i]) * kTile;
  const int64_t c0 = (int64_t)(local % t.tiles_c[i]) * kTile;
  const int rr = threadIdx.x >> 2;          // tile row
  const int cs = (threadIdx.x & 3) * 16;    // 16 columns per thread
  const int64_t r = r0 + rr;
  uint16_t h[16];
  if (r < j.rows) {
    int64_t sr = r;
    if (j.block_d > 0) {   // dst row (block, gate, unit) <- src row gate * D + block * 64 + unit
      const int64_t blk = r / (7 * 64), gte = (r % (7 * 64)) / 64, u = r % 64;
      sr = gte * j.block_d + blk * 64 + u;
    }
    const float* src = j.src + sr * j.ld_src;
    const int64_t c = c0 + cs;
    // (folded LayerNorm: col_scale[c] src - row_shift[sr], unfused as sc_ln_fold_prep's rowsum)
    const float sh = j.row_shift ? j.row_shift[sr] : 0.0f;
    auto val = [&](float x, int64_t cc) {
      return j.col_scale ? mul_sub_rn(j.col_scale[cc], x, sh) : x - sh;
    };
    if (c + 16 <= j.cols && (((uintptr_t)(src + c)) & 15) == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *(const float4*)(src + c + 4 * q);
        h[4 * q] = bf16_bits(val(x.x, c + 4 * q));
        h[4 * q + 1] = bf16_bits(val(x.y, c + 4 * q + 1));
        h[4 * q + 2] = bf16_bits(val(x.z, c + 4 * q + 2));
        h[4 * q + 3] = bf16_bits(val(x.w, c + 4 * q + 3));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        h[e] = (c + e < j.cols) ? bf16_bits(val(src[c + e], c + e)) : (uint16_t)0;
    }
    uint16_t* dst = (uint16_t*)j.dst + r * j.cols_pad;
    if (c + 16 <= j.cols_pad && (((uintptr_t)(dst + c)) & 15) == 0) {
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        u4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          w[e] = (uint32_t)h[8 * q + 2 * e] | ((uint32_t)h[8 * q + 2 * e + 1] << 16);
        *(u4*)(dst + c + 8 * q) = w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (c + e < j.cols_pad) dst[c + e] = h[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) h[e] = 0;
  }
  if (!j.dst_t || c0 >= j.cols) return;   // uniform per workgroup
#pragma unroll
  for (int e = 0; e < 16; ++e) tile[rr][cs + e] = h[e];
  __syncthreads();
  // transposed: dst_t[c][r0 + 16 q .. + 15] for tile column cc = threadIdx.x >> 2
  const int cc = threadIdx.x >> 2;
  const int rs = (threadIdx.x & 3) * 16;
  const int64_t c = c0 + cc;
  if (c >= j.cols) return;
  uint16_t* dt = (uint16_t*)j.dst_t + c * j.rows;
  const int64_t rb = r0 + rs;
  if (rb + 16 <= j.rows && (((uintptr_t)(dt + rb)) & 15) == 0) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      u4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (uint32_t)tile[rs + 8 * q + 2 * e][cc] |
               ((uint32_t)tile[rs + 8 * q + 2 * e + 1][cc] << 16);
      *(u4*)(dt + rb + 8 * q) = w;
    }
  } else {
    for (int e = 0; e < 16; ++e)
      if (rb + e < j.rows) dt[rb + e] = tile[rs + e][cc];
  }
}

// elements per sumsq workgroup so that the partials fit kMaxParts
int64_t sumsq_chunk(const sc_adam_tensor* t, int nt) {
  int64_t chunk = kStepChunk;
  for (;;) {
    int64_t parts = 0;
    for (int i = 0; i < nt; ++i) parts += (t[i].n + chunk - 1) / chunk;
    if (parts <= kMaxParts) return chunk;
    chunk *= 2;
  }
}

int check_tensors(const sc_adam_tensor* t, int nt, bool need_pmv, const char* what) {
  SC_REQUIRE(nt >= 0 && (nt == 0 || t), "%s: bad tensor table", what);
  for (int i = 0; i < nt; ++i) {
    SC_REQUIRE(t[i].n >= 0, "%s: tensor %d has negative length", what, i);
    SC_REQUIRE(t[i].n == 0 || t[i].g, "%s: tensor %d has a null gradient", what, i);
    SC_REQUIRE(!need_pmv || t[i].n == 0 || (t[i].p && t[i].m && t[i].v),
               "%s: tensor %d has a null param / moment", what, i);
    SC_REQUIRE(t[i].n < ((int64_t)1 << 40), "%s: tensor %d too long", what, i);
  }
  return 0;
}

// Fill launch tables of at most kMaxAdamT tensors (empty tensors skipped) and call f(table,
// grid) for each; returns the total chunk count.
template <typename F>
int64_t for_tables(const sc_adam_tensor* t, int nt, int64_t chunk, F&& f) {
  AdamTable tb{};
  tb.chunk = chunk;
  int64_t done = 0;
  int32_t chunks = 0;
  auto flush = [&]() {
    if (tb.nt == 0) return;
    tb.first[tb.nt] = chunks;
    f(tb, chunks);
    done += chunks;
    tb.part_base = (int32_t)done;
    tb.nt = 0;
    chunks = 0;
  };
  for (int i = 0; i < nt; ++i) {
    if (t[i].n == 0) continue;
    const int64_t c = (t[i].n + chunk - 1) / chunk;
    if (tb.nt == kMaxAdamT || chunks + c > (int64_t)1 << 30) flush();
    tb.p[tb.nt] = t[i].p;
    tb.g[tb.nt] = t[i].g;
    tb.m[tb.nt] = t[i].m;
    tb.v[tb.nt] = t[i].v;
    tb.n[tb.nt] = t[i].n;
    tb.first[tb.nt] = chunks;
    chunks += (int32_t)c;
    ++tb.nt;
  }
  flush();
  return done;
}

}  // namespace
}  // namespace sc

using namespace sc;

extern "C" int64_t sc_adam_parts(const sc_adam_tensor* t, int nt) {
  if (nt <= 0 || !t) return 0;
  const int64_t chunk = sumsq_chunk(t, nt);
  int64_t parts = 0;
  for (int i = 0; i < nt; ++i) parts += t[i].n > 0 ? (t[i].n + chunk - 1) / chunk : 0;
  return parts;
}

extern "C" int sc_adam_sumsq(const sc_adam_tensor* t, int nt, float* part, void* stream) {
  clear_error();
  if (int rc = check_tensors(t, nt, false, "sc_adam_sumsq")) return rc;
  if (sc_adam_parts(t, nt) == 0) return 0;
  SC_REQUIRE(part, "sc_adam_sumsq: null partial buffer");
  const int64_t chunk = sumsq_chunk(t, nt);
  hipStream_t st = (hipStream_t)stream;
  for_tables(t, nt, chunk, [&](const AdamTable& tb, int32_t grid) {
    hipLaunchKernelGGL(adam_sumsq_kernel, dim3(grid), dim3(kThreads), 0, st, tb, part);
  });
  return launch_status("sc_adam_sumsq");
}

extern "C" int sc_adam_step(const sc_adam_tensor* t, int nt, const float* part, int64_t nparts,
                            double max_norm, double lr, double beta1, double beta2, double eps,
                            double weight_decay, int decoupled, double step_size, double bc2_sqrt,
                            float* norm_out, void* stream) {
  clear_error();
  if (int rc = check_tensors(t, nt, true, "sc_adam_step")) return rc;
  SC_REQUIRE(!part || (nparts > 0 && nparts <= kMaxParts),
             "sc_adam_step: %lld partial sums (1..%d expected with a partial buffer)",
             (long long)nparts, kMaxParts);
  SC_REQUIRE(bc2_sqrt > 0.0f, "sc_adam_step: bias correction must be positive");
  StepScalars s{part, part ? nparts : 0, (float)max_norm, (float)(1.0 - beta1), (float)beta2,
                (float)(1.0 - beta2), (float)eps, (float)weight_decay,
                (float)(1.0 - lr * weight_decay), (float)step_size, (float)bc2_sqrt, decoupled,
                norm_out};
  hipStream_t st = (hipStream_t)stream;
  bool first = true;
  for_tables(t, nt, kStepChunk, [&](const AdamTable& tb, int32_t grid) {
    StepScalars sl = s;
    if (!first) sl.norm_out = nullptr;
    first = false;
    hipLaunchKernelGGL(adam_step_kernel, dim3(grid), dim3(kThreads), 0, st, tb, sl);
  });
  return launch_status("sc_adam_step");
}

extern "C" int sc_weight_images(const sc_image_job* jobs, int njobs, void* stream) {
  clear_error();
  SC_REQUIRE(njobs >= 0 && njobs <= kMaxJobs && (njobs == 0 || jobs),
             "sc_weight_images: 0..%d jobs per call", kMaxJobs);
  ImageTable tb{};
  int64_t tiles = 0;
  for (int i = 0; i < njobs; ++i) {
    const sc_image_job& j = jobs[i];
    SC_REQUIRE(j.rows >= 0 && j.cols >= 0 && j.cols_pad >= j.cols && j.ld_src >= j.cols,
               "sc_weight_images: job %d has a bad shape", i);
    SC_REQUIRE(j.rows == 0 || j.cols_pad == 0 || (j.src && j.dst),
               "sc_weight_images: job %d has a null pointer", i);
    SC_REQUIRE(j.block_d == 0 || (j.block_d % 64 == 0 && j.rows == 7 * j.block_d),
               "sc_weight_images: job %d: step-blocked rows need rows = 7 D, D %% 64 == 0", i);
    tb.j[tb.nj] = j;
    tb.first[tb.nj] = (int32_t)tiles;
    tb.tiles_c[tb.nj] = (int32_t)((j.cols_pad + kTile - 1) / kTile);
    tiles += ((j.rows + kTile - 1) / kTile) * tb.tiles_c[tb.nj];
    SC_REQUIRE(tiles < ((int64_t)1 << 30), "sc_weight_images: too many tiles");
    ++tb.nj;
  }
  if (tiles == 0) return 0;
  tb.first[tb.nj] = (int32_t)tiles;
  hipLaunchKernelGGL(images_kernel, dim3((unsigned)tiles), dim3(kThreads), 0, (hipStream_t)stream,
                     tb);
  return launch_status("sc_weight_images");
}
