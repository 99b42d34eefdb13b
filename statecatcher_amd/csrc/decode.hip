// Greedy CTC decoding on device, integer path bit-exact with the reference.
//
// Replaces decoder.py:3-30 `ctc_greedy_decoder` (torch.argmax over V, then a Python loop with
// one .item() host sync per frame, decoder.py:24).  Two kernels:
//   greedy_argmax_kernel   one wave per (b,t) row: first index of the maximum, a NaN counting
//                          as the maximum (torch.argmax semantics); lanes stride the row, then a
//                          64-lane (value, index) reduction that keeps the lower index on ties
//   greedy_collapse_kernel one workgroup per b: keep[t] = t < len && tok != blank &&
//                          tok != tok[t-1]; workgroup prefix sum of keep; compacted write.
// and, for streaming (one frame per call, statecatcher_amd/streaming.py):
//   greedy_step_kernel     one wave per stream: the same argmax, then the collapse against the
//                          stream's previous frame (prev[b], -1 at stream start as decoder.py's
//                          prev_token = None); emits the token or -1.  Masked frames (mask 0,
//                          past the stream's length) emit -1 and leave prev unchanged.
#include "sc_common.h"

namespace sc {

struct GreedyArgs {
  const void* x;
  int B, T, V, blank;
  int64_t sb, st;
  const int64_t* lengths;
  int32_t* tokens;
  int32_t* counts;
};

// a beats b?  (NaN beats everything; ties -> lower index)
__device__ __forceinline__ bool beats(float va, int ia, float vb, int ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return na && (!nb || ia < ib);
  if (va != vb) return va > vb;
  return ia < ib;
}

// argmax of one row by one wave (first maximal index, NaN maximal); the result in every lane.
// Aligned rows go by 16-byte pieces, kGu pieces per lane in flight at once (a row of V = 1024 is
// one memory round trip, not one per 64 elements); `beats` orders ties by index, so the order in
// which a lane visits its elements does not change the result.
template <int DT>
__device__ __forceinline__ int wave_argmax(const typename Elem<DT>::T* p, int V, int lane) {
  using E = Elem<DT>;
  float bv = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  constexpr int N = Vec16<DT>::N, kGu = 4;
  if (V % N == 0 && ((uintptr_t)p & 15) == 0) {
    const int nc = V / N;
    for (int c0 = lane; c0 < nc; c0 += 64 * kGu) {
      float xv[kGu][N];
#pragma unroll
      for (int u = 0; u < kGu; ++u) Vec16<DT>::ld(p + N * min(c0 + 64 * u, nc - 1), xv[u]);
#pragma unroll
      for (int u = 0; u < kGu; ++u) {
        if (c0 + 64 * u >= nc) break;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const int v = N * (c0 + 64 * u) + k;
          if (bi == 0x7fffffff || beats(xv[u][k], v, bv, bi)) {
            bv = xv[u][k];
            bi = v;
          }
        }
      }
    }
  } else {
    for (int v = lane; v < V; v += 64) {
      const float xv = E::ld(p[v]);
      if (bi == 0x7fffffff || beats(xv, v, bv, bi)) {
        bv = xv;
        bi = v;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (oi != 0x7fffffff && (bi == 0x7fffffff || beats(ov, oi, bv, bi))) {
      bv = ov;
      bi = oi;
    }
  }
  return bi;
}

template <int DT>
__global__ void __launch_bounds__(256) greedy_argmax_kernel(GreedyArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)a.B * a.T) return;
  const int b = (int)(row / a.T), t = (int)(row % a.T);
  const int tok = wave_argmax<DT>(
      (const typename Elem<DT>::T*)a.x + (int64_t)b * a.sb + (int64_t)t * a.st, a.V, lane);
  if (lane == 0) a.tokens[row] = tok;
}

struct GreedyStepArgs {
  const void* x;
  int B, V, blank;
  int64_t sb;
  const float* mask;
  int32_t* prev;
  int32_t* emit;
  int64_t emit_stride;
};

template <int DT>
__global__ void __launch_bounds__(256) greedy_step_kernel(GreedyStepArgs a) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.B) return;
  const int tok = wave_argmax<DT>((const typename Elem<DT>::T*)a.x + (int64_t)b * a.sb, a.V, lane);
  if (lane == 0) {
    const bool live = !a.mask || a.mask[b] != 0.0f;
    const int pv = a.prev[b];
    a.emit[(int64_t)b * a.emit_stride] = (live && tok != a.blank && tok != pv) ? tok : -1;
    if (live) a.prev[b] = tok;
  }
}

// F frames of one stream per wave, in frame order (prev carried in a register of lane 0)
struct GreedyFramesArgs {
  const void* x;
  int F, B, V, blank;
  int64_t sf, sb;
  const float* mask;
  int64_t mf;
  int32_t* prev;
  int32_t* emit;
  int64_t ef, eb;
};

template <int DT>
__global__ void __launch_bounds__(256) greedy_frames_kernel(GreedyFramesArgs a) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.B) return;
  int pv = a.prev[b];
  for (int f = 0; f < a.F; ++f) {
    const int tok = wave_argmax<DT>(
        (const typename Elem<DT>::T*)a.x + (int64_t)f * a.sf + (int64_t)b * a.sb, a.V, lane);
    if (lane == 0) {
      const bool live = !a.mask || a.mask[(int64_t)f * a.mf + b] != 0.0f;
      a.emit[(int64_t)f * a.ef + (int64_t)b * a.eb] = (live && tok != a.blank && tok != pv) ? tok : -1;
      if (live) pv = tok;
    }
  }
  if (lane == 0) a.prev[b] = pv;
}

__global__ void __launch_bounds__(1024) greedy_collapse_kernel(GreedyArgs a) {
  extern __shared__ __attribute__((aligned(16))) int sh[];   // T predictions + 16 wave sums
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int nthr = blockDim.x;
  int32_t* row = a.tokens + (int64_t)b * a.T;
  int len = (int)min<int64_t>(max<int64_t>(a.lengths[b], 0), a.T);
  for (int t = tid; t < a.T; t += nthr) sh[t] = row[t];
  __syncthreads();
  // each thread owns a contiguous span of steps
  const int per = (a.T + nthr - 1) / nthr;
  const int t0 = tid * per, t1 = min(t0 + per, len);
  int cnt = 0;
  for (int t = t0; t < t1; ++t) {
    const int tok = sh[t];
    cnt += (tok != a.blank && (t == 0 || tok != sh[t - 1])) ? 1 : 0;
  }
  // exclusive scan of cnt over the workgroup (wave scan + wave totals)
  const int lane = tid & 63, wv = tid >> 6;
  int inc = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  int* wsum = sh + a.T;
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int base = 0;
  for (int q = 0; q < wv; ++q) base += wsum[q];
  int pos = base + inc - cnt;
  for (int t = t0; t < t1; ++t) {
    const int tok = sh[t];
    if (tok != a.blank && (t == 0 || tok != sh[t - 1])) row[pos++] = tok;
  }
  if (tid == nthr - 1) a.counts[b] = base + inc;
}

template <int DT>
static void launch(const GreedyArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.T;
  hipLaunchKernelGGL((greedy_argmax_kernel<DT>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a);
  const int nthr = 1024;
  hipLaunchKernelGGL(greedy_collapse_kernel, dim3(a.B), dim3(nthr), (a.T + 16) * sizeof(int), st, a);
}

}  // namespace sc

using namespace sc;

extern "C" int sc_ctc_greedy_decode(const void* log_probs, int dtype, int B, int T, int V,
                                    int64_t stride_b, int64_t stride_t, const int64_t* lengths,
                                    int blank, int32_t* tokens, int32_t* counts, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16,
             "sc_ctc_greedy_decode: unsupported dtype %d", dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && V > 0, "sc_ctc_greedy_decode: bad shape");
  SC_REQUIRE(T <= 16000, "sc_ctc_greedy_decode: T=%d exceeds the 16000-step LDS row", T);
  if (B == 0) return 0;
  SC_REQUIRE(counts && lengths, "sc_ctc_greedy_decode: null pointer");
  SC_REQUIRE(T == 0 || (log_probs && tokens), "sc_ctc_greedy_decode: null pointer");
  GreedyArgs a{log_probs, B, T, V, blank, stride_b, stride_t, lengths, tokens, counts};
  hipStream_t st = (hipStream_t)stream;
  if (T == 0) {
    zero_async(counts, sizeof(int32_t) * B, st);
    return launch_status("sc_ctc_greedy_decode");
  }
  switch (dtype) {
    case SC_F32: launch<SC_F32>(a, st); break;
    case SC_BF16: launch<SC_BF16>(a, st); break;
    default: launch<SC_F16>(a, st); break;
  }
  return launch_status("sc_ctc_greedy_decode");
}

extern "C" int sc_ctc_greedy_step(const void* logits, int dtype, int B, int V, int64_t stride_b,
                                  const float* mask, int blank, int32_t* prev, int32_t* emit,
                                  int64_t emit_stride, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16,
             "sc_ctc_greedy_step: unsupported dtype %d", dtype);
  SC_REQUIRE(B >= 0 && V > 0, "sc_ctc_greedy_step: bad shape");
  if (B == 0) return 0;
  SC_REQUIRE(logits && prev && emit, "sc_ctc_greedy_step: null pointer");
  GreedyStepArgs a{logits, B, V, blank, stride_b, mask, prev, emit, emit_stride};
  const dim3 grid((unsigned)((B + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case SC_F32: hipLaunchKernelGGL(greedy_step_kernel<SC_F32>, grid, dim3(256), 0, st, a); break;
    case SC_BF16: hipLaunchKernelGGL(greedy_step_kernel<SC_BF16>, grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(greedy_step_kernel<SC_F16>, grid, dim3(256), 0, st, a); break;
  }
  return launch_status("sc_ctc_greedy_step");
}

extern "C" int sc_ctc_greedy_frames(const void* logits, int dtype, int F, int B, int V,
                                    int64_t stride_f, int64_t stride_b, const float* mask,
                                    int64_t mask_f, int blank, int32_t* prev, int32_t* emit,
                                    int64_t emit_f, int64_t emit_b, void* stream) {
  clear_error();
  SC_REQUIRE(dtype == SC_F32 || dtype == SC_BF16 || dtype == SC_F16,
             "sc_ctc_greedy_frames: unsupported dtype %d", dtype);
  SC_REQUIRE(F >= 0 && B >= 0 && V > 0, "sc_ctc_greedy_frames: bad shape");
  if (B == 0 || F == 0) return 0;
  SC_REQUIRE(logits && prev && emit, "sc_ctc_greedy_frames: null pointer");
  GreedyFramesArgs a{logits, F, B, V, blank, stride_f, stride_b, mask, mask_f, prev, emit, emit_f,
                     emit_b};
  const dim3 grid((unsigned)((B + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case SC_F32: hipLaunchKernelGGL(greedy_frames_kernel<SC_F32>, grid, dim3(256), 0, st, a); break;
    case SC_BF16: hipLaunchKernelGGL(greedy_frames_kernel<SC_BF16>, grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(greedy_frames_kernel<SC_F16>, grid, dim3(256), 0, st, a); break;
  }
  return launch_status("sc_ctc_greedy_frames");
}
