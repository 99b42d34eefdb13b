// RCCL-footprint probe (verdict r4, item 1 / weak 10): what a data-parallel step's gradient
// all-reduce costs the compute kernels it overlaps on ONE GPU.  RCCL's ring kernels occupy a few
// dozen CUs for the whole all-reduce and stream its bytes through them; this kernel does the same
// with local memory: `wgs` persistent workgroups (one per CU they land on) copy `bytes` from src to
// dst in 16-KiB chunks, pausing `sleep` s_sleep units after each chunk to pace the stream (xGMI
// delivers an 8-GPU ring's 2 (N - 1) / N x 40 MB per GPU in ~0.2-0.5 ms, far below a local copy).
// Not part of the product library: bench.py --rccl-footprint loads it (build: tools/footprint.sh).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) footprint_kernel(const float4* __restrict__ src,
                                                        float4* __restrict__ dst, int64_t n4,
                                                        int sleep) {
  constexpr int64_t kChunk = 1024;   // float4 per chunk = 16 KiB
  const int64_t nchunks = (n4 + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t base = c * kChunk;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + k * 256 + threadIdx.x;
      if (i < n4) dst[i] = src[i];
    }
    for (int s = 0; s < sleep; ++s) __builtin_amdgcn_s_sleep(127);
  }
}

extern "C" int sc_probe_footprint(const void* src, void* dst, int64_t bytes, int wgs, int sleep,
                                  void* stream) {
  if (wgs <= 0 || bytes < 16) return 1;
  hipLaunchKernelGGL(footprint_kernel, dim3(wgs), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)src, (float4*)dst, bytes / 16, sleep);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
