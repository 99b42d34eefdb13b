// FETCH_SIZE / WRITE_SIZE calibration probe (tool, not product): one kernel per access pattern,
// each moving a KNOWN byte count once, so rocprofv3's counters can be converted to bytes for the
// patterns the mLSTM walks use (MI355X_MICROARCH.md, HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
//   rd_stream     16 B per lane, contiguous (the guide's calibrated case: FETCH_SIZE = bytes / 2)
//   rd_seg192     16 B per lane, 192-B row segments at a 4624-B row stride (q / k rows of the
//                 xLSTM's fused projection, DQ = 96 bf16, N = 2312 columns)
//   rd_seg384     the same with 384-B segments (v rows, DV = 192)
//   rd_seg128     the same with 128-B segments (one 64-column block of a v row: mlstm_fw_walk)
//   rd_seg<192,1> 16 B per lane, contiguous 192-B rows (a [BH][T][96] bf16 operand)
//   wr_stream     16 B per lane contiguous stores
//   wr_seg192     16 B per lane, 192-B segments at 4624 B (dq / dk written into the gradient
//                 of the fused projection)
//   wr_2b_tile    2 B per lane in 16 x 16 bf16 tiles (an MFMA accumulator written element-wise:
//                 lane -> (row 4 (lane >> 4) + r, column lane & 15), r = 0..3)
//
// build: hipcc -O3 --offload-arch=gfx950 tools/fetch_probe.hip -o build/fetch_probe
// run:   rocprofv3 --pmc FETCH_SIZE -f csv -d OUT -o run -- build/fetch_probe   (and WRITE_SIZE)
// It prints each kernel's byte count; tools/fetch_probe.py turns the two counter CSVs into factors.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t kRows = 400000;   // rows of the segmented patterns (400k x 4624 B = 1.85 GB span)
constexpr int64_t kStride = 4624;   // bytes per fused-projection row

__global__ void rd_stream(const u32x4* p, int64_t n, uint32_t* sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

// one wave per row segment of SEG bytes (SEG / 16 lanes active); TAG only names the kernel
template <int SEG, int TAG>
__global__ void rd_seg(const char* p, int64_t rows, int64_t stride, uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  u32x4 acc = {0, 0, 0, 0};
  for (int64_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4)
    if (lane < SEG / 16) acc ^= *(const u32x4*)(p + r * stride + 16 * lane);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

__global__ void wr_stream(u32x4* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = u32x4{(uint32_t)i, 1, 2, 3};
}

template <int SEG>
__global__ void wr_seg(char* p, int64_t rows, int64_t stride) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4)
    if (lane < SEG / 16) *(u32x4*)(p + r * stride + 16 * lane) = u32x4{(uint32_t)r, 1, 2, 3};
}

// tiles of 16 rows x 16 bf16 columns, row pitch `pitch` bytes, six tiles across each 192-B row
// segment; each wave writes one tile with four 2-byte stores per lane
__global__ void wr_2b_tile(uint16_t* p, int64_t tiles, int64_t pitch) {
  const int lane = threadIdx.x & 63;
  for (int64_t t = blockIdx.x * 4 + (threadIdx.x >> 6); t < tiles; t += (int64_t)gridDim.x * 4) {
    char* base = (char*)p + (t / 6) * 16 * pitch + (t % 6) * 32;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *(uint16_t*)(base + (4 * (lane >> 4) + r) * pitch + 2 * (lane & 15)) = (uint16_t)(t + r);
  }
}

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main() {
  const int64_t span = kRows * kStride;
  char* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, span));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, span));
  const dim3 g(2048), b(256);
  // each kernel twice: the second launch's counters are the ones the script reads
  for (int it = 0; it < 2; ++it) {
    hipLaunchKernelGGL(rd_stream, g, b, 0, 0, (const u32x4*)buf, span / 16, sink);
    hipLaunchKernelGGL((rd_seg<192, 0>), g, b, 0, 0, buf, kRows, kStride, sink);
    hipLaunchKernelGGL((rd_seg<384, 0>), g, b, 0, 0, buf, kRows, kStride, sink);
    hipLaunchKernelGGL((rd_seg<128, 0>), g, b, 0, 0, buf + 1536, kRows, kStride, sink);
    hipLaunchKernelGGL((rd_seg<192, 1>), g, b, 0, 0, buf, kRows, (int64_t)192, sink);
    hipLaunchKernelGGL(wr_stream, g, b, 0, 0, (u32x4*)buf, span / 16);
    hipLaunchKernelGGL((wr_seg<192>), g, b, 0, 0, buf, kRows, kStride);
    hipLaunchKernelGGL(wr_2b_tile, g, b, 0, 0, (uint16_t*)buf, (kRows / 16) * 6, kStride);
  }
  CK(hipDeviceSynchronize());
  printf("rd_stream %lld\n", (long long)span);
  printf("rd_seg<192, 0> %lld\n", (long long)(kRows * 192));
  printf("rd_seg<384, 0> %lld\n", (long long)(kRows * 384));
  printf("rd_seg<128, 0> %lld\n", (long long)(kRows * 128));
  printf("rd_seg<192, 1> %lld\n", (long long)(kRows * 192));
  printf("wr_stream %lld\n", (long long)span);
  printf("wr_seg<192> %lld\n", (long long)(kRows * 192));
  printf("wr_2b_tile %lld\n", (long long)((kRows / 16) * 6 * 512));
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
