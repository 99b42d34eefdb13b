// Ablation probe for the forward LucyRNN scan's memory pipeline (research tool, not product).
// Variants of a forward-scan-shaped kernel at B=32, T=1500, D=512, bf16 gates:
//   COMPUTE  full per-step math vs a trivial use of every loaded word
//   BARRIER  the two LDS-composed barrier phases per 64-step super-chunk vs none
//   NBUF     register prefetch depth in super-chunks (2 = current + next, 3 = two ahead)
//   DPL      hidden units per lane (1: 2-byte loads, WG = 64 d; 2: 4-byte loads, WG = 128 d)
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -I statecatcher_amd/csrc \
//        tools/scan_probe.hip -o build/scan_probe
//   (+ -DWITH_LIB statecatcher_amd/libstatecatcher_hip.so -Wl,-rpath,$PWD/statecatcher_amd to
//   time the shipped kernel through the C ABI in the same harness)
#include <cstdio>
#include <algorithm>
#include <vector>

#include "sc_common.h"
#include "statecatcher.h"

using namespace sc;

constexpr int B = 32, T = 1500, D = 512, CH = 64;

__device__ __forceinline__ float tanh_like(float x) { return sigm(2.f * x) * 2.f - 1.f; }

template <int NW, int LC, int NBUF, bool COMPUTE, bool BARRIER, int DPL>
__global__ void __launch_bounds__(NW * 64) probe(const uint16_t* gates, uint16_t* out) {
  using W = typename std::conditional<DPL == 1, uint16_t, uint32_t>::type;
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int d0 = (blockIdx.x * 64 + lane) * DPL;
  __shared__ float2 agg[NW][64];
  const Buf<W> gb(gates + (int64_t)b * T * 7 * D);
  const Buf<W> ob(out + (int64_t)b * T * D);
  const uint32_t vg = d0 * 2;
  const int nsc = (T + CH - 1) / CH;
  uint32_t buf[NBUF][LC][7];
  auto load = [&](uint32_t (&bf)[LC][7], int k) {
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const uint32_t so = (uint32_t)min(k * CH + w * LC + j, T - 1) * 7 * D * 2;
#pragma unroll
      for (int g = 0; g < 7; ++g) bf[j][g] = (uint32_t)gb.ldw(vg, so + g * D * 2);
    }
  };
  float s = 0.f, h = 0.f;
  auto body = [&](const uint32_t (&cur)[LC][7], int k) __attribute__((always_inline)) {
    const int t0 = k * CH + w * LC;
    float x[LC * DPL], acc = 1.f, bb = 0.f;
#pragma unroll
    for (int j = 0; j < LC; ++j)
#pragma unroll
      for (int p = 0; p < DPL; ++p) {
        float g[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) g[q] = __uint_as_float((cur[j][q] >> (16 * p)) << 16);
        if (COMPUTE) {
          const float rc2 = (g[0] * g[0] + g[1] * g[1]) * 0.5f + 1e-6f;
          const float q2 = (g[2] * g[2] + g[3] * g[3]) * 0.5f + 1e-6f;
          const float zg = sigm(g[1] * rsq(rc2));
          const float dec = sigm(g[5] * rsq(g[5] * g[5] + 1e-6f));
          const float alp = sigm(g[6] * rsq(g[6] * g[6] + 1e-6f));
          const float hn = g[4] * rsq(g[4] * g[4] + 1e-6f);
          const float iq = rsq(q2);
          const float u = alp * (g[2] * iq) * (g[3] * iq) * rcp(q2 + 1e-6f);
          s = dec * s + u;
          x[j * DPL + p] = zg * h + (1.f - zg) * tanh_like(hn + s);
          acc *= dec;
          bb = bb * dec + u;
        } else {
          x[j * DPL + p] = g[0] + g[1] + g[2] + g[3] + g[4] + g[5] + g[6];
          acc += x[j * DPL + p];
        }
      }
    if (BARRIER) {
      agg[w][lane] = make_float2(acc, bb);
      lds_barrier();
      for (int q = 0; q < w; ++q) { const float2 m = agg[q][lane]; s = m.x * s + m.y; }
      lds_barrier();
      for (int q = 0; q < w; ++q) { const float2 m = agg[q][lane]; h = m.x * h + m.y; }
    }
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      if (t0 + j < T) {
        if (DPL == 1) {
          ob.st((W)(__float_as_uint(x[j] + h) >> 16), vg, (uint32_t)(t0 + j) * D * 2);
        } else {
          const uint32_t lo = __float_as_uint(x[j * DPL] + h) >> 16;
          const uint32_t hi = __float_as_uint(x[j * DPL + DPL - 1] + h) & 0xffff0000u;
          ob.st((W)(lo | hi), vg, (uint32_t)(t0 + j) * D * 2);
        }
      }
    }
  };
  load(buf[0], 0);
  if (NBUF > 2) load(buf[1], 1);
  for (int k = 0; k < nsc; k += NBUF) {
#pragma unroll
    for (int r = 0; r < NBUF; ++r) {
      if (k + r >= nsc) break;
      load(buf[(r + NBUF - 1) % NBUF], k + r + NBUF - 1);
      body(buf[r], k + r);
    }
  }
}


// Timing: NROT gate buffers used round-robin (1.4 GB, far beyond the 256 MB Infinity Cache,
// so no launch reads gates a previous launch left in cache), 20 warmup launches, then ROUNDS
// rounds of ITERS launches; min and median of the per-round means.
constexpr int NROT = 4, ROUNDS = 7, ITERS = 30;
static const uint16_t* g_rot[NROT];
template <typename F>
void time_variant(const char* name, F launch, size_t lds) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 20; ++i) launch(g_rot[i % NROT]);
  std::vector<double> r;
  for (int q = 0; q < ROUNDS; ++q) {
    (void)hipEventRecord(e0);
    for (int i = 0; i < ITERS; ++i) launch(g_rot[i % NROT]);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    r.push_back(ms * 1e3 / ITERS);
  }
  std::sort(r.begin(), r.end());
  const double bytes = (double)B * T * D * 8 * 2;
  printf("%-46s min %7.1f us  med %7.1f us  %6.1f GB/s %5.1f%%  (lds %zu, %s)\n", name, r[0],
         r[ROUNDS / 2], bytes / r[0] * 1e-3, bytes / r[0] * 1e-3 / 80.0, lds,
         hipGetErrorString(hipGetLastError()));
}

template <int NW, int LC, int NBUF, bool COMPUTE, bool BARRIER, int DPL>
void run(const char* name, const uint16_t*, uint16_t* o) {
  dim3 grid(D / (64 * DPL), B);
  time_variant(name, [&](const uint16_t* g) {
    hipLaunchKernelGGL((probe<NW, LC, NBUF, COMPUTE, BARRIER, DPL>), grid, dim3(NW * 64), 0, 0, g, o);
  }, 0);
}

// LDS-DMA variant: each wave stages its LC steps x 7 gates x 64 d (bf16) into a private LDS
// buffer with 16-byte buffer_load...lds pieces, NBUF buffers, the DMA for super-chunk k+NBUF-1
// issued during k, and the one for k+1 retired (counted vmcnt) before barrier B of k.
// MODE 0: gates [B][T][7][D] (128-B rows); 1: [B][D/64][T][7][64] (a WG's stream contiguous);
// 2: [B][T][D/64][7][64] (weight rows permuted: 896-B rows per step).
template <int NW, int LC, int MODE, int NBUF, bool GLOBAL = false>
__global__ void __launch_bounds__(NW * 64) probe_glds(const uint16_t* gates, uint16_t* out) {
  constexpr int SC = NW * LC;                   // steps per super-chunk
  constexpr int PIECES = LC * 7 * 8;            // 16-B pieces per wave per super-chunk
  constexpr int NI = (PIECES + 63) / 64;        // DMA instructions per wave per super-chunk
  constexpr int WBUF = NI * 64 * 16;            // bytes per wave buffer
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float2 agg[NW * 64];
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int b = blockIdx.y, db = blockIdx.x;
  unsigned char* mybuf = smem + w * NBUF * WBUF;
  const uint16_t* gbase = MODE == 1 ? gates + ((int64_t)b * (D / 64) + db) * T * 7 * 64
                        : MODE == 2 ? gates + (int64_t)b * T * 7 * D + db * 7 * 64
                                    : gates + (int64_t)b * T * 7 * D + db * 64;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)gbase, 0, 0x7fffffff, 0x00020000);
  const Buf<uint16_t> ob(out + (int64_t)b * T * D);
  const int nsc = (T + SC - 1) / SC;
  auto issue = [&](int k) {
    const int slot = k % NBUF;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (i * 64 + 64 > PIECES && lane >= PIECES - i * 64) continue;
      const int p = i * 64 + lane;
      const int j = p / 56, g = (p / 8) % 7, sub = p % 8;
      const int t = min(k * SC + w * LC + j, T - 1);
      const uint32_t voff = MODE == 1 ? (uint32_t)((t * 7 + g) * 128 + sub * 16)
                          : MODE == 2 ? (uint32_t)((t * 7 * D + g * 64) * 2 + sub * 16)
                                      : (uint32_t)(((t * 7 + g) * D) * 2 + sub * 16);
      const uint32_t la = uniform((int)(uint32_t)(size_t)(__attribute__((address_space(3))) void*)(mybuf + slot * WBUF + i * 1024));
      uint32_t keep;
      if (GLOBAL) {
        const void* src = (const char*)gbase + voff;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(la) : "memory");
      } else {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(rs), "s"(la) : "memory");
      }
    }
  };
  float s = 0.f, h = 0.f;
#pragma unroll
  for (int k = 0; k < NBUF - 1; ++k) issue(k);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  for (int k = 0; k < nsc; ++k) {
    const uint16_t* wb = (const uint16_t*)(mybuf + (k % NBUF) * WBUF);
    float g[LC][7];
#pragma unroll
    for (int j = 0; j < LC; ++j)
#pragma unroll
      for (int q = 0; q < 7; ++q) g[j][q] = __uint_as_float((uint32_t)wb[(j * 7 + q) * 64 + lane] << 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool more = k + NBUF - 1 < nsc;
    if (more) issue(k + NBUF - 1);
    const int t0 = k * SC + w * LC;
    float x[LC], acc = 1.f, bb = 0.f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const float rc2 = (g[j][0] * g[j][0] + g[j][1] * g[j][1]) * 0.5f + 1e-6f;
      const float q2 = (g[j][2] * g[j][2] + g[j][3] * g[j][3]) * 0.5f + 1e-6f;
      const float zg = sigm(g[j][1] * rsq(rc2));
      const float dec = sigm(g[j][5] * rsq(g[j][5] * g[j][5] + 1e-6f));
      const float alp = sigm(g[j][6] * rsq(g[j][6] * g[j][6] + 1e-6f));
      const float hn = g[j][4] * rsq(g[j][4] * g[j][4] + 1e-6f);
      const float iq = rsq(q2);
      const float u = alp * (g[j][2] * iq) * (g[j][3] * iq) * rcp(q2 + 1e-6f);
      s = dec * s + u;
      x[j] = zg * h + (1.f - zg) * tanh_like(hn + s);
      acc *= dec;
      bb = bb * dec + u;
    }
    agg[w * 64 + lane] = make_float2(acc, bb);
    lds_barrier();
    for (int q = 0; q < w; ++q) { const float2 m = agg[q * 64 + lane]; s = m.x * s + m.y; }
    // retire the DMA for k+1; the one for k+NBUF-1 (issued last) may stay in flight
    if (NBUF == 2 || !more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (NI == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (NI == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    for (int q = 0; q < w; ++q) { const float2 m = agg[q * 64 + lane]; h = m.x * h + m.y; }
#pragma unroll
    for (int j = 0; j < LC; ++j)
      if (t0 + j < T) ob.st((uint16_t)(__float_as_uint(x[j] + h) >> 16), lane * 2, (uint32_t)(t0 + j) * D * 2);
  }
}

template <int NW, int LC, int MODE, int NBUF, bool GLOBAL = false>
void run_glds(const char* name, const uint16_t*, uint16_t* o) {
  constexpr int NI = (LC * 7 * 8 + 63) / 64;
  const size_t lds = NBUF * NW * NI * 1024;
  auto kfn = probe_glds<NW, LC, MODE, NBUF, GLOBAL>;
  (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid(D / 64, B);
  time_variant(name, [&](const uint16_t* g) {
    hipLaunchKernelGGL(kfn, grid, dim3(NW * 64), lds, 0, g, o);
  }, lds);
}

int main() {
  uint16_t* o;
  (void)hipMalloc(&o, (size_t)B * T * D * 2);
  std::vector<uint16_t> h((size_t)B * T * 7 * D);
  for (int r = 0; r < NROT; ++r) {
    uint16_t* g;
    (void)hipMalloc(&g, (size_t)B * T * 7 * D * 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3f00 + (uint16_t)(((i + r) * 2654435761u) >> 24);
    (void)hipMemcpy(g, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    g_rot[r] = g;
  }
  const uint16_t* g = g_rot[0];
#ifdef WITH_LIB
  const bool with_lib = true;
#else
  const bool with_lib = false;
#endif
  float *bias, *st0, *sout, *ckpt;
  (void)hipMalloc(&bias, 7 * D * 4);
  (void)hipMemset(bias, 0, 7 * D * 4);
  (void)hipMalloc(&st0, B * D * 4);
  (void)hipMemset(st0, 0, B * D * 4);
  (void)hipMalloc(&sout, B * D * 4);
  (void)hipMalloc(&ckpt, (size_t)B * ((T + 63) / 64) * 2 * D * 4);
  for (int rep = 0; rep < 1; ++rep) {
    run<16, 4, 2, true, true, 1>("reg NW16 LC4 compute barrier (=old prod)", g, o);
    run<16, 4, 2, false, false, 1>("reg NW16 LC4 loads+stores only", g, o);
    run_glds<16, 4, 0, 2>("glds standard (buffer)", g, o);
    run_glds<16, 4, 0, 2, true>("glds standard (global)", g, o);
    run_glds<16, 4, 1, 2>("glds blocked (buffer)", g, o);
    run_glds<16, 4, 2, 2>("glds permuted (buffer)", g, o);
    run_glds<16, 4, 2, 2, true>("glds permuted (global)", g, o);
    run_glds<12, 4, 2, 3>("glds NW12 LC4 permuted nbuf3", g, o);
    if (with_lib) {   // the shipped kernel through the C ABI, step-blocked gates, same harness
      time_variant("libstatecatcher fwd (blocked, bias, ckpt)", [&](const uint16_t* gg) {
        sc_lucy_scan_fwd(gg, SC_BF16, bias, st0, st0, o, sout, nullptr, B, T, D, (int64_t)T * 7 * D, 7 * D,
                         64, 448, (int64_t)T * D, D, ckpt, nullptr);
      }, 0);
      time_variant("libstatecatcher fwd (blocked, no bias/ckpt)", [&](const uint16_t* gg) {
        sc_lucy_scan_fwd(gg, SC_BF16, nullptr, st0, st0, o, sout, nullptr, B, T, D, (int64_t)T * 7 * D, 7 * D,
                         64, 448, (int64_t)T * D, D, nullptr, nullptr);
      }, 0);
    }
  }
  return 0;
}
