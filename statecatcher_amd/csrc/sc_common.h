// Shared device helpers for the statecatcher gfx950 kernels (CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "statecatcher.h"

namespace sc {

// ------------------------------------------------------------------ errors (host) ------------
void set_error(const char* fmt, ...);
void clear_error();
// Converts the launch status of the kernel(s) just enqueued into the ABI return code.
int launch_status(const char* what);
// Zeroes `bytes` bytes at dst on `st` with a kernel (colsum.hip).  Used instead of
// hipMemsetAsync everywhere: inside a captured HIP graph (graphs.GraphedSegments) a captured
// hipMemsetAsync was not ordered before the next kernel on replay -- the RNN-T lattice's
// shift maxima, cleared by one, came out as garbage from the second replay on
// (tools/graph_diag5.py).  Kernel nodes keep stream order.
void zero_async(void* dst, size_t bytes, hipStream_t st);

#define SC_REQUIRE(cond, ...)            \
  do {                                   \
    if (!(cond)) {                       \
      ::sc::set_error(__VA_ARGS__);      \
      return SC_EINVAL;                  \
    }                                    \
  } while (0)

// ------------------------------------------------------------------ element types ------------
// Storage type + fp32 conversion per ABI dtype code.  Stores round to nearest-even.
template <int DT> struct Elem;
// ldw(): convert a raw load result held ZERO-EXTENDED in a 32-bit register.  Prefetch buffers
// hold raw words this way on purpose: with 16-bit element types hipcc packs pairs of loaded
// halves with v_perm right after the load, which forces an s_waitcnt on every prefetch load.
template <> struct Elem<SC_F32> {
  using T = float;
  static __device__ __forceinline__ float ld(T v) { return v; }
  static __device__ __forceinline__ float ldw(uint32_t w) { return __uint_as_float(w); }
  static __device__ __forceinline__ T st(float f) { return f; }
};
template <> struct Elem<SC_BF16> {
  // clang's native bf16: conversions lower to v_cvt_pk_bf16_f32 (RNE, NaN kept) on gfx950 and
  // 16-bit register packing works as for _Float16.
  using T = __bf16;
  static __device__ __forceinline__ float ld(T v) { return (float)v; }
  static __device__ __forceinline__ float ldw(uint32_t w) { return __uint_as_float(w << 16); }
  static __device__ __forceinline__ T st(float f) { return (T)f; }
};
template <> struct Elem<SC_F16> {
  using T = _Float16;
  static __device__ __forceinline__ float ld(T v) { return (float)v; }
  static __device__ __forceinline__ float ldw(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)w);
  }
  static __device__ __forceinline__ T st(float f) { return (T)f; }
};

// 16-byte vectors of an element type: N elements per 16 bytes, converted to / from fp32.
template <int DT> struct Vec16 {
  using T = typename Elem<DT>::T;
  static constexpr int N = 16 / (int)sizeof(T);
  typedef uint32_t raw_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ void ld(const T* p, float (&f)[N]) {
    const raw_t r = *(const raw_t*)p;
    if constexpr (N == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) f[i] = __uint_as_float(r[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[2 * i] = Elem<DT>::ldw(r[i] & 0xffffu);
        f[2 * i + 1] = Elem<DT>::ldw(r[i] >> 16);
      }
    }
  }
  static __device__ __forceinline__ void st(T* p, const float (&f)[N]) {
    raw_t r;
    if constexpr (N == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(f[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const T lo = Elem<DT>::st(f[2 * i]), hi = Elem<DT>::st(f[2 * i + 1]);
        r[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) |
               ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
      }
    }
    *(raw_t*)p = r;
  }
};

// ------------------------------------------------------------------ fast math ----------------
// Single-instruction transcendentals (v_exp_f32 / v_rcp_f32 / v_rsq_f32, ~1 ulp).
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float log2_(float x) { return __builtin_amdgcn_logf(x); }
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
__device__ __forceinline__ float fexp(float x) { return exp2_(x * kLog2e); }
__device__ __forceinline__ float flog(float x) { return log2_(x) * kLn2; }
// sigmoid(x) = 1 / (1 + e^-x): saturates cleanly to 0 / 1 (rcp(inf) = 0).
__device__ __forceinline__ float sigm(float x) { return rcp(1.0f + exp2_(-x * kLog2e)); }

// ------------------------------------------------------------------ buffer I/O ---------------
// Raw buffer loads/stores through a wave-uniform descriptor: the per-lane part of the address
// is a 32-bit VGPR offset that stays constant over a whole scan (the column), the per-step part
// (time, gate plane) is a scalar SGPR offset.  Saves the two VGPRs per in-flight load that a
// 64-bit flat address costs, which is what lets deep register prefetch fit.
template <int BYTES> struct RawIO;
template <> struct RawIO<2> {
  static __device__ __forceinline__ uint16_t ld(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, v, s, 0);
  }
  static __device__ __forceinline__ void st(uint16_t x, __amdgpu_buffer_rsrc_t r, uint32_t v,
                                            uint32_t s) {
    __builtin_amdgcn_raw_buffer_store_b16(x, r, v, s, 0);
  }
};
template <> struct RawIO<4> {
  static __device__ __forceinline__ uint32_t ld(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, v, s, 0);
  }
  static __device__ __forceinline__ void st(uint32_t x, __amdgpu_buffer_rsrc_t r, uint32_t v,
                                            uint32_t s) {
    __builtin_amdgcn_raw_buffer_store_b32(x, r, v, s, 0);
  }
};

template <typename T>
struct Buf {
  using Raw = RawIO<sizeof(T)>;
  __amdgpu_buffer_rsrc_t r;
  // base must be wave-uniform (kernel argument + blockIdx arithmetic only).
  __device__ __forceinline__ explicit Buf(const void* base)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000)) {}
  __device__ __forceinline__ T ld(uint32_t voff, uint32_t soff) const {
    return __builtin_bit_cast(T, Raw::ld(r, voff, soff));
  }
  // raw element bits, zero-extended to 32 bits (see Elem::ldw)
  __device__ __forceinline__ uint32_t ldw(uint32_t voff, uint32_t soff) const {
    return (uint32_t)Raw::ld(r, voff, soff);
  }
  __device__ __forceinline__ void st(T x, uint32_t voff, uint32_t soff) const {
    using U = decltype(Raw::ld(r, 0, 0));
    Raw::st(__builtin_bit_cast(U, x), r, voff, soff);
  }
};

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// ------------------------------------------------------------------ LDS-DMA ------------------
// global_load_lds_{ushort,dword,dwordx4}: each active lane copies PW bytes from its own global
// address straight into LDS at (wave-uniform lds_addr) + lane * PW; no VGPR destination.
// Issued from inline asm on purpose: hipcc's waitcnt model would otherwise treat the pending
// LDS write as aliasing every later LDS access and drain it (vmcnt(0)) at the next ds_read or
// ds_write.  The issuing wave retires it with dma_wait() (counts stores too on gfx9) and other
// waves may read the bytes only after a barrier that follows that wait.
template <int PW>
__device__ __forceinline__ void dma_to_lds(const void* src, uint32_t lds_addr) {
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);   // M0 operand: keep it in an SGPR
  uint32_t keep;
  if constexpr (PW == 16) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
  } else if constexpr (PW == 4) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
  } else {
    static_assert(PW == 2, "LDS-DMA piece width must be 2, 4 or 16 bytes");
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_ushort %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
  }
}
// Same copy with a wave-uniform 64-bit base in SGPRs plus a per-lane 32-bit byte offset
// (the saddr form): a loop that walks time with loop-invariant lane offsets issues each piece
// as one instruction, with no per-lane 64-bit address arithmetic.
template <int PW>
__device__ __forceinline__ void dma_to_lds_s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
  {   // the base is wave-uniform by contract: say so where the compiler cannot prove it (a
      // preceding exec-masked DMA leaves it unsure), so the saddr operand stays in SGPRs
    const uint64_t u = (uint64_t)(uintptr_t)sbase;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    sbase = (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  }
  uint32_t keep;
  if constexpr (PW == 16) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
  } else if constexpr (PW == 4) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
  } else {
    static_assert(PW == 2, "LDS-DMA piece width must be 2, 4 or 16 bytes");
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_ushort %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
  }
}
// 32-bit LDS address of a __shared__ pointer, made wave-uniform (it goes to M0)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)uniform((int)(uint32_t)(size_t)(__attribute__((address_space(3))) const void*)p);
}
// Retire (in hipcc's waitcnt model) the global loads that produced v before a loop: hipcc cannot
// see the asm dma_wait()s, so a first use of such a value inside a DMA-pipelined loop gets a
// vmcnt(0) in EVERY iteration, draining the in-flight DMA.  Passing the values through an empty
// asm makes the one wait happen here instead.
template <int N>
__device__ __forceinline__ void settle(float (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}
// g * w - m with the product rounded on its own (an opaque v_mul_f32: hipcc's default fp-contract
// would fuse it into an fma in one kernel and not in another).  Kernels that must round a value
// identically (the folded LayerNorm's weight image and its row sums) share this one expression.
__device__ __forceinline__ float mul_sub_rn(float g, float w, float m) {
  float p;
  asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p) : "v"(g), "v"(w));
  return p - m;
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Retire every DMA but the N youngest vector-memory LOADS.  Loads complete in issue order among
// themselves; stores may complete out of order with them, but they only make the counter larger:
// with at most N operations outstanding and the N youngest loads possibly among them, every
// older load has completed.  (Valid only when no other load was issued after those N.)
template <int N>
__device__ __forceinline__ void dma_wait_younger() {
  static_assert(N >= 0 && N <= 63, "gfx9 vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_read_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Workgroup barrier that orders LDS only.  __syncthreads() carries a workgroup fence that makes
// the compiler drain outstanding global loads (vmcnt(0)); the scans keep their next
// super-chunk's gate loads in flight across barriers, so the fence is restricted to LDS.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------------------------------------------ wave reductions ---------
// over the 64 lanes through DPP (quad perms, row mirrors, row broadcasts), result read from lane
// 63: a dozen VALU cycles instead of six LDS round trips of __shfl_xor
// v_max_f32 as one instruction: fmaxf makes LLVM canonicalise operands it cannot prove canonical
// (an extra v_max each); callers never hold a NaN they must quiet
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int CTRL, int RMASK, bool MAX>
__device__ __forceinline__ float dpp_step(float v) {
  const float o = __int_as_float(__builtin_amdgcn_update_dpp(
      __float_as_int(MAX ? v : 0.0f), __float_as_int(v), CTRL, RMASK, 0xf, false));
  return MAX ? vmax(v, o) : v + o;
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce_dpp(float x) {
  x = dpp_step<0xB1, 0xf, MAX>(x);    // quad_perm [1,0,3,2]
  x = dpp_step<0x4E, 0xf, MAX>(x);    // quad_perm [2,3,0,1]
  x = dpp_step<0x141, 0xf, MAX>(x);   // row_half_mirror
  x = dpp_step<0x140, 0xf, MAX>(x);   // row_mirror: every lane holds its row's result
  x = dpp_step<0x142, 0xa, MAX>(x);   // row_bcast:15 into rows 1, 3
  x = dpp_step<0x143, 0xc, MAX>(x);   // row_bcast:31 into rows 2, 3: lane 63 holds the result
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
__device__ __forceinline__ float wave_max_dpp(float x) { return wave_reduce_dpp<true>(x); }
__device__ __forceinline__ float wave_sum_dpp(float x) { return wave_reduce_dpp<false>(x); }

}  // namespace sc
