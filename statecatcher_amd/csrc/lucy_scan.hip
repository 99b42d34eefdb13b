// LucyRNN gated recurrent scan, forward and backward, for gfx950 (CDNA4, wave64).
//
// Replaces the reference Triton kernel rnn_forward_unfused_rmsnorm
// (speechcatcher-asr/statecatcher lucyrnn_triton.py:179-244), which runs one scalar program per
// (b, d) chain stepping serially over T, and adds the backward the reference lacks.
//
// Math per chain and step (gate planes r,z,k,v,h_pre,decay,alpha; lucyrnn_triton.py:205-242):
//   zg  = sigm(z / sqrt((r^2+z^2)/2 + eps))         dec = sigm(decay / sqrt(decay^2 + eps))
//   alp = sigm(alpha / sqrt(alpha^2 + eps))         hn  = h_pre / sqrt(h_pre^2 + eps)
//   kv  = (k/rkv)(v/rkv)/(rkv^2 + eps), rkv = sqrt((k^2+v^2)/2 + eps)
//   s_t = dec*s_{t-1} + alp*kv                      c = tanh(hn + s_t) (as 2 sigm(2x) - 1)
//   h_t = (1-zg)*c + zg*h_{t-1}
// Gates depend only on the layer input, so both recurrences are first-order LINEAR scans
// (SURVEY F5): s is affine in s_{t-1}; given s, h is affine in h_{t-1}.
//
// Decomposition (MI355X-first): one workgroup = one batch row b x one 64-wide column block of
// hidden units (lane = d) x NW waves that split TIME.  Time is walked in super-chunks of 64
// steps; wave w owns steps [w*LC, (w+1)*LC) of the super-chunk.  Per super-chunk each wave
//   1. computes the elementwise gate terms of its LC steps (gates read ONCE from HBM),
//   2. publishes its s-segment as an affine map (prod dec, local scan) in LDS, barrier,
//      composes the maps of the waves before it with the carried state -> exact s,
//   3. computes c = tanh(hn + s) and publishes its h-segment map, barrier, composes -> exact h,
//   4. stores h (out) and hands the super-chunk's final (s, h) to the next one through LDS.
// B*ceil(D/64) workgroups x 16 waves: 256 x 16 at the B=32, D=512 training shape, one per CU.
//
// Gate stream (measured, tools/scan_probe.hip): the gates never pass through VGPRs on their
// way in.  Each wave copies its LC steps x 7 gate rows of 64 units into a private LDS slot with
// LDS-DMA (global_load_lds, 16-byte pieces), the copy of super-chunk k+1 in flight while k
// computes, and reads its operands back with ds_read.  Versus register prefetch of 2-byte
// elements this frees ~56 VGPRs per lane and lifts the probe kernel from 49% to 53% of HBM
// peak; with the step-blocked gate layout (stride_g_cb = 448, a step's 7 x 64 gates contiguous
// -> 896-byte runs instead of seven 128-byte rows) it reaches 60%.
//
// The forward checkpoints (s, h) at every super-chunk start (B*ceil(T/64)*2*D floats, 1/32 of the
// output); the backward walks super-chunks in reverse, recomputes s, c, h from the gates it
// reads anyway (no re-read of `out`), then runs the two adjoint scans the same chunked way:
//   Gh_t = dout_t + zg_{t+1} Gh_{t+1}
//   Gs_t = Gh_t (1-zg_t)(1-c_t^2) + dec_{t+1} Gs_{t+1},   Gs_{T-1} += ds_last
// and writes the 7 gate gradients.  Algorithmic HBM bytes per (b,t,d): fwd 7e + e (+ckpt),
// bwd 7e + e + 7e.

#include <atomic>
#include <initializer_list>
#include <type_traits>

#include "sc_common.h"

namespace sc {

// SC_ABL: ablation bitmask for tools/abl_bench.sh only (never set in a shipped build):
//   1 trivial gate-gradient math, 2 no dgates stores, 4 no cross-wave compositions,
//   8 backward barriers B1-B3 removed (wrong results; timing only)
#ifndef SC_ABL
#define SC_ABL 0
#endif
// SC_SCAN_LW (forward): retire the next super-chunk's gate DMA at the END of the current one
// (just before its own output stores) instead of before its second barrier, so the DMA has the
// whole super-chunk to land.  (The backward keeps its wait before B2: its checkpoint rows are one
// shared copy that other waves read after B2, and per-wave copies measured 3% slower in-step.)  The slots are wave-private: the issuing wave's own vmcnt orders its later
// ds_reads, no barrier needed (MI355X_MICROARCH.md item 7).  SC_FWD_FD: LDS slots per wave in the
// forward (2: two super-chunks in flight, 16-bit gates).  SC_FWD_CSW: forward prefix
// compositions with the wave's position as a compile-time count (one LDS round trip).
#ifndef SC_SCAN_LW
#define SC_SCAN_LW 1
#endif
#ifndef SC_FWD_FD
#define SC_FWD_FD 1
#endif
#ifndef SC_FWD_CSW
#define SC_FWD_CSW 0
#endif

constexpr int kChunk = 64;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));   // time steps per super-chunk (== NW * LC for every variant)
constexpr float kEps = 1e-6f;

struct ScanFwdArgs {
  const void* gates;
  const float* bias;   // optional fp32 [7,D] gate bias added on load (NULL: gates are biased)
  const float* h0;
  const float* s0;
  void* out;
  float* s_out;
  float* h_out;   // optional fp32 [B,D]: h after the last step, unrounded (the segment carry)
  float* ckpt;
  int B, T, D, nsc;
  int64_t g_bt, g_td, g_cd, g_cb, o_bt, o_bd;
  // optional split-precision planes (16-bit out only, same strides as out): out_dup = out again,
  // out_lo = h - out in the same 16-bit type.  [out | out_dup | out_lo] against [Wh | Wl | Wh]
  // is one bf16 GEMM with the error of an fp32 one (sc_lucy_scan_fwd_split)
  void* out_dup;
  void* out_lo;
  // the inter-layer LayerNorm folded into the projection (sc_lucy_scan_fwd_ln; D % 64 == 0):
  //   ln_r    [7,D] fp32 row sums of the bf16 folded weight W'' (NULL: no fold).  The gates the
  //           GEMM wrote are u = h W''^T of the RAW previous output h; on load they become
  //           rstd (u - mean r) + b' (b' = gate_bias), i.e. exactly LN(h) W^T + b
  //   rec_in  [B][T][D/64] (mean, M2) records of h's 64-unit blocks (the previous scan's rec_out)
  //   ln_stat [B][T] (rstd, mean) out: the combined statistics (block 0 writes them; NULL: none)
  //   rec_out [B][T][D/64] (mean, M2) records of THIS output's 16-bit values (NULL: none)
  const float* ln_r;
  const float2* rec_in;
  float2* ln_stat;
  float2* rec_out;
  float ln_eps;
};

struct ScanBwdArgs {
  const void* gates;
  const float* bias;
  const float* ckpt;
  const void* dout;
  const float* ds_last;
  void* dgates;
  float* dh0;
  float* ds0;
  float* dbias;   // optional [B,7,D]: sum over t of dgates (gate-projection bias gradient part)
  int B, T, D, nsc;
  int64_t g_bt, g_td, g_cd, g_cb, d_bt, d_bd, dg_bt, dg_td, dg_cd, dg_cb;
  // the folded LayerNorm (sc_lucy_scan_bwd_ln): gates rebuilt as in the forward from ln_r and
  // the forward's ln_stat [B][T] (rstd, mean); the stored dgates are d gates / d u = rstd dL/dg
  // (what the projection's input and weight gradients consume); dbias stays dL/dg
  const float* ln_r;
  const float2* ln_stat;
};

// LDS-DMA piece geometry: a 64-unit row of T elements is PPR pieces of PW bytes.  A partial
// last column block (D % 64 != 0) clamps pieces past its end onto its last valid piece.
template <typename T, int PW> struct Pieces {
  static constexpr int EPP = PW / (int)sizeof(T);   // elements per piece
  static constexpr int PPR = 64 / EPP;              // pieces per row
  static_assert(EPP >= 1 && 64 % EPP == 0, "piece width");
};
// Bytes per element in an LDS slot.  global_load_lds_ushort writes each lane's 2 bytes at a
// 4-byte lane stride (measured), so the one-element path of 16-bit types pads to 4 bytes.
template <typename T, int PW> struct LdsElem {
  static constexpr int BYTES = PW == 2 ? 4 : (int)sizeof(T);
  static __device__ __forceinline__ T get(const unsigned char* slot, int idx) {
    return *(const T*)(slot + idx * BYTES);
  }
};

// Elementwise part of lucyrnn_triton.py:213-235 for one (step, chain).
__device__ __forceinline__ void step_terms(float r, float z, float k, float v, float hp, float dc,
                                           float al, float& zg, float& dec, float& u, float& hn) {
  const float rc2 = (r * r + z * z) * 0.5f + kEps;
  const float q = (k * k + v * v) * 0.5f + kEps;     // rkv^2
  zg = sigm(z * rsq(rc2));
  dec = sigm(dc * rsq(dc * dc + kEps));
  const float alp = sigm(al * rsq(al * al + kEps));
  hn = hp * rsq(hp * hp + kEps);
  const float iq = rsq(q);
  const float kv = (k * iq) * (v * iq) * rcp(q + kEps);
  u = alp * kv;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 rsq2(f2 x) { return f2{rsq(x.x), rsq(x.y)}; }
__device__ __forceinline__ f2 rcp2(f2 x) { return f2{rcp(x.x), rcp(x.y)}; }
// sigmoid / tanh of two values: the scale and the 1 + e run as packed fp32, the exp2 and rcp
// per component
__device__ __forceinline__ f2 sigm2(f2 x) {
  const f2 t = x * f2{-kLog2e, -kLog2e};
  return rcp2(f2{1.0f, 1.0f} + f2{exp2_(t.x), exp2_(t.y)});
}
__device__ __forceinline__ f2 tanh2(f2 x) {   // 2 sigm(2x) - 1
  const f2 t = x * f2{-2.0f * kLog2e, -2.0f * kLog2e};
  const f2 r = rcp2(f2{1.0f, 1.0f} + f2{exp2_(t.x), exp2_(t.y)});
  return r + r - f2{1.0f, 1.0f};
}
// Two fp32 values rounded to the element type (one v_cvt_pk_bf16_f32 for bf16).
template <int DT> struct Pair {
  using T = typename Elem<DT>::T;
  typedef T t2 __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ t2 st(f2 v) { return __builtin_convertvector(v, t2); }
};

// step_terms for two steps at once (packed fp32 for the elementwise math)
__device__ __forceinline__ void step_terms2(f2 r, f2 z, f2 k, f2 v, f2 hp, f2 dc, f2 al, f2& zg,
                                            f2& dec, f2& u, f2& hn) {
  const f2 eps = {kEps, kEps}, half = {0.5f, 0.5f};
  const f2 rc2 = (r * r + z * z) * half + eps;
  const f2 q = (k * k + v * v) * half + eps;
  zg = sigm2(z * rsq2(rc2));
  dec = sigm2(dc * rsq2(dc * dc + eps));
  const f2 alp = sigm2(al * rsq2(al * al + eps));
  hn = hp * rsq2(hp * hp + eps);
  const f2 iq = rsq2(q);
  u = alp * ((k * iq) * (v * iq) * rcp2(q + eps));
}

__device__ __forceinline__ float tanh_sig(float x) { return sigm(2.0f * x) * 2.0f - 1.0f; }

// Gradient of one step w.r.t. its 7 raw gates, given the step's adjoints.
//   gh   = dL/dh_t (total), dpre = dL/d(hn + s_t), gs = dL/ds_t (total); zg and dec are the
//   step's gates, kept in registers from the recompute (their sigmoids are not redone).
__device__ __forceinline__ void gate_grads(float r, float z, float k, float v, float hp, float dc,
                                           float al, float zg, float dec, float gh, float dpre,
                                           float gs, float hprev, float sprev, float c,
                                           float (&o)[7]) {
  const float rc2 = (r * r + z * z) * 0.5f + kEps;
  const float irc = rsq(rc2);
  const float ird = rsq(dc * dc + kEps);
  const float ira = rsq(al * al + kEps);
  const float alp = sigm(al * ira);
  const float irh = rsq(hp * hp + kEps);
  const float q = (k * k + v * v) * 0.5f + kEps;
  const float iq = rsq(q);
  const float iqe = rcp(q + kEps);
  // zg = sigm(z / rho_c): d/dz = (r^2/2 + eps)/rho_c^3, d/dr = -z r / (2 rho_c^3)
  const float d_zn = gh * (hprev - c) * zg * (1.0f - zg) * (irc * irc * irc);
  o[0] = -d_zn * z * r * 0.5f;
  o[1] = d_zn * (r * r * 0.5f + kEps);
  // kv = k v f(q), f = 1/(q (q+eps)), f' = -(2q+eps) f^2, dq/dk = k, dq/dv = v
  const float d_kv = gs * alp;
  const float f = iq * iq * iqe;
  const float fp = -(2.0f * q + kEps) * f * f;
  o[2] = d_kv * v * (f + k * k * fp);
  o[3] = d_kv * k * (f + v * v * fp);
  // x / sqrt(x^2 + eps): derivative eps / rho^3
  o[4] = dpre * kEps * (irh * irh * irh);
  o[5] = gs * sprev * dec * (1.0f - dec) * kEps * (ird * ird * ird);
  o[6] = gs * (k * v * f) * alp * (1.0f - alp) * kEps * (ira * ira * ira);
}

// gate_grads for two steps at once: the elementwise math runs as packed fp32 (v_pk_fma_f32 /
// v_pk_mul_f32 on two steps per instruction); the transcendentals stay per component.

__device__ __forceinline__ void gate_grads2(f2 r, f2 z, f2 k, f2 v, f2 hp, f2 dc, f2 al, f2 zg,
                                            f2 dec, f2 gh, f2 dpre, f2 gs, f2 hprev, f2 sprev,
                                            f2 c, f2 (&o)[7]) {
  const f2 one = {1.0f, 1.0f}, eps = {kEps, kEps}, half = {0.5f, 0.5f};
  const f2 rc2 = (r * r + z * z) * half + eps;
  const f2 irc = rsq2(rc2);
  const f2 ird = rsq2(dc * dc + eps);
  const f2 ira = rsq2(al * al + eps);
  const f2 alp = sigm2(al * ira);
  const f2 irh = rsq2(hp * hp + eps);
  const f2 q = (k * k + v * v) * half + eps;
  const f2 iq = rsq2(q);
  const f2 iqe = rcp2(q + eps);
  const f2 d_zn = gh * (hprev - c) * zg * (one - zg) * (irc * irc * irc);
  o[0] = -d_zn * z * r * half;
  o[1] = d_zn * (r * r * half + eps);
  const f2 d_kv = gs * alp;
  const f2 f = iq * iq * iqe;
  const f2 fp = -(q + q + eps) * f * f;
  o[2] = d_kv * v * (f + k * k * fp);
  o[3] = d_kv * k * (f + v * v * fp);
  o[4] = dpre * eps * (irh * irh * irh);
  o[5] = gs * sprev * dec * (one - dec) * eps * (ird * ird * ird);
  o[6] = gs * (k * v * f) * alp * (one - alp) * eps * (ira * ira * ira);
}

// step_terms2 for the backward's recompute, which also returns the seven per-step
// coefficients of the gate gradients (the transcendentals are shared with the recompute, so the
// gradient phase needs neither the raw gates nor a second pass of rsq / rcp / exp):
//   dr = gh (h_{t-1} - c) cf0    dz = gh (h_{t-1} - c) cf1    dk = gs cf2    dv = gs cf3
//   dh_pre = dpre cf4            ddecay = gs s_{t-1} cf5      dalpha = gs cf6
// (gh = dL/dh_t, gs = dL/ds_t, dpre = dL/d(hn + s_t); same formulas as gate_grads).
__device__ __forceinline__ void step_terms_bwd2(f2 r, f2 z, f2 k, f2 v, f2 hp, f2 dc, f2 al,
                                                f2& zg, f2& dec, f2& u, f2& hn, f2 (&cf)[7]) {
  const f2 one = {1.0f, 1.0f}, eps = {kEps, kEps}, half = {0.5f, 0.5f};
  const f2 rc2 = (r * r + z * z) * half + eps;
  const f2 q = (k * k + v * v) * half + eps;
  const f2 irc = rsq2(rc2);
  zg = sigm2(z * irc);
  const f2 ird = rsq2(dc * dc + eps);
  dec = sigm2(dc * ird);
  const f2 ira = rsq2(al * al + eps);
  const f2 alp = sigm2(al * ira);
  const f2 irh = rsq2(hp * hp + eps);
  hn = hp * irh;
  const f2 iq = rsq2(q);
  const f2 f = iq * iq * rcp2(q + eps);
  const f2 kv = k * v * f;
  u = alp * kv;
  const f2 kz = zg * (one - zg) * (irc * irc * irc);
  cf[0] = -kz * z * r * half;
  cf[1] = kz * (r * r * half + eps);
  const f2 fp = -(q + q + eps) * f * f;
  cf[2] = alp * v * (f + k * k * fp);
  cf[3] = alp * k * (f + v * v * fp);
  cf[4] = eps * (irh * irh * irh);
  cf[5] = dec * (one - dec) * eps * (ird * ird * ird);
  cf[6] = kv * alp * (one - alp) * eps * (ira * ira * ira);
}

// Cross-wave composition of the per-wave affine segment maps m_q = (a, b): x -> a x + b, read
// from LDS.  prefix: x <- m_{w-1} o ... o m_0 (x); suffix: x <- m_{w+1} o ... o m_{NW-1} (x)
// (reverse time).  Work stays proportional to the wave's position (the chain runs only over
// the maps it needs: the VALU is the scarce resource); maps are fetched four at a time so the
// LDS latency is paid once per four links.
template <int NW>
__device__ __forceinline__ float compose_prefix(const float2 (*agg)[64], int lane, int w, float x) {
  int q = 0;
  for (; q + 4 <= w; q += 4) {
    const float2 m0 = agg[q][lane], m1 = agg[q + 1][lane], m2 = agg[q + 2][lane],
                 m3 = agg[q + 3][lane];
    x = fmaf(m0.x, x, m0.y);
    x = fmaf(m1.x, x, m1.y);
    x = fmaf(m2.x, x, m2.y);
    x = fmaf(m3.x, x, m3.y);
  }
  for (; q < w; ++q) {
    const float2 m = agg[q][lane];
    x = fmaf(m.x, x, m.y);
  }
  return x;
}
template <int NW>
__device__ __forceinline__ float compose_suffix(const float2 (*agg)[64], int lane, int w, float x) {
  int q = NW - 1;
  for (; q - 4 >= w; q -= 4) {
    const float2 m0 = agg[q][lane], m1 = agg[q - 1][lane], m2 = agg[q - 2][lane],
                 m3 = agg[q - 3][lane];
    x = fmaf(m0.x, x, m0.y);
    x = fmaf(m1.x, x, m1.y);
    x = fmaf(m2.x, x, m2.y);
    x = fmaf(m3.x, x, m3.y);
  }
  for (; q > w; --q) {
    const float2 m = agg[q][lane];
    x = fmaf(m.x, x, m.y);
  }
  return x;
}

// Prefix composition with the wave's position as a compile-time count: one uniform branch picks
// the instance, whose W map fetches all issue before the first link (one LDS round trip instead
// of one per group of four).  Forward only: the backward has no registers for 2 W map values.
template <int W>
__device__ __forceinline__ float prefix_fixed(const float2 (*agg)[64], int lane, float x) {
  if constexpr (W > 0) {
    float2 m[W];
#pragma unroll
    for (int q = 0; q < W; ++q) m[q] = agg[q][lane];
#pragma unroll
    for (int q = 0; q < W; ++q) x = fmaf(m[q].x, x, m[q].y);
  }
  return x;
}
template <int NW, int W = 0>
__device__ __forceinline__ float compose_prefix_sw(const float2 (*agg)[64], int lane, int w, float x) {
  if constexpr (W == NW - 1)
    return prefix_fixed<W>(agg, lane, x);
  else
    return w == W ? prefix_fixed<W>(agg, lane, x) : compose_prefix_sw<NW, W + 1>(agg, lane, w, x);
}

// ------------------------------------------------------------------------ forward ----------
// Reductions over aligned groups of N lanes (N = 2, 4, 8, 16) through DPP: every lane of a group
// ends with the group's sum.
template <int N>
__device__ __forceinline__ float group_sum_dpp(float x) {
  static_assert(N == 2 || N == 4 || N == 8 || N == 16, "group of 2..16 lanes");
  x = dpp_step<0xB1, 0xf, false>(x);                       // quad_perm [1,0,3,2]
  if constexpr (N >= 4) x = dpp_step<0x4E, 0xf, false>(x);   // quad_perm [2,3,0,1]
  if constexpr (N >= 8) x = dpp_step<0x141, 0xf, false>(x);  // row_half_mirror
  if constexpr (N >= 16) x = dpp_step<0x140, 0xf, false>(x);  // row_mirror
  return x;
}

// FD: LDS slots per wave (fetch depth), ring by super-chunk index.  LN (the folded inter-layer
// LayerNorm, ScanFwdArgs::ln_r): bit 1 = this layer's gates are u = h W''^T of the previous raw
// output (combine its block records, rebuild the gates on load); bit 2 = write this output's
// block records.  NB = D / 64 column blocks per row (LN only).
template <int DT, int NW, int LC, int PW, int FD, bool SPLIT = false, int LN = 0, int NB = 8>
__global__ void __launch_bounds__(NW * 64)
lucy_scan_fwd_kernel(ScanFwdArgs a) {
  static_assert(NW * LC == kChunk, "super-chunk must be 64 steps");
  using E = Elem<DT>;
  using T = typename E::T;
  using P = Pieces<T, PW>;
  constexpr int ROWS = LC * 7;                       // gate rows per wave per super-chunk
  constexpr int PIECES = ROWS * P::PPR;
  constexpr int NI = (PIECES + 63) / 64;             // DMA instructions per wave per super-chunk
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int blk = blockIdx.x;
  const int d = blk * 64 + lane;
  const bool dok = d < a.D;
  const int dc = dok ? d : a.D - 1;
  const int pcmax = (min(64, a.D - blk * 64) - 1) / P::EPP;

  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  __shared__ float2 aggS[NW][64];
  __shared__ float2 aggH[NW][64];
  __shared__ float carS[2][64];
  __shared__ float carH[2][64];
  // (LN & 1) the input's block records of the wave's LC steps, [step][block], by LDS-DMA with
  // the gates (16-byte pieces of two blocks of one step)
  constexpr int RECN = (LN & 1) ? LC * NB : 2;
  static_assert(!(LN & 1) || (RECN <= 64 && NB % 2 == 0), "LN fold: LC * NB <= 64, NB even");
  __shared__ __attribute__((aligned(16))) float2 recS[(LN & 1) ? FD : 1][(LN & 1) ? NW : 1][RECN];
  using L = LdsElem<T, PW>;
  constexpr int SLOTB = ROWS * 64 * L::BYTES;                       // wave-private [LC][7][64]
  const unsigned char* slots = dyn_lds + w * FD * SLOTB;            // FD of them
  const uint32_t slots_lds = lds_addr(slots);

  const T* gsrc = (const T*)a.gates + (int64_t)b * a.g_bt + (int64_t)blk * a.g_cb;
  const Buf<T> obuf((T*)a.out + (int64_t)b * a.o_bt);
  const Buf<T> dbuf(SPLIT ? (T*)a.out_dup + (int64_t)b * a.o_bt : (T*)a.out);
  const Buf<T> lbuf(SPLIT ? (T*)a.out_lo + (int64_t)b * a.o_bt : (T*)a.out);
  const uint32_t vo = (uint32_t)d * sizeof(T);
  const uint32_t otd = (uint32_t)(a.o_bd * sizeof(T));
  if (w == 0) {
    carS[0][lane] = dok ? a.s0[(int64_t)b * a.D + d] : 0.0f;
    carH[0][lane] = dok ? a.h0[(int64_t)b * a.D + d] : 0.0f;
  }
  float gb[7], fr[7];
#pragma unroll
  for (int g = 0; g < 7; ++g) {
    gb[g] = a.bias ? a.bias[g * a.D + dc] : 0.0f;
    fr[g] = (LN & 1) ? a.ln_r[g * a.D + dc] : 0.0f;
  }
  settle(gb);
  settle(fr);
  const int Tm1 = a.T - 1;
  // (LN & 1) the records of super-chunk k's LC steps for this wave: lane p < LC NB / 2 copies
  // blocks 2 (p % (NB/2)) .. +1 of step p / (NB/2) (time clamped like the gates)
  auto issue_rec = [&](int k) __attribute__((always_inline)) {
    if constexpr ((LN & 1) != 0) {
      constexpr int NP = LC * NB / 2;
      if (lane < NP) {
        const int j = lane / (NB / 2), q2 = lane % (NB / 2);
        const int t = min(k * kChunk + w * LC + j, Tm1);
        dma_to_lds<16>(a.rec_in + ((int64_t)b * a.T + t) * NB + 2 * q2,
                       lds_addr(&recS[(LN & 1) ? k % FD : 0][(LN & 1) ? w : 0][0]));
      }
    }
  };
  // Past the end of the sequence the clamped step re-reads row T-1 (never out of bounds).
  auto issue = [&](int k) __attribute__((always_inline)) {
    issue_rec(k);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int p = i * 64 + lane;
      if (PIECES % 64 == 0 || p < PIECES) {
        const int row = p / P::PPR, pc = p % P::PPR;
        const int j = row / 7, g = row - 7 * (row / 7);
        const int t = min(k * kChunk + w * LC + j, Tm1);
        dma_to_lds<PW>(gsrc + (int64_t)t * a.g_td + (int64_t)g * a.g_cd + min(pc, pcmax) * P::EPP,
                       slots_lds + (uint32_t)((k % FD) * SLOTB) + i * 64 * (PW == 2 ? 4 : PW));
      }
    }
  };
  // Pieces of a super-chunk wholly inside the sequence need no time clamp: loop-invariant
  // per-lane byte offsets from the wave's first step, one saddr DMA each (16-byte pieces).
  constexpr bool kFast = NI <= 16;   // (one-element pieces: too many offsets to hold)
  uint32_t voff[kFast ? NI : 1];
#pragma unroll
  for (int i = 0; i < (kFast ? NI : 0); ++i) {
    const int p = min(i * 64 + lane, PIECES - 1);
    const int row = p / P::PPR, pc = p % P::PPR;
    voff[i] = (uint32_t)((row / 7) * a.g_td + (row % 7) * a.g_cd + min(pc, pcmax) * P::EPP) *
              (uint32_t)sizeof(T);
  }
  auto issue_next = [&](int k) __attribute__((always_inline)) {
    if (kFast && (k + 1) * kChunk <= a.T) {
      issue_rec(k);
      const T* gt = gsrc + ((int64_t)k * kChunk + w * LC) * a.g_td;
#pragma unroll
      for (int i = 0; i < (kFast ? NI : 0); ++i)
        if (PIECES % 64 == 0 || i * 64 + lane < PIECES)
          dma_to_lds_s<PW>(gt, voff[i], slots_lds + (uint32_t)((k % FD) * SLOTB) + i * 64 * (PW == 2 ? 4 : PW));
    } else {
      issue(k);
    }
  };
  // retire super-chunk k+1's DMA; with two slots, k+2's (the only younger loads) may fly on
  constexpr int NIR = NI + ((LN & 1) ? 1 : 0);   // (+ the records piece)
  auto wait_next = [&](int k) __attribute__((always_inline)) {
    if (FD == 2 && k + 2 < a.nsc) dma_wait_younger<NIR>();
    else dma_wait();
  };
  if (a.nsc > 0) issue(0);
  if (FD == 2 && a.nsc > 1) issue(1);
  wait_next(-1);
  lds_barrier();
  // One super-chunk.  FULL: every step inside the sequence and every lane inside D (no
  // per-step conditions); the tail super-chunk and a partial column block take the guarded one.
  auto chunk = [&](int k, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    constexpr int LP = LC / 2;
    const int t0 = k * kChunk + w * LC;
    f2 zg[LP], dec[LP], u[LP], x[LP], wz[LP];
    float gv[LC][7];
    const unsigned char* slot = slots + (k % FD) * SLOTB;
    if constexpr ((LN & 1) != 0) {
      // the LayerNorm statistics of the input rows: Chan's combination of the NB block records
      // of each step over a group of NB lanes (lane = step * NB + block)
      const float2 rq = recS[(LN & 1) ? k % FD : 0][(LN & 1) ? w : 0][lane % RECN];
      const float mean = group_sum_dpp<NB>(rq.x) * (1.0f / NB);
      const float dm = rq.x - mean;
      const float m2 = group_sum_dpp<NB>(fmaf(64.0f * dm, dm, rq.y));
      const float rstd = rsq(m2 * (1.0f / (64 * NB)) + a.ln_eps);
      if (a.ln_stat && blk == 0 && lane % NB == 0 && lane < RECN && k * kChunk + w * LC + lane / NB < a.T)
        a.ln_stat[(int64_t)b * a.T + k * kChunk + w * LC + lane / NB] = make_float2(rstd, mean);
#pragma unroll
      for (int j = 0; j < LC; ++j) {
        const float rs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rstd), j * NB));
        const float mu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mean), j * NB));
        const float rm = -rs * mu;
#pragma unroll
        for (int g = 0; g < 7; ++g)   // rstd (u - mean r) + b'
          gv[j][g] = fmaf(E::ld(L::get(slot, (j * 7 + g) * 64 + lane)), rs, fmaf(rm, fr[g], gb[g]));
      }
    } else {
#pragma unroll
      for (int j = 0; j < LC; ++j)
#pragma unroll
        for (int g = 0; g < 7; ++g) gv[j][g] = E::ld(L::get(slot, (j * 7 + g) * 64 + lane)) + gb[g];
    }
    lds_read_wait();              // slot consumed: it may be refilled with super-chunk k+FD
    if (k + FD < a.nsc) issue_next(k + FD);
#pragma unroll
    for (int p = 0; p < LP; ++p) {   // two steps per packed instruction
      const int j = 2 * p;
      step_terms2(f2{gv[j][0], gv[j + 1][0]}, f2{gv[j][1], gv[j + 1][1]},
                  f2{gv[j][2], gv[j + 1][2]}, f2{gv[j][3], gv[j + 1][3]},
                  f2{gv[j][4], gv[j + 1][4]}, f2{gv[j][5], gv[j + 1][5]},
                  f2{gv[j][6], gv[j + 1][6]}, zg[p], dec[p], u[p], x[p]);
      if constexpr (!FULL) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          if (t0 + j + h2 >= a.T) {   // identity step past the end of the sequence
            zg[p][h2] = 1.0f; dec[p][h2] = 1.0f; u[p][h2] = 0.0f; x[p][h2] = 0.0f;
          }
        }
      }
    }
    float As = 1.0f, Bs = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      As *= dec[j >> 1][j & 1];
      Bs = fmaf(dec[j >> 1][j & 1], Bs, u[j >> 1][j & 1]);
    }
    aggS[w][lane] = make_float2(As, Bs);
    lds_barrier();
    float s = carS[k & 1][lane];
    const float s_in = s;
    s = SC_FWD_CSW ? compose_prefix_sw<NW>(aggS, lane, w, s) : compose_prefix<NW>(aggS, lane, w, s);
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      s = fmaf(dec[j >> 1][j & 1], s, u[j >> 1][j & 1]);
      x[j >> 1][j & 1] += s;
    }
#pragma unroll
    for (int p = 0; p < LP; ++p) {   // c = tanh(hn + s) and (1 - zg) c, two steps at a time
      x[p] = tanh2(x[p]);
      wz[p] = x[p] - zg[p] * x[p];
    }
    float Ah = 1.0f, Bh = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      Ah *= zg[j >> 1][j & 1];
      Bh = fmaf(zg[j >> 1][j & 1], Bh, wz[j >> 1][j & 1]);
    }
    if (w == NW - 1) carS[(k + 1) & 1][lane] = s;
    aggH[w][lane] = make_float2(Ah, Bh);
    if (!SC_SCAN_LW) wait_next(k);   // super-chunk k+1 has landed in this wave's slot
    lds_barrier();
    float h = carH[k & 1][lane];
    const float h_in = h;
    h = SC_FWD_CSW ? compose_prefix_sw<NW>(aggH, lane, w, h) : compose_prefix<NW>(aggH, lane, w, h);
    float hs[LC];
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      h = fmaf(zg[j >> 1][j & 1], h, wz[j >> 1][j & 1]);
      hs[j] = h;
    }
    if (w == NW - 1) carH[(k + 1) & 1][lane] = h;
    // late wait: retire super-chunk k+1's DMA before this super-chunk's own stores (a store
    // issued before a full vmcnt wait would be drained with it)
    if (SC_SCAN_LW) wait_next(k);
    if (w == 0 && a.ckpt && dok) {
      a.ckpt[((int64_t)(b * a.nsc + k) * 2) * a.D + d] = s_in;
      a.ckpt[((int64_t)(b * a.nsc + k) * 2 + 1) * a.D + d] = h_in;
    }
#pragma unroll
    for (int j = 0; j < LC; ++j)
      if (FULL || (dok && t0 + j < a.T)) {
        const T hi = E::st(hs[j]);
        obuf.st(hi, vo, (uint32_t)(t0 + j) * otd);
        if constexpr (SPLIT) {
          dbuf.st(hi, vo, (uint32_t)(t0 + j) * otd);
          lbuf.st(E::st(hs[j] - E::ld(hi)), vo, (uint32_t)(t0 + j) * otd);
        }
      }
    if constexpr ((LN & 2) != 0) {
      // (mean, M2) of each step's 64 stored (rounded) values, shifted by unit 0's value: the
      // 2 LC sums transposed over the wave (three halving exchanges, then a group-of-8 sum), so
      // lane l ends with sum (l >> 3) & 7 -- 22 exchanges per super-chunk, not 2 LC reductions
      static_assert(LC == 4, "record butterfly written for 4 steps per wave");
      float v[8], ref[LC];
#pragma unroll
      for (int j = 0; j < LC; ++j) {
        const float hb = E::ld(E::st(hs[j]));
        ref[j] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(hb)));
        const float dl = hb - ref[j];
        v[2 * j] = dl;
        v[2 * j + 1] = dl * dl;
      }
      const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
      float u4[4], u2[2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        u4[i] = (b5 ? v[i + 4] : v[i]) + __shfl_xor(b5 ? v[i] : v[i + 4], 32);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        u2[i] = (b4 ? u4[i + 2] : u4[i]) + __shfl_xor(b4 ? u4[i] : u4[i + 2], 16);
      float y = (b3 ? u2[1] : u2[0]) + __shfl_xor(b3 ? u2[0] : u2[1], 8);
      y = group_sum_dpp<8>(y);
      const float ysq = __shfl_xor(y, 8);   // lane 16 j: sum 2 j (dl) here, 2 j + 1 (dl^2) there
      const int j = lane >> 4;
      const float r = j == 0 ? ref[0] : j == 1 ? ref[1] : j == 2 ? ref[2] : ref[3];
      if ((lane & 15) == 0 && t0 + j < a.T)
        a.rec_out[((int64_t)b * a.T + t0 + j) * NB + blk] =
            make_float2(fmaf(y, 1.0f / 64, r), fmaxf(ysq - y * y * (1.0f / 64), 0.0f));
    }
  };
  const bool blk_full = (blk + 1) * 64 <= a.D;
  for (int k = 0; k < a.nsc; ++k) {
    if (blk_full && (k + 1) * kChunk <= a.T)
      chunk(k, std::true_type{});
    else
      chunk(k, std::false_type{});
  }
  lds_barrier();
  if (w == 0 && dok) {
    a.s_out[(int64_t)b * a.D + d] = carS[a.nsc & 1][lane];
    if (a.h_out) a.h_out[(int64_t)b * a.D + d] = carH[a.nsc & 1][lane];
  }
}

// ------------------------------------------------------------------------ backward ---------
// NBUF = 2: two LDS slots per wave, the raw gates stay in LDS for the gate-gradient phase while
// the next super-chunk lands in the other slot (16-bit gates).  NBUF = 1 (fp32, whose two slots
// would not fit in LDS): the raw gates are copied to VGPRs and the slot is refilled at once.
// WST: the 7 gate gradients of each step are written back into the wave's LDS slot over the raw
// gates they were computed from, then stored as whole 16-byte pieces (3.5 wave-instructions per
// super-chunk instead of 28 two-byte stores).  Needs NBUF = 2 and 16-byte aligned dgates.
// LN: the folded inter-layer LayerNorm.  1 (sc_lucy_scan_bwd_ln with ln_r): the gates are
// u = h W''^T, rebuilt as rstd (u - mean r) + b' on load; 2 (ln_r NULL): the projection GEMM has
// already applied the fold (sc_gemm_tn_ln_bf16 wrote rstd (u - mean r)), the gates take b' alone.
// Both store d/du = rstd dL/dgate.
template <int DT, int NW, int LC, int PW, int NBUF, bool WST, int LN = 0>
__global__ void __launch_bounds__(NW * 64)
lucy_scan_bwd_kernel(ScanBwdArgs a) {
  static_assert(NW * LC == kChunk, "super-chunk must be 64 steps");
  using E = Elem<DT>;
  using T = typename E::T;
  using P = Pieces<T, PW>;
  constexpr int GROWS = LC * 7;                      // gate rows, then LC rows of dout
  constexpr int ROWS = LC * 8;
  constexpr int PIECES = ROWS * P::PPR;
  constexpr int NI = (PIECES + 63) / 64;
  static_assert(!WST || (NBUF == 2 && PW == 16), "staged stores need two 16-bit slots");
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int blk = blockIdx.x;
  const int d = blk * 64 + lane;
  const bool dok = d < a.D;
  const int dc = dok ? d : a.D - 1;
  const int pcmax = (min(64, a.D - blk * 64) - 1) / P::EPP;

  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
  __shared__ float2 aggA[NW][64];   // s maps      (B1)
  __shared__ float2 aggB[NW][64];   // h maps      (B2)
  __shared__ float2 aggC[NW][64];   // Gh maps     (B1)
  __shared__ float2 aggD[NW][64];   // Gs maps     (B2)
  __shared__ float carGh[2][64];
  __shared__ float carGs[2][64];
  __shared__ float ckS[2][2][64];   // (s, h) checkpoint of the super-chunk, shared by all waves
  // (LN) the input rows' (rstd, mean) of the wave's LC steps, by LDS-DMA with the gates
  static_assert(!LN || (NBUF == 2 && WST), "LN fold: 16-bit gates with staged stores");
  __shared__ __attribute__((aligned(16))) float2 stS[LN ? NBUF : 1][LN ? NW : 1][LN ? LC : 1];
  using L = LdsElem<T, PW>;
  unsigned char* slots = dyn_lds + w * NBUF * ROWS * 64 * L::BYTES;   // [NBUF][LC*8][64]
  const uint32_t slots_lds = lds_addr(slots);

  const T* gsrc = (const T*)a.gates + (int64_t)b * a.g_bt + (int64_t)blk * a.g_cb;
  const T* dsrc = (const T*)a.dout + (int64_t)b * a.d_bt + (int64_t)blk * 64;
  const float* cksrc = a.ckpt + (int64_t)b * a.nsc * 2 * a.D + dc;
  const Buf<T> dgbuf((T*)a.dgates + (int64_t)b * a.dg_bt + (int64_t)blk * a.dg_cb);
  const uint32_t vo = (uint32_t)lane * sizeof(T);
  if (w == 0) {
    carGh[0][lane] = 0.0f;
    carGs[0][lane] = (a.ds_last && dok) ? a.ds_last[(int64_t)b * a.D + d] : 0.0f;
  }
  float gb[LN ? 1 : 7];
  // (LN) the folded bias b' and the row sums r of the folded weight, per gate and lane, in LDS
  // (the fold's gate rebuild has no registers to spare)
  __shared__ float2 fbS[LN ? 7 : 1][64];
  if constexpr (LN) {
    if (w < 7)
      fbS[LN ? w : 0][lane] = make_float2(a.bias[w * a.D + dc], LN == 1 ? a.ln_r[w * a.D + dc] : 0.0f);
  } else {
#pragma unroll
    for (int g = 0; g < 7; ++g) gb[g] = a.bias ? a.bias[g * a.D + dc] : 0.0f;
    settle(gb);
  }
  const int Tm1 = a.T - 1;
  // (LN) the statistics of super-chunk k's LC steps: lane p < 2 LC copies word p % 2 of step
  // p / 2 (time clamped)
  auto issue_stat = [&](int it) __attribute__((always_inline)) {
    if constexpr (LN) {
      if (lane < 2 * LC) {
        const int k = a.nsc - 1 - it;
        const int t = min(k * kChunk + w * LC + (lane >> 1), Tm1);
        dma_to_lds<4>((const float*)(a.ln_stat + (int64_t)b * a.T + t) + (lane & 1),
                      lds_addr(&stS[LN ? it % NBUF : 0][LN ? w : 0][0]));
      }
    }
  };
  auto issue = [&](int it) __attribute__((always_inline)) {
    const int k = a.nsc - 1 - it;
    issue_stat(it);
    const uint32_t base = slots_lds + (uint32_t)((it % NBUF) * ROWS * 64 * L::BYTES);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int p = i * 64 + lane;
      if (PIECES % 64 == 0 || p < PIECES) {
        const int row = p / P::PPR, pc = p % P::PPR;
        const int col = min(pc, pcmax) * P::EPP;
        const T* src;
        if (row < GROWS) {
          const int j = row / 7, g = row - 7 * (row / 7);
          const int t = min(k * kChunk + w * LC + j, Tm1);
          src = gsrc + (int64_t)t * a.g_td + (int64_t)g * a.g_cd + col;
        } else {
          const int t = min(k * kChunk + w * LC + (row - GROWS), Tm1);
          src = dsrc + (int64_t)t * a.d_bd + col;
        }
        dma_to_lds<PW>(src, base + i * 64 * (PW == 2 ? 4 : PW));
      }
    }
    if (w == 0) {
      dma_to_lds<4>(cksrc + (int64_t)(k * 2) * a.D, lds_addr(&ckS[it & 1][0][0]));
      dma_to_lds<4>(cksrc + (int64_t)(k * 2 + 1) * a.D, lds_addr(&ckS[it & 1][1][0]));
    }
  };
  // Every super-chunk after the first one issued (the tail, k = nsc - 1) lies wholly inside
  // the sequence, so its pieces need no time clamp: each lane's byte offset from the wave's
  // first step is loop-invariant, and a piece is one saddr DMA off a uniform time base.  An
  // instruction's 64 pieces are all gate rows or all dout rows (GROWS * PPR % 64 == 0).
  static_assert((GROWS * P::PPR) % 64 == 0 && PIECES % 64 == 0, "uniform row kind per DMA");
  // The offsets are the same for every wave (the wave's first step is in the uniform base) and
  // live in LDS, not VGPRs: the backward needs every register for its gate-gradient
  // coefficients, and a spilled offset's scratch reload would wait vmcnt(0) on the DMA in flight.
  constexpr int NIF = NI <= 16 ? NI : 1;
  // dgates laid out like gates (always, from the module): the staged gradient stores of a full
  // super-chunk reuse the gate rows' lane offsets
  const bool same_layout = NI <= 16 && a.dg_td == a.g_td && a.dg_cd == a.g_cd;
  __shared__ uint32_t voffT[NIF][64];
  if constexpr (NI <= 16) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (i % NW != w) continue;
      const int p = i * 64 + lane;
      const int row = p / P::PPR, pc = p % P::PPR;
      const int col = min(pc, pcmax) * P::EPP;
      voffT[i][lane] = (uint32_t)(row < GROWS ? (row / 7) * a.g_td + (row % 7) * a.g_cd + col
                                              : (row - GROWS) * a.d_bd + col) *
                       (uint32_t)sizeof(T);
    }
  }
  auto issue_full = [&](int it) __attribute__((always_inline)) {
    const int k = a.nsc - 1 - it;
    issue_stat(it);
    const uint32_t base = slots_lds + (uint32_t)((it % NBUF) * ROWS * 64 * L::BYTES);
    const int64_t t = (int64_t)k * kChunk + w * LC;
    const T* gt = gsrc + t * a.g_td;
    const T* dt = dsrc + t * a.d_bd;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      dma_to_lds_s<PW>((i * 64) / P::PPR < GROWS ? (const void*)gt : (const void*)dt, voffT[i][lane],
                       base + i * 64 * (PW == 2 ? 4 : PW));
    if (w == 0) {
      const float* ck = a.ckpt + ((int64_t)b * a.nsc + k) * 2 * a.D;
      dma_to_lds_s<4>(ck, (uint32_t)dc * 4u, lds_addr(&ckS[it & 1][0][0]));
      dma_to_lds_s<4>(ck + a.D, (uint32_t)dc * 4u, lds_addr(&ckS[it & 1][1][0]));
    }
  };
  // (one-element pieces take 64 instructions per super-chunk: too many offsets to hold)
  auto issue_next = [&](int it) __attribute__((always_inline)) {
    if constexpr (NI <= 16) issue_full(it); else issue(it);
  };
  // bias-gradient partial sums: NBUF = 2 of the fp32 gradients, even / odd steps in the two
  // halves; NBUF = 1 (raw gates held in VGPRs) of the stored values, one register per gate
  f2 bacc[7];
  float bacc1[7];
#pragma unroll
  for (int g = 0; g < 7; ++g) {
    bacc[g] = f2{0.0f, 0.0f};
    bacc1[g] = 0.0f;
  }
  if (a.nsc > 0) issue(0);
  dma_wait();
  lds_barrier();
  // One super-chunk.  FULL: every step is inside the sequence and every lane inside D, so the
  // body carries no per-step conditions (one basic block the scheduler can interleave); the
  // tail super-chunk and a partial column block take the guarded instance.
  auto chunk = [&](int it, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    constexpr int LP = LC / 2;   // step pairs: per-step values live as packed (even, odd) pairs
    const int k = a.nsc - 1 - it;
    const int t0 = k * kChunk + w * LC;
    unsigned char* slot = slots + (it % NBUF) * ROWS * 64 * L::BYTES;
    if (NBUF == 2 && it + 1 < a.nsc) issue_next(it + 1);     // into the other slot
    const float s_ck = ckS[it & 1][0][lane];
    const float h_ck = ckS[it & 1][1][lane];
    f2 zg[LP], dec[LP], u[LP], x[LP], dj[LP], sv[LP], hv[LP], wz[LP];
    // NBUF = 2: the gate-gradient coefficients of step_terms_bwd2 (0-3 stashed in the slot
    // once its raw gates are consumed).  NBUF = 1 refills the slot at once: the raw gates stay
    // in VGPRs and gate_grads2 recomputes from them.
    f2 cf[LP][7];
    float rg[NBUF == 1 ? LC : 1][7];
    // ---- recompute the forward of this super-chunk ----
#pragma unroll
    for (int p = 0; p < LP; ++p) {
      const int j = 2 * p;
      f2 g7[7];
      f2 lrs = {1.0f, 1.0f}, lrm = {0.0f, 0.0f};   // (LN) rstd and -rstd mean of the two steps
      if constexpr (LN) {
        const float2 s0 = stS[LN ? it % NBUF : 0][LN ? w : 0][j];
        const float2 s1 = stS[LN ? it % NBUF : 0][LN ? w : 0][j + 1];
        lrs = f2{s0.x, s1.x};
        lrm = -lrs * f2{s0.y, s1.y};
      }
#pragma unroll
      for (int g = 0; g < 7; ++g) {
        const f2 raw = f2{E::ld(L::get(slot, (j * 7 + g) * 64 + lane)),
                          E::ld(L::get(slot, ((j + 1) * 7 + g) * 64 + lane))};
        if constexpr (LN == 1) {   // rstd (u - mean r) + b', as the forward rebuilt it
          const float2 fb = fbS[LN ? g : 0][lane];
          g7[g] = raw * lrs + (lrm * f2{fb.y, fb.y} + f2{fb.x, fb.x});
        } else if constexpr (LN == 2) {   // (the GEMM applied rstd and mean) + b'
          const float fbx = fbS[LN ? g : 0][lane].x;
          g7[g] = raw + f2{fbx, fbx};
        } else {
          g7[g] = raw + gb[LN ? 0 : g];
        }
        if constexpr (NBUF == 1) {
          rg[j][g] = g7[g].x;
          rg[j + 1][g] = g7[g].y;
        }
      }
      if constexpr (NBUF == 2)
        step_terms_bwd2(g7[0], g7[1], g7[2], g7[3], g7[4], g7[5], g7[6], zg[p], dec[p], u[p],
                        x[p], cf[p]);
      else
        step_terms2(g7[0], g7[1], g7[2], g7[3], g7[4], g7[5], g7[6], zg[p], dec[p], u[p], x[p]);
      dj[p] = f2{E::ld(L::get(slot, (GROWS + j) * 64 + lane)),
                 E::ld(L::get(slot, (GROWS + j + 1) * 64 + lane))};
      if constexpr (!FULL) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          if (t0 + j + h2 >= a.T) {   // identity step past the end of the sequence
            zg[p][h2] = 1.0f; dec[p][h2] = 1.0f; u[p][h2] = 0.0f; x[p][h2] = 0.0f;
            dj[p][h2] = 0.0f;
          }
        }
      }
    }
    // Stash cf0-3 as [pair][coefficient][lane] f2 over the consumed raw gates: the gradient
    // phase reads them back pair by pair before it writes that pair's gradients, whose bytes
    // [1792 p, 1792 (p + 1)) never reach a later pair's stash [2048 p', ...) (p' > p).
    f2* stash = (f2*)slot;
    if constexpr (NBUF == 2) {
#pragma unroll
      for (int p = 0; p < LP; ++p)
#pragma unroll
        for (int c = 0; c < 4; ++c) stash[(p * 4 + c) * 64 + lane] = cf[p][c];
    }
    float As = 1.0f, Bs = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      As *= dec[j >> 1][j & 1];
      Bs = fmaf(dec[j >> 1][j & 1], Bs, u[j >> 1][j & 1]);
    }
    if constexpr (NBUF == 1) {
      lds_read_wait();
      if (it + 1 < a.nsc) issue_next(it + 1);                // refill the slot just read
    }
    // The Gh adjoint depends only on zg and dout, so its segment map is published with the
    // s map (one barrier); Gs needs c = tanh(hn + s) and goes out with the h map.
    float Ph = 1.0f, Qh = 0.0f;   // adjoint of h: C_t = zg_t Gh_t flows to step t-1
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      Qh = zg[j >> 1][j & 1] * (dj[j >> 1][j & 1] + Qh);
      Ph *= zg[j >> 1][j & 1];
    }
    aggA[w][lane] = make_float2(As, Bs);
    aggC[w][lane] = make_float2(Ph, Qh);
    if (!(SC_ABL & 8)) lds_barrier();                          // B1
    float s = s_ck;
    if (!(SC_ABL & 4)) s = compose_prefix<NW>(aggA, lane, w, s);
    // s chain (serial), then c = tanh(hn + s) and (1 - zg) c two steps per instruction
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      sv[j >> 1][j & 1] = s;
      s = fmaf(dec[j >> 1][j & 1], s, u[j >> 1][j & 1]);
      x[j >> 1][j & 1] += s;
    }
#pragma unroll
    for (int p = 0; p < LP; ++p) {
      x[p] = tanh2(x[p]);
      wz[p] = x[p] - zg[p] * x[p];
      if constexpr (NBUF == 2) cf[p][5] *= sv[p];
    }
    float Ah = 1.0f, Bh = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      Ah *= zg[j >> 1][j & 1];
      Bh = fmaf(zg[j >> 1][j & 1], Bh, wz[j >> 1][j & 1]);
    }
    float C = carGh[it & 1][lane];
    if (!(SC_ABL & 4)) C = compose_suffix<NW>(aggC, lane, w, C);
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      u[j >> 1][j & 1] = dj[j >> 1][j & 1] + C;                // Gh_t
      C = zg[j >> 1][j & 1] * u[j >> 1][j & 1];
    }
    if (w == 0) carGh[(it + 1) & 1][lane] = C;
    // dL/d(hn + s_t) = Gh_t (1 - zg_t)(1 - c_t^2), two steps per instruction
    f2 dp[LP];
#pragma unroll
    for (int p = 0; p < LP; ++p) dp[p] = (u[p] - u[p] * zg[p]) * (f2{1.0f, 1.0f} - x[p] * x[p]);
    // adjoint of s: Cs_t = dec_t Gs_t flows to step t-1
    float Ps = 1.0f, Qs = 0.0f;
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      Qs = dec[j >> 1][j & 1] * (dp[j >> 1][j & 1] + Qs);
      Ps *= dec[j >> 1][j & 1];
    }
    aggB[w][lane] = make_float2(Ah, Bh);
    aggD[w][lane] = make_float2(Ps, Qs);
    dma_wait();                   // the next super-chunk (and its checkpoint) has landed
    lds_barrier();                                             // B2
    float h = h_ck;
    if (!(SC_ABL & 4)) h = compose_prefix<NW>(aggB, lane, w, h);
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      if constexpr (NBUF == 2)
        hv[j >> 1][j & 1] = u[j >> 1][j & 1] * (h - x[j >> 1][j & 1]);   // Gh_t (h_{t-1} - c_t)
      else
        hv[j >> 1][j & 1] = h;
      h = fmaf(zg[j >> 1][j & 1], h, wz[j >> 1][j & 1]);
    }
    float Cs = carGs[it & 1][lane];
    if (!(SC_ABL & 4)) Cs = compose_suffix<NW>(aggD, lane, w, Cs);
    f2 gsj[LP];
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {   // the serial part of the Gs scan
      gsj[j >> 1][j & 1] = dp[j >> 1][j & 1] + Cs;
      Cs = dec[j >> 1][j & 1] * gsj[j >> 1][j & 1];
    }
    // gate gradients, two steps per packed instruction
#pragma unroll
    for (int p = 0; p < LP; ++p) {
      const int jp = 2 * p;
      f2 o[7];
      if constexpr (NBUF == 2) {
        const f2 gz = hv[p];   // Gh_t (h_{t-1} - c_t)
        o[0] = gz * stash[(p * 4 + 0) * 64 + lane];
        o[1] = gz * stash[(p * 4 + 1) * 64 + lane];
        o[2] = gsj[p] * stash[(p * 4 + 2) * 64 + lane];
        o[3] = gsj[p] * stash[(p * 4 + 3) * 64 + lane];
        o[4] = dp[p] * cf[p][4];
        o[5] = gsj[p] * cf[p][5];   // cf5 carries s_{t-1} (folded after the s scan)
        o[6] = gsj[p] * cf[p][6];
      } else {
        f2 g7[7];
#pragma unroll
        for (int g = 0; g < 7; ++g) g7[g] = f2{rg[jp][g], rg[jp + 1][g]};
        gate_grads2(g7[0], g7[1], g7[2], g7[3], g7[4], g7[5], g7[6], zg[p], dec[p], u[p], dp[p],
                    gsj[p], hv[p], sv[p], x[p], o);
      }
      if (SC_ABL & 1) {
#pragma unroll
        for (int g = 0; g < 7; ++g) o[g] = gsj[p];
      }
      if constexpr (FULL && NBUF == 2) {
#pragma unroll
        for (int g = 0; g < 7; ++g) bacc[g] += o[g];
      }
      f2 lrs = {1.0f, 1.0f};   // (LN) the stored gradient is d/du = rstd d/dg
      if constexpr (LN) {
        lrs = f2{stS[LN ? it % NBUF : 0][LN ? w : 0][jp].x, stS[LN ? it % NBUF : 0][LN ? w : 0][jp + 1].x};
        if constexpr (FULL) {
#pragma unroll
          for (int g = 0; g < 7; ++g) o[g] *= lrs;
        }
      }
      if constexpr (FULL && WST) {   // both steps' gradients rounded by one v_cvt_pk_bf16_f32
#pragma unroll
        for (int g = 0; g < 7; ++g) {
          const auto pr = Pair<DT>::st(o[g]);
          ((T*)slot)[(jp * 7 + g) * 64 + lane] = pr.x;          // over its raw gate
          ((T*)slot)[((jp + 1) * 7 + g) * 64 + lane] = pr.y;
        }
      } else {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int j = jp + h2;
          if (FULL || (dok && t0 + j < a.T)) {
            const uint32_t so = (uint32_t)((t0 + j) * a.dg_td * sizeof(T));
#pragma unroll
            for (int g = 0; g < 7; ++g) {
              const float og = o[g][h2];
              const T ogt = E::st(LN ? og * lrs[h2] : og);
              if constexpr (WST) ((T*)slot)[(j * 7 + g) * 64 + lane] = ogt;   // over its raw gate
              else if (!(SC_ABL & 2)) dgbuf.st(ogt, vo, so + (uint32_t)(g * a.dg_cd * sizeof(T)));
              if constexpr (NBUF == 1) bacc1[g] += E::ld(ogt);
              else if constexpr (!FULL) bacc[g][h2] += og;
            }
          }
        }
      }
    }
    if constexpr (WST) {   // staged gradients -> HBM in 16-byte pieces (same wave: LDS in order)
      constexpr int SP = LC * 7 * 8;
#pragma unroll
      for (int i = 0; i < (SP + 63) / 64; ++i) {
        const int p = i * 64 + lane;
        if (SP % 64 == 0 || p < SP) {
          const int row = p >> 3, pc = p & 7;
          const int j = row / 7, g = row - 7 * (row / 7);
          if ((FULL || (t0 + j < a.T && pc <= pcmax)) && !(SC_ABL & 2)) {
            const v4u v = *(const v4u*)(slot + p * 16);
            if constexpr (FULL)   // lane offset from the gate DMA table, time in soffset
              __builtin_amdgcn_raw_buffer_store_b128(v, dgbuf.r, voffT[i][lane],
                                                     (uint32_t)(t0 * a.dg_td * sizeof(T)), 0);
            else
              __builtin_amdgcn_raw_buffer_store_b128(   // (a batch row is < 2 GiB: 32-bit math)
                  v, dgbuf.r,
                  ((uint32_t)(t0 + j) * (uint32_t)a.dg_td + (uint32_t)g * (uint32_t)a.dg_cd +
                   (uint32_t)pc * 8u) * (uint32_t)sizeof(T),
                  0, 0);
          }
        }
      }
    }
    if (w == 0) carGs[(it + 1) & 1][lane] = Cs;
  };
  // (WST: the FULL body stores through the gate offset table, so dgates must share the layout)
  const bool blk_full = (blk + 1) * 64 <= a.D && (!WST || same_layout);
  for (int it = 0; it < a.nsc; ++it) {
    // (NBUF = 1 keeps 56 raw gates in VGPRs: the freer schedule of the FULL body would spill)
    if constexpr (NBUF == 2) {
      if (blk_full && (a.nsc - it) * kChunk <= a.T) {
        chunk(it, std::true_type{});
        continue;
      }
    }
    chunk(it, std::false_type{});
  }
  lds_barrier();
  if (w == 0 && dok) {
    a.dh0[(int64_t)b * a.D + d] = carGh[a.nsc & 1][lane];
    a.ds0[(int64_t)b * a.D + d] = carGs[a.nsc & 1][lane];
  }
  if (a.dbias) {   // reduce the per-wave partials over the NW waves (fixed order: deterministic)
#pragma unroll
    for (int g = 0; g < 7; ++g) {
      aggA[w][lane].x = NBUF == 1 ? bacc1[g] : bacc[g].x + bacc[g].y;
      lds_barrier();
      if (w == 0) {
        float acc = 0.0f;
        for (int q = 0; q < NW; ++q) acc += aggA[q][lane].x;
        if (dok) a.dbias[((int64_t)b * 7 + g) * a.D + d] = acc;
      }
      lds_barrier();
    }
  }
}

// ------------------------------------------------------------------------ launchers --------
// 16 waves x 4 steps per wave (one 16-wave workgroup per CU at B*D/64 = 256), every dtype.
#ifndef SC_FWD_NW
#define SC_FWD_NW 16
#endif
constexpr int kNW = SC_FWD_NW, kLC = kChunk / SC_FWD_NW;
#ifndef SC_BWD_NW
#define SC_BWD_NW 8
#endif
constexpr int kBNW = SC_BWD_NW, kBLC = kChunk / SC_BWD_NW;

// > 64 KiB of dynamic LDS must be opted into per kernel (gfx950 has 160 KiB per CU).  Called
// once per kernel instantiation (function-local static): the call costs host time per launch.
template <typename K>
static bool set_lds_limit(K kernel, size_t bytes) {
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes) == hipSuccess;
}

template <int DT, int PW, bool SPLIT = false, int LN = 0, int NB = 8>
static void launch_fwd(const ScanFwdArgs& a, hipStream_t st) {
  using T = typename Elem<DT>::T;
  constexpr int FD = (SC_FWD_FD >= 2 && LdsElem<T, PW>::BYTES == 2) ? 2 : 1;   // 2 x 56 KiB fit
  auto kern = lucy_scan_fwd_kernel<DT, kNW, kLC, PW, FD, SPLIT, LN, NB>;
  const size_t lds = (size_t)FD * kNW * kLC * 7 * 64 * LdsElem<T, PW>::BYTES;
  static const bool lds_ok = set_lds_limit(kern, lds);
  (void)lds_ok;
  dim3 grid((a.D + 63) / 64, a.B);
  hipLaunchKernelGGL(kern, grid, dim3(kNW * 64), lds, st, a);
}

template <int DT, int PW, bool WST, int LN = 0>
static void launch_bwd(const ScanBwdArgs& a, hipStream_t st) {
  using T = typename Elem<DT>::T;
  // two slots per wave fit only for 2-byte LDS elements (160 KiB per CU)
  constexpr int NBUF = LdsElem<T, PW>::BYTES == 2 ? 2 : 1;
  auto kern = lucy_scan_bwd_kernel<DT, kBNW, kBLC, PW, NBUF, WST, LN>;
  const size_t lds = (size_t)NBUF * kBNW * kBLC * 8 * 64 * LdsElem<T, PW>::BYTES;
  static const bool lds_ok = set_lds_limit(kern, lds);
  (void)lds_ok;
  dim3 grid((a.D + 63) / 64, a.B);
  hipLaunchKernelGGL(kern, grid, dim3(kBNW * 64), lds, st, a);
}

// 16-byte pieces need a 16-byte aligned base and every stride and D in whole pieces; otherwise
// pieces of one element (2 or 4 bytes) handle any layout.
static bool wide_pieces(const void* p, int esize, int D, std::initializer_list<int64_t> strides) {
  const int epp = 16 / esize;
  if ((uintptr_t)p % 16 || D % epp) return false;
  for (int64_t s : strides)
    if (s % epp) return false;
  return true;
}

// the LN-fold instances (16-bit gates, 16-byte pieces, D = 64 NB): fold bit 1, records bit 2
template <int DT, bool SPLIT, int NB>
static void dispatch_fwd_ln(const ScanFwdArgs& a, int mode, hipStream_t st) {
  switch (mode) {
    case 1: launch_fwd<DT, 16, SPLIT, 1, NB>(a, st); break;
    case 2: launch_fwd<DT, 16, SPLIT, 2, NB>(a, st); break;
    default: launch_fwd<DT, 16, SPLIT, 3, NB>(a, st); break;
  }
}
template <int DT, bool SPLIT>
static void dispatch_fwd_ln_nb(const ScanFwdArgs& a, int mode, hipStream_t st) {
  if (a.D == 512) dispatch_fwd_ln<DT, SPLIT, 8>(a, mode, st);
  else dispatch_fwd_ln<DT, SPLIT, 16>(a, mode, st);
}

template <int DT>
static void dispatch_fwd(const ScanFwdArgs& a, hipStream_t st) {
  constexpr int es = (int)sizeof(typename Elem<DT>::T);
  const bool wide = wide_pieces(a.gates, es, a.D, {a.g_bt, a.g_td, a.g_cd, a.g_cb});
  if constexpr (es == 2) {
    const int mode = (a.ln_r ? 1 : 0) | (a.rec_out ? 2 : 0);
    if (mode) {   // (scan_fwd checked wide pieces and D)
      if (a.out_lo) dispatch_fwd_ln_nb<DT, true>(a, mode, st);
      else dispatch_fwd_ln_nb<DT, false>(a, mode, st);
      return;
    }
    if (a.out_lo) {
      if (wide) launch_fwd<DT, 16, true>(a, st);
      else launch_fwd<DT, es, true>(a, st);
      return;
    }
  }
  if (wide) launch_fwd<DT, 16>(a, st);
  else launch_fwd<DT, es>(a, st);
}

template <int DT>
static void dispatch_bwd(const ScanBwdArgs& a, hipStream_t st) {
  constexpr int es = sizeof(typename Elem<DT>::T);
  if constexpr (es == 2) {
    if (a.ln_stat) {   // (scan_bwd checked the layout)
      if (a.ln_r) launch_bwd<DT, 16, true, 1>(a, st);
      else launch_bwd<DT, 16, true, 2>(a, st);
      return;
    }
  }
  if (wide_pieces(a.gates, es, a.D, {a.g_bt, a.g_td, a.g_cd, a.g_cb}) &&
      wide_pieces(a.dout, es, a.D, {a.d_bt, a.d_bd})) {
    if (es == 2 && wide_pieces(a.dgates, es, a.D, {a.dg_bt, a.dg_td, a.dg_cd, a.dg_cb}))
      launch_bwd<DT, 16, es == 2>(a, st);
    else
      launch_bwd<DT, 16, false>(a, st);
  } else {
    launch_bwd<DT, es, false>(a, st);
  }
}

}  // namespace sc

using namespace sc;

extern "C" int sc_lucy_scan_chunk(void) { return kChunk; }

extern "C" int64_t sc_lucy_scan_ckpt_numel(int B, int T, int D) {
  if (B < 0 || T < 0 || D < 0) return 0;
  return (int64_t)B * ((T + kChunk - 1) / kChunk) * 2 * D;
}

static int check_dtype(int dt) { return dt == SC_F32 || dt == SC_BF16 || dt == SC_F16; }

struct LnFold {   // sc_lucy_scan_fwd_ln's extra arguments (all NULL: no fold, no records)
  const float* r = nullptr;
  const float* rec_in = nullptr;
  float* stat = nullptr;
  float* rec_out = nullptr;
  float eps = 1e-5f;
};

static int scan_fwd(const void* gates, int gates_dtype, const float* gate_bias, const float* h0,
                    const float* s0, void* out, float* s_out, float* h_out, int B, int T, int D,
                    int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                    int64_t stride_g_cb, int64_t stride_o_bt, int64_t stride_o_bd, float* ckpt,
                    void* out_dup, void* out_lo, void* stream, const LnFold& ln = LnFold{}) {
  SC_REQUIRE(check_dtype(gates_dtype), "sc_lucy_scan_fwd: unsupported gates dtype %d", gates_dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && D >= 0, "sc_lucy_scan_fwd: negative shape B=%d T=%d D=%d", B, T, D);
  SC_REQUIRE(B <= 65535, "sc_lucy_scan_fwd: B=%d exceeds grid limit 65535", B);
  if (B == 0 || D == 0) return 0;
  SC_REQUIRE(h0 && s0 && s_out, "sc_lucy_scan_fwd: null state pointer");
  SC_REQUIRE(T == 0 || (gates && out), "sc_lucy_scan_fwd: null gates/out pointer");
  SC_REQUIRE(stride_g_bt >= 0 && stride_g_td >= 0 && stride_g_cd >= 0 && stride_g_cb >= 0 &&
                 stride_o_bt >= 0 && stride_o_bd >= 0,
             "sc_lucy_scan_fwd: negative stride");
  SC_REQUIRE((int64_t)T * stride_o_bd * 4 < (1ll << 31),
             "sc_lucy_scan_fwd: one batch row of out spans >= 2 GiB");
  if (ln.r || ln.rec_out) {
    const int es = gates_dtype == SC_F32 ? 4 : 2;
    SC_REQUIRE(es == 2, "sc_lucy_scan_fwd_ln: the LayerNorm fold needs 16-bit gates");
    SC_REQUIRE(D == 512 || D == 1024, "sc_lucy_scan_fwd_ln: D=%d must be 512 or 1024", D);
    SC_REQUIRE(wide_pieces(gates, es, D, {stride_g_bt, stride_g_td, stride_g_cd, stride_g_cb}),
               "sc_lucy_scan_fwd_ln: gates must be 16-byte aligned with 16-byte strides");
    SC_REQUIRE(!ln.r || (ln.rec_in && gate_bias), "sc_lucy_scan_fwd_ln: the fold needs rec_in and "
               "the folded bias b' as gate_bias");
  }
  ScanFwdArgs a{gates, gate_bias, h0, s0, out, s_out, h_out, ckpt, B, T, D, (T + kChunk - 1) / kChunk,
                stride_g_bt, stride_g_td, stride_g_cd, stride_g_cb, stride_o_bt, stride_o_bd,
                out_dup, out_lo, ln.r, (const float2*)ln.rec_in, (float2*)ln.stat,
                (float2*)ln.rec_out, ln.eps};
  hipStream_t st = (hipStream_t)stream;
  switch (gates_dtype) {
    case SC_F32: dispatch_fwd<SC_F32>(a, st); break;
    case SC_BF16: dispatch_fwd<SC_BF16>(a, st); break;
    default: dispatch_fwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_lucy_scan_fwd");
}

extern "C" int sc_lucy_scan_fwd(const void* gates, int gates_dtype, const float* gate_bias,
                                const float* h0,
                                const float* s0, void* out, float* s_out, float* h_out, int B,
                                int T, int D,
                                int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                                int64_t stride_g_cb, int64_t stride_o_bt, int64_t stride_o_bd,
                                float* ckpt, void* stream) {
  clear_error();
  return scan_fwd(gates, gates_dtype, gate_bias, h0, s0, out, s_out, h_out, B, T, D, stride_g_bt,
                  stride_g_td, stride_g_cd, stride_g_cb, stride_o_bt, stride_o_bd, ckpt, nullptr,
                  nullptr, stream);
}

extern "C" int sc_lucy_scan_fwd_split(const void* gates, int gates_dtype, const float* gate_bias,
                                      const float* h0, const float* s0, void* out, void* out_dup,
                                      void* out_lo, float* s_out, float* h_out, int B, int T, int D,
                                      int64_t stride_g_bt, int64_t stride_g_td,
                                      int64_t stride_g_cd, int64_t stride_g_cb,
                                      int64_t stride_o_bt, int64_t stride_o_bd, float* ckpt,
                                      void* stream) {
  clear_error();
  SC_REQUIRE(gates_dtype == SC_BF16 || gates_dtype == SC_F16,
             "sc_lucy_scan_fwd_split: the split planes need a 16-bit out (dtype %d)", gates_dtype);
  SC_REQUIRE(T == 0 || (out_dup && out_lo), "sc_lucy_scan_fwd_split: null out_dup/out_lo");
  return scan_fwd(gates, gates_dtype, gate_bias, h0, s0, out, s_out, h_out, B, T, D, stride_g_bt,
                  stride_g_td, stride_g_cd, stride_g_cb, stride_o_bt, stride_o_bd, ckpt, out_dup,
                  out_lo, stream);
}

extern "C" int sc_lucy_scan_fwd_ln(const void* gates, int gates_dtype, const float* gate_bias,
                                   const float* h0, const float* s0, void* out, void* out_dup,
                                   void* out_lo, float* s_out, float* h_out, int B, int T, int D,
                                   int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                                   int64_t stride_g_cb, int64_t stride_o_bt, int64_t stride_o_bd,
                                   float* ckpt, const float* ln_r, const float* ln_rec_in,
                                   float* ln_stat, float* ln_rec_out, float ln_eps, void* stream) {
  clear_error();
  SC_REQUIRE((out_dup == nullptr) == (out_lo == nullptr),
             "sc_lucy_scan_fwd_ln: out_dup and out_lo come together");
  LnFold ln;
  ln.r = ln_r;
  ln.rec_in = ln_rec_in;
  ln.stat = ln_stat;
  ln.rec_out = ln_rec_out;
  ln.eps = ln_eps;
  return scan_fwd(gates, gates_dtype, gate_bias, h0, s0, out, s_out, h_out, B, T, D, stride_g_bt,
                  stride_g_td, stride_g_cd, stride_g_cb, stride_o_bt, stride_o_bd, ckpt, out_dup,
                  out_lo, stream, ln);
}

static int scan_bwd(const void* gates, int gates_dtype, const float* gate_bias, const float* ckpt,
                    const void* dout, const float* ds_last, void* dgates, float* dh0, float* ds0,
                    float* dbias, int B, int T, int D, int64_t stride_g_bt, int64_t stride_g_td,
                    int64_t stride_g_cd, int64_t stride_g_cb, int64_t stride_d_bt,
                    int64_t stride_d_bd, int64_t stride_dg_bt, int64_t stride_dg_td,
                    int64_t stride_dg_cd, int64_t stride_dg_cb, const float* ln_r,
                    const float* ln_stat, void* stream);

extern "C" int sc_lucy_scan_bwd(const void* gates, int gates_dtype, const float* gate_bias,
                                const float* ckpt,
                                const void* dout, const float* ds_last, void* dgates, float* dh0,
                                float* ds0, float* dbias, int B, int T, int D, int64_t stride_g_bt,
                                int64_t stride_g_td, int64_t stride_g_cd, int64_t stride_g_cb,
                                int64_t stride_d_bt, int64_t stride_d_bd, int64_t stride_dg_bt,
                                int64_t stride_dg_td, int64_t stride_dg_cd, int64_t stride_dg_cb,
                                void* stream) {
  clear_error();
  return scan_bwd(gates, gates_dtype, gate_bias, ckpt, dout, ds_last, dgates, dh0, ds0, dbias, B,
                  T, D, stride_g_bt, stride_g_td, stride_g_cd, stride_g_cb, stride_d_bt,
                  stride_d_bd, stride_dg_bt, stride_dg_td, stride_dg_cd, stride_dg_cb, nullptr,
                  nullptr, stream);
}

extern "C" int sc_lucy_scan_bwd_ln(const void* gates, int gates_dtype, const float* gate_bias,
                                   const float* ckpt, const void* dout, const float* ds_last,
                                   void* dgates, float* dh0, float* ds0, float* dbias, int B, int T,
                                   int D, int64_t stride_g_bt, int64_t stride_g_td,
                                   int64_t stride_g_cd, int64_t stride_g_cb, int64_t stride_d_bt,
                                   int64_t stride_d_bd, int64_t stride_dg_bt, int64_t stride_dg_td,
                                   int64_t stride_dg_cd, int64_t stride_dg_cb, const float* ln_r,
                                   const float* ln_stat, void* stream) {
  clear_error();
  SC_REQUIRE(ln_stat && gate_bias, "sc_lucy_scan_bwd_ln: null ln_stat / gate_bias");
  SC_REQUIRE(gates_dtype != SC_F32, "sc_lucy_scan_bwd_ln: the LayerNorm fold needs 16-bit gates");
  SC_REQUIRE((D == 512 || D == 1024) && wide_pieces(gates, 2, D, {stride_g_bt, stride_g_td, stride_g_cd, stride_g_cb}) &&
                 wide_pieces(dout, 2, D, {stride_d_bt, stride_d_bd}) &&
                 wide_pieces(dgates, 2, D, {stride_dg_bt, stride_dg_td, stride_dg_cd, stride_dg_cb}),
             "sc_lucy_scan_bwd_ln: 16-byte aligned gates / dout / dgates with 16-byte strides, "
             "D = 512 or 1024");
  return scan_bwd(gates, gates_dtype, gate_bias, ckpt, dout, ds_last, dgates, dh0, ds0, dbias, B,
                  T, D, stride_g_bt, stride_g_td, stride_g_cd, stride_g_cb, stride_d_bt,
                  stride_d_bd, stride_dg_bt, stride_dg_td, stride_dg_cd, stride_dg_cb, ln_r,
                  ln_stat, stream);
}

static int scan_bwd(const void* gates, int gates_dtype, const float* gate_bias, const float* ckpt,
                    const void* dout, const float* ds_last, void* dgates, float* dh0, float* ds0,
                    float* dbias, int B, int T, int D, int64_t stride_g_bt, int64_t stride_g_td,
                    int64_t stride_g_cd, int64_t stride_g_cb, int64_t stride_d_bt,
                    int64_t stride_d_bd, int64_t stride_dg_bt, int64_t stride_dg_td,
                    int64_t stride_dg_cd, int64_t stride_dg_cb, const float* ln_r,
                    const float* ln_stat, void* stream) {
  SC_REQUIRE(check_dtype(gates_dtype), "sc_lucy_scan_bwd: unsupported gates dtype %d", gates_dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && D >= 0, "sc_lucy_scan_bwd: negative shape B=%d T=%d D=%d", B, T, D);
  SC_REQUIRE(B <= 65535, "sc_lucy_scan_bwd: B=%d exceeds grid limit 65535", B);
  if (B == 0 || D == 0) return 0;
  SC_REQUIRE(dh0 && ds0, "sc_lucy_scan_bwd: null dh0/ds0");
  if (T == 0 && dbias) zero_async(dbias, sizeof(float) * 7 * B * D, (hipStream_t)stream);
  SC_REQUIRE(T == 0 || (gates && ckpt && dout && dgates),
             "sc_lucy_scan_bwd: null gates/ckpt/dout/dgates pointer");
  SC_REQUIRE(stride_g_bt >= 0 && stride_g_td >= 0 && stride_g_cd >= 0 && stride_g_cb >= 0 &&
                 stride_d_bt >= 0 && stride_d_bd >= 0 && stride_dg_bt >= 0 && stride_dg_td >= 0 &&
                 stride_dg_cd >= 0 && stride_dg_cb >= 0,
             "sc_lucy_scan_bwd: negative stride");
  SC_REQUIRE(((int64_t)T * stride_dg_td + 7 * stride_dg_cd) * 4 < (1ll << 31),
             "sc_lucy_scan_bwd: one batch row of dgates spans >= 2 GiB");
  ScanBwdArgs a{gates, gate_bias, ckpt, dout, ds_last, dgates, dh0, ds0, dbias, B, T, D,
                (T + kChunk - 1) / kChunk,
                stride_g_bt, stride_g_td, stride_g_cd, stride_g_cb, stride_d_bt, stride_d_bd,
                stride_dg_bt, stride_dg_td, stride_dg_cd, stride_dg_cb, ln_r,
                (const float2*)ln_stat};
  hipStream_t st = (hipStream_t)stream;
  switch (gates_dtype) {
    case SC_F32: dispatch_bwd<SC_F32>(a, st); break;
    case SC_BF16: dispatch_bwd<SC_BF16>(a, st); break;
    default: dispatch_bwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_lucy_scan_bwd");
}
