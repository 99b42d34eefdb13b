// CTC loss forward (alpha, beta, nll) and gradient for gfx950, with log_softmax fused.
//
// Replaces the reference's loss layer `enc_out.log_softmax(-1).transpose(0,1)` +
// nn.CTCLoss(blank=0, zero_infinity=True) (model.py:68-71, train.py:142), i.e. ATen's
// ctc_loss/_ctc_loss_backward.  Semantics kept: blank-extended label sequence of 2U+1 states,
// log-space recursions, nll = -log p(l|x) (+inf when infeasible), gradient
//   grad[t,v] = scale_b * (exp(lp[t,v]) - exp(lcab[t,v] + nll - lp[t,v]))   (t < in_len)
// which ATen returns for log-prob inputs and which equals d nll / d logits when the
// log_softmax is fused (is_logits=1).  The time axis is never transposed: x stays [B,T,V].
//
// Kernels (all on the caller's stream):
//   ctc_emit_kernel   one wave per (b,t) row: log-sum-exp over V (logits only), then the
//                     emission log-probs of the row's 2U+1 states, base 2, into lpe[b,t,:],
//                     shifted by the row's largest one, c_t (kept in cst[b,t]).  Every path takes
//                     exactly one emission per frame, so the shift moves every path by the same
//                     sum_t c_t: exact, and it keeps the lattice's fp32 values near 0, where their
//                     rounding is small (unshifted, a value ~ -10 bits per step away from its
//                     re-centring carried 3e-3 of relative error into the T=1500 posteriors;
//                     tools/ctc_precision.py)
//   ctc_chain_kernel  per b: for every target position the next position with the same label,
//                     so label occupancies are summed in a fixed order (deterministic, no atomics)
//   ctc_lin_kernel    (Umax <= 255, SC_CTC_LIN=1) the lattice in linear probability space, fp64,
//                     renormalised every 16 steps by exact powers of two: five full-rate fp64
//                     adds / multiplies per state pair and step instead of five exp2 / log2; one
//                     wave computes, two more store its rows as fp32 logs (lin_produce /
//                     lin_consume); a sequence with an emission or a wave that would underflow
//                     goes to ctc_x64_kernel
//   ctc_ab_kernel     (the default) one workgroup per (sequence, direction): 2B workgroups run alpha forward
//                     and beta backward concurrently.  Two states (a blank and its label) per
//                     lane; each wave also carries a K-pair halo of its neighbour's pairs so it
//                     advances K steps with DPP wave_shr:1 / wave_shl:1 only (no LDS, no
//                     barrier), then exchanges halos through LDS.  Emission rows are prefetched
//                     16 steps ahead.
//                     Values live in base-2 log space with a finite "dead" sentinel (branch-free
//                     log-sum-exp) and are re-centred on the workgroup max every 16 steps; the
//                     running offset is kept in fp64 (at T=1500 |alpha| ~ 1e4, where an fp32
//                     ulp would put ~0.5% error into the posteriors).
//                     A re-centring that finds the maximum more than kDrift bits below the last
//                     one flags the sequence (sharp[b]): its fp32 values have drifted far enough
//                     from 0 that their rounding reaches the posteriors
//   ctc_x64_kernel    (flagged sequences, U <= 255) the lattice again, exactly: one wave, values
//                     as fp64 mantissa + int exponent (no under- or overflow), emissions from the
//                     logits in fp64, rows stored relative to each step's largest value
//   ctc_grad_kernel   one wave per (b,t) row: label occupancies into an LDS row of V
//                     log-sums, then one coalesced 16-byte pass writing the gradient row
#include "sc_common.h"

#ifndef SC_CTC_ABL   // ablation bitmask (timing studies only; results are wrong when set):
#define SC_CTC_ABL 0  // 1 no halo exchange, 2 no per-step stores, 4 max instead of log-sum-exp,
#endif                // (ctc_lin_kernel) 8 no renormalisation, 16 no emission loads
#ifndef SC_CTC_KMAX   // most steps between halo exchanges (8 or 16)
#define SC_CTC_KMAX 16
#endif
// SC_CTC_FLAGX: the halo exchanges that do not re-centre hand the halo to the one neighbour that
// reads it through an LDS flag (the writer's exchange count) instead of a workgroup barrier; the
// re-centring exchanges keep the barrier (they need the workgroup maximum).  0: every exchange
// on the barrier (A/B only).
// Measured (tools/r5_ctc.sh, scan_bench ctc_fwd at C2 size, alternated): flags 233.6 us vs
// barriers 211.6 us -- the chained waits (wave w on w - 1 on w - 2 ...) cost more than the
// barrier they replace, so the barrier stays.
#ifndef SC_CTC_FLAGX
#define SC_CTC_FLAGX 0
#endif
// SC_CTC_WMV: 1 = the re-centring exchange reads the wave maxima as float4s.  Measured slower
// (tools/r5_pc.sh, scan_bench ctc_fwd: 211.4-212.0 us vs 199.9-200.0 us for the scalar loop)
#ifndef SC_CTC_WMV
#define SC_CTC_WMV 0
#endif
#ifndef SC_CTC_FLAG_SLEEP   // (SC_CTC_FLAGX) s_sleep in the flag spin
#define SC_CTC_FLAG_SLEEP 1
#endif

namespace sc {

constexpr float kNegInf = -__builtin_huge_valf();

struct CtcWs {
  float* lse;     // [B,T]      natural-log row normaliser (logits input)
  double* lse64;  // [B,T]      the same, row max + log(sum) kept in fp64 (the exact lattice and
                  //            the gradient's log-probs: an fp32 lse of a row ~1e3 is 6e-5 off)
  float* lpe;     // [B,T,Sp]   base-2 emission log-probs of the blank-extended states
  float* alpha;   // [B,T,Sp]   base-2, relative to offA
  float* beta;    // [B,T,Sp]   base-2, relative to offB
  double* offA;   // [B,T+1]    base-2 offsets: entry n = offset after the n-th re-centring (at
  double* offB;   // [B,T+1]    step i = 2Kn - 1 of the direction), so step i has entry (i+1)/2K
                  //            (the exact lattice re-centres every step: entry i + 1)
  float* cst;     // [B,T]      base-2 per-row emission shift c_t (lpe = log2 p - c_t)
  double* ll2s;   // [B]        base-2 log-likelihood of the SHIFTED lattice (log2 p - sum_t c_t)
  int* chain;     // [B,Um]
  int* first;     // [B,Um]
  // one-wave family (Umax <= 255) only:
  float* ylin;    // [B,T,Sp]   linear shifted emissions 2^(lpe) (0: dead)
  int* flag;      // [B]        a live emission below 2^-kTiny: the linear lattice is not used
  int* sharp;     // [B]        the log-space lattice drifted more than kDrift bits between two
                  //            re-centrings: ctc_x64_kernel recomputes the sequence exactly
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// states per lane for a given max state count
static int states_per_lane(int S) { return (S + 63) / 64; }

static int lin_ppl(int Umax);

static size_t ws_layout(int B, int T, int Umax, CtcWs* w, void* base) {
  const int S = 2 * Umax + 1;
  const int Sp = 64 * states_per_lane(S);
  const bool lin = lin_ppl(Umax) > 0;
  const size_t ab = 4;   // alpha / beta: fp32 base-2 log rows (every lattice)
  const int Um = Umax > 0 ? Umax : 1;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p + off;
    off += align256(bytes);
    return (void*)r;
  };
  CtcWs t;
  t.lse = (float*)take((size_t)B * T * 4);
  t.lse64 = (double*)take((size_t)B * T * 8);
  t.lpe = (float*)take((size_t)B * T * Sp * 4);
  t.alpha = (float*)take((size_t)B * T * Sp * ab);
  t.beta = (float*)take((size_t)B * T * Sp * ab);
  t.offA = (double*)take((size_t)B * (T + 1) * 8);
  t.offB = (double*)take((size_t)B * (T + 1) * 8);
  t.cst = (float*)take((size_t)B * T * 4);
  t.ll2s = (double*)take((size_t)B * 8);
  t.chain = (int*)take((size_t)B * Um * 4);
  t.first = (int*)take((size_t)B * Um * 4);
  t.ylin = lin ? (float*)take((size_t)B * T * Sp * 4) : nullptr;
  t.flag = lin ? (int*)take((size_t)B * 4) : nullptr;
  t.sharp = (int*)take((size_t)B * 4);
  if (w) *w = t;
  return off;
}

// log2(2^a + 2^b), base-2 log-sum-exp
__device__ __forceinline__ float lse2_b2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == kNegInf) return kNegInf;
  return m + log2_(exp2_(a - m) + exp2_(b - m));
}


struct CtcArgs {
  const void* x;
  int is_logits, B, T, V, S, Sp, Umax, blank;
  int kh;   // steps between halo exchanges of ctc_ab_kernel (re-centring every 2 kh steps)
  int lin;      // the linear-domain lattice (ctc_lin_kernel) runs
  int64_t sb, stt;
  const int64_t* tg;
  int64_t tgs;
  const int64_t* in_lens;
  const int64_t* tgt_lens;
  float* nll;
  CtcWs ws;
  const float* scale;
  void* grad;
  // optional emission logits (sc_ctc_*_ex): ex[b][t][0] the blank's logit, ex[b][t][1 + u] label
  // u's, fp32 — what the lattice and the gradient's emission columns read instead of x
  const float* ex;
  int64_t exb, ext;
};

__device__ __forceinline__ int clampi(int64_t v, int lo, int hi) {
  return (int)(v < lo ? lo : (v > hi ? hi : v));
}

// label of blank-extended state s (clamped into [0, V) so no load leaves the row; out-of-range
// targets are undefined input, as in ATen)
__device__ __forceinline__ int state_label(const int64_t* tg, int s, int blank, int V) {
  int lab = (s & 1) ? (int)tg[(s - 1) >> 1] : blank;
  return lab < 0 ? 0 : (lab >= V ? V - 1 : lab);
}

// ---------------------------------------------------------------------------- emissions -----
constexpr float kTiny = 120.0f;   // (2^-120: a normal fp32 with 6 bits of headroom)

template <int DT>
__global__ void __launch_bounds__(256) ctc_emit_kernel(CtcArgs a) {
  using E = Elem<DT>;
  using T = typename E::T;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)a.B * a.T) return;
  const int b = (int)(row / a.T), t = (int)(row % a.T);
  if (t >= clampi(a.in_lens[b], 0, a.T)) return;     // rows past in_len are never read
  const T* p = (const T*)a.x + (int64_t)b * a.sb + (int64_t)t * a.stt;
  const int Sb = 2 * clampi(a.tgt_lens[b], 0, a.Umax) + 1;
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  const float* exr = a.ex ? a.ex + (int64_t)b * a.exb + (int64_t)t * a.ext : nullptr;
  // the row's state logits, gathered ONCE and before the row reduction (their loads overlap
  // it): up to kGx per lane in registers (Sp <= 512, U <= 255), else gathered again below
  constexpr int kGx = 8;
  auto state_logit = [&](int s) {
    // (ex column: 0 for the blank states, 1 + u for label state 2u + 1)
    return exr ? exr[(s & 1) ? (s + 1) >> 1 : 0] : E::ld(p[state_label(tg, s, a.blank, a.V)]);
  };
  const bool inreg = a.Sp <= 64 * kGx;
  float xs[kGx];
  if (inreg) {   // (clamped states: every load unconditional, all in flight together)
    if (exr) {
#pragma unroll
      for (int j = 0; j < kGx; ++j) {
        const int s = min(lane + 64 * j, Sb - 1);
        xs[j] = exr[(s & 1) ? (s + 1) >> 1 : 0];
      }
    } else {
      int lab[kGx];
#pragma unroll
      for (int j = 0; j < kGx; ++j) lab[j] = state_label(tg, min(lane + 64 * j, Sb - 1), a.blank, a.V);
#pragma unroll
      for (int j = 0; j < kGx; ++j) xs[j] = E::ld(p[lab[j]]);
    }
  }
  float lse = 0.0f;
  if (a.is_logits) {
    float m = kNegInf, l = 0.0f;
    constexpr int N = Vec16<DT>::N;
    if ((a.V % N) == 0 && ((uintptr_t)p & 15) == 0) {   // 16-byte loads (online max per chunk)
      for (int c = lane; c < a.V / N; c += 64) {
        float xv[N];
        Vec16<DT>::ld(p + N * c, xv);
        float cm = xv[0];
#pragma unroll
        for (int k = 1; k < N; ++k) cm = fmaxf(cm, xv[k]);
        const float mn = fmaxf(m, cm);
        float cs = 0.0f;
#pragma unroll
        for (int k = 0; k < N; ++k) cs += fexp(xv[k] - mn);
        l = l * fexp(m - mn) + cs;
        m = mn;
      }
    } else {
      for (int v = lane; v < a.V; v += 64) {
        const float xv = E::ld(p[v]);
        const float mn = fmaxf(m, xv);
        l = l * fexp(m - mn) + fexp(xv - mn);
        m = mn;
      }
    }
    // the row max, then every lane's partial sum rescaled to it and summed (NaN in l
    // propagates as before)
    const float M = wave_max_dpp(m);
    l = wave_sum_dpp(m == kNegInf ? 0.0f : l * fexp(m - M));
    lse = M + flog(l);
    if (lane == 0) {
      a.ws.lse[row] = lse;
      a.ws.lse64[row] = (double)M + (double)flog(l);
    }
  }
  float* out = a.ws.lpe + row * a.Sp;
  auto lp2x = [&](float xl) { return fmaxf((xl - lse) * kLog2e, -1e30f); };
  auto lp2 = [&](int s) { return lp2x(state_logit(s)); };
  float c = -1e30f;
  if (inreg) {
#pragma unroll
    for (int j = 0; j < kGx; ++j)
      if (lane + 64 * j < Sb) c = fmaxf(c, lp2x(xs[j]));
  } else {
    for (int s = lane; s < Sb; s += 64) c = fmaxf(c, lp2(s));
  }
  c = wave_max_dpp(c);
  if (!(c > -1e29f)) c = 0.0f;   // every state dead (or NaN): no shift, the sentinel stays
  bool tiny = false;
  auto put = [&](int s, float e) {
    out[s] = e;
    if (a.lin) {
      // linear emission for ctc_lin_kernel; a live one below 2^-kTiny sends the sequence to the
      // log-space lattice (fp32 would lose it, and it may carry every path)
      tiny |= e > -1e29f && e < -kTiny;
      a.ws.ylin[row * a.Sp + s] = e > -1e29f ? exp2_(e) : 0.0f;
    }
  };
  if (inreg) {
#pragma unroll
    for (int j = 0; j < kGx; ++j) {
      const int s = lane + 64 * j;
      if (s < a.Sp) put(s, s < Sb ? fmaxf(lp2x(xs[j]) - c, -1e30f) : -1e30f);
    }
  } else {
    for (int s = lane; s < a.Sp; s += 64) put(s, s < Sb ? fmaxf(lp2(s) - c, -1e30f) : -1e30f);
  }
  if (lane == 0) a.ws.cst[row] = c;
  if (a.lin && __ballot(tiny) && lane == 0) a.ws.flag[b] = 1;   // (every writer stores 1)
}

// ---------------------------------------------------------------------------- chains --------
__global__ void __launch_bounds__(256) ctc_chain_kernel(CtcArgs a) {
  // one wave per target position u (4 per workgroup): the next and any earlier position with
  // the same label, 64 candidates per ballot
  __shared__ int lt[1024];   // the target row (Umax <= 1007)
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  const int Um = a.Umax > 0 ? a.Umax : 1;
  for (int u = threadIdx.x; u < Ub; u += blockDim.x) lt[u] = (int)tg[u];
  __syncthreads();
  if (blockIdx.y == 0 && threadIdx.x == 0) a.ws.sharp[b] = 0;   // (ctc_ab's drift flag)
  const int u = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (u >= Um) return;
  int nxt = -1, first = 0;
  if (u < Ub) {
    const int lab = lt[u];
    for (int q0 = u + 1; q0 < Ub; q0 += 64) {
      const int q = q0 + lane;
      const unsigned long long hit = __ballot(q < Ub && lt[q] == lab);
      if (hit) {
        nxt = q0 + __ffsll(hit) - 1;
        break;
      }
    }
    first = 1;
    for (int q0 = 0; q0 < u; q0 += 64) {
      const int q = q0 + lane;
      if (__ballot(q < u && lt[q] == lab)) {
        first = 0;
        break;
      }
    }
  }
  if (lane == 0) {
    a.ws.chain[(int64_t)b * Um + u] = nxt;
    a.ws.first[(int64_t)b * Um + u] = first;
  }
}

// ---------------------------------------------------------------------------- alpha / beta --
__device__ __forceinline__ float shr1(float v) {   // value of lane-1 (lane 0: dead)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-1e30f), __float_as_int(v),
                                                     0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float shl1(float v) {   // value of lane+1 (lane 63: dead)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-1e30f), __float_as_int(v),
                                                     0x130, 0xf, 0xf, false));
}

// Branch-free log2-sum-exp for the lattice: "dead" states carry kDead (finite), so no -inf
// test is needed; exp2 of anything ~kDead below the max is exactly 0.
constexpr float kDead = -1e30f;
// a re-centring that finds the lattice's maximum this many bits below the last one sends the
// sequence to the exact lattice (ctc_x64_kernel): |values| ~ 512 round by ~3e-5 per step
constexpr float kDrift = 512.0f;
__device__ __forceinline__ float lse3_live(float a, float b, float c) {
  const float m = fmaxf(fmaxf(a, b), c);
  if (SC_CTC_ABL & 4) return m;
  // the max term is exp2(0) = 1: two exponentials (median and minimum), not three
  const float md = __builtin_amdgcn_fmed3f(a, b, c);
  const float lo = fminf(fminf(a, b), c);
  return m + log2_(1.0f + exp2_(md - m) + exp2_(lo - m));
}

constexpr int kAbP = 16;   // emission prefetch depth (steps)

#ifndef SC_CTC_V2   // 1: lattice step without canonicalising max/min, emission selects or a swap
#define SC_CTC_V2 1
#endif
// max / min / max3 / min3 as single instructions: fmaxf & co. make LLVM canonicalise loop-carried
// operands first (one extra v_max per value per step); the lattice never holds NaN it must quiet
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// lane shifts with bound_ctrl: the lane with no source neighbour reads 0, not a "dead" value.
// That lane is always a halo lane (alpha: lane 0, beta: lane 63 of every wave), whose values
// are never published and are overwritten at each exchange; saves the v_mov of an old value.
__device__ __forceinline__ float shr1z(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float shl1z(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}
typedef float f2v __attribute__((ext_vector_type(2)));
// (lse2(a2, b2) + e.x, lse3(a3, b3, c3) + e.y) in base 2: the max terms are exp2(0) = 1; the
// emission pair joins the maxima while the exponentials run, and the two results leave as one
// packed pair (what the store and the next step's DPP read)
__device__ __forceinline__ f2v lse23(float a2, float b2, float a3, float b3, float c3, f2v e) {
  const float m2 = vmax(a2, b2), l2 = vmin(a2, b2);
  const float m3 = vmax3(a3, b3, c3), d3 = __builtin_amdgcn_fmed3f(a3, b3, c3);
  const float l3 = vmin3(a3, b3, c3);
  const f2v me = f2v{m2, m3} + e;
  const f2v s = f2v{1.0f, 1.0f} + f2v{exp2_(l2 - m2), exp2_(d3 - m3)};
  return me + f2v{log2_(s.x), log2_(s.y + exp2_(l3 - m3))};
}


__device__ __forceinline__ float lse2_live(float a, float b) {
  const float m = fmaxf(a, b);
  if (SC_CTC_ABL & 4) return m;
  return m + log2_(1.0f + exp2_(fminf(a, b) - m));
}

// One workgroup per (sequence, direction).  Each lane holds a PAIR of blank-extended states,
// p -> (blank 2p, label 2p+1), so one step is
//   alpha:  B' = lse(B, L[p-1]) + e(2p);    L' = lse(L, B, skip ? L[p-1] : dead) + e(2p+1)
//   beta:   B' = lse(B, L) + e(2p);         L' = lse(L, B[p+1], skip ? L[p+1] : dead) + e(2p+1)
// i.e. one DPP lane shift (two independent ones for beta) and two independent log-sum-exps per
// step, half the lanes of a state-per-lane layout.  Wave w computes 64 consecutive pairs: OW =
// 64 - K it OWNS plus a K-pair halo owned by the neighbouring wave (left for alpha, right for
// beta); a missing neighbour corrupts one more halo pair per step, so for K steps the owned
// pairs stay exact with no communication, then they are published to LDS, one barrier, and the
// halo lanes re-read theirs (every second such exchange also re-centres on the workgroup max).
template <int K, bool BETA>
__device__ __forceinline__ void ab_run(const CtcArgs& a, int b, int Tb, int Ub) {
  constexpr int OW = 64 - K;      // owned pairs per wave
  constexpr int kAbP = K > 16 ? K : 16;   // emission prefetch depth: a multiple of K
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = uniform(tid >> 6);
  const int nw = blockDim.x >> 6;
  const int p = BETA ? w * OW + lane : w * OW + lane - K;
  const bool own = BETA ? (lane < OW) : (lane >= K);
  const bool liveB = p >= 0 && p <= Ub;    // state 2p   < 2Ub + 1
  const bool liveL = p >= 0 && p < Ub;     // state 2p+1 < 2Ub + 1
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  bool skip = false;   // alpha: 2p-1 -> 2p+1 allowed;  beta: 2p+3 -> 2p+1 allowed
  if (liveL) {
    const int lab = (int)tg[p];
    if (!BETA) {
      skip = p >= 1 && lab != a.blank && lab != (int)tg[p - 1];
    } else if (p + 1 < Ub) {
      const int l2 = (int)tg[p + 1];
      skip = l2 != a.blank && l2 != lab;
    }
  }
  extern __shared__ __attribute__((aligned(16))) float2 full2[];   // [2][nw*OW] published pairs
  __shared__ __attribute__((aligned(16))) float wmax[16];
  __shared__ int xflag[16];   // (SC_CTC_FLAGX) exchanges published by each wave
  if (SC_CTC_FLAGX) {
    if (tid < 16) xflag[tid] = 0;
    lds_barrier();
  }
  const int nst = nw * OW;
  const int pc = p < 0 ? 0 : (2 * p >= a.Sp ? a.Sp / 2 - 1 : p);   // clamped for addressing only
  const float2* lrow = (const float2*)(a.ws.lpe + (int64_t)b * a.T * a.Sp) + pc;
  const int64_t rs = a.Sp / 2;   // row stride in pairs
  // Per-step outputs through buffer descriptors: lanes that must not write (halo lanes, pairs
  // past the row; every lane but 0 for the offset) get an out-of-range offset, which the buffer
  // unit drops, so the stores need no exec-mask branch in the step loop.
  constexpr uint32_t kDrop = 0x80000000u;
  const uint32_t rowb = (uint32_t)(a.Sp * 4);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (BETA ? a.ws.beta : a.ws.alpha) + (int64_t)b * a.T * a.Sp, 0, (int)(rowb * (uint32_t)a.T),
      0x00020000);
  const uint32_t ovo = (own && 2 * p < a.Sp) ? (uint32_t)(8 * pc) : kDrop;
  double* offn = (BETA ? a.ws.offB : a.ws.offA) + (int64_t)b * (a.T + 1);
  if (tid == 0) offn[0] = 0.0;
  auto tstep = [&](int i) { return BETA ? Tb - 1 - i : i; };
  float2 bufA[kAbP], bufB[kAbP];
#if SC_CTC_V2
  // emission pairs through a buffer descriptor: lanes outside the row (alpha's leading halo,
  // pairs past Sp) get an out-of-range offset and read 0, which keeps a dead state dead (its
  // inputs are all dead); live lanes past 2 Ub + 1 read the -1e30 padding ctc_emit wrote
  const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
      a.ws.lpe + (int64_t)b * a.T * a.Sp, 0, (int)(rowb * (uint32_t)a.T), 0x00020000);
  const uint32_t evo = (p >= 0 && 2 * p < a.Sp) ? (uint32_t)(8 * p) : kDrop;
  auto load = [&](float2 (&buf)[kAbP], int i0) {
#pragma unroll
    for (int j = 0; j < kAbP; ++j)
      buf[j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                                              ers, evo, (uint32_t)tstep(min(i0 + j, Tb - 1)) * rowb, 0));
  };
#else
  auto load = [&](float2 (&buf)[kAbP], int i0) {
#pragma unroll
    for (int j = 0; j < kAbP; ++j) buf[j] = lrow[(int64_t)tstep(min(i0 + j, Tb - 1)) * rs];
  };
#endif
  auto emit = [&](int t, float vB, float vL) {
    __builtin_amdgcn_raw_buffer_store_b64(
        __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, make_float2(vB, vL)), ors,
        ovo, (uint32_t)t * rowb, 0);
  };
  float vB = kDead, vL = kDead;
  double off = 0.0;
  int exch = 0;
  auto body = [&](const float2 (&buf)[kAbP], int i0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < kAbP; ++j) {
      const int i = i0 + j;
      if (i >= Tb) break;
#if SC_CTC_V2
      if (i == 0) {
        vB = (liveB && p == (BETA ? Ub : 0)) ? buf[j].x : kDead;
        vL = (liveL && p == (BETA ? Ub - 1 : 0)) ? buf[j].y : kDead;
      } else if (!BETA) {
        const float lp = shr1z(vL);
        const f2v r = lse23(vB, lp, vL, vB, skip ? lp : kDead, f2v{buf[j].x, buf[j].y});
        vB = r.x;
        vL = r.y;
      } else {
        const float bn = shl1z(vB);
        const float ln = shl1z(vL);
        const f2v r = lse23(vB, vL, vL, bn, skip ? ln : kDead, f2v{buf[j].x, buf[j].y});
        vB = r.x;
        vL = r.y;
      }
#else
      const float eB = liveB ? buf[j].x : kDead;
      const float eL = liveL ? buf[j].y : kDead;
      if (i == 0) {
        vB = (liveB && p == (BETA ? Ub : 0)) ? eB : kDead;
        vL = (liveL && p == (BETA ? Ub - 1 : 0)) ? eL : kDead;
      } else if (!BETA) {
        const float lp = shr1(vL);
        const float nB = lse2_live(vB, lp) + eB;
        vL = lse3_live(vL, vB, skip ? lp : kDead) + eL;
        vB = nB;
      } else {
        const float bn = shl1(vB);
        const float ln = shl1(vL);
        const float nB = lse2_live(vB, vL) + eB;
        vL = lse3_live(vL, bn, skip ? ln : kDead) + eL;
        vB = nB;
      }
#endif
      if (!(SC_CTC_ABL & 1) && j % K == K - 1) {   // halo exchange (+ re-centre every 2nd)
        const int par = exch & 1;
        const bool norm = par == 1;
        if (own) full2[par * nst + p] = make_float2(vB, vL);
        // (buffer 0 is written only at the exchanges that do not re-centre: the barrier of the
        // re-centring exchange between two of them orders every read before the next write)
        if (SC_CTC_FLAGX && !norm) {
          // the halo comes from one neighbour (alpha: wave w - 1, beta: w + 1): publish this
          // wave's count after its pairs (one wave's LDS operations complete in order), then wait
          // for the neighbour's
          lds_read_wait();   // (every lane's pairs written before lane 0's count)
          if (lane == 0)
            __hip_atomic_store(&xflag[w], exch + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int nb = BETA ? w + 1 : w - 1;
          if (nb >= 0 && nb < nw) {
            while (__hip_atomic_load(&xflag[nb], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= exch)
              if (SC_CTC_FLAG_SLEEP) __builtin_amdgcn_s_sleep(1);
          }
          if (!own) {
            const bool has = p >= 0 && p < nst;
            const float2 q = has ? full2[par * nst + p] : make_float2(kDead, kDead);
            vB = q.x;
            vL = q.y;
          }
          ++exch;
          if (!(SC_CTC_ABL & 2)) emit(tstep(i), vB, vL);
          continue;
        }
        if (norm) {
          float m = own ? fmaxf(vB, vL) : kDead;
#if SC_CTC_V2
          m = wave_max_dpp(m);
#else
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
#endif
          if (lane == 0) wmax[w] = m;
        }
        lds_barrier();
        if (!own) {
          const bool has = p >= 0 && p < nst;
          const float2 q = has ? full2[par * nst + p] : make_float2(kDead, kDead);
          vB = q.x;
          vL = q.y;
        }
        if (norm) {
          float m = kDead;
#if SC_CTC_WMV
#pragma unroll
          for (int q4 = 0; q4 < 16; q4 += 4) {   // (nw <= 16: four 16-byte reads, unused slots skipped)
            if (q4 < nw) {
              const float4 wm = *(const float4*)&wmax[q4];
              m = fmaxf(m, q4 + 0 < nw ? wm.x : kDead);
              m = fmaxf(m, q4 + 1 < nw ? wm.y : kDead);
              m = fmaxf(m, q4 + 2 < nw ? wm.z : kDead);
              m = fmaxf(m, q4 + 3 < nw ? wm.w : kDead);
            }
          }
#else
          for (int q = 0; q < nw; ++q) m = fmaxf(m, wmax[q]);
#endif
          if (m > 0.5f * kDead) {   // all dead (infeasible): keep the sentinel
            vB -= m;
            vL -= m;
            off += (double)m;
            // values that drifted this far below their re-centring carry fp32 rounding of
            // ~|m| 2^-24 per step into the posteriors: the exact lattice redoes the sequence
            if (tid == 0 && m < -kDrift) a.ws.sharp[b] = 1;
          }
          if (tid == 0) offn[(exch + 1) >> 1] = off;
        }
        ++exch;
      }
      if (!(SC_CTC_ABL & 2)) emit(tstep(i), vB, vL);
    }
  };
  load(bufA, 0);
  for (int i0 = 0; i0 < Tb; i0 += 2 * kAbP) {
    load(bufB, i0 + kAbP);
    body(bufA, i0);
    if (i0 + kAbP >= Tb) break;
    load(bufA, i0 + 2 * kAbP);
    body(bufB, i0 + kAbP);
  }
  if (!BETA) {
    // sum_t c_t, the emission shift of every path, in fp64 and a fixed order
    __shared__ double csum[16];
    double cs = 0.0;
    for (int t = tid; t < Tb; t += blockDim.x) cs += (double)a.ws.cst[(int64_t)b * a.T + t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o);
    if (lane == 0) csum[w] = cs;
    // log p = log2sum(alpha_{Tb-1}(2Ub), alpha_{Tb-1}(2Ub-1)) + off, gathered over the workgroup
    float c = lse2_live((own && p == Ub) ? vB : kDead, (own && p == Ub - 1) ? vL : kDead);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float co = __shfl_xor(c, o);
      const float m = fmaxf(c, co);
      c = m + log2_(exp2_(c - m) + exp2_(co - m));
    }
    lds_barrier();
    if (lane == 0) wmax[w] = c;
    lds_barrier();
    if (tid == 0) {
      float cc = kDead;
      double ctot = 0.0;
      for (int q = 0; q < nw; ++q) {
        const float m = fmaxf(cc, wmax[q]);
        cc = m + log2_(exp2_(cc - m) + exp2_(wmax[q] - m));
        ctot += csum[q];
      }
      const bool dead = cc < 0.5f * kDead;
      const double ll2s = (double)cc + off;
      a.ws.ll2s[b] = dead ? -__builtin_huge_val() : ll2s;
      a.nll[b] = dead ? __builtin_huge_valf() : (float)(-(ll2s + ctot) * 0.6931471805599453);
    }
  }
}

template <int K>
__global__ void __launch_bounds__(1024) ctc_ab_kernel(CtcArgs a) {
  const bool is_beta = blockIdx.x >= a.B;
  const int b = is_beta ? blockIdx.x - a.B : blockIdx.x;
  const int Tb = clampi(a.in_lens[b], 0, a.T);
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  if (Tb == 0) {
    if (!is_beta && threadIdx.x == 0) {
      a.nll[b] = (Ub == 0) ? 0.0f : __builtin_huge_valf();
      a.ws.ll2s[b] = (Ub == 0) ? 0.0 : -__builtin_huge_val();
    }
    return;
  }
  if (is_beta) ab_run<K, true>(a, b, Tb, Ub);
  else ab_run<K, false>(a, b, Tb, Ub);
}

// The one-wave lattices (ctc_lin_kernel, ctc_x64_kernel) hold PPL pairs of states per lane
// (PPL <= 4: U <= 255; C2's U <= 150 takes PPL = 3): lane l holds pairs p = l PPL .. l PPL +
// PPL - 1, so a step needs one DPP lane shift and no halo, LDS or barrier.
constexpr int kAb1R = 16;   // the linear lattice's renormalisation period (steps)
constexpr int kAb1P = 16;   // its emission prefetch depth (steps)

// Linear-domain lattice (SC_CTC_LIN=1, Umax <= 255).  The pair-per-lane layout above, but
// the values are probabilities in fp64: one step of a pair is
//   alpha:  B' = (B + L[p-1]) e(2p);          L' = (L + B + skip L[p-1]) e(2p+1)
//   beta:   B' = (B + L) e(2p);               L' = (L + B[p+1] + skip L[p+1]) e(2p+1)
// five fp64 adds / multiplies (gfx950's vector ALU issues them at the fp32 rate) instead of five
// exp2 / log2 at the transcendental rate, and exact 0 is "dead" (the DPP shifts' bound_ctrl zero
// is the right boundary value).  Every kAb1R steps the wave max is renormalised into [0.5, 1) by
// an exact power of two (v_ldexp_f64: no rounding), its exponent added to the fp64 offset that
// the gradient reads exactly as the log-space kernels' re-centring offsets.
//
// One workgroup of three waves per (sequence, direction).  Wave 0 runs the recurrence and
// leaves each 16-step chunk of rows in an LDS slot; waves 1 and 2 turn the previous chunk into
// fp32 base-2 logs (frexp exponent + v_log_f32 of the mantissa) and store it.  So wave 0 issues no
// global store: its vmcnt holds only the emission prefetch (a wait for a prefetched row would
// otherwise also wait for every older row store — one workgroup of one wave that stored its own
// rows measured 217 us at C2, no faster than the multi-wave log-space kernel), and the rows
// are the same fp32 log-space rows the gradient reads from every other lattice.
// fp64 keeps 2^1022 of range below the wave max between renormalisations (fp32 log space keeps
// all of it; a state 2^1022 below the max that later carries the likelihood is the one case the
// two differ).  A sequence whose live emissions reach below 2^-kTiny (the emit kernel's flag), and
// a direction whose wave max or final likelihood underflows to 0, are flagged (sharp[b]) and
// recomputed by ctc_x64_kernel.
__device__ __forceinline__ double dpp_shr1d(double v) {   // lane-1's value (lane 0: 0)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1d(double v) {   // lane+1's value (lane 63: 0)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
typedef double d2v __attribute__((ext_vector_type(2)));

constexpr int kLinC = kAb1P;   // steps per chunk (LDS slot)

// base-2 log of a non-negative double as fp32 (0 -> the dead sentinel): exact exponent plus the
// mantissa's v_log_f32
__device__ __forceinline__ float log2d(double v) {
  int e;
  const double m = frexp(v, &e);
  return v > 0.0 ? (float)e + log2_((float)m) : kDead;
}

// wave 0: the recurrence over chunks; returns false on underflow (log space then decides)
template <int PPL, bool BETA>
__device__ __forceinline__ bool lin_produce(const CtcArgs& a, int b, int Tb, int Ub, d2v* slots,
                                            int* fail_lds) {
  const int lane = threadIdx.x;
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  const int npairs = a.Sp / 2;
  double skip[PPL];
  uint32_t vo[PPL];   // emission pair byte offsets (kDrop past the row)
  constexpr uint32_t kDrop = 0x80000000u;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int p = lane * PPL + j;
    bool sk = false;
    if (p < Ub) {
      const int lab = (int)tg[p];
      if (!BETA) {
        sk = p >= 1 && lab != a.blank && lab != (int)tg[p - 1];
      } else if (p + 1 < Ub) {
        const int l2 = (int)tg[p + 1];
        sk = l2 != a.blank && l2 != lab;
      }
    }
    skip[j] = sk ? 1.0 : 0.0;
    vo[j] = p < npairs ? (uint32_t)(8 * p) : kDrop;
  }
  const uint32_t rowb = (uint32_t)(a.Sp * 4);
  const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
      a.ws.ylin + (int64_t)b * a.T * a.Sp, 0, (int)(rowb * (uint32_t)a.T), 0x00020000);
  double* offn = (BETA ? a.ws.offB : a.ws.offA) + (int64_t)b * (a.T + 1);
  if (lane == 0) offn[0] = 0.0;
  auto tstep = [&](int i) { return BETA ? Tb - 1 - i : i; };
  f2v bufA[kLinC][PPL], bufB[kLinC][PPL];
  auto load = [&](f2v (&buf)[kLinC][PPL], int i0) {
#pragma unroll
    for (int s = 0; s < kLinC; ++s) {
      const uint32_t so = (uint32_t)tstep(min(i0 + s, Tb - 1)) * rowb;
#pragma unroll
      for (int j = 0; j < PPL; ++j)
        buf[s][j] = (SC_CTC_ABL & 16) ? f2v{0.5f, 0.25f}
                                      : __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(ers, vo[j], so, 0));
    }
  };
  double vB[PPL], vL[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) vB[j] = vL[j] = 0.0;
  double off = 0.0;
  bool fail = false;
  // one chunk of steps into slot (chunk & 1); false when the wave underflowed
  auto body = [&](const f2v (&buf)[kLinC][PPL], int ci) __attribute__((always_inline)) {
    d2v* slot = slots + (size_t)(ci & 1) * kLinC * PPL * 64;
#pragma unroll
    for (int s = 0; s < kLinC; ++s) {
      const int i = ci * kLinC + s;
      if (i >= Tb) break;
      if (i == 0) {
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const int p = lane * PPL + j;
          vB[j] = (p <= Ub && p == (BETA ? Ub : 0)) ? (double)buf[s][j].x : 0.0;
          vL[j] = (p < Ub && p == (BETA ? Ub - 1 : 0)) ? (double)buf[s][j].y : 0.0;
        }
      } else if (!BETA) {
        double prevL[PPL];
        prevL[0] = dpp_shr1d(vL[PPL - 1]);
#pragma unroll
        for (int j = 1; j < PPL; ++j) prevL[j] = vL[j - 1];
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const double nb = (vB[j] + prevL[j]) * (double)buf[s][j].x;
          const double nl = __builtin_fma(skip[j], prevL[j], vL[j] + vB[j]) * (double)buf[s][j].y;
          vB[j] = nb;
          vL[j] = nl;
        }
      } else {
        double nB[PPL], nL[PPL];
        nB[PPL - 1] = dpp_shl1d(vB[0]);
        nL[PPL - 1] = dpp_shl1d(vL[0]);
#pragma unroll
        for (int j = 0; j + 1 < PPL; ++j) {
          nB[j] = vB[j + 1];
          nL[j] = vL[j + 1];
        }
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const double nb = (vB[j] + vL[j]) * (double)buf[s][j].x;
          const double nl = __builtin_fma(skip[j], nL[j], vL[j] + nB[j]) * (double)buf[s][j].y;
          vB[j] = nb;
          vL[j] = nl;
        }
      }
      if (!(SC_CTC_ABL & 8) && (i + 1) % kAb1R == 0) {   // renormalise the wave max to [0.5, 1)
        double m = 0.0;
#pragma unroll
        for (int j = 0; j < PPL; ++j) m = fmax(m, fmax(vB[j], vL[j]));
        int e = 0;
        (void)frexp(m, &e);
        const float E = wave_max_dpp(m > 0.0 ? (float)e : -1e9f);
        if (E < -1e8f) {   // every state underflowed (or the lattice died): log space instead
          fail = true;
          return;
        }
        const int ie = (int)E;
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          vB[j] = ldexp(vB[j], -ie);
          vL[j] = ldexp(vL[j], -ie);
        }
        off += (double)ie;
        if (lane == 0) offn[(i + 1) / kAb1R] = off;
      }
#pragma unroll
      for (int j = 0; j < PPL; ++j) slot[(s * PPL + j) * 64 + lane] = d2v{vB[j], vL[j]};
    }
  };
  const int nch = (Tb + kLinC - 1) / kLinC;
  load(bufA, 0);
  for (int ci = 0; ci < nch; ++ci) {
    if (!fail) {
      if ((ci & 1) == 0) {
        if (ci + 1 < nch) load(bufB, (ci + 1) * kLinC);
        body(bufA, ci);
      } else {
        if (ci + 1 < nch) load(bufA, (ci + 1) * kLinC);
        body(bufB, ci);
      }
    }
    if (lane == 0) *fail_lds = fail ? 1 : 0;
    __syncthreads();   // chunk ci is in its slot (or the lattice failed); consumers take it
  }
  if (fail) return false;
  if (!BETA) {
    // P = alpha_{Tb-1}(2Ub) + alpha_{Tb-1}(2Ub-1), fixed-order fp64 sums
    double c = 0.0;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int p = lane * PPL + j;
      if (p == Ub) c += vB[j];
      if (p == Ub - 1) c += vL[j];
    }
    double cs = 0.0;
    for (int t = lane; t < Tb; t += 64) cs += (double)a.ws.cst[(int64_t)b * a.T + t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      c += __shfl_xor(c, o);
      cs += __shfl_xor(cs, o);
    }
    if (!(c > 0.0)) return false;   // underflowed at the end (or infeasible): log space decides
    if (lane == 0) {
      const double ll2s = log2(c) + off;
      a.ws.ll2s[b] = ll2s;
      a.nll[b] = (float)(-(ll2s + cs) * 0.6931471805599453);
    }
  }
  return true;
}

// waves 1 and 2: chunk ci - 1's rows (slot (ci - 1) & 1) as fp32 base-2 logs into alpha / beta,
// half of the chunk's steps each, while wave 0 computes chunk ci
template <int PPL, bool BETA>
__device__ __forceinline__ void lin_consume(const CtcArgs& a, int b, int Tb, const d2v* slots,
                                            const int* fail_lds) {
  const int lane = threadIdx.x & 63, half = (threadIdx.x >> 6) - 1;
  const int npairs = a.Sp / 2;
  constexpr uint32_t kDrop = 0x80000000u;
  uint32_t vo[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int p = lane * PPL + j;
    vo[j] = p < npairs ? (uint32_t)(8 * p) : kDrop;
  }
  const uint32_t rowb = (uint32_t)(a.Sp * 4);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (BETA ? a.ws.beta : a.ws.alpha) + (int64_t)b * a.T * a.Sp, 0, (int)(rowb * (uint32_t)a.T),
      0x00020000);
  const int nch = (Tb + kLinC - 1) / kLinC;
  bool stop = false;
  auto consume = [&](int ci) {
    const d2v* slot = slots + (size_t)(ci & 1) * kLinC * PPL * 64;
#pragma unroll
    for (int s2 = 0; s2 < kLinC / 2; ++s2) {
      const int s = half * (kLinC / 2) + s2, i = ci * kLinC + s;
      if (i >= Tb) break;
      const uint32_t so = (uint32_t)(BETA ? Tb - 1 - i : i) * rowb;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const d2v v = slot[(s * PPL + j) * 64 + lane];
        if (!(SC_CTC_ABL & 2))
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, f2v{log2d(v.x), log2d(v.y)}),
              ors, vo[j], so, 0);
      }
    }
  };
  for (int ci = 0; ci < nch; ++ci) {
    __syncthreads();   // chunk ci produced (wave 0); chunk ci - 1 consumed by both waves
    if (!stop) stop = *fail_lds != 0;
    if (!stop) consume(ci);
  }
}

template <int PPL>
__global__ void __launch_bounds__(192) ctc_lin_kernel(CtcArgs a) {
  // two 16-step slots of PPL pairs x 64 lanes of (B, L) fp64
  __shared__ d2v slots[2 * kLinC * PPL * 64];
  __shared__ int fail_lds;
  const bool is_beta = blockIdx.x >= a.B;
  const int b = is_beta ? blockIdx.x - a.B : blockIdx.x;
  const int Tb = clampi(a.in_lens[b], 0, a.T);
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  const int w = uniform(threadIdx.x >> 6);
  if (Tb == 0) {
    if (!is_beta && threadIdx.x == 0) {
      a.nll[b] = (Ub == 0) ? 0.0f : __builtin_huge_valf();
      a.ws.ll2s[b] = (Ub == 0) ? 0.0 : -__builtin_huge_val();
    }
    return;
  }
  // (uniform over the workgroup: every wave takes the same branch, so the barriers match)
  const bool tiny = a.ws.flag[b] != 0;
  bool lin = !tiny;
  if (lin) {
    if (w == 0) {
      lin = is_beta ? lin_produce<PPL, true>(a, b, Tb, Ub, slots, &fail_lds)
                    : lin_produce<PPL, false>(a, b, Tb, Ub, slots, &fail_lds);
    } else {
      if (is_beta) lin_consume<PPL, true>(a, b, Tb, slots, &fail_lds);
      else lin_consume<PPL, false>(a, b, Tb, slots, &fail_lds);
      __builtin_amdgcn_s_waitcnt(0);   // (the stores retire before a fallback rewrites rows)
    }
    __syncthreads();
  }
  // an underflow (or a flagged emission): ctc_x64_kernel recomputes the sequence exactly
  if (!lin && threadIdx.x == 0) a.ws.sharp[b] = 1;
}


// ------------------------------------------------- exact lattice for sharp sequences --------
// ctc_x64_kernel recomputes, ONE wave per (sequence, direction), every sequence whose log-space
// lattice drifted more than kDrift bits between two re-centrings (sharp[b], set by ctc_ab_kernel).
// That happens when the best alignment must pay emissions hundreds of bits below the frame's best
// (logits x 100 over a small vocabulary: log-probs of -2000 nats): an fp32 log-space value of
// magnitude ~1e4 carries 1e-3 of rounding per step, and an fp32 EMISSION of magnitude 3e3 is
// already 1e-4 off before the lattice adds it.  Here every value is an extended-range number: an
// fp64 mantissa in [0.5, 1) (0: dead) and an int exponent, so a state never under- or overflows
// and the recurrence rounds at 2^-53.  Emissions come straight from the logits in fp64 (the
// row's lse kept as max + log(sum), ws.lse64): e = x log2(e) - lse log2(e) - c_t, split into
// the integer floor k and 2^frac.  One step of a pair:
//   alpha:  B' = (B + L[p-1]) e(2p);          L' = (L + B + skip L[p-1]) e(2p+1)
//   beta:   B' = (B + L) e(2p);               L' = (L + B[p+1] + skip L[p+1]) e(2p+1)
// with the sums aligned to their largest exponent (v_ldexp_f64, exact but for what falls below
// 2^-53 of it).  Each step's row is stored as the fp32 base-2 log relative to that step's largest
// exponent O_t (entry i + 1 of the offsets: the gradient reads a sharp sequence's offsets per
// step), so the live states' stored values sit near 0 whatever the drift.
constexpr int kXDeadE = -(1 << 29);
constexpr int kX64P = 16;   // steps per emission prefetch chunk
constexpr double kLog2eD = 1.4426950408889634;

struct Xv {
  double m;
  int e;
};
__device__ __forceinline__ Xv xnorm(double m, int e) {   // m >= 0 -> [0.5, 1) 2^e, 0 -> dead
  int x;
  const double mm = frexp(m, &x);
  return m > 0.0 ? Xv{mm, e + x} : Xv{0.0, kXDeadE};
}
__device__ __forceinline__ Xv xadd2(Xv a, Xv b) {
  const int E = max(a.e, b.e);
  return Xv{ldexp(a.m, a.e - E) + ldexp(b.m, b.e - E), E};
}
__device__ __forceinline__ Xv xadd3(Xv a, Xv b, Xv c) {
  const int E = max(max(a.e, b.e), c.e);
  return Xv{ldexp(a.m, a.e - E) + ldexp(b.m, b.e - E) + ldexp(c.m, c.e - E), E};
}
template <bool RIGHT>
__device__ __forceinline__ Xv xdpp(Xv v) {   // lane -1's (RIGHT) / lane +1's value, else dead
  constexpr int ctl = RIGHT ? 0x138 : 0x130;
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v.m), ctl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v.m), ctl, 0xf, 0xf, false);
  const int e = __builtin_amdgcn_update_dpp(kXDeadE, v.e, ctl, 0xf, 0xf, false);
  return Xv{__hiloint2double(hi, lo), e};
}
// emission factor of logit x at a step with q = lse log2(e) + c_t: (2^frac, floor) as an Xv
__device__ __forceinline__ Xv xemit(float x, double q, bool live) {
  const double e2 = (double)x * kLog2eD - q;
  if (!live || !(e2 > -1e300)) return Xv{0.0, kXDeadE};
  const double k = floor(e2);
  return xnorm((double)exp2_((float)(e2 - k)), (int)k);
}

template <int PPL, int DT, bool BETA>
__device__ __forceinline__ void x64_run(const CtcArgs& a, int b, int Tb, int Ub) {
  using E = Elem<DT>;
  const int lane = threadIdx.x;
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  const int npairs = a.Sp / 2;
  bool skip[PPL], liveB[PPL], liveL[PPL];
  uint32_t cB[PPL], cL[PPL];   // byte offsets of the pair's blank / label logit in a row
  uint32_t vo[PPL];            // byte offset of pair p in a lattice row (kDrop past it)
  constexpr uint32_t kDrop = 0x80000000u;
  const bool ex = a.ex != nullptr;
  const uint32_t esz = ex ? 4u : (uint32_t)sizeof(typename E::T);
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int p = lane * PPL + j;
    skip[j] = false;
    liveB[j] = p <= Ub;
    liveL[j] = p < Ub;
    int lab = a.blank;
    if (p < Ub) {
      lab = (int)tg[p];
      if (!BETA) {
        skip[j] = p >= 1 && lab != a.blank && lab != (int)tg[p - 1];
      } else if (p + 1 < Ub) {
        const int l2 = (int)tg[p + 1];
        skip[j] = l2 != a.blank && l2 != lab;
      }
    }
    lab = lab < 0 ? 0 : (lab >= a.V ? a.V - 1 : lab);
    cB[j] = ex ? 0u : (uint32_t)a.blank * esz;
    cL[j] = ex ? (uint32_t)(p < Ub ? 1 + p : 0) * 4u : (uint32_t)lab * esz;
    vo[j] = p < npairs ? (uint32_t)(8 * p) : kDrop;
  }
  // logits (or the emission-logit side array) of this sequence, rows at t * row stride
  const void* xb = ex ? (const void*)(a.ex + (int64_t)b * a.exb)
                      : (const void*)((const typename E::T*)a.x + (int64_t)b * a.sb);
  const uint32_t xrow = ex ? (uint32_t)a.ext * 4u : (uint32_t)a.stt * esz;
  const Buf<float> xf(xb);
  const Buf<typename E::T> xe(xb);
  auto ldx = [&](uint32_t col, uint32_t so) -> uint32_t {
    return ex ? __float_as_uint(xf.ld(col, so)) : xe.ldw(col, so);
  };
  auto cvt = [&](uint32_t w) { return ex ? __uint_as_float(w) : E::ldw(w); };
  const uint32_t rowb = (uint32_t)(a.Sp * 4);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (BETA ? a.ws.beta : a.ws.alpha) + (int64_t)b * a.T * a.Sp, 0, (int)(rowb * (uint32_t)a.T),
      0x00020000);
  double* offn = (BETA ? a.ws.offB : a.ws.offA) + (int64_t)b * (a.T + 1);
  const double* lse64 = a.ws.lse64 + (int64_t)b * a.T;
  const float* cst = a.ws.cst + (int64_t)b * a.T;
  if (lane == 0) offn[0] = 0.0;
  auto tstep = [&](int i) { return BETA ? Tb - 1 - i : i; };
  // a chunk's raw logits (blank, label per pair and step) and, on lane s, step s's q
  uint32_t wA[kX64P][PPL][2], wB[kX64P][PPL][2];
  double qA, qB;
  auto load = [&](uint32_t (&w)[kX64P][PPL][2], double& q, int i0) {
#pragma unroll
    for (int s = 0; s < kX64P; ++s) {
      const uint32_t so = (uint32_t)tstep(min(i0 + s, Tb - 1)) * xrow;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        w[s][j][0] = ldx(cB[j], so);
        w[s][j][1] = ldx(cL[j], so);
      }
    }
    const int t = tstep(min(i0 + (lane & (kX64P - 1)), Tb - 1));
    q = (a.is_logits ? lse64[t] * kLog2eD : 0.0) + (double)cst[t];
  };
  Xv vB[PPL], vL[PPL];
#pragma unroll
  for (int j = 0; j < PPL; ++j) vB[j] = vL[j] = Xv{0.0, kXDeadE};
  const Xv dead{0.0, kXDeadE};
  auto body = [&](const uint32_t (&w)[kX64P][PPL][2], double qv, int i0) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < kX64P; ++s) {
      const int i = i0 + s;
      if (i >= Tb) break;
      const double q = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(qv), s),
                                        __builtin_amdgcn_readlane(__double2loint(qv), s));
      Xv eB[PPL], eL[PPL];
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        eB[j] = xemit(cvt(w[s][j][0]), q, liveB[j]);
        eL[j] = xemit(cvt(w[s][j][1]), q, liveL[j]);
      }
      if (i == 0) {
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const int p = lane * PPL + j;
          vB[j] = p == (BETA ? Ub : 0) ? eB[j] : dead;
          vL[j] = p == (BETA ? Ub - 1 : 0) ? eL[j] : dead;
        }
      } else if (!BETA) {
        Xv prevL[PPL];
        prevL[0] = xdpp<true>(vL[PPL - 1]);
#pragma unroll
        for (int j = 1; j < PPL; ++j) prevL[j] = vL[j - 1];
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const Xv nb = xadd2(vB[j], prevL[j]);
          const Xv nl = xadd3(vL[j], vB[j], skip[j] ? prevL[j] : dead);
          vB[j] = xnorm(nb.m * eB[j].m, nb.e + eB[j].e);
          vL[j] = xnorm(nl.m * eL[j].m, nl.e + eL[j].e);
        }
      } else {
        Xv nB[PPL], nL[PPL];
        nB[PPL - 1] = xdpp<false>(vB[0]);
        nL[PPL - 1] = xdpp<false>(vL[0]);
#pragma unroll
        for (int j = 0; j + 1 < PPL; ++j) {
          nB[j] = vB[j + 1];
          nL[j] = vL[j + 1];
        }
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const Xv nb = xadd2(vB[j], vL[j]);
          const Xv nl = xadd3(vL[j], nB[j], skip[j] ? nL[j] : dead);
          vB[j] = xnorm(nb.m * eB[j].m, nb.e + eB[j].e);
          vL[j] = xnorm(nl.m * eL[j].m, nl.e + eL[j].e);
        }
      }
      // the row, relative to its largest exponent
      int mx = kXDeadE;
#pragma unroll
      for (int j = 0; j < PPL; ++j) mx = max(mx, max(vB[j].e, vL[j].e));
      const int O = (int)wave_max_dpp((float)mx);
      const bool alive = O > kXDeadE / 2;
      if (lane == 0) offn[i + 1] = alive ? (double)O : 0.0;
      const uint32_t so = (uint32_t)tstep(i) * rowb;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const float rb = vB[j].m > 0.0 ? (float)(vB[j].e - O) + log2_((float)vB[j].m) : kDead;
        const float rl = vL[j].m > 0.0 ? (float)(vL[j].e - O) + log2_((float)vL[j].m) : kDead;
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, f2v{rb, rl}), ors,
            vo[j], so, 0);
      }
    }
  };
  load(wA, qA, 0);
  for (int i0 = 0; i0 < Tb; i0 += 2 * kX64P) {
    load(wB, qB, i0 + kX64P);
    body(wA, qA, i0);
    if (i0 + kX64P >= Tb) break;
    load(wA, qA, i0 + 2 * kX64P);
    body(wB, qB, i0 + kX64P);
  }
  if (!BETA) {
    // P = alpha_{Tb-1}(2Ub) + alpha_{Tb-1}(2Ub-1); sum_t c_t; both in a fixed order
    Xv c = dead;
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int p = lane * PPL + j;
      if (p == Ub) c = xadd2(c, vB[j]);
      if (p == Ub - 1) c = xadd2(c, vL[j]);
    }
    double cs = 0.0;
    for (int t = lane; t < Tb; t += 64) cs += (double)cst[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const Xv co{__shfl_xor(c.m, o), __shfl_xor(c.e, o)};
      c = xadd2(c, co);
      cs += __shfl_xor(cs, o);
    }
    if (lane == 0) {
      const bool deadP = !(c.m > 0.0);
      const double ll2s = (double)c.e + log2(c.m);
      a.ws.ll2s[b] = deadP ? -__builtin_huge_val() : ll2s;
      a.nll[b] = deadP ? __builtin_huge_valf() : (float)(-(ll2s + cs) * 0.6931471805599453);
    }
  }
}

template <int PPL, int DT>
__global__ void __launch_bounds__(64) ctc_x64_kernel(CtcArgs a) {
  const bool is_beta = blockIdx.x >= a.B;
  const int b = is_beta ? blockIdx.x - a.B : blockIdx.x;
  if (a.ws.sharp[b] == 0) return;   // (uniform: the common case costs one load)
  const int Tb = clampi(a.in_lens[b], 0, a.T);
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  if (Tb == 0) return;
  // sharp[b] = 2: this sequence's rows and offsets are the exact lattice's (one offset per step),
  // which is what the gradient reads them as.  A flagged sequence this kernel does not redo
  // (U > 255: no launch) keeps sharp[b] = 1 and the log-space rows and offsets.
  if (threadIdx.x == 0) a.ws.sharp[b] = 2;
  if (is_beta) x64_run<PPL, DT, true>(a, b, Tb, Ub);
  else x64_run<PPL, DT, false>(a, b, Tb, Ub);
}

// pairs per lane of the exact lattice (0: U > 255, not built)
static int x64_ppl(int Umax) {
  const int ppl = (Umax + 1 + 63) / 64;
  return ppl <= 4 ? ppl : 0;
}

// pairs per lane of the one-wave lattice family (0: the multi-wave kernel).  Off unless
// SC_CTC_LIN=1 in the environment.  Measured at C2 (tools/scan_bench.py --only ctc, ablation
// builds of tools/ctc_abl.sh; profiles/r4_lattice_ab.md): emit + chain + lattice 256 us against
// 211 us for the multi-wave log-space kernel, and the gradient 60 us slower on the fp64 rows.
// Dropping the per-step stores (ABL 2) takes 62 us off: vmcnt retires loads and stores in issue
// order, so waiting for a prefetched emission row also waits for the older row stores.
static int lin_ppl(int Umax) {
  static const bool on = [] {
    const char* e = getenv("SC_CTC_LIN");
    return e && e[0] == '1';
  }();
  const int ppl = (Umax + 1 + 63) / 64;
  return (on && ppl <= 4) ? ppl : 0;
}

// K (steps between halo exchanges) so that ceil((Umax + 1) / (64 - K)) waves of state pairs fit
// a 1024-thread group
static int ab_halo_k(int Umax) {
  auto waves = [&](int K) { return (Umax + 1 + (64 - K) - 1) / (64 - K); };
  for (int K : {SC_CTC_KMAX, 4, 2, 1})
    if (waves(K) <= 16) {
      // a wider halo with the same wave count: fewer exchanges (barriers) per step
      if (SC_CTC_KMAX == 16 && K == 16 && waves(24) == waves(16)) return 24;
      return K;
    }
  return 0;
}

// ---------------------------------------------------------------------------- gradient ------
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One WAVE per (b,t) row (4 rows per workgroup, no workgroup barriers): label occupancies into a
// per-wave LDS row of V base-2 log-sums, then the gradient row with 16-byte accesses.
template <int DT, int GT>
__global__ void __launch_bounds__(256) ctc_grad_kernel(CtcArgs a) {
  using E = Elem<DT>;
  using G = Elem<GT>;
  extern __shared__ __attribute__((aligned(16))) float lcab_all[];   // [4][V + 4]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
  if (row >= (int64_t)a.B * a.T) return;
  // the row's label occupancies by column (base-2 log-sums; -inf off the emission columns).  With
  // emission logits (a.ex) an emission column holds its finished gradient value instead: softmax
  // term and occupancy both from the exact logit, so the output pass only needs "is it -inf"
  float* lcab = lcab_all + w * (a.V + 4);
  const int b = (int)(row / a.T), t = (int)(row % a.T);
  const int Tb = clampi(a.in_lens[b], 0, a.T);
  typename G::T* g = (typename G::T*)a.grad + row * a.V;
  const float sc = a.scale[b];
  const bool gvec = (a.V & 7) == 0 && ((uintptr_t)g & 15) == 0;
  if (t >= Tb || sc == 0.0f) {
    if (gvec) {
      const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int c = lane; c < (a.V >> 3); c += 64) {
        if constexpr (Vec16<GT>::N == 8) {
          Vec16<GT>::st(g + 8 * c, z);
        } else {
          Vec16<GT>::st(g + 8 * c, *(const float(*)[4])&z[0]);
          Vec16<GT>::st(g + 8 * c + 4, *(const float(*)[4])&z[4]);
        }
      }
    } else {
      for (int v = lane; v < a.V; v += 64) g[v] = G::st(0.0f);
    }
    return;
  }
  const int Ub = clampi(a.tgt_lens[b], 0, a.Umax);
  const int Sb = 2 * Ub + 1;
  const int Um = a.Umax > 0 ? a.Umax : 1;
  const int64_t* tg = a.tg + (int64_t)b * a.tgs;
  for (int v = lane; v < a.V; v += 64) lcab[v] = kNegInf;
  wave_lds_sync();
  const float* exr = a.ex ? a.ex + (int64_t)b * a.exb + (int64_t)t * a.ext : nullptr;
  const float* al = a.ws.alpha + ((int64_t)b * a.T + t) * a.Sp;
  const float* be = a.ws.beta + ((int64_t)b * a.T + t) * a.Sp;
  // exp(lcab + nll - lp) = 2^(lcab2 + offA + offB + c_t - ll2s - lp*log2e): the lattice holds
  // alpha_t - sum_{t'<=t} c and beta_t - sum_{t'>=t} c, so alpha + beta carries c_t once more than
  // the shifted log-likelihood ll2s; offsets folded in fp64
  // steps per re-centring (a sequence the exact lattice recomputed, sharp[b] == 2, has one
  // offset per step; a flagged one it did not redo, sharp[b] == 1, keeps the log-space offsets)
  const int per = a.ws.sharp[b] == 2 ? 1 : 2 * a.kh;
  const float koff = (float)(a.ws.offA[(int64_t)b * (a.T + 1) + (t + 1) / per] +
                             a.ws.offB[(int64_t)b * (a.T + 1) + (Tb - t) / per] +
                             (double)a.ws.cst[(int64_t)b * a.T + t] - a.ws.ll2s[b]);
  const int* chain = a.ws.chain + (int64_t)b * Um;
  const int* first = a.ws.first + (int64_t)b * Um;
  // the log-probs as (x - lse) - lse_lo: lse's fp32 rounding (6e-5 at |lse| ~ 1e3) taken out
  const float lse = a.is_logits ? a.ws.lse[(int64_t)b * a.T + t] : 0.0f;
  const float lse_lo = a.is_logits ? (float)(a.ws.lse64[(int64_t)b * a.T + t] - (double)lse) : 0.0f;
  // (ex) the finished gradient of an emission column from its exact logit and occupancy
  auto exact_grad = [&](float logit, float occ2) {
    const float lp2 = ((logit - lse) - lse_lo) * kLog2e;
    return (exp2_(lp2) - exp2_(occ2 + koff - lp2)) * sc;
  };
  float m = kNegInf, l = 0.0f;   // blank-label occupancy (base 2), per lane
  for (int s = lane; s < Sb; s += 64) {
    const int lab = (s & 1) ? (int)tg[(s - 1) >> 1] : a.blank;
    const float val = al[s] + be[s];
    if (lab == a.blank) {
      const float mn = fmaxf(m, val);
      if (mn != kNegInf) {
        l = l * exp2_(m - mn) + exp2_(val - mn);
        m = mn;
      }
    } else {
      const int u = (s - 1) >> 1;
      if (first[u]) {
        float acc = val;
        for (int q = chain[u]; q >= 0; q = chain[q])
          acc = lse2_b2(acc, al[2 * q + 1] + be[2 * q + 1]);
        if (lab >= 0 && lab < a.V) lcab[lab] = exr ? exact_grad(exr[1 + u], acc) : acc;
      }
    }
  }
  {   // the blank occupancy's log-sum-exp over the lanes (DPP: max, then rescaled sum)
    const float M = wave_max_dpp(m);
    l = wave_sum_dpp(m == kNegInf ? 0.0f : l * exp2_(m - M));
    m = M;
  }
  if (lane == 0 && a.blank >= 0 && a.blank < a.V) {
    const float ob = (m == kNegInf) ? kNegInf : m + log2_(l);
    lcab[a.blank] = exr ? exact_grad(exr[0], ob) : ob;
  }
  wave_lds_sync();
  const typename E::T* xr = (const typename E::T*)a.x + (int64_t)b * a.sb + (int64_t)t * a.stt;
  // grad = (softmax - occupancy) * scale
  if (gvec && ((uintptr_t)xr & 15) == 0) {
    for (int c = lane; c < (a.V >> 3); c += 64) {
      float xv[8], gv[8];
      if constexpr (Vec16<DT>::N == 8) {
        Vec16<DT>::ld(xr + 8 * c, xv);
      } else {
        Vec16<DT>::ld(xr + 8 * c, *(float(*)[4])&xv[0]);
        Vec16<DT>::ld(xr + 8 * c + 4, *(float(*)[4])&xv[4]);
      }
      const float4 l0 = *(const float4*)&lcab[8 * c], l1 = *(const float4*)&lcab[8 * c + 4];
      const float lc[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float lp2 = ((xv[k] - lse) - lse_lo) * kLog2e;
        gv[k] = (exp2_(lp2) - exp2_(lc[k] + koff - lp2)) * sc;
        if (a.ex && lc[k] != kNegInf) gv[k] = lc[k];   // (an emission column's finished value)
      }
      if constexpr (Vec16<GT>::N == 8) {
        Vec16<GT>::st(g + 8 * c, gv);
      } else {
        Vec16<GT>::st(g + 8 * c, *(float(*)[4])&gv[0]);
        Vec16<GT>::st(g + 8 * c + 4, *(float(*)[4])&gv[4]);
      }
    }
    return;
  }
  for (int v = lane; v < a.V; v += 64) {
    const float lp2 = ((E::ld(xr[v]) - lse) - lse_lo) * kLog2e;
    const float lc = lcab[v];
    const float gv = (a.ex && lc != kNegInf) ? lc : (exp2_(lp2) - exp2_(lc + koff - lp2)) * sc;
    g[v] = G::st(gv);
  }
}

static void launch_ab(const CtcArgs& a, hipStream_t st);

template <int DT>
static void launch_fwd(const CtcArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.B * a.T;
  if (a.lin) zero_async(a.ws.flag, (size_t)a.B * sizeof(int), st);   // tiny[b]
  hipLaunchKernelGGL((ctc_emit_kernel<DT>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(ctc_chain_kernel, dim3(a.B, ((a.Umax > 0 ? a.Umax : 1) + 3) / 4), dim3(256), 0,
                     st, a);
  switch (a.lin ? lin_ppl(a.Umax) : 0) {
    case 1: hipLaunchKernelGGL((ctc_lin_kernel<1>), dim3(2 * a.B), dim3(192), 0, st, a); break;
    case 2: hipLaunchKernelGGL((ctc_lin_kernel<2>), dim3(2 * a.B), dim3(192), 0, st, a); break;
    case 3: hipLaunchKernelGGL((ctc_lin_kernel<3>), dim3(2 * a.B), dim3(192), 0, st, a); break;
    case 4: hipLaunchKernelGGL((ctc_lin_kernel<4>), dim3(2 * a.B), dim3(192), 0, st, a); break;
    default: launch_ab(a, st); break;
  }
  // the sequences a lattice flagged (sharp[b]) again, exactly; the others' workgroups exit at
  // once.  U <= 255 only (the pairs fit one wave, 4 per lane): a flagged sequence with a longer
  // target keeps the log-space result, whose fp32 drift at such sharpness is ~1e-3 .. 1e-2
  // relative in the gradient (tests/test_gpu_ctc.py::test_ctc_sharp_long_targets_keep_log_space)
  switch (x64_ppl(a.Umax)) {
    case 1: hipLaunchKernelGGL((ctc_x64_kernel<1, DT>), dim3(2 * a.B), dim3(64), 0, st, a); break;
    case 2: hipLaunchKernelGGL((ctc_x64_kernel<2, DT>), dim3(2 * a.B), dim3(64), 0, st, a); break;
    case 3: hipLaunchKernelGGL((ctc_x64_kernel<3, DT>), dim3(2 * a.B), dim3(64), 0, st, a); break;
    case 4: hipLaunchKernelGGL((ctc_x64_kernel<4, DT>), dim3(2 * a.B), dim3(64), 0, st, a); break;
    default: break;
  }
}

static void launch_ab(const CtcArgs& a, hipStream_t st) {
  const int K = a.kh;
  const int nw = (a.Umax + 1 + (64 - K) - 1) / (64 - K);
  const size_t sh = 2 * (size_t)nw * (64 - K) * sizeof(float2);
  switch (K) {
#if SC_CTC_KMAX == 16
    case 24: hipLaunchKernelGGL((ctc_ab_kernel<24>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    case 16: hipLaunchKernelGGL((ctc_ab_kernel<16>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
#endif
    case 8: hipLaunchKernelGGL((ctc_ab_kernel<8>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    case 4: hipLaunchKernelGGL((ctc_ab_kernel<4>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    case 2: hipLaunchKernelGGL((ctc_ab_kernel<2>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
    default: hipLaunchKernelGGL((ctc_ab_kernel<1>), dim3(2 * a.B), dim3(64 * nw), sh, st, a); break;
  }
}

template <int DT, int GT>
static void launch_bwd(const CtcArgs& a, hipStream_t st) {
  // 4 rows (waves) per workgroup while their LDS rows fit the default 64 KB, else 1
  const int R = 4 * (a.V + 4) * (int)sizeof(float) <= 65536 ? 4 : 1;
  hipLaunchKernelGGL((ctc_grad_kernel<DT, GT>), dim3((unsigned)(((int64_t)a.B * a.T + R - 1) / R)),
                     dim3(64 * R), R * (a.V + 4) * sizeof(float), st, a);
}

// nn.CTCLoss(reduction='mean', zero_infinity=True) on device in one launch: loss =
// mean_b(z_b / max(U_b, 1)) with z_b = 0 where nll_b is infinite, and the per-sequence factor
// d loss / d nll_b = (finite ? 1 / (B max(U_b, 1)) : 0) for the backward.  One workgroup, fixed
// summation order.
__global__ void __launch_bounds__(256) ctc_mean_kernel(const float* nll, const int64_t* tgt_lens,
                                                       int B, float* loss, float* factor) {
  __shared__ float part[256];
  float acc = 0.0f;
  for (int b = threadIdx.x; b < B; b += 256) {
    const float u = (float)(tgt_lens[b] > 1 ? tgt_lens[b] : 1);
    const float v = nll[b];
    const bool fin = !__builtin_isinf(v);
    acc += fin ? v / u : 0.0f;
    factor[b] = fin ? 1.0f / ((float)B * u) : 0.0f;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = part[0] / (float)B;
}

// The CTC head's emission-column operand (ops._emission_logits): row (b, c) of out is
// [bf16(w_r) | bf16(w_r - bf16(w_r)) | bf16(w_r)] for r = blank (c = 0) or targets[b][c - 1]
// (clamped into [0, V)), and bout[b][c] = bias[r] — one launch instead of the split image's
// casts, a concatenation and two gathers.  One wave per row, 16-byte loads, 8-byte stores.
__global__ void __launch_bounds__(256) ctc_split_rows_kernel(const float* w, int64_t ldw,
                                                             const float* bias, int V, int K,
                                                             const int64_t* tg, int64_t tgs, int U1,
                                                             int blank, __bf16* out, float* bout,
                                                             int B) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * U1) return;
  const int b = (int)(row / U1), c = (int)(row % U1);
  int r = c == 0 ? blank : (int)tg[(int64_t)b * tgs + c - 1];
  r = r < 0 ? 0 : (r >= V ? V - 1 : r);
  const float* wr = w + (int64_t)r * ldw;
  __bf16* o = out + row * 3 * (int64_t)K;
  typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
  for (int k = 4 * lane; k < K; k += 256) {
    const float4 v = *(const float4*)(wr + k);
    const bf4 hi = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    const bf4 lo = {(__bf16)(v.x - (float)hi[0]), (__bf16)(v.y - (float)hi[1]),
                    (__bf16)(v.z - (float)hi[2]), (__bf16)(v.w - (float)hi[3])};
    *(bf4*)(o + k) = hi;
    *(bf4*)(o + K + k) = lo;
    *(bf4*)(o + 2 * K + k) = hi;
  }
  if (lane == 0) bout[row] = bias ? bias[r] : 0.0f;
}

}  // namespace sc

using namespace sc;

extern "C" int sc_ctc_split_rows(const float* w, int64_t ldw, const float* bias, int V, int K,
                                 const int64_t* targets, int64_t target_stride, int max_target_len,
                                 int blank, void* out, float* bias_out, int B, void* stream) {
  clear_error();
  SC_REQUIRE(B >= 0 && V > 0 && K > 0 && max_target_len >= 0, "sc_ctc_split_rows: bad shape");
  if (B == 0) return 0;
  SC_REQUIRE(w && out && bias_out && (max_target_len == 0 || targets),
             "sc_ctc_split_rows: null pointer");
  SC_REQUIRE(K % 4 == 0 && ldw % 4 == 0 && (uintptr_t)w % 16 == 0 && (uintptr_t)out % 8 == 0,
             "sc_ctc_split_rows: rows must be 16-byte aligned (K %% 4, ldw %% 4)");
  SC_REQUIRE(blank >= 0 && blank < V, "sc_ctc_split_rows: blank outside [0, V)");
  const int U1 = max_target_len + 1;
  const int64_t rows = (int64_t)B * U1;
  hipLaunchKernelGGL(ctc_split_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, w, ldw, bias, V, K, targets, target_stride, U1, blank,
                     (__bf16*)out, bias_out, B);
  return launch_status("sc_ctc_split_rows");
}

extern "C" size_t sc_ctc_workspace_bytes(int B, int T, int max_target_len) {
  if (B <= 0 || T <= 0 || max_target_len < 0) return 256;
  return ws_layout(B, T, max_target_len, nullptr, nullptr);
}

static int ctc_check(const void* x, int x_dtype, int B, int T, int V, int max_target_len,
                     const int64_t* targets, const int64_t* in_lens, const int64_t* tgt_lens,
                     int blank, const void* ws, size_t wsb, const char* who) {
  SC_REQUIRE(x_dtype == SC_F32 || x_dtype == SC_BF16 || x_dtype == SC_F16,
             "%s: unsupported dtype %d", who, x_dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && V > 0 && max_target_len >= 0, "%s: bad shape", who);
  SC_REQUIRE(ab_halo_k(max_target_len) > 0,
             "%s: max target length %d exceeds %d", who, max_target_len, 16 * 63 - 1);
  SC_REQUIRE(blank >= 0 && blank < V, "%s: blank %d outside [0, %d)", who, blank, V);
  SC_REQUIRE((int64_t)B * T <= 0x7fffffff, "%s: B*T too large", who);
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(x && in_lens && tgt_lens && ws, "%s: null pointer", who);
  SC_REQUIRE(max_target_len == 0 || targets, "%s: null targets", who);
  const size_t need = ws_layout(B, T, max_target_len, nullptr, nullptr);
  SC_REQUIRE(wsb >= need, "%s: workspace %zu < %zu bytes", who, wsb, need);
  return 0;
}

static CtcArgs make_args(const void* x, int is_logits, int B, int T, int V, int64_t sb, int64_t st,
                         const int64_t* targets, int64_t tgs, int umax, const int64_t* in_lens,
                         const int64_t* tgt_lens, int blank, float* nll, const void* ws,
                         const float* scale, void* grad) {
  CtcArgs a;
  a.x = x;
  a.is_logits = is_logits;
  a.B = B;
  a.T = T;
  a.V = V;
  a.S = 2 * umax + 1;
  a.Sp = 64 * states_per_lane(a.S);
  a.Umax = umax;
  // steps per re-centring / 2 (the gradient's offset index): the one-wave lattices re-centre
  // every kAb1R steps, the multi-wave one at every second halo exchange
  a.lin = lin_ppl(umax) > 0;
  a.kh = a.lin ? kAb1R / 2 : ab_halo_k(umax);
  a.blank = blank;
  a.sb = sb;
  a.stt = st;
  a.tg = targets;
  a.tgs = tgs;
  a.in_lens = in_lens;
  a.tgt_lens = tgt_lens;
  a.nll = nll;
  ws_layout(B, T, umax, &a.ws, (void*)ws);
  a.scale = scale;
  a.grad = grad;
  a.ex = nullptr;
  a.exb = a.ext = 0;
  return a;
}

static int ex_check(const float* ex, int64_t ex_stride_b, int64_t ex_stride_t, int is_logits,
                    int T, int max_target_len, const char* who) {
  if (!ex) return 0;
  SC_REQUIRE(is_logits, "%s: emission logits need is_logits = 1", who);
  SC_REQUIRE(ex_stride_t >= max_target_len + 1 && ex_stride_b >= (int64_t)T * ex_stride_t,
             "%s: emission logits rows of max_target_len + 1 = %d", who, max_target_len + 1);
  return 0;
}

extern "C" int sc_ctc_fwd_ex(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                             int64_t stride_b, int64_t stride_t, const int64_t* targets,
                             int64_t target_stride, int max_target_len, const int64_t* in_lens,
                             const int64_t* tgt_lens, int blank, const float* ex,
                             int64_t ex_stride_b, int64_t ex_stride_t, float* nll, void* workspace,
                             size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = ctc_check(x, x_dtype, B, T, V, max_target_len, targets, in_lens, tgt_lens, blank,
                     workspace, workspace_bytes, "sc_ctc_fwd");
  if (rc) return rc;
  if (B == 0) return 0;
  SC_REQUIRE(nll, "sc_ctc_fwd: null nll");
  SC_REQUIRE(T > 0, "sc_ctc_fwd: T == 0 is handled by the caller");
  if ((rc = ex_check(ex, ex_stride_b, ex_stride_t, is_logits, T, max_target_len, "sc_ctc_fwd_ex")))
    return rc;
  CtcArgs a = make_args(x, is_logits, B, T, V, stride_b, stride_t, targets, target_stride,
                        max_target_len, in_lens, tgt_lens, blank, nll, workspace, nullptr, nullptr);
  a.ex = ex;
  a.exb = ex_stride_b;
  a.ext = ex_stride_t;
  hipStream_t st = (hipStream_t)stream;
  switch (x_dtype) {
    case SC_F32: launch_fwd<SC_F32>(a, st); break;
    case SC_BF16: launch_fwd<SC_BF16>(a, st); break;
    default: launch_fwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_ctc_fwd");
}

extern "C" int sc_ctc_fwd(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                          int64_t stride_b, int64_t stride_t, const int64_t* targets,
                          int64_t target_stride, int max_target_len, const int64_t* in_lens,
                          const int64_t* tgt_lens, int blank, float* nll, void* workspace,
                          size_t workspace_bytes, void* stream) {
  return sc_ctc_fwd_ex(x, x_dtype, is_logits, B, T, V, stride_b, stride_t, targets, target_stride,
                       max_target_len, in_lens, tgt_lens, blank, nullptr, 0, 0, nll, workspace,
                       workspace_bytes, stream);
}

extern "C" int sc_ctc_bwd_ex(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                             int64_t stride_b, int64_t stride_t, const int64_t* targets,
                             int64_t target_stride, int max_target_len, const int64_t* in_lens,
                             const int64_t* tgt_lens, int blank, const float* ex,
                             int64_t ex_stride_b, int64_t ex_stride_t, const float* nll,
                             const float* scale, void* grad, int grad_dtype, const void* workspace,
                             size_t workspace_bytes, void* stream) {
  clear_error();
  int rc = ctc_check(x, x_dtype, B, T, V, max_target_len, targets, in_lens, tgt_lens, blank,
                     workspace, workspace_bytes, "sc_ctc_bwd");
  if (rc) return rc;
  if (B == 0 || T == 0) return 0;
  SC_REQUIRE(grad_dtype == SC_F32 || grad_dtype == SC_BF16 || grad_dtype == SC_F16,
             "sc_ctc_bwd: unsupported grad dtype %d", grad_dtype);
  SC_REQUIRE(nll && scale && grad, "sc_ctc_bwd: null pointer");
  if ((rc = ex_check(ex, ex_stride_b, ex_stride_t, is_logits, T, max_target_len, "sc_ctc_bwd_ex")))
    return rc;
  CtcArgs a = make_args(x, is_logits, B, T, V, stride_b, stride_t, targets, target_stride,
                        max_target_len, in_lens, tgt_lens, blank, (float*)nll, workspace, scale,
                        grad);
  a.ex = ex;
  a.exb = ex_stride_b;
  a.ext = ex_stride_t;
  hipStream_t st = (hipStream_t)stream;
#define SC_CTC_BWD(DT)                                               \
  switch (grad_dtype) {                                              \
    case SC_F32: launch_bwd<DT, SC_F32>(a, st); break;               \
    case SC_BF16: launch_bwd<DT, SC_BF16>(a, st); break;             \
    default: launch_bwd<DT, SC_F16>(a, st); break;                   \
  }
  switch (x_dtype) {
    case SC_F32: SC_CTC_BWD(SC_F32) break;
    case SC_BF16: SC_CTC_BWD(SC_BF16) break;
    default: SC_CTC_BWD(SC_F16) break;
  }
#undef SC_CTC_BWD
  return launch_status("sc_ctc_bwd");
}

extern "C" int sc_ctc_bwd(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                          int64_t stride_b, int64_t stride_t, const int64_t* targets,
                          int64_t target_stride, int max_target_len, const int64_t* in_lens,
                          const int64_t* tgt_lens, int blank, const float* nll,
                          const float* scale, void* grad, int grad_dtype, const void* workspace,
                          size_t workspace_bytes, void* stream) {
  return sc_ctc_bwd_ex(x, x_dtype, is_logits, B, T, V, stride_b, stride_t, targets, target_stride,
                       max_target_len, in_lens, tgt_lens, blank, nullptr, 0, 0, nll, scale, grad,
                       grad_dtype, workspace, workspace_bytes, stream);
}

extern "C" int sc_ctc_mean(const float* nll, const int64_t* tgt_lens, int B, float* loss,
                           float* factor, void* stream) {
  clear_error();
  SC_REQUIRE(B > 0, "sc_ctc_mean: B must be positive");
  SC_REQUIRE(nll && tgt_lens && loss && factor, "sc_ctc_mean: null pointer");
  hipLaunchKernelGGL(ctc_mean_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, nll, tgt_lens, B,
                     loss, factor);
  return launch_status("sc_ctc_mean");
}
