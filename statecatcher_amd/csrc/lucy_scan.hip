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
// Decomposition (MI355X-first): one workgroup = one batch row b x 64 hidden units (lane = d,
// coalesced 64-wide rows of the [B,T,7,D] gates) x NW waves that split TIME.  Time is walked in
// super-chunks of 64 steps; wave w owns steps [w*LC, (w+1)*LC) of the super-chunk.  Per
// super-chunk each wave
//   1. computes the elementwise gate terms of its LC steps from registers (gates read ONCE),
//   2. publishes its s-segment as an affine map (prod dec, local scan) in LDS, barrier,
//      composes the maps of the waves before it with the carried state -> exact s,
//   3. computes c = tanh(hn + s) and publishes its h-segment map, barrier, composes -> exact h,
//   4. stores h (out) and hands the super-chunk's final (s, h) to the next one through LDS.
// The next super-chunk's gates are loaded into registers while the current one computes, and
// the barriers order LDS only, so those loads stay in flight (HBM stream never drains).
// B*D/64 workgroups x NW waves: 256 x 8 = 2048 waves at the B=32, D=512 training shape.
//
// The forward checkpoints (s, h) at every super-chunk start (B*ceil(T/64)*2*D floats, 1/32 of the
// output); the backward walks super-chunks in reverse, recomputes s, c, h from the gates it
// reads anyway (no re-read of `out`), then runs the two adjoint scans the same chunked way:
//   Gh_t = dout_t + zg_{t+1} Gh_{t+1}
//   Gs_t = Gh_t (1-zg_t)(1-c_t^2) + dec_{t+1} Gs_{t+1},   Gs_{T-1} += ds_last
// and writes the 7 gate gradients.  Algorithmic HBM bytes per (b,t,d): fwd 7e + e (+ckpt),
// bwd 7e + e + 7e.

#include "sc_common.h"

namespace sc {

constexpr int kChunk = 64;   // time steps per super-chunk (== NW * LC for every variant)
constexpr float kEps = 1e-6f;

struct ScanFwdArgs {
  const void* gates;
  const float* bias;   // optional fp32 [7,D] gate bias added on load (NULL: gates are biased)
  const float* h0;
  const float* s0;
  void* out;
  float* s_out;
  float* ckpt;
  int B, T, D, nsc;
  int64_t g_bt, g_td, g_cd, o_bt, o_bd;
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
  int64_t g_bt, g_td, g_cd, d_bt, d_bd, dg_bt, dg_td, dg_cd;
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

__device__ __forceinline__ float tanh_sig(float x) { return sigm(2.0f * x) * 2.0f - 1.0f; }

// Gradient of one step w.r.t. its 7 raw gates, given the step's adjoints.
//   gh   = dL/dh_t (total), dpre = dL/d(hn + s_t), gs = dL/ds_t (total)
__device__ __forceinline__ void gate_grads(float r, float z, float k, float v, float hp, float dc,
                                           float al, float gh, float dpre, float gs, float hprev,
                                           float sprev, float c, float (&o)[7]) {
  const float rc2 = (r * r + z * z) * 0.5f + kEps;
  const float irc = rsq(rc2);
  const float zg = sigm(z * irc);
  const float ird = rsq(dc * dc + kEps);
  const float dec = sigm(dc * ird);
  const float ira = rsq(al * al + kEps);
  const float alp = sigm(al * ira);
  const float irh = rsq(hp * hp + kEps);
  const float q = (k * k + v * v) * 0.5f + kEps;
  const float iq = rsq(q);
  const float iqe = rcp(q + kEps);
  const float kv = (k * iq) * (v * iq) * iqe;
  // zg = sigm(z / rho_c): d/dz = (r^2/2 + eps)/rho_c^3, d/dr = -z r / (2 rho_c^3)
  const float d_zn = gh * (hprev - c) * zg * (1.0f - zg);
  const float irc3 = irc * irc * irc;
  o[0] = -d_zn * z * r * 0.5f * irc3;
  o[1] = d_zn * (r * r * 0.5f + kEps) * irc3;
  // kv = k v f(q), f = 1/(q (q+eps)), f' = -(2q+eps) f^2, dq/dk = k, dq/dv = v
  const float d_kv = gs * alp;
  const float f = iq * iq * iqe;
  const float fp = -(2.0f * q + kEps) * f * f;
  o[2] = d_kv * v * (f + k * k * fp);
  o[3] = d_kv * k * (f + v * v * fp);
  // x / sqrt(x^2 + eps): derivative eps / rho^3
  o[4] = dpre * kEps * (irh * irh * irh);
  o[5] = gs * sprev * dec * (1.0f - dec) * kEps * (ird * ird * ird);
  o[6] = gs * kv * alp * (1.0f - alp) * kEps * (ira * ira * ira);
}

// ------------------------------------------------------------------------ forward ----------
template <int DT, int NW, int LC>
__global__ void __launch_bounds__(NW * 64)
lucy_scan_fwd_kernel(ScanFwdArgs a) {
  static_assert(NW * LC == kChunk, "super-chunk must be 64 steps");
  using E = Elem<DT>;
  using T = typename E::T;
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int d = blockIdx.x * 64 + lane;
  const bool dok = d < a.D;
  const int dc = dok ? d : a.D - 1;           // clamped column: loads never leave the row

  __shared__ float2 aggS[NW][64];
  __shared__ float2 aggH[NW][64];
  __shared__ float carS[2][64];
  __shared__ float carH[2][64];

  // per-row buffer descriptors; lane offset = column, scalar offset = (t, gate)
  const Buf<T> gbuf((const T*)a.gates + (int64_t)b * a.g_bt);
  const Buf<T> obuf((T*)a.out + (int64_t)b * a.o_bt);
  const uint32_t vg = (uint32_t)dc * sizeof(T);
  const uint32_t vo = (uint32_t)d * sizeof(T);
  const uint32_t gtd = (uint32_t)(a.g_td * sizeof(T)), gcd = (uint32_t)(a.g_cd * sizeof(T));
  const uint32_t otd = (uint32_t)(a.o_bd * sizeof(T));
  if (w == 0) {
    carS[0][lane] = dok ? a.s0[(int64_t)b * a.D + d] : 0.0f;
    carH[0][lane] = dok ? a.h0[(int64_t)b * a.D + d] : 0.0f;
  }

  // Two register buffers used ping-pong (explicitly, so no register copy ever waits on a
  // load that is still in flight): super-chunk k+1 streams in while k computes.
  uint32_t bufA[LC][7], bufB[LC][7];   // raw gate words (Elem::ldw)
  float gb[7];
#pragma unroll
  for (int g = 0; g < 7; ++g) gb[g] = a.bias ? a.bias[g * a.D + dc] : 0.0f;
  const int Tm1 = a.T - 1;
  auto load = [&](uint32_t (&buf)[LC][7], int k) {
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const uint32_t so = (uint32_t)min(k * kChunk + w * LC + j, Tm1) * gtd;
#pragma unroll
      for (int g = 0; g < 7; ++g) buf[j][g] = gbuf.ldw(vg, so + g * gcd);
    }
  };
  auto body = [&](const uint32_t (&cur)[LC][7], int k) __attribute__((always_inline)) {
    const int t0 = k * kChunk + w * LC;
    float zg[LC], dec[LC], u[LC], x[LC];
    float As = 1.0f, Bs = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      if (t0 + j < a.T) {
        step_terms(E::ldw(cur[j][0]) + gb[0], E::ldw(cur[j][1]) + gb[1], E::ldw(cur[j][2]) + gb[2],
                   E::ldw(cur[j][3]) + gb[3], E::ldw(cur[j][4]) + gb[4], E::ldw(cur[j][5]) + gb[5],
                   E::ldw(cur[j][6]) + gb[6], zg[j], dec[j], u[j], x[j]);
      } else {  // identity step past the end of the sequence
        zg[j] = 1.0f; dec[j] = 1.0f; u[j] = 0.0f; x[j] = 0.0f;
      }
      As *= dec[j];
      Bs = dec[j] * Bs + u[j];
    }
    aggS[w][lane] = make_float2(As, Bs);
    lds_barrier();
    float s = carS[k & 1][lane];
    if (w == 0 && a.ckpt && dok) a.ckpt[((int64_t)(b * a.nsc + k) * 2) * a.D + d] = s;
    for (int q = 0; q < w; ++q) {
      const float2 m = aggS[q][lane];
      s = m.x * s + m.y;
    }
    float Ah = 1.0f, Bh = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      s = dec[j] * s + u[j];
      x[j] = tanh_sig(x[j] + s);
      Ah *= zg[j];
      Bh = zg[j] * Bh + (1.0f - zg[j]) * x[j];
    }
    if (w == NW - 1) carS[(k + 1) & 1][lane] = s;
    aggH[w][lane] = make_float2(Ah, Bh);
    lds_barrier();
    float h = carH[k & 1][lane];
    if (w == 0 && a.ckpt && dok) a.ckpt[((int64_t)(b * a.nsc + k) * 2 + 1) * a.D + d] = h;
    for (int q = 0; q < w; ++q) {
      const float2 m = aggH[q][lane];
      h = m.x * h + m.y;
    }
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      h = zg[j] * h + (1.0f - zg[j]) * x[j];
      if (dok && t0 + j < a.T) obuf.st(E::st(h), vo, (uint32_t)(t0 + j) * otd);
    }
    if (w == NW - 1) carH[(k + 1) & 1][lane] = h;
  };
  if (a.nsc > 0) load(bufA, 0);
  lds_barrier();
  // Prefetches are unconditional: past the end the clamped time index re-reads row T-1 (a cache
  // hit); a branch around them would make hipcc's vmcnt bookkeeping fall back to full drains.
  for (int k = 0; k < a.nsc; k += 2) {
    load(bufB, k + 1);
    body(bufA, k);
    if (k + 1 >= a.nsc) break;
    load(bufA, k + 2);
    body(bufB, k + 1);
  }
  lds_barrier();
  if (w == 0 && dok) a.s_out[(int64_t)b * a.D + d] = carS[a.nsc & 1][lane];
}

// ------------------------------------------------------------------------ backward ---------
template <int DT, int NW, int LC>
__global__ void __launch_bounds__(NW * 64)
lucy_scan_bwd_kernel(ScanBwdArgs a) {
  static_assert(NW * LC == kChunk, "super-chunk must be 64 steps");
  using E = Elem<DT>;
  using T = typename E::T;
  const int lane = threadIdx.x & 63;
  const int w = uniform(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int d = blockIdx.x * 64 + lane;
  const bool dok = d < a.D;
  const int dc = dok ? d : a.D - 1;

  __shared__ float2 aggA[NW][64];
  __shared__ float2 aggB[NW][64];
  __shared__ float carGh[2][64];
  __shared__ float carGs[2][64];
  __shared__ float stS[NW][LC][64];   // s_{t-1} per step (recomputed forward), LDS not VGPRs
  __shared__ float stH[NW][LC][64];   // h_{t-1}
  // 16-bit gates: the current super-chunk's raw gates are parked in LDS (wave-private rows) so
  // their registers are free while the next super-chunk's prefetch is in flight.
  constexpr bool kStage = sizeof(T) == 2;
  __shared__ uint16_t rawS[kStage ? NW : 1][LC][7][64];

  const Buf<T> gbuf((const T*)a.gates + (int64_t)b * a.g_bt);
  const Buf<T> dbuf((const T*)a.dout + (int64_t)b * a.d_bt);
  const Buf<T> obuf((T*)a.dgates + (int64_t)b * a.dg_bt);
  const uint32_t vg = (uint32_t)dc * sizeof(T);
  const uint32_t vo = (uint32_t)d * sizeof(T);
  const uint32_t gtd = (uint32_t)(a.g_td * sizeof(T)), gcd = (uint32_t)(a.g_cd * sizeof(T));
  const uint32_t dtd = (uint32_t)(a.d_bd * sizeof(T));
  const uint32_t otd = (uint32_t)(a.dg_td * sizeof(T)), ocd = (uint32_t)(a.dg_cd * sizeof(T));
  if (w == 0) {
    carGh[0][lane] = 0.0f;
    carGs[0][lane] = (a.ds_last && dok) ? a.ds_last[(int64_t)b * a.D + d] : 0.0f;
  }

  uint32_t bufA[LC][7], bufB[LC][7];   // raw gate words (Elem::ldw), ping-pong
  uint32_t dbA[LC], dbB[LC];
  // gate bias through LDS (one word per lane and gate): at 128 VGPRs the backward has no room
  // for 7 more live registers
  __shared__ float gbS[7][64];
  if (w == 0) {
#pragma unroll
    for (int g = 0; g < 7; ++g) gbS[g][lane] = a.bias ? a.bias[g * a.D + dc] : 0.0f;
  }
#define gb(g) gbS[g][lane]
  float ckA[2], ckB[2];                // (s, h) checkpoint at the super-chunk start
  const Buf<float> cbuf(a.ckpt + (int64_t)b * a.nsc * 2 * a.D);
  const uint32_t vc = (uint32_t)dc * 4;
  const int Tm1 = a.T - 1;
  // checkpoint words first: they are then the OLDEST loads of the group, so consuming them
  // never waits on the gate stream behind them
  auto load = [&](uint32_t (&buf)[LC][7], uint32_t (&db)[LC], float (&ck)[2], int k) {
    ck[0] = cbuf.ld(vc, (uint32_t)(k * 2) * a.D * 4);
    ck[1] = cbuf.ld(vc, (uint32_t)(k * 2 + 1) * a.D * 4);
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const uint32_t t = (uint32_t)min(k * kChunk + w * LC + j, Tm1);
#pragma unroll
      for (int g = 0; g < 7; ++g) buf[j][g] = gbuf.ldw(vg, t * gtd + g * gcd);
      db[j] = dbuf.ldw(vg, t * dtd);
    }
  };
  float bacc[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // bias-gradient partial sums
  auto body = [&](const uint32_t (&cur)[LC][7], const uint32_t (&dcur)[LC], const float (&ck)[2],
                  int it) __attribute__((always_inline)) {
    const int k = a.nsc - 1 - it;
    const int t0 = k * kChunk + w * LC;
    const float s_ck = ck[0];
    const float h_ck = ck[1];
    float zg[LC], dec[LC], u[LC], x[LC];
    // ---- recompute the forward of this super-chunk ----
    float As = 1.0f, Bs = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      if constexpr (kStage) {
#pragma unroll
        for (int g = 0; g < 7; ++g) rawS[w][j][g][lane] = (uint16_t)cur[j][g];
      }
      if (t0 + j < a.T) {
        step_terms(E::ldw(cur[j][0]) + gb(0), E::ldw(cur[j][1]) + gb(1), E::ldw(cur[j][2]) + gb(2),
                   E::ldw(cur[j][3]) + gb(3), E::ldw(cur[j][4]) + gb(4), E::ldw(cur[j][5]) + gb(5),
                   E::ldw(cur[j][6]) + gb(6), zg[j], dec[j], u[j], x[j]);
      } else {
        zg[j] = 1.0f; dec[j] = 1.0f; u[j] = 0.0f; x[j] = 0.0f;
      }
      As *= dec[j];
      Bs = dec[j] * Bs + u[j];
    }
    aggA[w][lane] = make_float2(As, Bs);
    lds_barrier();                                             // B1
    float s = s_ck;
    for (int q = 0; q < w; ++q) {
      const float2 m = aggA[q][lane];
      s = m.x * s + m.y;
    }
    float Ah = 1.0f, Bh = 0.0f;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      stS[w][j][lane] = s;
      s = dec[j] * s + u[j];
      x[j] = tanh_sig(x[j] + s);
      Ah *= zg[j];
      Bh = zg[j] * Bh + (1.0f - zg[j]) * x[j];
    }
    aggB[w][lane] = make_float2(Ah, Bh);
    lds_barrier();                                             // B2
    float h = h_ck;
    for (int q = 0; q < w; ++q) {
      const float2 m = aggB[q][lane];
      h = m.x * h + m.y;
    }
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      stH[w][j][lane] = h;
      h = zg[j] * h + (1.0f - zg[j]) * x[j];
    }
    // ---- adjoint of h: C_t = zg_t Gh_t flows to step t-1 ----
    float Ph = 1.0f, Qh = 0.0f;
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      const float dj = (t0 + j < a.T) ? E::ldw(dcur[j]) : 0.0f;
      Qh = zg[j] * (dj + Qh);
      Ph *= zg[j];
    }
    aggA[w][lane] = make_float2(Ph, Qh);
    lds_barrier();                                             // B3
    float C = carGh[it & 1][lane];
    for (int q = NW - 1; q > w; --q) {
      const float2 m = aggA[q][lane];
      C = m.x * C + m.y;
    }
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      const float dj = (t0 + j < a.T) ? E::ldw(dcur[j]) : 0.0f;
      u[j] = dj + C;                                            // Gh_t
      C = zg[j] * u[j];
    }
    if (w == 0) carGh[(it + 1) & 1][lane] = C;
    // ---- adjoint of s: Cs_t = dec_t Gs_t flows to step t-1 ----
    float Ps = 1.0f, Qs = 0.0f;
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      Qs = dec[j] * (u[j] * (1.0f - zg[j]) * (1.0f - x[j] * x[j]) + Qs);
      Ps *= dec[j];
    }
    aggB[w][lane] = make_float2(Ps, Qs);
    lds_barrier();                                             // B4
    float Cs = carGs[it & 1][lane];
    for (int q = NW - 1; q > w; --q) {
      const float2 m = aggB[q][lane];
      Cs = m.x * Cs + m.y;
    }
#pragma unroll
    for (int j = LC - 1; j >= 0; --j) {
      const float dpre = u[j] * (1.0f - zg[j]) * (1.0f - x[j] * x[j]);
      const float gs = dpre + Cs;
      Cs = dec[j] * gs;
      if (dok && t0 + j < a.T) {
        float o[7], g7[7];
#pragma unroll
        for (int g = 0; g < 7; ++g)
          g7[g] = (kStage ? E::ldw((uint32_t)rawS[w][j][g][lane]) : E::ldw(cur[j][g])) + gb(g);
        gate_grads(g7[0], g7[1], g7[2], g7[3], g7[4], g7[5], g7[6], u[j], dpre, gs,
                   stH[w][j][lane], stS[w][j][lane], x[j], o);
        const uint32_t so = (uint32_t)(t0 + j) * otd;
#pragma unroll
        for (int g = 0; g < 7; ++g) {
          const T og = E::st(o[g]);
          obuf.st(og, vo, so + g * ocd);
          bacc[g] += E::ld(og);   // sum what is stored, so db == dgates.sum() exactly as a GEMM sees it
        }
      }
    }
    if (w == 0) carGs[(it + 1) & 1][lane] = Cs;
  };
  if (a.nsc > 0) load(bufA, dbA, ckA, a.nsc - 1);
  lds_barrier();
  for (int it = 0; it < a.nsc; it += 2) {
    load(bufB, dbB, ckB, max(a.nsc - 2 - it, 0));
    body(bufA, dbA, ckA, it);
    if (it + 1 >= a.nsc) break;
    load(bufA, dbA, ckA, max(a.nsc - 3 - it, 0));
    body(bufB, dbB, ckB, it + 1);
  }
  lds_barrier();
  if (w == 0 && dok) {
    a.dh0[(int64_t)b * a.D + d] = carGh[a.nsc & 1][lane];
    a.ds0[(int64_t)b * a.D + d] = carGs[a.nsc & 1][lane];
  }
#undef gb
  if (a.dbias) {   // reduce the per-wave partials over the NW waves (fixed order: deterministic)
#pragma unroll
    for (int g = 0; g < 7; ++g) {
      stS[w][0][lane] = bacc[g];
      lds_barrier();
      if (w == 0) {
        float acc = 0.0f;
        for (int q = 0; q < NW; ++q) acc += stS[q][0][lane];
        if (dok) a.dbias[((int64_t)b * 7 + g) * a.D + d] = acc;
      }
      lds_barrier();
    }
  }
}

// ------------------------------------------------------------------------ launchers --------
// Wave split of the 64-step super-chunk.  NW=8 x LC=8: 8 waves per workgroup (one workgroup
// per CU at B*D/64 = 256).  Selected per dtype from measurements.
template <int DT> struct FwdCfg { static constexpr int NW = 16, LC = 4; };
template <int DT> struct BwdCfg { static constexpr int NW = 16, LC = 4; };

template <int DT>
static void launch_fwd(const ScanFwdArgs& a, hipStream_t st) {
  constexpr int NW = FwdCfg<DT>::NW, LC = FwdCfg<DT>::LC;
  dim3 grid((a.D + 63) / 64, a.B);
  hipLaunchKernelGGL((lucy_scan_fwd_kernel<DT, NW, LC>), grid, dim3(NW * 64), 0, st, a);
}

template <int DT>
static void launch_bwd(const ScanBwdArgs& a, hipStream_t st) {
  constexpr int NW = BwdCfg<DT>::NW, LC = BwdCfg<DT>::LC;
  dim3 grid((a.D + 63) / 64, a.B);
  hipLaunchKernelGGL((lucy_scan_bwd_kernel<DT, NW, LC>), grid, dim3(NW * 64), 0, st, a);
}

}  // namespace sc

using namespace sc;

extern "C" int sc_lucy_scan_chunk(void) { return kChunk; }

extern "C" int64_t sc_lucy_scan_ckpt_numel(int B, int T, int D) {
  if (B < 0 || T < 0 || D < 0) return 0;
  return (int64_t)B * ((T + kChunk - 1) / kChunk) * 2 * D;
}

static int check_dtype(int dt) { return dt == SC_F32 || dt == SC_BF16 || dt == SC_F16; }

extern "C" int sc_lucy_scan_fwd(const void* gates, int gates_dtype, const float* gate_bias,
                                const float* h0,
                                const float* s0, void* out, float* s_out, int B, int T, int D,
                                int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                                int64_t stride_o_bt, int64_t stride_o_bd, float* ckpt,
                                void* stream) {
  clear_error();
  SC_REQUIRE(check_dtype(gates_dtype), "sc_lucy_scan_fwd: unsupported gates dtype %d", gates_dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && D >= 0, "sc_lucy_scan_fwd: negative shape B=%d T=%d D=%d", B, T, D);
  SC_REQUIRE(B <= 65535, "sc_lucy_scan_fwd: B=%d exceeds grid limit 65535", B);
  if (B == 0 || D == 0) return 0;
  SC_REQUIRE(h0 && s0 && s_out, "sc_lucy_scan_fwd: null state pointer");
  SC_REQUIRE(T == 0 || (gates && out), "sc_lucy_scan_fwd: null gates/out pointer");
  ScanFwdArgs a{gates, gate_bias, h0, s0, out, s_out, ckpt, B, T, D, (T + kChunk - 1) / kChunk,
                stride_g_bt, stride_g_td, stride_g_cd, stride_o_bt, stride_o_bd};
  hipStream_t st = (hipStream_t)stream;
  switch (gates_dtype) {
    case SC_F32: launch_fwd<SC_F32>(a, st); break;
    case SC_BF16: launch_fwd<SC_BF16>(a, st); break;
    default: launch_fwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_lucy_scan_fwd");
}

extern "C" int sc_lucy_scan_bwd(const void* gates, int gates_dtype, const float* gate_bias,
                                const float* ckpt,
                                const void* dout, const float* ds_last, void* dgates, float* dh0,
                                float* ds0, float* dbias, int B, int T, int D, int64_t stride_g_bt,
                                int64_t stride_g_td, int64_t stride_g_cd, int64_t stride_d_bt,
                                int64_t stride_d_bd, int64_t stride_dg_bt, int64_t stride_dg_td,
                                int64_t stride_dg_cd, void* stream) {
  clear_error();
  SC_REQUIRE(check_dtype(gates_dtype), "sc_lucy_scan_bwd: unsupported gates dtype %d", gates_dtype);
  SC_REQUIRE(B >= 0 && T >= 0 && D >= 0, "sc_lucy_scan_bwd: negative shape B=%d T=%d D=%d", B, T, D);
  SC_REQUIRE(B <= 65535, "sc_lucy_scan_bwd: B=%d exceeds grid limit 65535", B);
  if (B == 0 || D == 0) return 0;
  SC_REQUIRE(dh0 && ds0, "sc_lucy_scan_bwd: null dh0/ds0");
  if (T == 0 && dbias) (void)hipMemsetAsync(dbias, 0, sizeof(float) * 7 * B * D, (hipStream_t)stream);
  SC_REQUIRE(T == 0 || (gates && ckpt && dout && dgates),
             "sc_lucy_scan_bwd: null gates/ckpt/dout/dgates pointer");
  ScanBwdArgs a{gates, gate_bias, ckpt, dout, ds_last, dgates, dh0, ds0, dbias, B, T, D,
                (T + kChunk - 1) / kChunk,
                stride_g_bt, stride_g_td, stride_g_cd, stride_d_bt, stride_d_bd,
                stride_dg_bt, stride_dg_td, stride_dg_cd};
  hipStream_t st = (hipStream_t)stream;
  switch (gates_dtype) {
    case SC_F32: launch_bwd<SC_F32>(a, st); break;
    case SC_BF16: launch_bwd<SC_BF16>(a, st); break;
    default: launch_bwd<SC_F16>(a, st); break;
  }
  return launch_status("sc_lucy_scan_bwd");
}
