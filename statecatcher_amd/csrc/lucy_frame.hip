// Streaming frame of the native LucyRNN (infer mode) as a short chain of fused kernels — SURVEY
// §8(f) row 2: the reference's per-frame loop lucyrnn.py:172-184, LucyRNNCell.forward
// (lucyrnn.py:44-70) at T = 1, with the state resident in HBM in fp32 between calls.
//
// A frame of B streams is, per layer (u = LN_in(a) etc. as in lucyrnn.py:45-68):
//   lucy_frame_gemm  PRO_NONE / EPI_STATS  a = x W_in^T + b_in, plus per-row LayerNorm partial
//                                          statistics of a (one record per 32 output columns)
//   lucy_frame_gemm  PRO_LN / EPI_CELL     g = LN_in(a) W_g^T + b_g, the workgroup owning 16 units
//                                          of EVERY gate, so the cell's elementwise part runs in
//                                          its epilogue: s' = sigmoid(dl) s + k v (state, masked),
//                                          then unfused: y = u + s' (the input of W_h); fused:
//                                          hp = h_pre + s'; z and hp with their row statistics
//   lucy_frame_gemm  PRO_NONE / EPI_STATS  (unfused) hp = y W_h^T + b_h, statistics of hp
//   lucy_frame_cellb                       h = (1 - sigmoid(LN_z z)) tanh(LN_h hp)
//                                              + sigmoid(LN_z z) h_prev, masked; the next input
// and after the last layer the output projection (lucy_frame_gemm PRO_NONE / EPI_PLAIN) and the
// greedy step (sc_ctc_greedy_step, decode.hip).  The W_r rows are never computed: the reference
// evaluates sigmoid(LN_r(W_r u)) and never uses it.
//
// LayerNorm (nn.LayerNorm: biased variance, eps inside the rsqrt) is split over the producing GEMM
// and its consumer: every producer workgroup writes (n, mean, M2) of its columns per row, the
// consumer combines the records (Chan's parallel formula) and normalises on load — no separate
// LayerNorm launch and no second pass over the activations.
//
// GEMM tiling (B streams x N outputs x K, B <= a few hundred: skinny): one wave computes one 16 x 16
// output tile over a K slice on MFMA — v_mfma_f32_16x16x4_f32 for fp32 weights (exact f32 products,
// the reference's arithmetic), v_mfma_f32_16x16x32_bf16 for bf16 weights (activations rounded to
// bf16 on load, fp32 accumulate); a workgroup holds NT tiles x KS K-slices, summed through LDS.
// Activations between kernels are fp32.
#include "sc_common.h"

#include <algorithm>

// SC_FRAME_ABL: ablation bitmask for tools timing only (never set in a shipped build; wrong
// results): 1 no MFMAs (fp32 weights), 2 no epilogue stores, 4 no weight loads, 8 no A-row loads
#ifndef SC_FRAME_ABL
#define SC_FRAME_ABL 0
#endif

namespace sc {

enum { FR_PLAIN = 0, FR_STATS = 1, FR_CELL_UNFUSED = 2, FR_CELL_FUSED = 3 };

struct FrameGemmArgs {
  const float* x;        // [B][ldx] fp32 activations (the A operand, before the prologue)
  int64_t ldx;
  int K;                 // reduction length
  const float* ln_w;     // PRO_LN: LayerNorm weight / bias over K (NULL: no prologue)
  const float* ln_b;
  const float4* st_in;   // PRO_LN: [nst_in][B] (n, mean, M2, -) records of x's rows
  int nst_in;
  float eps;
  const void* w;         // [N][ldw] weights (fp32 or bf16): output column j = row j
  int64_t ldw;
  const float* bias;     // [N]
  int B, N;
  int gstride;           // EPI_CELL: W row of gate g, unit d = g * gstride + d (gstride = D)
  // outputs
  float* y;              // PLAIN / STATS: [B][ldy]; CELL: y (unfused) or hp (fused) [B][D]
  int64_t ldy;
  float4* st_out;        // STATS: [ceil(N / 32)][B]; CELL: [D / 16][B] records of y/hp (fused)
  float* z;              // CELL: raw z [B][D]
  float4* st_z;          // CELL: [D / 16][B] records of z
  float* s;              // CELL: fp32 state [B][D], in place
  const float* mask;     // CELL: [B] or NULL
};

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Chan's combination of (n, mean, M2) records -> (mean, rstd) of the full row
__device__ __forceinline__ void combine_stats(const float4* rec, int nrec, int64_t stride,
                                              float eps, float& mean, float& rstd) {
  float n = 0.0f, sm = 0.0f;
  for (int i = 0; i < nrec; ++i) {
    const float4 r = rec[i * stride];
    n += r.x;
    sm += r.x * r.y;
  }
  mean = sm / n;
  float m2 = 0.0f;
  for (int i = 0; i < nrec; ++i) {
    const float4 r = rec[i * stride];
    const float d = r.y - mean;
    m2 += r.z + r.x * d * d;
  }
  rstd = 1.0f / sqrtf(m2 / n + eps);
}

// Chan's combination of two (n, mean, M2) records
__device__ __forceinline__ float4 chan2(float4 a, float4 b) {
  const float n = a.x + b.x;
  if (n == 0.0f) return a;
  const float d = b.y - a.y, f = b.x / n;
  return make_float4(n, a.y + d * f, a.z + b.z + d * d * a.x * f, 0.0f);
}
// the records of lanes l, l ^ 1, ..., l ^ (W - 1) combined (xor butterflies over W lanes): every
// lane of the group ends with the group's total
template <int W>
__device__ __forceinline__ float4 chan_xor(float4 r) {
#pragma unroll
  for (int o = 1; o < W; o <<= 1) {
    const float4 q = make_float4(__shfl_xor(r.x, o), __shfl_xor(r.y, o), __shfl_xor(r.z, o), 0.0f);
    r = chan2(r, q);
  }
  return r;
}
// (mean, rstd) of one row from its nrec <= 64 records (stride apart), one record per lane
__device__ __forceinline__ float2 row_stats_wave(const float4* rec, int nrec, int64_t stride,
                                                 float eps, int lane) {
  float4 r = lane < nrec ? rec[(int64_t)lane * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
  r = chan_xor<64>(r);
  return make_float2(r.y, 1.0f / sqrtf(r.z / r.x + eps));
}

// (n, mean, M2) of 16 values held by the 16 lanes of a lane group (xor butterflies within it)
__device__ __forceinline__ float4 stats16(float v) {
  float sm = v;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) sm += __shfl_xor(sm, o);
  const float mean = sm * (1.0f / 16.0f);
  float d = (v - mean) * (v - mean);
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) d += __shfl_xor(d, o);
  return make_float4(16.0f, mean, d, 0.0f);
}

// One workgroup: rows r0 .. r0 + 15, NT output tiles x KS K-slices (one wave each).
//   PLAIN / STATS: tile t = columns n0 + 16 t .. (n0 = blockIdx.x * 16 NT)
//   CELL: tile t = gate t, units d0 .. d0 + 15 (d0 = 16 blockIdx.x), W rows t * gstride + d
// (bx, by) = the workgroup's column block and 16-row block; the kernels below pass blockIdx
template <bool BF16W, bool LN, int EPI, int NT, int KS>
__device__ __forceinline__ void frame_gemm_body(const FrameGemmArgs& a, const int bx, const int by) {
  __shared__ float part[NT * KS][16][17];   // per-wave 16 x 16 partial sums (padded rows)
  __shared__ float stat[16][2];             // PRO_LN: (mean, rstd) of the workgroup's rows
  extern __shared__ __attribute__((aligned(16))) float xs[];   // the A rows [16][kpitch]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform: scalar)
  const int t = w % NT, ks = w / NT;
  const int r0 = by * 16;
  constexpr bool CELL = EPI == FR_CELL_UNFUSED || EPI == FR_CELL_FUSED;
  constexpr int KSTEP = BF16W ? 32 : 16;
  const int cbase = CELL ? bx * 16 + t * a.gstride : (bx * NT + t) * 16;
  const int nsteps = (a.K + KSTEP - 1) / KSTEP;
  const int kpad = nsteps * KSTEP, kpitch = kpad + 4;   // +4 floats: conflict-free row reads
  const int col = cbase + (lane & 15);
  const bool cok = CELL || col < a.N;
  const int sb = (int)((int64_t)nsteps * ks / KS), se = (int)((int64_t)nsteps * (ks + 1) / KS);
  const int q = lane >> 4;
  constexpr int NTH = 64 * NT * KS;
  // Latency chain of a frame kernel: one memory round trip for everything the MFMAs need (the
  // first weight chunk, the A rows, the LayerNorm records and parameters, the epilogue's bias /
  // state / mask), then the MFMAs, then the epilogue.  So every one of those loads is issued
  // before the first wait.
  constexpr int SMAXF = 8;   // fp32: steps per weight chunk (few registers: two workgroups per CU)
  constexpr int SMAXB = 8;                      // bf16
  float4 wf[BF16W ? 1 : SMAXF];
  bf16x8 wh[BF16W ? SMAXB : 1];
  const float* wrf = (const float*)a.w + (int64_t)(cok ? col : 0) * a.ldw;
  const __bf16* wrh = (const __bf16*)a.w + (int64_t)(cok ? col : 0) * a.ldw;
  auto load_chunk = [&](int c0) __attribute__((always_inline)) {
    if constexpr (!BF16W) {
#pragma unroll
      for (int i = 0; i < SMAXF; ++i)
        wf[i] = (SC_FRAME_ABL & 4) ? make_float4((float)c0, 1.f, 1.f, 1.f)
                                   : *(const float4*)(wrf + min((c0 + i) * 16 + 4 * q, a.K - 4));
    } else {
#pragma unroll
      for (int i = 0; i < SMAXB; ++i) wh[i] = *(const bf16x8*)(wrh + min((c0 + i) * 32 + 8 * q, a.K - 8));
    }
  };
  load_chunk(sb);
  // epilogue operands
  float e_bias[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, e_s = 0.f, e_m = 1.f;
  {
    if constexpr (CELL) {
      if (w < 4) {
        const int rr = 4 * w + q, rc = min(r0 + rr, a.B - 1), d = bx * 16 + (lane & 15);
#pragma unroll
        for (int g = 0; g < (EPI == FR_CELL_FUSED ? 5 : 4); ++g) e_bias[g] = a.bias[g * a.gstride + d];
        e_s = a.s[(int64_t)rc * a.gstride + d];
        if (a.mask) e_m = a.mask[rc];
      }
    } else {
      if (w < NT && cok) e_bias[0] = a.bias[col];
    }
  }
  // The workgroup's 16 A rows (LayerNorm applied, rows past B and columns past K zero) into LDS
  // with coalesced 16-byte loads: every wave then reads its fragments from LDS, and no global
  // load of the MFMA loop depends on a row or K condition.  Up to 4 pieces per thread are loaded
  // before the LayerNorm statistics are combined.
  {
    const int per_row = kpad / 4;   // float4 pieces per row
    const int npc = 16 * per_row;
    for (int i0 = 0; i0 < npc; i0 += 4 * NTH) {
      float4 v[4], lw[4], lb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = i0 + j * NTH + threadIdx.x;
        const int rr = i / per_row, k = 4 * (i % per_row), r = r0 + rr;
        v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < npc && r < a.B && k < a.K) {   // (K % 4 == 0: a piece is wholly in or out)
          if (!(SC_FRAME_ABL & 8)) v[j] = *(const float4*)(a.x + (int64_t)r * a.ldx + k);
          if (LN) {
            lw[j] = *(const float4*)(a.ln_w + k);
            lb[j] = *(const float4*)(a.ln_b + k);
          }
        }
      }
      if (LN && i0 == 0) {   // the row statistics, once per workgroup, while the pieces load
        if (a.nst_in <= 64) {   // wave w: rows w, w + nwaves, ...; one record per lane
          for (int rr = w; rr < 16; rr += NT * KS) {
            const float2 st = row_stats_wave(a.st_in + min(r0 + rr, a.B - 1), a.nst_in, a.B,
                                             a.eps, lane);
            if (lane == 0) {
              stat[rr][0] = st.x;
              stat[rr][1] = st.y;
            }
          }
        } else if (threadIdx.x < 16) {
          const int r = min(r0 + (int)threadIdx.x, a.B - 1);
          float mean, rstd;
          combine_stats(a.st_in + r, a.nst_in, a.B, a.eps, mean, rstd);
          stat[threadIdx.x][0] = mean;
          stat[threadIdx.x][1] = rstd;
        }
        __syncthreads();
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = i0 + j * NTH + threadIdx.x;
        const int rr = i / per_row, k = 4 * (i % per_row), r = r0 + rr;
        if (i < npc) {
          if (LN && r < a.B && k < a.K) {
            const float mu = stat[rr][0], rs = stat[rr][1];
            v[j].x = (v[j].x - mu) * rs * lw[j].x + lb[j].x;
            v[j].y = (v[j].y - mu) * rs * lw[j].y + lb[j].y;
            v[j].z = (v[j].z - mu) * rs * lw[j].z + lb[j].z;
            v[j].w = (v[j].w - mu) * rs * lw[j].w + lb[j].w;
          }
          *(float4*)(xs + rr * kpitch + k) = v[j];
        }
      }
    }
    __syncthreads();
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* xrow = xs + (lane & 15) * kpitch;
  // A chunk runs SMAX steps: a load past the slice or past K reads a clamped address (always
  // inside the matrix) and the LDS operand's k slots there are zeroed by a select (no branch
  // around a load, no per-step wait).  Columns past N read W row 0 and are never stored.
  if constexpr (!BF16W) {
    for (int c0 = sb; c0 < se; c0 += SMAXF) {
      if (c0 != sb) load_chunk(c0);
      float4 xb[SMAXF];
#pragma unroll
      for (int i = 0; i < SMAXF; ++i) xb[i] = *(const float4*)(xrow + min((c0 + i) * 16, kpad - 16) + 4 * q);
      __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead of the MFMAs (no sinking)
#pragma unroll
      for (int i = 0; i < SMAXF; ++i) {
        const bool in = c0 + i < se && (c0 + i) * 16 + 4 * q < a.K;
        float4 xa = xb[i];
        xa.x = in ? xa.x : 0.f;
        xa.y = in ? xa.y : 0.f;
        xa.z = in ? xa.z : 0.f;
        xa.w = in ? xa.w : 0.f;
        // k slot q of MFMA j is k0 + j for both operands: the sum runs over the same k set
        if (SC_FRAME_ABL & 1) {
          acc0[0] += xa.x * wf[i].x + xa.z * wf[i].z;
          acc1[0] += xa.y * wf[i].y + xa.w * wf[i].w;
          continue;
        }
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.x, wf[i].x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.y, wf[i].y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.z, wf[i].z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa.w, wf[i].w, acc1, 0, 0, 0);
      }
    }
  } else {
    const bf16x8 zero8 = {};
    for (int c0 = sb; c0 < se; c0 += SMAXB) {
      if (c0 != sb) load_chunk(c0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < SMAXB; ++i) {
        const bool in = c0 + i < se && (c0 + i) * 32 + 8 * q < a.K;
        const int kx = min((c0 + i) * 32, kpad - 32) + 8 * q;
        const float4 x0 = *(const float4*)(xrow + kx), x1 = *(const float4*)(xrow + kx + 4);
        const bf16x8 av = {(__bf16)x0.x, (__bf16)x0.y, (__bf16)x0.z, (__bf16)x0.w,
                           (__bf16)x1.x, (__bf16)x1.y, (__bf16)x1.z, (__bf16)x1.w};
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(in ? av : zero8, wh[i], acc0, 0, 0, 0);
      }
    }
  }
  // C layout: column lane & 15, rows 4 (lane >> 4) + i
#pragma unroll
  for (int i = 0; i < 4; ++i) part[w][4 * q + i][lane & 15] = acc0[i] + acc1[i];
  __syncthreads();
  // sum the K slices into slot t (waves ks = 0)
  if (KS > 1 && ks == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = part[t][4 * q + i][lane & 15];
#pragma unroll
      for (int s = 1; s < KS; ++s) v += part[t + s * NT][4 * q + i][lane & 15];
      part[t][4 * q + i][lane & 15] = v;
    }
  }
  if (KS > 1) __syncthreads();
  if constexpr (!CELL) {
    // tile t (waves w < NT): bias, store, row statistics over the workgroup's 16 NT columns
    if (w < NT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + 4 * q + i, c = cbase + (lane & 15);
        const float v = part[w][4 * q + i][lane & 15] + e_bias[0];
        part[w][4 * q + i][lane & 15] = v;
        if (r < a.B && c < a.N) a.y[(int64_t)r * a.ldy + c] = v;
      }
    }
    if (EPI == FR_STATS) {
      // per tile (wave w < NT) and row 4 q + i: (16, mean, M2) of its 16 columns by xor
      // butterflies within each 16-lane group, then the NT tiles' records per row combined
      __shared__ float4 trec[NT][16];
      if (w < NT) {
        const int ncol = min(16 * NT, a.N - bx * 16 * NT);
        const bool live = (lane & 15) + 16 * w < ncol;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = part[w][4 * q + i][lane & 15];
          const float4 r = chan_xor<16>(live ? make_float4(1.0f, v, 0.0f, 0.0f)
                                             : make_float4(0.f, 0.f, 0.f, 0.f));
          if ((lane & 15) == 0) trec[w][4 * q + i] = r;
        }
      }
      __syncthreads();
      if (threadIdx.x < 16) {
        const int rr = threadIdx.x;
        float4 r = trec[0][rr];
#pragma unroll
        for (int t2 = 1; t2 < NT; ++t2) r = chan2(r, trec[t2][rr]);
        if (r0 + rr < a.B) a.st_out[(int64_t)bx * a.B + r0 + rr] = make_float4(r.x, r.y, r.z, 0.0f);
      }
    }
  } else {
    // the cell's elementwise part for the 16 x 16 (row, unit) elements: one per lane of wave 0..3
    if (w < 4) {
      const int rr = 4 * w + q, r = r0 + rr, d = bx * 16 + (lane & 15);
      const int D = a.gstride;
      const bool ok = r < a.B;
      auto gate = [&](int g) { return part[g][rr][lane & 15] + e_bias[g]; };
      const float z = gate(0), k = gate(1), v = gate(2);
      const float dl = gate(EPI == FR_CELL_FUSED ? 4 : 3);
      const float m = e_m;
      const float sp = e_s;
      const float sn = (1.0f / (1.0f + expf(-dl))) * sp + k * v;
      float o;
      if (EPI == FR_CELL_FUSED) {
        o = gate(3) + sn;                                   // hp = h_pre + s'
      } else {
        o = xs[rr * kpitch + d] + sn;                       // y = u + s', u = LN_in(a)
      }
      const float4 sz = stats16(z), so = stats16(o);
      if (SC_FRAME_ABL & 2) {
        asm volatile("" ::"v"(sz.x), "v"(so.x), "v"(sn), "v"(z), "v"(o));
      } else if (ok) {
        a.s[(int64_t)r * D + d] = m * sn + (1.0f - m) * sp;
        a.z[(int64_t)r * D + d] = z;
        a.y[(int64_t)r * D + d] = o;
        if ((lane & 15) == 0) {
          a.st_z[(int64_t)bx * a.B + r] = sz;
          if (a.st_out) a.st_out[(int64_t)bx * a.B + r] = so;
        }
      }
    }
  }
}

// (at most 128 VGPRs: four waves per SIMD, two 8-wave or one 16-wave workgroup per CU)
template <bool BF16W, bool LN, int EPI, int NT, int KS>
__global__ void __launch_bounds__(64 * NT * KS, 4) lucy_frame_gemm(FrameGemmArgs a) {
  frame_gemm_body<BF16W, LN, EPI, NT, KS>(a, blockIdx.x, blockIdx.y);
}

// Up to kMaxFrameJobs independent GEMMs of one epilogue kind in ONE launch (blockIdx.z = job):
// the layers of a frame block run as a wavefront over (frame, layer), so the jobs of a launch are
// different layers at different frames (streaming.py).  Workgroups past a job's column or row
// blocks leave at once (uniformly, before any barrier).
constexpr int kMaxFrameJobs = 8;
struct FrameGemmJobs {
  FrameGemmArgs j[kMaxFrameJobs];
};
template <bool BF16W, bool LN, int EPI, int NT, int KS>
__global__ void __launch_bounds__(64 * NT * KS, 4) lucy_frame_gemm_multi(FrameGemmJobs jobs) {
  const FrameGemmArgs& a = jobs.j[blockIdx.z];
  constexpr bool CELL = EPI == FR_CELL_UNFUSED || EPI == FR_CELL_FUSED;
  const int nblk = CELL ? a.gstride / 16 : (a.N + 16 * NT - 1) / (16 * NT);
  if ((int)blockIdx.x >= nblk || (int)blockIdx.y * 16 >= a.B) return;
  frame_gemm_body<BF16W, LN, EPI, NT, KS>(a, blockIdx.x, blockIdx.y);
}

// h = (1 - zg) c + zg h_prev (masked), zg = sigmoid(LN_z z), c = tanh(LN_h hp): one workgroup of
// 256 threads per row
struct FrameCellArgs {
  const float* z;
  const float4* st_z;   // [nst_z][B] or NULL (no LayerNorm)
  int nst_z;
  const float* hp;
  const float4* st_h;   // [nst_h][B] or NULL
  int nst_h;
  const float *lnz_w, *lnz_b, *lnh_w, *lnh_b;
  float eps;
  float* h;             // fp32 state [B][D], in place
  float* out;           // next layer input [B][ldo] fp32
  int64_t ldo;
  const float* mask;
  int B, D;
};

__device__ __forceinline__ void frame_cellb_body(const FrameCellArgs& a, const int r) {
  __shared__ float st[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // every operand of the row is loaded before the statistics are combined (one memory latency)
  constexpr int kPer = 4;   // D <= 1024: up to 4 units per thread in registers
  float zv[kPer], hv[kPer], hpv[kPer];
  const bool regs = a.D <= 256 * kPer;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int d = threadIdx.x + 256 * j;
    if (regs && d < a.D) {
      const int64_t i = (int64_t)r * a.D + d;
      zv[j] = a.z[i];
      hpv[j] = a.hp[i];
      hv[j] = a.h[i];
    }
  }
  // (wave 0: LN_z's records, wave 1: LN_h's; one record per lane, xor butterflies)
  if (w == 0) {
    float2 s2 = make_float2(0.0f, 1.0f);
    if (a.lnz_w) {
      if (a.nst_z <= 64) s2 = row_stats_wave(a.st_z + r, a.nst_z, a.B, a.eps, lane);
      else combine_stats(a.st_z + r, a.nst_z, a.B, a.eps, s2.x, s2.y);
    }
    if (lane == 0) { st[0] = s2.x; st[1] = s2.y; }
  } else if (w == 1) {
    float2 s2 = make_float2(0.0f, 1.0f);
    if (a.lnh_w) {
      if (a.nst_h <= 64) s2 = row_stats_wave(a.st_h + r, a.nst_h, a.B, a.eps, lane);
      else combine_stats(a.st_h + r, a.nst_h, a.B, a.eps, s2.x, s2.y);
    }
    if (lane == 0) { st[2] = s2.x; st[3] = s2.y; }
  }
  __syncthreads();
  const float m = a.mask ? a.mask[r] : 1.0f;
  if (regs) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int d = threadIdx.x + 256 * j;
      if (d < a.D) {
        float z = zv[j], hp = hpv[j];
        if (a.lnz_w) z = (z - st[0]) * st[1] * a.lnz_w[d] + a.lnz_b[d];
        if (a.lnh_w) hp = (hp - st[2]) * st[3] * a.lnh_w[d] + a.lnh_b[d];
        const float zg = 1.0f / (1.0f + expf(-z));
        const float hv2 = (1.0f - zg) * tanhf(hp) + zg * hv[j];
        const float hn = m * hv2 + (1.0f - m) * hv[j];
        a.h[(int64_t)r * a.D + d] = hn;
        a.out[(int64_t)r * a.ldo + d] = hn;
      }
    }
    return;
  }
  for (int d = threadIdx.x; d < a.D; d += 256) {
    const int64_t i = (int64_t)r * a.D + d;
    float z = a.z[i], hp = a.hp[i];
    if (a.lnz_w) z = (z - st[0]) * st[1] * a.lnz_w[d] + a.lnz_b[d];
    if (a.lnh_w) hp = (hp - st[2]) * st[3] * a.lnh_w[d] + a.lnh_b[d];
    const float zg = 1.0f / (1.0f + expf(-z));
    const float hprev = a.h[i];
    const float hv = (1.0f - zg) * tanhf(hp) + zg * hprev;
    const float hn = m * hv + (1.0f - m) * hprev;
    a.h[i] = hn;
    a.out[(int64_t)r * a.ldo + d] = hn;
  }
}

__global__ void __launch_bounds__(256) lucy_frame_cellb(FrameCellArgs a) {
  frame_cellb_body(a, blockIdx.x);
}
struct FrameCellJobs {
  FrameCellArgs j[kMaxFrameJobs];
};
__global__ void __launch_bounds__(256) lucy_frame_cellb_multi(FrameCellJobs jobs) {
  const FrameCellArgs& a = jobs.j[blockIdx.y];
  if ((int)blockIdx.x >= a.B) return;
  frame_cellb_body(a, blockIdx.x);
}

template <bool BF16W, bool LN, int EPI, int NT, int KS>
static void launch_gemm(const FrameGemmArgs& a, int nblk, hipStream_t st) {
  const int kstep = BF16W ? 32 : 16;
  const size_t lds = (size_t)16 * (((a.K + kstep - 1) / kstep) * kstep + 4) * sizeof(float);
  static bool big_lds = false;   // (the A rows of K > ~800 exceed the default 64 KB window)
  if (lds > 48 * 1024 && !big_lds) {
    (void)hipFuncSetAttribute((const void*)lucy_frame_gemm<BF16W, LN, EPI, NT, KS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
    big_lds = true;
  }
  hipLaunchKernelGGL((lucy_frame_gemm<BF16W, LN, EPI, NT, KS>), dim3(nblk, (a.B + 15) / 16),
                     dim3(64 * NT * KS), lds, st, a);
}

template <bool BF16W, bool LN, int EPI, int NT, int KS>
static void launch_gemm_multi(const FrameGemmJobs& jobs, int nj, hipStream_t st) {
  const int kstep = BF16W ? 32 : 16;
  constexpr bool CELL = EPI == FR_CELL_UNFUSED || EPI == FR_CELL_FUSED;
  size_t lds = 0;
  int gx = 1, gy = 1;
  for (int i = 0; i < nj; ++i) {
    const FrameGemmArgs& a = jobs.j[i];
    lds = std::max(lds, (size_t)16 * (((a.K + kstep - 1) / kstep) * kstep + 4) * sizeof(float));
    gx = std::max(gx, CELL ? a.gstride / 16 : (a.N + 16 * NT - 1) / (16 * NT));
    gy = std::max(gy, (a.B + 15) / 16);
  }
  static bool big_lds = false;
  if (lds > 48 * 1024 && !big_lds) {
    (void)hipFuncSetAttribute((const void*)lucy_frame_gemm_multi<BF16W, LN, EPI, NT, KS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
    big_lds = true;
  }
  hipLaunchKernelGGL((lucy_frame_gemm_multi<BF16W, LN, EPI, NT, KS>), dim3(gx, gy, nj),
                     dim3(64 * NT * KS), lds, st, jobs);
}

template <bool BF16W, bool LN>
static void dispatch_gemm_multi(int epi, const FrameGemmJobs& jobs, int nj, hipStream_t st) {
  switch (epi) {   // (the tilings of dispatch_gemm below)
    case FR_PLAIN: launch_gemm_multi<BF16W, LN, FR_PLAIN, 2, 4>(jobs, nj, st); break;
    case FR_STATS: launch_gemm_multi<BF16W, LN, FR_STATS, 2, 4>(jobs, nj, st); break;
    case FR_CELL_UNFUSED: launch_gemm_multi<BF16W, LN, FR_CELL_UNFUSED, 4, 2>(jobs, nj, st); break;
    default: launch_gemm_multi<BF16W, LN, FR_CELL_FUSED, 5, 2>(jobs, nj, st); break;
  }
}

template <bool BF16W, bool LN>
static void dispatch_gemm(int epi, int ngate, const FrameGemmArgs& a, hipStream_t st) {
  switch (epi) {
    // (K split over 3-4 waves: a wave's share of K = 512 is one weight chunk, one memory
    // latency; PLAIN / STATS 32 columns per workgroup, so a 512-wide output is 16 x B/16
    // workgroups)
    case FR_PLAIN: launch_gemm<BF16W, LN, FR_PLAIN, 2, 4>(a, (a.N + 31) / 32, st); break;
    case FR_STATS: launch_gemm<BF16W, LN, FR_STATS, 2, 4>(a, (a.N + 31) / 32, st); break;
    // (the gate GEMMs keep 2 K-slices: at 4 the 16-wave workgroups ran one per CU and took
    // 23.5 us against 19.3 us at B = 256, profiles/r4_stream_frame.md)
    case FR_CELL_UNFUSED:
      launch_gemm<BF16W, LN, FR_CELL_UNFUSED, 4, 2>(a, a.gstride / 16, st); break;
    default: launch_gemm<BF16W, LN, FR_CELL_FUSED, 5, 2>(a, a.gstride / 16, st); break;
  }
  (void)ngate;
}

}  // namespace sc

using namespace sc;

// the argument checks of one frame GEMM (0, or the error code with the message set)
static int frame_gemm_check(const char* fn, int epi, int w_dtype, const float* x, int64_t ldx,
                            int K, const float* ln_w, const float* ln_b, const void* st_in,
                            int nst_in, const void* w, int64_t ldw, const float* bias, int B, int N,
                            float* y, void* st_out, float* z, void* st_z, float* s) {
  SC_REQUIRE(epi >= FR_PLAIN && epi <= FR_CELL_FUSED, "%s: bad epilogue %d", fn, epi);
  SC_REQUIRE(w_dtype == SC_F32 || w_dtype == SC_BF16, "%s: weights fp32 or bf16", fn);
  SC_REQUIRE(B >= 0 && K > 0 && N > 0, "%s: bad shape B=%d K=%d N=%d", fn, B, K, N);
  if (B == 0) return 0;
  SC_REQUIRE(x && w && bias && y, "%s: null pointer", fn);
  SC_REQUIRE(ldx % 4 == 0 && ldw % 8 == 0 && K % 4 == 0 && (uintptr_t)x % 16 == 0 &&
                 (uintptr_t)w % 16 == 0,
             "%s: rows must be 16-byte aligned (ldx %% 4, ldw %% 8, K %% 4)", fn);
  SC_REQUIRE(w_dtype == SC_F32 || K % 8 == 0, "%s: bf16 weights need K %% 8 == 0", fn);
  SC_REQUIRE(K <= 2048, "%s: K = %d above 2048 (the A rows live in LDS)", fn, K);
  SC_REQUIRE(!ln_w || ((uintptr_t)ln_w % 16 == 0 && (uintptr_t)ln_b % 16 == 0),
             "%s: LayerNorm parameters must be 16-byte aligned", fn);
  SC_REQUIRE((ln_w == nullptr) == (ln_b == nullptr) && (!ln_w || (st_in && nst_in > 0)),
             "%s: LayerNorm prologue needs weight, bias and statistics", fn);
  const bool cell = epi >= FR_CELL_UNFUSED;
  const int ng = epi == FR_CELL_FUSED ? 5 : 4;
  if (cell) {
    SC_REQUIRE(N % (16 * ng) == 0, "%s: N = %d gates x D, D a multiple of 16", fn, N);
    SC_REQUIRE(z && st_z && s, "%s: cell outputs / state missing", fn);
    SC_REQUIRE(epi == FR_CELL_FUSED || K == N / ng, "%s: unfused cell needs K == D", fn);
  } else {
    SC_REQUIRE(epi == FR_PLAIN || st_out, "%s: statistics output missing", fn);
  }
  return 0;
}

static FrameGemmArgs frame_gemm_args(int epi, const float* x, int64_t ldx, int K, const float* ln_w,
                                     const float* ln_b, const void* st_in, int nst_in, float eps,
                                     const void* w, int64_t ldw, const float* bias, int B, int N,
                                     float* y, int64_t ldy, void* st_out, float* z, void* st_z,
                                     float* s, const float* mask) {
  const bool cell = epi >= FR_CELL_UNFUSED;
  const int ng = epi == FR_CELL_FUSED ? 5 : 4;
  FrameGemmArgs a;
  a.x = x; a.ldx = ldx; a.K = K; a.ln_w = ln_w; a.ln_b = ln_b; a.st_in = (const float4*)st_in;
  a.nst_in = nst_in; a.eps = eps; a.w = w; a.ldw = ldw; a.bias = bias; a.B = B; a.N = N;
  a.gstride = cell ? N / ng : 16;
  a.y = y; a.ldy = ldy; a.st_out = (float4*)st_out; a.z = z; a.st_z = (float4*)st_z; a.s = s;
  a.mask = mask;
  return a;
}

extern "C" int sc_lucy_frame_gemm(int epi, const float* x, int64_t ldx, int K, const float* ln_w,
                                  const float* ln_b, const void* st_in, int nst_in, float eps,
                                  const void* w, int w_dtype, int64_t ldw, const float* bias,
                                  int B, int N, float* y, int64_t ldy, void* st_out, float* z,
                                  void* st_z, float* s, const float* mask, void* stream) {
  clear_error();
  const int rc = frame_gemm_check("sc_lucy_frame_gemm", epi, w_dtype, x, ldx, K, ln_w, ln_b, st_in,
                                  nst_in, w, ldw, bias, B, N, y, st_out, z, st_z, s);
  if (rc || B == 0) return rc;
  const FrameGemmArgs a = frame_gemm_args(epi, x, ldx, K, ln_w, ln_b, st_in, nst_in, eps, w, ldw,
                                          bias, B, N, y, ldy, st_out, z, st_z, s, mask);
  const int ng = epi == FR_CELL_FUSED ? 5 : 4;
  hipStream_t st = (hipStream_t)stream;
  if (w_dtype == SC_BF16) {
    if (ln_w) dispatch_gemm<true, true>(epi, ng, a, st);
    else dispatch_gemm<true, false>(epi, ng, a, st);
  } else {
    if (ln_w) dispatch_gemm<false, true>(epi, ng, a, st);
    else dispatch_gemm<false, false>(epi, ng, a, st);
  }
  return launch_status("sc_lucy_frame_gemm");
}

extern "C" int sc_lucy_frame_gemm_multi(int epi, int w_dtype, float eps,
                                        const sc_frame_gemm_job* jobs, int njobs, void* stream) {
  clear_error();
  SC_REQUIRE(njobs >= 0 && njobs <= kMaxFrameJobs && (njobs == 0 || jobs),
             "sc_lucy_frame_gemm_multi: 0..%d jobs per call", kMaxFrameJobs);
  FrameGemmJobs fj{};
  int nj = 0, with_ln = -1;
  for (int i = 0; i < njobs; ++i) {
    const sc_frame_gemm_job& j = jobs[i];
    const int rc = frame_gemm_check("sc_lucy_frame_gemm_multi", epi, w_dtype, j.x, j.ldx, j.K,
                                    j.ln_w, j.ln_b, j.st_in, j.nst_in, j.w, j.ldw, j.bias, j.B,
                                    j.N, j.y, j.st_out, j.z, j.st_z, j.s);
    if (rc) return rc;
    if (j.B == 0) continue;
    SC_REQUIRE(with_ln < 0 || with_ln == (j.ln_w != nullptr),
               "sc_lucy_frame_gemm_multi: every job of a call with or every job without the "
               "LayerNorm prologue");
    with_ln = j.ln_w != nullptr;
    fj.j[nj++] = frame_gemm_args(epi, j.x, j.ldx, j.K, j.ln_w, j.ln_b, j.st_in, j.nst_in, eps,
                                 j.w, j.ldw, j.bias, j.B, j.N, j.y, j.ldy, j.st_out, j.z, j.st_z,
                                 j.s, j.mask);
  }
  if (nj == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (w_dtype == SC_BF16) {
    if (with_ln) dispatch_gemm_multi<true, true>(epi, fj, nj, st);
    else dispatch_gemm_multi<true, false>(epi, fj, nj, st);
  } else {
    if (with_ln) dispatch_gemm_multi<false, true>(epi, fj, nj, st);
    else dispatch_gemm_multi<false, false>(epi, fj, nj, st);
  }
  return launch_status("sc_lucy_frame_gemm_multi");
}

static int frame_cellb_check(const char* fn, const float* z, const void* st_z, int nst_z,
                             const float* hp, const void* st_h, int nst_h, const float* lnz_w,
                             const float* lnz_b, const float* lnh_w, const float* lnh_b, float* h,
                             float* out, int B, int D) {
  SC_REQUIRE(B >= 0 && D > 0, "%s: bad shape", fn);
  if (B == 0) return 0;
  SC_REQUIRE(z && hp && h && out, "%s: null pointer", fn);
  SC_REQUIRE((lnz_w == nullptr) == (lnz_b == nullptr) && (lnh_w == nullptr) == (lnh_b == nullptr) &&
                 (!lnz_w || (st_z && nst_z > 0)) && (!lnh_w || (st_h && nst_h > 0)),
             "%s: LayerNorm needs weight, bias and statistics", fn);
  return 0;
}

extern "C" int sc_lucy_frame_cellb(const float* z, const void* st_z, int nst_z, const float* hp,
                                   const void* st_h, int nst_h, const float* lnz_w,
                                   const float* lnz_b, const float* lnh_w, const float* lnh_b,
                                   float eps, float* h, float* out, int64_t ldo, const float* mask,
                                   int B, int D, void* stream) {
  clear_error();
  const int rc = frame_cellb_check("sc_lucy_frame_cellb", z, st_z, nst_z, hp, st_h, nst_h, lnz_w,
                                   lnz_b, lnh_w, lnh_b, h, out, B, D);
  if (rc || B == 0) return rc;
  FrameCellArgs a{z, (const float4*)st_z, nst_z, hp, (const float4*)st_h, nst_h, lnz_w, lnz_b,
                  lnh_w, lnh_b, eps, h, out, ldo, mask, B, D};
  hipLaunchKernelGGL(lucy_frame_cellb, dim3(B), dim3(256), 0, (hipStream_t)stream, a);
  return launch_status("sc_lucy_frame_cellb");
}

extern "C" int sc_lucy_frame_cellb_multi(float eps, const sc_frame_cell_job* jobs, int njobs,
                                         void* stream) {
  clear_error();
  SC_REQUIRE(njobs >= 0 && njobs <= kMaxFrameJobs && (njobs == 0 || jobs),
             "sc_lucy_frame_cellb_multi: 0..%d jobs per call", kMaxFrameJobs);
  FrameCellJobs fj{};
  int nj = 0, gx = 1;
  for (int i = 0; i < njobs; ++i) {
    const sc_frame_cell_job& j = jobs[i];
    const int rc = frame_cellb_check("sc_lucy_frame_cellb_multi", j.z, j.st_z, j.nst_z, j.hp,
                                     j.st_h, j.nst_h, j.lnz_w, j.lnz_b, j.lnh_w, j.lnh_b, j.h,
                                     j.out, j.B, j.D);
    if (rc) return rc;
    if (j.B == 0) continue;
    fj.j[nj++] = FrameCellArgs{j.z, (const float4*)j.st_z, j.nst_z, j.hp, (const float4*)j.st_h,
                               j.nst_h, j.lnz_w, j.lnz_b, j.lnh_w, j.lnh_b, eps, j.h, j.out,
                               j.ldo, j.mask, j.B, j.D};
    gx = std::max(gx, j.B);
  }
  if (nj == 0) return 0;
  hipLaunchKernelGGL(lucy_frame_cellb_multi, dim3(gx, nj), dim3(256), 0, (hipStream_t)stream, fj);
  return launch_status("sc_lucy_frame_cellb_multi");
}
