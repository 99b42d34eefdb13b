// Feature frontend on the GPU: the reference's make_frontend (model.py:250-279), applied under
// no_grad at train.py:473-475 — torchaudio MFCC(n_mfcc=80, dct ortho, log_mels) or
// MelSpectrogram + AmplitudeToDB(top_db=80), with n_fft = win = 400, hop = 160, 80 HTK mel
// bands, center=False, power 2.
//
// fbank_kernel: one wave per frame (a workgroup's 4 waves take 4 frames at a time, grid-stride
// over all B x frames).  Per frame, all in LDS / registers, fp32:
//   window      x[n] = audio[f*160 + n] * hann_periodic[n]
//   DFT-400     as 20 x 20 (Cooley-Tukey, n = 20 n1 + n2, k = k1 + 20 k2):
//                 Y[n2][k1]  = sum_n1 x[20 n1 + n2] W^(20 n1 k1),  times the twiddle W^(n2 k1)
//                 X[k1+20k2] = sum_n2 Y[n2][k1] W^(20 n2 k2)        (W = e^{-2 pi i / 400})
//               only the 201 one-sided bins of the second stage are formed; power = |X|^2
//   mel         80 triangular HTK bands, weights evaluated from the 82 band edges (no table)
//   MFCC        log(mel + 1e-6), orthonormal DCT-II (matrix in LDS)    | mel: 10 log10(max(mel,
//                                                                      | 1e-10)), the batch max
//                                                                      | by an ordered atomicMax
// fbank_topdb_kernel (mel only): x = max(x, batch max - 80).
// Tables (twiddles, window, band edges, DCT) are built once per workgroup in LDS.
#include <algorithm>

#include "sc_common.h"

namespace sc {

constexpr int kNfft = 400, kHop = 160, kBins = 201, kMels = 80;

struct FbankArgs {
  const float* audio;
  int B;
  int64_t N, sa;     // samples per row, row stride
  int64_t F;         // frames per row
  int kind;          // 0 MFCC, 1 log-mel dB
  float sr;
  float* out;        // [B][F][80]
  unsigned* dbmax;   // ordered-int running max (kind 1)
};

__device__ __forceinline__ unsigned order_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float order_val(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float hz_to_mel(float f) { return 2595.0f * log10f(1.0f + f / 700.0f); }
__device__ __forceinline__ float mel_to_hz(float m) { return 700.0f * (exp10f(m / 2595.0f) - 1.0f); }

__global__ void __launch_bounds__(256) fbank_kernel(FbankArgs a) {
  __shared__ float cosT[kNfft], sinT[kNfft], win[kNfft];
  __shared__ float fpts[kMels + 2];
  __shared__ float dct[kMels * kMels];            // [m][c]
  __shared__ float xs[4][kNfft];
  __shared__ float2 ys[4][kNfft];
  __shared__ float pw[4][kBins + 3];
  __shared__ float lm[4][kMels];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kNfft; i += 256) {
    float s, c;
    sincospif((float)i / (kNfft / 2), &s, &c);   // angle 2 pi i / 400
    cosT[i] = c;
    sinT[i] = s;
    win[i] = 0.5f - 0.5f * c;                    // torch.hann_window(400), periodic
  }
  if (tid < kMels + 2) {
    const float mmax = hz_to_mel(0.5f * a.sr);
    fpts[tid] = mel_to_hz(mmax * (float)tid / (float)(kMels + 1));
  }
  if (a.kind == 0) {
    const float s0 = sqrtf(1.0f / kMels), s1 = sqrtf(2.0f / kMels);
    for (int i = tid; i < kMels * kMels; i += 256) {
      const int m = i / kMels, c = i % kMels;
      dct[i] = cospif((m + 0.5f) * c / kMels) * (c == 0 ? s0 : s1);
    }
  }
  __syncthreads();
  const float df = 0.5f * a.sr / (kBins - 1);      // bin spacing of linspace(0, sr/2, 201)
  const int64_t total = (int64_t)a.B * a.F;
  float* x = xs[w];
  float2* y = ys[w];
  float* p = pw[w];
  float* l = lm[w];
  float runmax = -__builtin_huge_valf();
  for (int64_t fr = (int64_t)blockIdx.x * 4 + w; fr < total; fr += (int64_t)gridDim.x * 4) {
    const int b = (int)(fr / a.F);
    const int64_t f = fr % a.F;
    const float* src = a.audio + (int64_t)b * a.sa + f * kHop;
    for (int n = lane; n < kNfft; n += 64) x[n] = src[n] * win[n];
    wave_lds_sync();
    // stage 1: o = n2 * 20 + k1
    for (int o = lane; o < kNfft; o += 64) {
      const int n2 = o / 20, k1 = o - 20 * (o / 20);
      float re = 0.0f, im = 0.0f;
      int idx = 0;                                  // 20 n1 k1 mod 400
#pragma unroll 4
      for (int n1 = 0; n1 < 20; ++n1) {
        const float v = x[20 * n1 + n2];
        re = fmaf(v, cosT[idx], re);
        im = fmaf(-v, sinT[idx], im);
        idx += 20 * k1;
        idx -= idx >= kNfft ? kNfft : 0;
      }
      const int tw = (n2 * k1) % kNfft;             // twiddle W^(n2 k1)
      const float c = cosT[tw], s = sinT[tw];
      y[o] = make_float2(re * c + im * s, im * c - re * s);
    }
    wave_lds_sync();
    // stage 2: one-sided bins k = k1 + 20 k2 < 201
    for (int k = lane; k < kBins; k += 64) {
      const int k1 = k - 20 * (k / 20), k2 = k / 20;
      float re = 0.0f, im = 0.0f;
      int idx = 0;                                  // 20 n2 k2 mod 400
#pragma unroll 4
      for (int n2 = 0; n2 < 20; ++n2) {
        const float2 v = y[n2 * 20 + k1];
        const float c = cosT[idx], s = sinT[idx];
        re += v.x * c + v.y * s;
        im += v.y * c - v.x * s;
        idx += 20 * k2;
        idx -= idx >= kNfft ? kNfft : 0;
      }
      p[k] = re * re + im * im;
    }
    wave_lds_sync();
    // mel bands
    float* orow = a.out + fr * kMels;
    for (int m = lane; m < kMels; m += 64) {
      const float f0 = fpts[m], f1 = fpts[m + 1], f2 = fpts[m + 2];
      const float i01 = 1.0f / (f1 - f0), i12 = 1.0f / (f2 - f1);
      const int k0 = max(0, (int)floorf(f0 / df)), k2 = min(kBins - 1, (int)ceilf(f2 / df));
      float acc = 0.0f;
      for (int k = k0; k <= k2; ++k) {
        const float fk = df * (float)k;
        const float wk = fmaxf(0.0f, fminf((fk - f0) * i01, (f2 - fk) * i12));
        acc = fmaf(wk, p[k], acc);
      }
      if (a.kind == 0) {
        l[m] = logf(acc + 1e-6f);
      } else {
        const float db = 10.0f * log10f(fmaxf(acc, 1e-10f));
        orow[m] = db;
        runmax = fmaxf(runmax, db);
      }
    }
    if (a.kind == 0) {
      wave_lds_sync();
      for (int c = lane; c < kMels; c += 64) {
        float acc = 0.0f;
#pragma unroll 8
        for (int m = 0; m < kMels; ++m) acc = fmaf(l[m], dct[m * kMels + c], acc);
        orow[c] = acc;
      }
    }
    wave_lds_sync();   // the wave's scratch is reused by its next frame
  }
  if (a.kind == 1) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) runmax = fmaxf(runmax, __shfl_xor(runmax, o));
    if (lane == 0 && runmax > -__builtin_huge_valf()) atomicMax(a.dbmax, order_key(runmax));
  }
}

__global__ void __launch_bounds__(256) fbank_topdb_kernel(float* out, int64_t n,
                                                          const unsigned* dbmax) {
  const float lo = order_val(*dbmax) - 80.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = fmaxf(out[i], lo);
}

}  // namespace sc

using namespace sc;

extern "C" int64_t sc_fbank_frames(int64_t n_samples) {
  return n_samples < kNfft ? 0 : 1 + (n_samples - kNfft) / kHop;
}

extern "C" size_t sc_fbank_workspace_bytes(void) { return 256; }

extern "C" int sc_fbank(const float* audio, int B, int64_t n_samples, int64_t audio_stride,
                        int kind, float sample_rate, float* out, void* workspace,
                        size_t workspace_bytes, void* stream) {
  clear_error();
  SC_REQUIRE(kind == 0 || kind == 1, "sc_fbank: kind must be 0 (mfcc) or 1 (mel), got %d", kind);
  SC_REQUIRE(B >= 0 && n_samples >= 0 && sample_rate > 0.0f, "sc_fbank: bad shape / rate");
  const int64_t F = sc_fbank_frames(n_samples);
  if (B == 0 || F == 0) return 0;
  SC_REQUIRE(audio && out, "sc_fbank: null pointer");
  SC_REQUIRE(audio_stride >= n_samples, "sc_fbank: row stride %lld < samples %lld",
             (long long)audio_stride, (long long)n_samples);
  SC_REQUIRE(kind == 0 || (workspace && workspace_bytes >= 4), "sc_fbank: mel needs the workspace");
  hipStream_t st = (hipStream_t)stream;
  FbankArgs a{audio, B, n_samples, audio_stride, F, kind, sample_rate, out, (unsigned*)workspace};
  if (kind == 1) zero_async(workspace, 4, st);
  const int64_t frames = (int64_t)B * F;
  const unsigned grid = (unsigned)std::min<int64_t>((frames + 3) / 4, 2048);
  hipLaunchKernelGGL(fbank_kernel, dim3(grid), dim3(256), 0, st, a);
  if (kind == 1) {
    const int64_t n = frames * kMels;
    hipLaunchKernelGGL(fbank_topdb_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)),
                       dim3(256), 0, st, out, n, (const unsigned*)workspace);
  }
  return launch_status("sc_fbank");
}
