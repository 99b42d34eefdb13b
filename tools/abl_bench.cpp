// Times sc_lucy_scan_fwd / sc_lucy_scan_bwd from several builds of the library (ablation
// variants, tools/abl_bench.sh) in one process with rotating inputs (C2 shape, bf16,
// step-blocked gates).  usage: abl_bench lib1.so [lib2.so ...]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int B = 32, T = 1500, D = 512, NROT = 4;
typedef int (*fwd_t)(const void*, int, const float*, const float*, const float*, void*, float*, int,
                     int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, float*, void*);
typedef int (*bwd_t)(const void*, int, const float*, const float*, const void*, const float*, void*,
                     float*, float*, float*, int, int, int, int64_t, int64_t, int64_t, int64_t,
                     int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, void*);

template <typename F>
double time_it(F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 8; ++i) f(i);
  std::vector<double> r;
  for (int q = 0; q < 5; ++q) {
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) f(i);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    r.push_back(ms * 1e3 / 20);
  }
  std::sort(r.begin(), r.end());
  return r[0];
}

int main(int argc, char** argv) {
  const size_t ng = (size_t)B * T * 7 * D, nd = (size_t)B * T * D;
  std::vector<uint16_t> h(ng);
  void *g[NROT], *dout, *dg, *out;
  float *st, *sout, *ck[NROT], *dh, *ds, *db, *bias;
  for (int r = 0; r < NROT; ++r) {
    for (size_t i = 0; i < ng; ++i) h[i] = 0x3e00 + (uint16_t)(((i + 7 * r) * 2654435761u) >> 22) % 0x200;
    (void)hipMalloc(&g[r], ng * 2);
    (void)hipMemcpy(g[r], h.data(), ng * 2, hipMemcpyHostToDevice);
    (void)hipMalloc(&ck[r], (size_t)B * 24 * 2 * D * 4);
  }
  (void)hipMalloc(&dout, nd * 2);
  (void)hipMemcpy(dout, h.data(), nd * 2, hipMemcpyHostToDevice);
  (void)hipMalloc(&dg, ng * 2);
  (void)hipMalloc(&out, nd * 2);
  (void)hipMalloc(&st, B * D * 4);
  (void)hipMemset(st, 0, B * D * 4);
  (void)hipMalloc(&sout, B * D * 4);
  (void)hipMalloc(&dh, B * D * 4);
  (void)hipMalloc(&ds, B * D * 4);
  (void)hipMalloc(&db, B * 7 * D * 4);
  (void)hipMalloc(&bias, 7 * D * 4);
  (void)hipMemset(bias, 0, 7 * D * 4);
  const int64_t gbt = (int64_t)T * 7 * D, gtd = 7 * D, gcd = 64, gcb = 448;
  for (int a = 1; a < argc; ++a) {
    void* lib = dlopen(argv[a], RTLD_NOW | RTLD_LOCAL);
    if (!lib) { printf("%s: %s\n", argv[a], dlerror()); continue; }
    auto fwd = (fwd_t)dlsym(lib, "sc_lucy_scan_fwd");
    auto bwd = (bwd_t)dlsym(lib, "sc_lucy_scan_bwd");
    for (int r = 0; r < NROT; ++r)
      fwd(g[r], 1, bias, st, st, out, sout, B, T, D, gbt, gtd, gcd, gcb, (int64_t)T * D, D, ck[r], nullptr);
    const double tf = time_it([&](int i) {
      fwd(g[i % NROT], 1, bias, st, st, out, sout, B, T, D, gbt, gtd, gcd, gcb, (int64_t)T * D, D,
          ck[i % NROT], nullptr);
    });
    const double tb = time_it([&](int i) {
      bwd(g[i % NROT], 1, bias, ck[i % NROT], dout, nullptr, dg, dh, ds, db, B, T, D, gbt, gtd, gcd,
          gcb, (int64_t)T * D, D, gbt, gtd, gcd, gcb, nullptr);
    });
    const double bf = (double)nd * 16 + B * 24 * 2 * D * 4, bb = (double)nd * 30 + B * 24 * 2 * D * 4;
    printf("%-40s fwd %7.1f us %5.1f%%   bwd %7.1f us %5.1f%%  (%s)\n", argv[a], tf,
           bf / tf * 1e-6 / 8e3 * 100, tb, bb / tb * 1e-6 / 8e3 * 100,
           hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
