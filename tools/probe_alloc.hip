// probe_alloc.hip — does where a client stack lives in HBM change the reduce's rate?  The same
// product kernel (reduce_kernel_rowmajor, NS geometry) over K separately allocated stacks of one
// shape, some from hipMalloc, some from hipExtMallocWithFlags(hipDeviceMallocContiguous), timed in
// interleaved rounds in one process.  Bench lines of one config differ by ~2% between processes
// on one box (DESIGN.md §4 finding 20); if the stacks of one process differ alike, placement is
// the cause.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iflearn_amd/csrc \
//         tools/probe_alloc.hip -o tools/probe_alloc
//   tools/probe_alloc [n=100] [ncols=25610176] [stacks=6] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fa_device.hpp"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

using namespace fa;

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int n = argc > 1 ? atoi(argv[1]) : 100;
  const int64_t ncols = argc > 2 ? atoll(argv[2]) : 25610176;
  const int k = argc > 3 ? atoi(argv[3]) : 6;
  const int rounds = argc > 4 ? atoi(argv[4]) : 5;
  const int64_t stride = (ncols + 63) / 64 * 64;
  const size_t bytes = (size_t)n * stride * 4;
  std::vector<float*> stacks;
  std::vector<int> contiguous;
  for (int i = 0; i < k; ++i) {
    float* p = nullptr;
    const bool want_c = i % 2 == 1;
    if (want_c) {
      const hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&p), bytes, hipDeviceMallocContiguous);
      if (e != hipSuccess) {
        fprintf(stderr, "contiguous alloc %d failed: %s; using hipMalloc\n", i, hipGetErrorString(e));
        (void)hipGetLastError();
        p = nullptr;
      }
    }
    if (!p) CK(hipMalloc(&p, bytes));
    stacks.push_back(p);
    contiguous.push_back(want_c && p);
    hipLaunchKernelGGL(fill_uniform_kernel, dim3(4096, n), dim3(256), 0, 0, p, stride, stride, 2024ull, (int64_t)0,
                       (int64_t)0);
  }
  float *w, *out;
  CK(hipMalloc(&w, n * 4));
  CK(hipMalloc(&out, stride * 4));
  std::vector<float> ones(n, 1.0f);
  CK(hipMemcpy(w, ones.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  Epi<double> e{};
  e.denom = (double)n;
  e.out32 = out;
  const double algo = (double)n * ncols * 4 + ncols * 4;
  printf("# n=%d ncols=%lld stacks=%d (odd: hipDeviceMallocContiguous) bytes/launch=%.0f\n", n, (long long)ncols, k,
         algo);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<std::vector<float>> t(k);
  for (int r = 0; r < rounds; ++r) {
    for (int i = 0; i < k; ++i) {
      auto launch = [&] {
        hipLaunchKernelGGL((reduce_kernel_rowmajor<AccF32, double, FA_OP_MEAN, 16, 1, 4, 3, true, 2>), dim3(192),
                           dim3(256), 0, 0, stacks[i], stride, n, w, (int64_t)0, ncols, e);
      };
      launch();
      CK(hipEventRecord(a, 0));
      for (int j = 0; j < 10; ++j) launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      t[i].push_back(ms / 10);
    }
  }
  for (int i = 0; i < k; ++i) {
    std::sort(t[i].begin(), t[i].end());
    const double med = t[i][t[i].size() / 2] * 1e3;
    printf("stack %d %-11s addr %p  med %.1f us  min %.1f us  %.2f%% of 8 TB/s\n", i,
           contiguous[i] ? "contiguous" : "hipMalloc", (void*)stacks[i], med, t[i][0] * 1e3,
           algo / (med * 1e-6) / 8e12 * 100);
  }
  return 0;
}
