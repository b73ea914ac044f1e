// Zero-copy PCIe probe: how fast can a kernel read (and write) pinned host memory, by access
// shape, against the copy engines (hipMemcpyAsync H2D / D2H) on the same buffers?
// The client-side update (flearn_amd/strategy/_update.py, zero_copy) reads w_local / w_glob
// straight from pinned staging; this says whether its ~44 GB/s is the link or the kernel.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/probe_zc.cpp -o tools/probe_zc
//   tools/probe_zc [MiB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// each thread reads U consecutive 16-B quads per step (U*16 B contiguous per lane), grid-stride
template <int U>
__global__ __launch_bounds__(256) void zc_read(const f4* __restrict__ src, int64_t nq, float* sink) {
  f4 acc = {0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t q = ((int64_t)blockIdx.x * 256 + threadIdx.x) * U; q < nq; q += stride) {
    f4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = q + u < nq ? __builtin_nontemporal_load(src + q + u) : f4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc += x[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[threadIdx.x] = acc.x;
}

// wave-contiguous form: lane l of a wave reads quad (base + u*64 + l): each load instruction
// covers 1 KiB contiguous per wave, U of them in flight
template <int U>
__global__ __launch_bounds__(256) void zc_read_wave(const f4* __restrict__ src, int64_t nq, float* sink) {
  f4 acc = {0, 0, 0, 0};
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t per_wave = 64 * U;
  const int64_t stride = (int64_t)gridDim.x * 4 * per_wave;
  for (int64_t b = ((int64_t)blockIdx.x * 4 + wv) * per_wave; b < nq; b += stride) {
    f4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = b + u * 64 + lane;
      x[u] = q < nq ? __builtin_nontemporal_load(src + q) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += x[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[threadIdx.x] = acc.x;
}

__global__ __launch_bounds__(256) void zc_write_wave(f4* __restrict__ dst, int64_t nq) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += stride)
    __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, (float)q}, dst + q);
}

// the client update's shape: per 4 elements, a f32 quad of w_local and two quads of f64 w_glob in,
// two quads of f64 out (12 B in, 8 B out per element), grid-stride
__global__ __launch_bounds__(256) void zc_update_shape(const f4* __restrict__ a, const f4* __restrict__ b,
                                                       f4* __restrict__ c, int64_t nquads) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nquads; q += stride) {
    f4 x = __builtin_nontemporal_load(a + q);
    f4 y0 = __builtin_nontemporal_load(b + 2 * q), y1 = __builtin_nontemporal_load(b + 2 * q + 1);
    __builtin_nontemporal_store(y0 + x.x, c + 2 * q);
    __builtin_nontemporal_store(y1 + x.y, c + 2 * q + 1);
  }
}

static double time_ms(hipStream_t s, int reps, const std::function<void()>& fn) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  fn();
  CK(hipStreamSynchronize(s));
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, s));
    fn();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 256;
  const size_t bytes = mib << 20;
  const int64_t nq = bytes / 16;
  void *h, *h2, *d;
  float* sink;
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&h2, bytes, hipHostMallocDefault));
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 4096));
  memset(h, 1, bytes);
  memset(h2, 1, bytes);
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int reps = 7;
  auto gbs = [&](double ms, size_t b) { return b / ms / 1e6; };
  printf("{\"mib\": %zu, \"results\": [\n", mib);
  double ms = time_ms(s, reps, [&] { CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s)); });
  printf("  {\"what\": \"dma h2d\", \"ms\": %.3f, \"gbs\": %.1f},\n", ms, gbs(ms, bytes));
  ms = time_ms(s, reps, [&] { CK(hipMemcpyAsync(h2, d, bytes, hipMemcpyDeviceToHost, s)); });
  printf("  {\"what\": \"dma d2h\", \"ms\": %.3f, \"gbs\": %.1f},\n", ms, gbs(ms, bytes));
  ms = time_ms(s, reps, [&] {
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(h2, (char*)d, bytes, hipMemcpyDeviceToHost, s2));
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, s2));
    CK(hipStreamWaitEvent(s, e, 0));
    CK(hipEventDestroy(e));
  });
  printf("  {\"what\": \"dma h2d + d2h concurrent\", \"ms\": %.3f, \"gbs_each\": %.1f},\n", ms, gbs(ms, bytes));
  const f4* src = (const f4*)h;
  for (int grid : {256, 512, 1024, 2048, 4096}) {
#define RUN(K, U, NAME)                                                                                      \
  ms = time_ms(s, reps, [&] { hipLaunchKernelGGL((K<U>), dim3(grid), dim3(256), 0, s, src, nq, sink); }); \
  printf("  {\"what\": \"%s U%d grid %d\", \"ms\": %.3f, \"gbs\": %.1f},\n", NAME, U, grid, ms, gbs(ms, bytes));
    RUN(zc_read, 1, "lane-contig read")
    RUN(zc_read, 4, "lane-contig read")
    RUN(zc_read_wave, 1, "wave-contig read")
    RUN(zc_read_wave, 4, "wave-contig read")
    RUN(zc_read_wave, 8, "wave-contig read")
#undef RUN
    ms = time_ms(s, reps, [&] { hipLaunchKernelGGL(zc_write_wave, dim3(grid), dim3(256), 0, s, (f4*)h2, nq); });
    printf("  {\"what\": \"write grid %d\", \"ms\": %.3f, \"gbs\": %.1f},\n", grid, ms, gbs(ms, bytes));
  }
  // the update's shape: read the host buffer while writing the other (full duplex?)
  ms = time_ms(s, reps, [&] {
    hipLaunchKernelGGL((zc_read_wave<4>), dim3(1024), dim3(256), 0, s, src, nq, sink);
    hipLaunchKernelGGL(zc_write_wave, dim3(1024), dim3(256), 0, s2, (f4*)h2, nq);
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, s2));
    CK(hipStreamWaitEvent(s, e, 0));
    CK(hipEventDestroy(e));
  });
  printf("  {\"what\": \"zc read + zc write concurrent\", \"ms\": %.3f, \"gbs_each\": %.1f},\n", ms, gbs(ms, bytes));
  ms = time_ms(s, reps, [&] {
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(zc_write_wave, dim3(512), dim3(256), 0, s2, (f4*)h2, nq);
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, s2));
    CK(hipStreamWaitEvent(s, e, 0));
    CK(hipEventDestroy(e));
  });
  printf("  {\"what\": \"dma h2d + zc write concurrent\", \"ms\": %.3f, \"gbs_each\": %.1f},\n", ms, gbs(ms, bytes));
  {  // update-shaped: local bytes/5 f32, glob and out 2 bytes/5 each (in 3/5, out 2/5 of 'bytes')
    const int64_t nqa = bytes / 5 / 16 / 4 * 4;
    for (int grid : {256, 512, 1024, 2048, 0}) {
      const int g = grid ? grid : (int)((nqa + 255) / 256);
      ms = time_ms(s, reps, [&] {
        hipLaunchKernelGGL(zc_update_shape, dim3(g), dim3(256), 0, s, (const f4*)h, (const f4*)h + nqa, (f4*)h2, nqa);
      });
      const double in = nqa * 48.0, out = nqa * 32.0;
      printf("  {\"what\": \"update-shaped grid %d\", \"ms\": %.3f, \"in_gbs\": %.1f, \"out_gbs\": %.1f, \"total_gbs\": %.1f}%s\n", g, ms,
             in / ms / 1e6, out / ms / 1e6, (in + out) / ms / 1e6, grid ? "," : "");
    }
  }
  printf("]}\n");
  CK(hipDeviceSynchronize());
  return 0;
}
