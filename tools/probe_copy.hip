// probe_copy.hip — stand-in for RCCL's all-gather traffic on ONE GPU (tools/overlap_probe.py):
// a grid-stride 16-B copy on a chosen number of blocks, launched on its own stream beside the
// aggregation reduce, so the reduce's slowdown from sharing CUs and HBM with a concurrent
// collective can be measured without a second GPU.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/probe_copy.hip -o tools/libprobe_copy.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void probe_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                    int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

extern "C" int probe_copy(void* dst, const void* src, int64_t n16, int32_t blocks, void* stream) {
  if (!dst || !src || n16 <= 0 || blocks <= 0) return -1;
  hipLaunchKernelGGL(probe_copy16, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint4*>(dst), static_cast<const uint4*>(src), n16);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// the same copy over one small buffer `reps` times (L2-resident: CU and cache traffic, no HBM)
__global__ __launch_bounds__(256) void probe_copy16_rep(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                        int64_t n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
      uint4 v = src[i];
      v.x += (unsigned)r;
      dst[i] = v;
    }
}

// ALU only: a dependent FMA chain per lane, one store per lane at the end (no memory traffic)
__global__ __launch_bounds__(256) void probe_spin_k(float* __restrict__ out, int iters) {
  float a = (float)threadIdx.x * 1e-3f, b = 1.0000001f, c = 1e-7f;
  for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, b, c);
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = a;
}

extern "C" int probe_copy_rep(void* dst, const void* src, int64_t n16, int32_t blocks, int32_t reps, void* stream) {
  if (!dst || !src || n16 <= 0 || blocks <= 0 || reps <= 0) return -1;
  hipLaunchKernelGGL(probe_copy16_rep, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint4*>(dst), static_cast<const uint4*>(src), n16, reps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int probe_spin(float* out, int32_t blocks, int32_t iters, void* stream) {
  if (!out || blocks <= 0 || iters <= 0) return -1;
  hipLaunchKernelGGL(probe_spin_k, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), out, iters);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// read-only stream (no stores but one per block): does the reduce suffer from foreign READS as
// much as from a copy's read + write mix (HBM bus turnaround)?
__global__ __launch_bounds__(256) void probe_read16(const uint4* __restrict__ src, int64_t n, uint4* __restrict__ sink) {
  uint4 acc = {0u, 0u, 0u, 0u};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 v = src[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x & 0x7fffffffu) == 0x12345678u) sink[blockIdx.x * 256 + threadIdx.x] = acc;  // keeps the loads
}

// write-only stream
__global__ __launch_bounds__(256) void probe_write16(uint4* __restrict__ dst, int64_t n) {
  const uint4 v = {1u, 2u, 3u, 4u};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = v;
}

extern "C" int probe_read(const void* src, int64_t n16, int32_t blocks, void* sink, void* stream) {
  if (!src || !sink || n16 <= 0 || blocks <= 0 || blocks > 4096) return -1;
  hipLaunchKernelGGL(probe_read16, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(src), n16, static_cast<uint4*>(sink));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int probe_write(void* dst, int64_t n16, int32_t blocks, void* stream) {
  if (!dst || n16 <= 0 || blocks <= 0) return -1;
  hipLaunchKernelGGL(probe_write16, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint4*>(dst), n16);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// the runtime's own copy of a device buffer to another address (hipMemcpyDeviceToDevice): for a
// pinned-host destination ROCclr runs its blit kernel (__amd_rocclr_copyBuffer) on the stream's
// queue; the fa_push contention probe compares it with fa_push into the same memory
extern "C" int probe_blit(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (!dst || !src || nbytes <= 0) return -1;
  return hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)) ==
                 hipSuccess ? 0 : -2;
}

// a stream whose kernels may run only on the CUs set in `mask` (words x 32 bits, CU i = bit i):
// does fencing a link-bound push onto a few CUs, and the reduce onto the others, remove the
// push's cost to the reduce?  (tools/overlap_probe.py --push-cus)
extern "C" int probe_stream_cumask(const uint32_t* mask, int32_t words, void** out) {
  if (!mask || words <= 0 || !out) return -1;
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask) != hipSuccess) return -2;
  *out = s;
  return 0;
}

extern "C" int probe_stream_cumask_get(void* stream, int32_t words, uint32_t* mask) {
  return hipExtStreamGetCUMask(static_cast<hipStream_t>(stream), (uint32_t)words, mask) == hipSuccess ? 0 : -2;
}

extern "C" int probe_stream_destroy(void* stream) {
  return hipStreamDestroy(static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -2;
}

// a paced push stand-in: like fa_push's kernel into ONE destination (U quads per lane per round),
// but every wave waits for its stores before its next loads (s_waitcnt vmcnt(0): on gfx9 the
// counter covers stores too), so at most U x 1 KiB per wave is in flight — about the link's
// bandwidth-delay product on few blocks instead of queues of stores backed up behind it.
typedef uint32_t pu4 __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void probe_push_paced_k(const pu4* __restrict__ s, int64_t quads,
                                                          pu4* __restrict__ d) {
  const int64_t G = (int64_t)gridDim.x * 256;
  for (int64_t q0 = (int64_t)blockIdx.x * 256 + threadIdx.x; q0 < quads; q0 += U * G) {
    pu4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = q0 + u * G;
      v[u] = q < quads ? __builtin_nontemporal_load(s + q) : pu4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = q0 + u * G;
      if (q < quads) d[q] = v[u];
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __threadfence_system();
}

extern "C" int probe_push_paced(void* dst, const void* src, int64_t n16, int32_t blocks, int32_t u, void* stream) {
  if (!dst || !src || n16 <= 0 || blocks <= 0) return -1;
  auto s = static_cast<hipStream_t>(stream);
  const pu4* a = static_cast<const pu4*>(src);
  pu4* b = static_cast<pu4*>(dst);
  if (u == 1) hipLaunchKernelGGL(probe_push_paced_k<1>, dim3((unsigned)blocks), dim3(256), 0, s, a, n16, b);
  else if (u == 2) hipLaunchKernelGGL(probe_push_paced_k<2>, dim3((unsigned)blocks), dim3(256), 0, s, a, n16, b);
  else if (u == 4) hipLaunchKernelGGL(probe_push_paced_k<4>, dim3((unsigned)blocks), dim3(256), 0, s, a, n16, b);
  else if (u == 8) hipLaunchKernelGGL(probe_push_paced_k<8>, dim3((unsigned)blocks), dim3(256), 0, s, a, n16, b);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
