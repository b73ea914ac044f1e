// probe_event_chain.hip — which cross-stream orderings does the HIP runtime keep?  (round 6)
//
// Round 5's copy-engine push gave wrong buckets when its pusher stream had high priority
// (profiles/r05/pipeline_queues/push_order_normal_vs_high_w8.json).  Its ordering was a CHAIN:
//   compute stream A: reduce kernel writes X
//   pusher stream B:  waits on an event recorded on A (torch's wait_stream), then — with nothing
//                     else queued on B — fa_push_dma records a fresh event E on B (destroyed at once)
//   peer stream C:    waits on E, then a copy-engine (NoCU) copy X -> Y
// This probe replays that chain in one process on one GPU, against variants that each change one
// thing, and counts copies that read X before the producer finished (Y != the value just written):
//   chain_destroy  the round-5 chain (E destroyed right after the wait)
//   chain_keep     E kept alive until the iteration ends            (cause candidate a)
//   direct         C waits on the event recorded on A itself         (cause candidate b)
//   chain_work     B runs a tiny kernel between its wait and recording E
//   chain_kernel   the chain, C runs a copy KERNEL instead of NoCU
//   chain_d2d      the chain, C uses plain hipMemcpyDeviceToDevice
// each with B at normal or high priority, and A = the null stream or a created stream.
// Join side: C's NoCU copy, an event recorded on C (destroyed or kept), B waits and runs a kernel
// that compares Y with X — counts consumers that ran before the copy had landed.
// Not product code; prints one JSON object.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_event_chain.hip -o tools/probe_event_chain
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

// every thread spins for `ticks` of the 100 MHz wall clock (bounded), then writes v over its part
__global__ __launch_bounds__(256) void slow_fill(float* __restrict__ x, int64_t n, float v, long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] = v;
}

__global__ __launch_bounds__(256) void copy_k(float* __restrict__ y, const float* __restrict__ x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = x[i];
}

// counts elements of y that differ from v (one vector atomic per block)
__global__ __launch_bounds__(256) void count_ne(const float* __restrict__ y, int64_t n, float v,
                                                unsigned long long* __restrict__ bad) {
  __shared__ unsigned s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  unsigned c = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) c += y[i] != v;
  atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0 && s) atomicAdd(bad, (unsigned long long)s);
}

// y vs x elementwise (the join consumer)
__global__ __launch_bounds__(256) void count_diff(const float* __restrict__ y, const float* __restrict__ x, int64_t n,
                                                  unsigned long long* __restrict__ bad) {
  __shared__ unsigned s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  unsigned c = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) c += y[i] != x[i];
  atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0 && s) atomicAdd(bad, (unsigned long long)s);
}

__global__ void tiny(float* p) {
  if (threadIdx.x == 0) p[0] += 1.0f;
}

enum Variant { CHAIN_DESTROY, CHAIN_KEEP, DIRECT, CHAIN_WORK, CHAIN_KERNEL, CHAIN_D2D, N_VARIANTS };
static const char* kNames[] = {"chain_destroy", "chain_keep", "direct", "chain_work", "chain_kernel", "chain_d2d"};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  const int64_t n = (int64_t)16 << 20;  // 64 MiB of fp32
  const long long spin = 200000;        // 2 ms at 100 MHz
  float *x, *y, *scratch;
  unsigned long long* bad;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&scratch, 256));
  CK(hipMalloc(&bad, 8));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  printf("{\"priority_range\": [%d, %d], \"iters\": %d, \"bytes\": %lld, \"results\": [\n", lo, hi, iters,
         (long long)(n * 4));
  bool first = true;
  float val = 1.0f;
  for (int a_null = 1; a_null >= 0; --a_null)
    for (int b_high = 0; b_high <= 1; ++b_high)
      for (int c_high = 0; c_high <= 1; ++c_high)
      for (int v = 0; v < N_VARIANTS; ++v) {
        hipStream_t A = nullptr, B, C;
        if (!a_null) CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
        CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, b_high ? hi : lo));
        CK(hipStreamCreateWithPriority(&C, hipStreamNonBlocking, c_high ? hi : lo));
        unsigned long long total_bad = 0;
        int bad_iters = 0;
        for (int it = 0; it < iters; ++it) {
          val += 1.0f;
          CK(hipMemsetAsync(bad, 0, 8, A));
          CK(hipMemsetAsync(y, 0, n * 4, A));
          CK(hipStreamSynchronize(A));
          hipLaunchKernelGGL(slow_fill, dim3(1024), dim3(256), 0, A, x, n, val, spin);
          hipEvent_t evA, E = nullptr;
          CK(hipEventCreateWithFlags(&evA, hipEventDisableTiming));
          CK(hipEventRecord(evA, A));
          if (v == DIRECT) {
            CK(hipStreamWaitEvent(C, evA, 0));
          } else {
            CK(hipStreamWaitEvent(B, evA, 0));  // torch's wait_stream
            if (v == CHAIN_WORK) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, B, scratch);
            CK(hipEventCreateWithFlags(&E, hipEventDisableTiming));
            CK(hipEventRecord(E, B));
            CK(hipStreamWaitEvent(C, E, 0));
            if (v == CHAIN_DESTROY || v == CHAIN_WORK || v == CHAIN_KERNEL || v == CHAIN_D2D) {
              CK(hipEventDestroy(E));
              E = nullptr;
            }
          }
          if (v == CHAIN_KERNEL)
            hipLaunchKernelGGL(copy_k, dim3(1024), dim3(256), 0, C, y, x, n);
          else
            CK(hipMemcpyAsync(y, x, n * 4, v == CHAIN_D2D ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToDeviceNoCU, C));
          CK(hipStreamSynchronize(C));
          CK(hipDeviceSynchronize());
          hipLaunchKernelGGL(count_ne, dim3(1024), dim3(256), 0, A, y, n, val, bad);
          unsigned long long h = 0;
          CK(hipMemcpyAsync(&h, bad, 8, hipMemcpyDeviceToHost, A));
          CK(hipStreamSynchronize(A));
          total_bad += h;
          bad_iters += h != 0;
          CK(hipEventDestroy(evA));
          if (E) CK(hipEventDestroy(E));
        }
        printf("%s{\"side\": \"producer\", \"variant\": \"%s\", \"A\": \"%s\", \"B\": \"%s\", \"C\": \"%s\", "
               "\"bad_iters\": %d, \"bad_elems\": %llu}",
               first ? "  " : ",\n  ", kNames[v], a_null ? "null" : "created", b_high ? "high" : "normal",
               c_high ? "high" : "normal", bad_iters, total_bad);
        first = false;
        fflush(stdout);
        if (A) CK(hipStreamDestroy(A));
        CK(hipStreamDestroy(B));
        CK(hipStreamDestroy(C));
      }
  // join side: C copies X -> Y on a copy engine; B waits on an event recorded on C and compares
  for (int b_high = 0; b_high <= 1; ++b_high)
    for (int c_high = 0; c_high <= 1; ++c_high)
    for (int keep = 0; keep <= 1; ++keep) {
      hipStream_t B, C;
      CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, b_high ? hi : lo));
      CK(hipStreamCreateWithPriority(&C, hipStreamNonBlocking, c_high ? hi : lo));
      unsigned long long total_bad = 0;
      int bad_iters = 0;
      for (int it = 0; it < iters; ++it) {
        val += 1.0f;
        hipLaunchKernelGGL(slow_fill, dim3(1024), dim3(256), 0, C, x, n, val, 1);
        CK(hipMemsetAsync(y, 0, n * 4, C));
        CK(hipMemsetAsync(bad, 0, 8, C));
        CK(hipStreamSynchronize(C));
        CK(hipMemcpyAsync(y, x, n * 4, hipMemcpyDeviceToDeviceNoCU, C));
        hipEvent_t E;
        CK(hipEventCreateWithFlags(&E, hipEventDisableTiming));
        CK(hipEventRecord(E, C));
        CK(hipStreamWaitEvent(B, E, 0));
        if (!keep) CK(hipEventDestroy(E));
        hipLaunchKernelGGL(count_diff, dim3(1024), dim3(256), 0, B, y, x, n, bad);
        unsigned long long h = 0;
        CK(hipMemcpyAsync(&h, bad, 8, hipMemcpyDeviceToHost, B));
        CK(hipStreamSynchronize(B));
        CK(hipDeviceSynchronize());
        if (keep) CK(hipEventDestroy(E));
        total_bad += h;
        bad_iters += h != 0;
      }
      printf(",\n  {\"side\": \"join\", \"variant\": \"%s\", \"B\": \"%s\", \"C\": \"%s\", \"bad_iters\": %d, "
             "\"bad_elems\": %llu}",
             keep ? "keep" : "destroy", b_high ? "high" : "normal", c_high ? "high" : "normal", bad_iters, total_bad);
      fflush(stdout);
      CK(hipStreamDestroy(B));
      CK(hipStreamDestroy(C));
    }
  printf("\n]}\n");
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(scratch));
  CK(hipFree(bad));
  return 0;
}
