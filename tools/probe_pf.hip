// probe_pf.hip — reduce_kernel_narrow vs reduce_kernel_narrow_pf (L2 prefetch waves) on narrow
// windows: every variant launched once under a host watchdog (progress on stderr, unbuffered),
// bitwise-checked against the narrow kernel, then timed in interleaved rounds, warm (back-to-back
// launches) and cold (a 1-GiB memset between launches evicts L2 and the Infinity Cache).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iflearn_amd/csrc \
//         tools/probe_pf.hip -o tools/probe_pf
//   tools/probe_pf [n=1000] [ncols=44426] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <type_traits>
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

namespace fa {
// Narrow windows with L2 prefetch waves.  reduce_kernel_narrow's one wave per 1-KiB chunk walks
// the N rows through at most 63 loads in flight (its vmcnt), so at 174 chunks the chip holds ~7 MB
// of requests and the serial sweep is latency-bound below the streaming roof.  Here each chunk's
// block adds NPF prefetch waves beside the consumer wave: lane l of a prefetch wave loads one
// dword of row r0 + l/8 at byte (l%8)*128 — one dword per 128-B line, so ONE instruction pulls 8
// rows (8 KiB) of the chunk into L2 — PD instructions deep, groups of 8 rows interleaved over the
// NPF waves.  The consumer runs the unchanged sequential sweep (bit-exact, list order) with its
// loads hitting L2 or merging with a prefetch in flight.  Prefetchers stay at most LEAD rows ahead
// of the consumer (its row index in LDS), so a chunk's prefetched lines are still in the XCD's
// 4-MiB L2 when the consumer reaches them.  The consumer never waits for a prefetcher.
template <class P, typename T, int OP, int D, int NPF, int PD, int LEAD, bool NTC, int RPI = 8>
__global__ __launch_bounds__(64 * (1 + NPF)) void reduce_kernel_narrow_pf(const float* __restrict__ stack,
                                                                          int64_t stride, int n,
                                                                          const typename P::w_t* __restrict__ w,
                                                                          int64_t col0, int64_t ncols, Epi<T> e) {
  static_assert(sizeof(typename P::x_t) == 4 && D <= 63 && PD <= 63, "4-byte rows; vmcnt counts 63 loads");
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  typedef typename vec4<float>::type XV;
  __shared__ int s_row;  // the consumer's next row (its progress), read by the prefetchers
  if (threadIdx.x == 0) s_row = 0;
  __syncthreads();
  const int64_t nquads = (ncols + 3) / 4;
  const int64_t qb = (int64_t)blockIdx.x * 64;
  const int64_t qe = qb + 64 < nquads ? qb + 64 : nquads;
  const int64_t cend = qe * 4 < ncols ? qe * 4 : ncols;
  if (cend <= qb * 4) return;
  const int cols = (int)(cend - qb * 4);
  const uint32_t bytes = (uint32_t)cols * 4u;
  const int64_t rb = stride * 4;
  const char* base = reinterpret_cast<const char*>(stack + col0 + qb * 4);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)threadIdx.x & 63;
  if (wave > 0) {  // prefetcher k = wave - 1: row groups k, k + NPF, ... of 8 rows
    // RPI rows per instruction: 8 = one dword per 128-B line of 8 rows (lane l: row l/8, line l%8);
    // 1 = one coalesced 16-B-per-lane row load, like the consumer's
    const int voff = RPI == 8 ? (lane >> 3) * (int)rb + (lane & 7) * 128 : lane * 16;
    typedef typename std::conditional<RPI == 8, int, XV>::type PT;
    PT pf[PD];
#pragma unroll
    for (int d = 0; d < PD; ++d) pf[d] = PT{};
    int spins = 0;
    for (int r0 = (wave - 1) * RPI; r0 < n; r0 += NPF * RPI * PD) {
#pragma unroll
      for (int d = 0; d < PD; ++d) {
        const int rr = r0 + d * NPF * RPI;
        // consume the load issued PD slots ago (an opaque use: the compiler waits for exactly that
        // one, vmcnt(PD - 1), instead of sinking a reassociable use to a drain after the batch)
        asm volatile("" ::"v"(pf[d]));
        if (d % 4 == 0) {  // pacing; relaxed workgroup-scope load (a volatile read drained vmcnt).
          // Bounded: a prefetcher never waits more than ~1 ms in all, whatever the consumer does
          for (; spins < 4096 && rr > __hip_atomic_load(&s_row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + LEAD;
               ++spins)
            __builtin_amdgcn_s_sleep(4);
        }
        // rows past n: empty range, the load is dropped (no branch, no phi)
        const int rows = n - rr < RPI ? n - rr : RPI;
        const uint32_t nrec = rows > 0 ? (uint32_t)((rows - 1) * rb) + bytes : 0u;
        const __amdgpu_buffer_rsrc_t r = row_rsrc(base + (int64_t)rr * rb, nrec);
        if constexpr (RPI == 8)
          pf[d] = (int)__builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0);
        else
          pf[d] = buf_load_quad<false>(r, voff, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < PD; ++d) asm volatile("" ::"v"(pf[d]));
    return;
  }
  const int voff = lane * 16;
  const char* lastp = base + (int64_t)(n - 1) * rb;
  const char* p = base + rb;
#define FA_NP_LOAD(dst, CLAMP)                                                         \
  {                                                                                      \
    const char* q_ = p;                                                                  \
    if (CLAMP) q_ = p <= lastp ? p : lastp;                                              \
    dst = buf_load_quad<NTC>(row_rsrc(q_, bytes), voff, 0);                              \
    p += rb;                                                                             \
    asm volatile("" : "+s"(p));                                                          \
  }
  typedef typename P::w_t WT;
  const __amdgpu_buffer_rsrc_t wr = row_rsrc(w, (uint32_t)n * (uint32_t)sizeof(WT));
  auto wload = [&](int first) {
    if constexpr (sizeof(WT) == 4)
      return __builtin_bit_cast(WT, __builtin_amdgcn_raw_buffer_load_b32(wr, (lane + first) * 4, 0, 0));
    else
      return __builtin_bit_cast(WT, __builtin_amdgcn_raw_buffer_load_b64(wr, (lane + first) * 8, 0, 0));
  };
  auto wlane = [](WT v, int l) {
    if constexpr (sizeof(WT) == 4) {
      return __builtin_bit_cast(WT, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    } else {
      const long long b = __builtin_bit_cast(long long, v);
      const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
      return __builtin_bit_cast(WT, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    }
  };
  WT wcur = wload(1);
  XV x[D];
#pragma unroll
  for (int d = 0; d < D; ++d) FA_NP_LOAD(x[d], true);
  AV acc = quad_mul<P>(w[0], buf_load_quad<NTC>(row_rsrc(base, bytes), voff, 0));
  int i = 1;
  for (; i + 2 * D <= n; i += D) {
    const WT wnext = wload(i + D);
    if (lane == 0) __hip_atomic_store(&s_row, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc = quad_axpy<P>(acc, wlane(wcur, d), x[d]);
      __builtin_amdgcn_sched_barrier(0);
      FA_NP_LOAD(x[d], false);
      __builtin_amdgcn_sched_barrier(0);
    }
    wcur = wnext;
  }
  if (lane == 0) __hip_atomic_store(&s_row, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // release the prefetchers
  for (; i < n; i += D) {
    const WT wnext = wload(i + D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const AV t = quad_axpy<P>(acc, wlane(wcur, d), x[d]);
      acc = i + d < n ? t : acc;
      __builtin_amdgcn_sched_barrier(0);
      FA_NP_LOAD(x[d], true);
      __builtin_amdgcn_sched_barrier(0);
    }
    wcur = wnext;
  }
#undef FA_NP_LOAD
  const AV accs[1] = {acc};
  finish_piece<T, OP, A, 1, 64, 1>(e, qb, cols, accs);
}

}  // namespace fa

using namespace fa;

struct Var {
  std::string name;
  std::function<void()> launch;
  std::vector<float> warm, cold;
};

template <int D>
Var narrow(const float* s, int64_t stride, int n, const float* w, int64_t ncols, Epi<double> e) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  return {"narrow D" + std::to_string(D),
          [=] {
            hipLaunchKernelGGL((reduce_kernel_narrow<AccF32, double, FA_OP_MEAN, D, 1, true>), dim3((unsigned)chunks),
                               dim3(64), 0, 0, s, stride, n, w, (int64_t)0, ncols, e);
          },
          {}, {}};
}

template <int D, int NPF, int PD, int LEAD, bool NTC, int RPI = 8>
Var pf(const float* s, int64_t stride, int n, const float* w, int64_t ncols, Epi<double> e) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  char name[96];
  snprintf(name, sizeof name, "pf D%d NPF%d PD%d L%d NT%d R%d", D, NPF, PD, LEAD, (int)NTC, RPI);
  return {name,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_narrow_pf<AccF32, double, FA_OP_MEAN, D, NPF, PD, LEAD, NTC, RPI>),
                               dim3((unsigned)chunks), dim3(64 * (1 + NPF)), 0, 0, s, stride, n, w, (int64_t)0, ncols, e);
          },
          {}, {}};
}

static bool wait_done(double limit_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(0);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) {
      fprintf(stderr, "stream error %s\n", hipGetErrorString(q));
      exit(1);
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) return false;
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int n = argc > 1 ? atoi(argv[1]) : 1000;
  const int64_t ncols = argc > 2 ? atoll(argv[2]) : 44426;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  const int64_t stride = (ncols + 63) / 64 * 64;
  float *stack, *w, *out;
  CK(hipMalloc(&stack, (size_t)n * stride * 4));
  CK(hipMalloc(&w, n * 4));
  CK(hipMalloc(&out, stride * 4));
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(4096, n), dim3(256), 0, 0, stack, stride, stride, 2024ull,
                     (int64_t)0, (int64_t)0);
  std::vector<float> ones(n, 1.0f);
  CK(hipMemcpy(w, ones.data(), n * 4, hipMemcpyHostToDevice));
  void* flush;
  CK(hipMalloc(&flush, (size_t)1 << 30));
  CK(hipDeviceSynchronize());
  Epi<double> e{};
  e.denom = (double)n;
  e.out32 = out;
  const double bytes = (double)n * ncols * 4 + ncols * 4;
  printf("# n=%d ncols=%lld stride=%lld bytes=%.0f\n", n, (long long)ncols, (long long)stride, bytes);

  std::vector<Var> vs;
  vs.push_back(narrow<40>(stack, stride, n, w, ncols, e));
  vs.push_back(narrow<32>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 32, 256, false>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 32, 100000, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 48, 100000, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 60, 100000, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 32, 80, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 48, 120, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 60, 160, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 1, 60, 160, true, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 2, 32, 160, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 2, 48, 200, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<20, 1, 60, 160, false, 1>(stack, stride, n, w, ncols, e));
  vs.push_back(pf<40, 3, 32, 200, false, 1>(stack, stride, n, w, ncols, e));
  std::vector<float> ref(ncols), got(ncols);
  for (size_t i = 0; i < vs.size(); ++i) {
    fprintf(stderr, "check %s ...", vs[i].name.c_str());
    CK(hipMemset(out, 0xff, stride * 4));
    vs[i].launch();
    if (!wait_done(5.0)) {
      fprintf(stderr, " HUNG (> 5 s)\n");
      printf("HUNG %s\n", vs[i].name.c_str());
      return 3;
    }
    CK(hipMemcpy(i == 0 ? ref.data() : got.data(), out, ncols * 4, hipMemcpyDeviceToHost));
    const bool ok = i == 0 || memcmp(ref.data(), got.data(), ncols * 4) == 0;
    fprintf(stderr, ok ? " ok\n" : " MISMATCH\n");
    if (!ok) {
      printf("MISMATCH %s\n", vs[i].name.c_str());
      return 2;
    }
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      v.launch();
      CK(hipEventRecord(a, 0));
      for (int k = 0; k < 10; ++k) v.launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.warm.push_back(ms / 10);
      for (int k = 0; k < 5; ++k) {
        CK(hipMemsetAsync(flush, (r + k) & 0xff, (size_t)1 << 30, 0));
        CK(hipEventRecord(a, 0));
        v.launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        v.cold.push_back(ms);
      }
    }
    fprintf(stderr, "round %d done\n", r);
  }
  printf("%-28s %10s %8s %10s %8s\n", "variant", "warm_us", "%8TB/s", "cold_us", "%8TB/s");
  for (auto& v : vs) {
    std::sort(v.warm.begin(), v.warm.end());
    std::sort(v.cold.begin(), v.cold.end());
    const double wm = v.warm[v.warm.size() / 2] * 1e3, cm = v.cold[v.cold.size() / 2] * 1e3;
    printf("%-28s %10.2f %8.2f %10.2f %8.2f\n", v.name.c_str(), wm, bytes / (wm * 1e-6) / 8e12 * 100, cm,
           bytes / (cm * 1e-6) / 8e12 * 100);
  }
  return 0;
}
