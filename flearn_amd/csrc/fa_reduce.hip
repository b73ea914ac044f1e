// fa_reduce.hip — gfx950 kernels + C ABI of the FedAVG-family aggregation engine.
//
// Hot path: Strategy.server_ensemble (flearn/common/strategy/strategy.py:102-130), i.e. for
// every element p of the flattened model bucket
//     acc = a0*x[0][p];  acc += a_n*x[n][p]  (n = 1..N-1, in list order);  w = acc / sum(a)
// followed optionally by the AVGM / FedOPT update (avgm.py:19-36, opt.py:23-65).
//
// Mapping (HBM-bound streaming reduce, 0.5 flop/B, no MFMA):
//   * one thread owns V quads (4 contiguous fp32 = one 16-B global_load_dwordx4); the V quads of
//     a thread are kThreads*4 elements apart, so each wave instruction reads 1 KiB contiguous of
//     one client row;
//   * the client loop runs down the rows in list order (bit-exact sequential fp32 sum, as numpy
//     does it) and is unrolled U deep, so each thread keeps U*V*16 B of loads in flight — the
//     HBM latency is covered by loads that are independent of the running sum;
//   * each client value is read exactly once per launch: loads are non-temporal;
//   * the epilogue (divide, optional momentum/adaptive update, f32/f64 stores) is fused, so the
//     only HBM traffic is N*P*4 of client reads plus the O(P) output/state bytes.
// This TU is compiled with -ffp-contract=off: a fused a*x+acc would change the fp32 rounding and
// break bit-parity with the reference.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <cstdio>
#include <string>

#include "flearn_amd.h"

namespace {

constexpr int kThreads = 256;

thread_local std::string g_last_error;

int fail(int code, const char* what) {
  g_last_error = what;
  return code;
}

template <typename T>
struct vec4 {
  typedef T type __attribute__((ext_vector_type(4)));
};

// 4 contiguous elements, 16-B aligned for fp32 (32-B for 8-byte types), read once.
template <typename T>
__device__ __forceinline__ typename vec4<T>::type load_quad(const T* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const typename vec4<T>::type*>(p));
}

template <typename T>
__device__ __forceinline__ typename vec4<T>::type load_quad_guarded(const T* p, int valid) {
  typename vec4<T>::type r = {T(0), T(0), T(0), T(0)};
  if (valid > 0) r[0] = p[0];
  if (valid > 1) r[1] = p[1];
  if (valid > 2) r[2] = p[2];
  if (valid > 3) r[3] = p[3];
  return r;
}

template <typename T>
__device__ __forceinline__ void store_quad(T* p, typename vec4<T>::type v, int valid) {
  if (valid == 4) {
    *reinterpret_cast<typename vec4<T>::type*>(p) = v;
  } else {
    if (valid > 0) p[0] = v[0];
    if (valid > 1) p[1] = v[1];
    if (valid > 2) p[2] = v[2];
  }
}

// ---------------------------------------------------------------------------------------------
// Accumulation policies: product dtype = sum dtype, chosen by numpy's promotion of the weight
// type against the tensor dtype (resolved on the host, see flearn_amd/bucket.py).
// ---------------------------------------------------------------------------------------------
struct AccF32 {  // fp32 tensors x Python-float/int or np.float32 weights
  typedef float x_t;
  typedef float w_t;
  typedef float acc_t;
  static __device__ __forceinline__ float mul(float w, float x) { return w * x; }
};
struct AccF32W64 {  // fp32 tensors x np.float64/np.int64 weights: promoted to f64
  typedef float x_t;
  typedef double w_t;
  typedef double acc_t;
  static __device__ __forceinline__ double mul(double w, float x) { return w * (double)x; }
};
struct AccF64 {  // f64 tensors (and int64 buffers cast to f64) x f64 weights
  typedef double x_t;
  typedef double w_t;
  typedef double acc_t;
  static __device__ __forceinline__ double mul(double w, double x) { return w * x; }
};
struct AccI64 {  // int64 buffers x Python-int weights: int64 arithmetic, wraps like numpy
  typedef int64_t x_t;
  typedef int64_t w_t;
  typedef int64_t acc_t;
  static __device__ __forceinline__ int64_t mul(int64_t w, int64_t x) {
    return (int64_t)((uint64_t)w * (uint64_t)x);
  }
};

template <typename A>
__device__ __forceinline__ A add(A a, A b) {
  return a + b;
}
template <>
__device__ __forceinline__ int64_t add<int64_t>(int64_t a, int64_t b) {
  return (int64_t)((uint64_t)a + (uint64_t)b);
}

// ---------------------------------------------------------------------------------------------
// Epilogue: mean in precision T (double for DIV64/W64, float for DIV32) and the optional
// server-side optimizer update, all in T with the reference's operation order.
// ---------------------------------------------------------------------------------------------
template <typename T>
struct Epi {
  T denom;
  const float* prev;
  T* v;
  T beta, eta, tau, beta2, c;  // c = 1 - beta2 (evaluated in double on the host, as Python does)
  float* out32;
  double* out64;
};

template <typename T>
__device__ __forceinline__ T sign_of(T x) {
  // np.sign: -1, 0, +1, NaN for NaN
  return x > T(0) ? T(1) : (x < T(0) ? T(-1) : (x == T(0) ? T(0) : x));
}

template <typename T, int OP>
__device__ __forceinline__ T update(const Epi<T>& e, T g, T l, T& vv) {
  if constexpr (OP == FA_OP_MEAN) {
    return g;
  } else {
    const T d = g - l;  // delta_w = w_glob - w_local            avgm.py:22-25 / opt.py:30-33
    if constexpr (OP == FA_OP_AVGM) {
      vv = d + e.beta * vv;  // v_t = delta + beta*v_t           avgm.py:31-32
      return l + vv;         // w_local + v_t                    avgm.py:34-35
    } else {
      const T m = d * d;  // np.multiply(delta, delta)            opt.py:52
      if constexpr (OP == FA_OP_ADAGRAD) {
        vv = vv + m;  //                                          opt.py:53-54
      } else if constexpr (OP == FA_OP_YOGI) {
        vv = vv - (e.c * m) * sign_of<T>(vv - m);  //             opt.py:55-58
      } else {
        vv = e.beta2 * vv + e.c * m;  //                          opt.py:59-60
      }
      return l + (e.eta * d) / (sqrt(vv) + e.tau);  //          opt.py:62-63
    }
  }
}

template <typename T, int OP, typename A>
__device__ __forceinline__ void finish_quad(const Epi<T>& e, int64_t c, int valid,
                                            typename vec4<A>::type acc) {
  typename vec4<T>::type w;
  typename vec4<T>::type vv = {T(0), T(0), T(0), T(0)};
  typename vec4<float>::type l = {0.f, 0.f, 0.f, 0.f};
  if constexpr (OP != FA_OP_MEAN) {
    if (valid == 4) {
      l = *reinterpret_cast<const typename vec4<float>::type*>(e.prev + c);
      vv = *reinterpret_cast<const typename vec4<T>::type*>(e.v + c);
    } else {
      l = load_quad_guarded(e.prev + c, valid);
      vv = load_quad_guarded(e.v + c, valid);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const T g = (T)acc[j] / e.denom;  // np.divide(w_glob, np.sum(a))  strategy.py:127-129
    T vj = vv[j];
    w[j] = update<T, OP>(e, g, (T)l[j], vj);
    vv[j] = vj;
  }
  if constexpr (OP != FA_OP_MEAN) store_quad<T>(e.v + c, vv, valid);
  if (e.out32) {
    typename vec4<float>::type o = {(float)w[0], (float)w[1], (float)w[2], (float)w[3]};
    store_quad<float>(e.out32 + c, o, valid);
  }
  if (e.out64) {
    typename vec4<double>::type o = {(double)w[0], (double)w[1], (double)w[2], (double)w[3]};
    store_quad<double>(e.out64 + c, o, valid);
  }
}

// ---------------------------------------------------------------------------------------------
// The reduce kernel.  Block b covers quads [b*kThreads*V, (b+1)*kThreads*V); thread t owns quads
// b*kThreads*V + v*kThreads + t, v < V.
// ---------------------------------------------------------------------------------------------
template <class P, typename T, int OP, int V, int U>
__global__ __launch_bounds__(kThreads) void reduce_kernel(
    const typename P::x_t* __restrict__ stack, int64_t stride, int n,
    const typename P::w_t* __restrict__ w, int64_t col0, int64_t ncols, Epi<T> e) {
  typedef typename P::x_t X;
  typedef typename P::acc_t A;
  typedef typename vec4<X>::type XV;
  typedef typename vec4<A>::type AV;

  const int64_t q0 = (int64_t)blockIdx.x * (kThreads * V) + threadIdx.x;
  const X* base = stack + col0;

  if ((q0 + (int64_t)(V - 1) * kThreads) * 4 + 4 <= ncols) {
    // ---- full tile: V aligned quads per thread ----
    AV acc[V];
    {
      const typename P::w_t w0 = w[0];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const XV x = load_quad(base + (q0 + v * kThreads) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[v][j] = P::mul(w0, x[j]);
      }
    }
    int i = 1;
    for (; i + U <= n; i += U) {
      XV x[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const X* row = base + (int64_t)(i + u) * stride;
#pragma unroll
        for (int v = 0; v < V; ++v) x[u][v] = load_quad(row + (q0 + v * kThreads) * 4);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const typename P::w_t wu = w[i + u];
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[v][j] = add<A>(acc[v][j], P::mul(wu, x[u][v][j]));
      }
    }
    for (; i < n; ++i) {
      const X* row = base + (int64_t)i * stride;
      const typename P::w_t wi = w[i];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const XV x = load_quad(row + (q0 + v * kThreads) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[v][j] = add<A>(acc[v][j], P::mul(wi, x[j]));
      }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) finish_quad<T, OP, A>(e, (q0 + v * kThreads) * 4, 4, acc[v]);
    return;
  }

  // ---- ragged tail (last block only): quad by quad, element-guarded ----
  for (int v = 0; v < V; ++v) {
    const int64_t c = (q0 + (int64_t)v * kThreads) * 4;
    if (c >= ncols) break;
    const int valid = (int)((ncols - c) < 4 ? (ncols - c) : 4);
    AV acc;
    {
      const XV x = load_quad_guarded(base + c, valid);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = P::mul(w[0], x[j]);
    }
    for (int i = 1; i < n; ++i) {
      const XV x = load_quad_guarded(base + (int64_t)i * stride + c, valid);
      const typename P::w_t wi = w[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = add<A>(acc[j], P::mul(wi, x[j]));
    }
    finish_quad<T, OP, A>(e, c, valid, acc);
  }
}

// Standalone update (client_receive form): g read from memory instead of reduced.
template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void apply_kernel(const float* __restrict__ local,
                                                         const T* __restrict__ glob, int64_t n,
                                                         Epi<T> e) {
  const int64_t c = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 4;
  if (c >= n) return;
  const int valid = (int)((n - c) < 4 ? (n - c) : 4);
  typename vec4<T>::type g = load_quad_guarded(glob + c, valid);
  // reuse finish_quad with denom == 1: T(g)/1 == g exactly
  finish_quad<T, OP, T>(e, c, valid, g);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void fill_uniform_kernel(float* __restrict__ dst,
                                                                int64_t stride, int64_t ncols,
                                                                uint64_t seed, int64_t row0,
                                                                int64_t colg0) {
  const int64_t r = blockIdx.y;
  const uint64_t key_row = (seed * 0xD1B54A32D192ED03ull) ^ ((uint64_t)(row0 + r) << 40);
  float* out = dst + r * stride;
  for (int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x; c < ncols;
       c += (int64_t)gridDim.x * kThreads) {
    const uint64_t h = splitmix64(key_row ^ (uint64_t)(colg0 + c));
    out[c] = (float)(h >> 40) * 0x1.0p-23f - 1.0f;
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
constexpr int kV = 2;  // quads per thread
constexpr int kU = 8;  // client unroll (loads in flight per thread = kU*kV*16 B for fp32)

template <typename X>
bool aligned_window(const X* stack, int64_t stride, int64_t col0) {
  const uintptr_t a = (uintptr_t)(stack + col0);
  return (a % (4 * sizeof(X))) == 0 && ((stride * (int64_t)sizeof(X)) % (4 * sizeof(X))) == 0;
}

int launch_check() {
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(err));
  return FA_OK;
}

template <class P, typename T, int OP>
int launch_reduce(const typename P::x_t* stack, int64_t stride, int n, const void* w, int64_t col0,
                  int64_t ncols, const Epi<T>& e, hipStream_t s) {
  const int64_t per_block = (int64_t)kThreads * kV * 4;
  const int64_t blocks = (ncols + per_block - 1) / per_block;
  if (blocks > 0x7fffffff) return fail(FA_ERR_ARG, "n_cols too large");
  hipLaunchKernelGGL((reduce_kernel<P, T, OP, kV, kU>), dim3((unsigned)blocks), dim3(kThreads), 0, s,
                     stack, stride, n, static_cast<const typename P::w_t*>(w), col0, ncols, e);
  return launch_check();
}

template <class P, typename T>
int dispatch_op(int op, const typename P::x_t* stack, int64_t stride, int n, const void* w,
                int64_t col0, int64_t ncols, const Epi<T>& e, hipStream_t s) {
  switch (op) {
    case FA_OP_MEAN: return launch_reduce<P, T, FA_OP_MEAN>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_AVGM: return launch_reduce<P, T, FA_OP_AVGM>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_ADAGRAD:
      return launch_reduce<P, T, FA_OP_ADAGRAD>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_YOGI: return launch_reduce<P, T, FA_OP_YOGI>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_ADAM: return launch_reduce<P, T, FA_OP_ADAM>(stack, stride, n, w, col0, ncols, e, s);
    default: return fail(FA_ERR_ARG, "unknown epilogue op");
  }
}

template <typename T>
int make_epi(const fa_epilogue* in, double denom, float* out32, double* out64, Epi<T>* e) {
  e->denom = (T)denom;
  e->prev = nullptr;
  e->v = nullptr;
  e->beta = e->eta = e->tau = e->beta2 = e->c = T(0);
  e->out32 = out32;
  e->out64 = out64;
  if (in && in->op != FA_OP_MEAN) {
    if (in->op < FA_OP_AVGM || in->op > FA_OP_ADAM) return fail(FA_ERR_ARG, "unknown epilogue op");
    if (!in->prev || !in->v) return fail(FA_ERR_ARG, "epilogue needs prev and v");
    e->prev = in->prev;
    e->v = static_cast<T*>(in->v);
    e->beta = (T)in->beta;
    e->eta = (T)in->eta;
    e->tau = (T)in->tau;
    e->beta2 = (T)in->beta2;
    e->c = (T)(1.0 - in->beta2);  // Python evaluates (1 - self.beta2) in double
  }
  return FA_OK;
}

bool aligned_to(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

// per-column arrays are accessed with 4-element vector loads/stores
int check_columns(const float* out32, const double* out64, const void* prev, const void* v,
                  size_t v_elem) {
  if (!aligned_to(out32, 16) || !aligned_to(out64, 32) || !aligned_to(prev, 16) ||
      !aligned_to(v, 4 * v_elem))
    return fail(FA_ERR_ALIGN, "output / prev / v arrays must be 4-element aligned");
  return FA_OK;
}

template <typename X>
int check_common(const X* stack, int64_t stride, int n, const void* w, int64_t col0,
                 int64_t ncols, const void* o1, const void* o2) {
  if (n <= 0) return fail(FA_ERR_ARG, "n_clients must be >= 1");
  if (ncols < 0 || col0 < 0 || stride < col0 + ncols) return fail(FA_ERR_ARG, "bad column window");
  if (!stack || !w) return fail(FA_ERR_ARG, "null stack or weights");
  if (!o1 && !o2) return fail(FA_ERR_ARG, "no output");
  if (!aligned_window(stack, stride, col0)) return fail(FA_ERR_ALIGN, "row window not 16-B aligned");
  return FA_OK;
}

}  // namespace

extern "C" {

int fa_abi_version(void) { return FA_ABI_VERSION; }

const char* fa_last_error(void) { return g_last_error.c_str(); }

int fa_reduce_f32(const float* stack, int64_t row_stride, int32_t n_clients, int32_t mode,
                  const void* weights, double denom, int64_t col_begin, int64_t n_cols,
                  const fa_epilogue* epi, float* out32, double* out64, void* stream) {
  int rc = check_common(stack, row_stride, n_clients, weights, col_begin, n_cols, out32, out64);
  if (rc) return rc;
  if (n_cols == 0) return FA_OK;
  const int op = epi ? epi->op : FA_OP_MEAN;
  if ((rc = check_columns(out32, out64, epi ? epi->prev : nullptr, epi ? epi->v : nullptr,
                          mode == FA_MODE_W32_DIV32 ? sizeof(float) : sizeof(double))))
    return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == FA_MODE_W32_DIV64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, out32, out64, &e))) return rc;
    return dispatch_op<AccF32, double>(op, stack, row_stride, n_clients, weights, col_begin, n_cols,
                                       e, s);
  }
  if (mode == FA_MODE_W32_DIV32) {
    Epi<float> e;
    if ((rc = make_epi<float>(epi, denom, out32, out64, &e))) return rc;
    return dispatch_op<AccF32, float>(op, stack, row_stride, n_clients, weights, col_begin, n_cols,
                                      e, s);
  }
  if (mode == FA_MODE_W64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, out32, out64, &e))) return rc;
    return dispatch_op<AccF32W64, double>(op, stack, row_stride, n_clients, weights, col_begin,
                                          n_cols, e, s);
  }
  return fail(FA_ERR_ARG, "unknown reduce mode");
}

int fa_reduce_f64(const double* stack, int64_t row_stride, int32_t n_clients,
                  const double* weights, double denom, int64_t col_begin, int64_t n_cols,
                  double* out64, void* stream) {
  int rc = check_common(stack, row_stride, n_clients, weights, col_begin, n_cols, out64, nullptr);
  if (rc) return rc;
  if (n_cols == 0) return FA_OK;
  if ((rc = check_columns(nullptr, out64, nullptr, nullptr, 8))) return rc;
  Epi<double> e;
  make_epi<double>(nullptr, denom, nullptr, out64, &e);
  return launch_reduce<AccF64, double, FA_OP_MEAN>(stack, row_stride, n_clients, weights, col_begin,
                                                   n_cols, e, static_cast<hipStream_t>(stream));
}

int fa_reduce_i64(const int64_t* stack, int64_t row_stride, int32_t n_clients,
                  const int64_t* weights, double denom, int64_t col_begin, int64_t n_cols,
                  double* out64, void* stream) {
  int rc = check_common(stack, row_stride, n_clients, weights, col_begin, n_cols, out64, nullptr);
  if (rc) return rc;
  if (n_cols == 0) return FA_OK;
  if ((rc = check_columns(nullptr, out64, nullptr, nullptr, 8))) return rc;
  Epi<double> e;
  make_epi<double>(nullptr, denom, nullptr, out64, &e);
  return launch_reduce<AccI64, double, FA_OP_MEAN>(stack, row_stride, n_clients, weights, col_begin,
                                                   n_cols, e, static_cast<hipStream_t>(stream));
}

int fa_opt_apply(int32_t prec, const fa_epilogue* epi, const float* local, const void* glob,
                 int64_t n, float* out32, double* out64, void* stream) {
  if (!epi || !local || !glob || n < 0) return fail(FA_ERR_ARG, "bad apply arguments");
  if (!out32 && !out64) return fail(FA_ERR_ARG, "no output");
  if (n == 0) return FA_OK;
  if (epi->op == FA_OP_MEAN) return fail(FA_ERR_ARG, "apply needs an optimizer op");
  const size_t ve = prec == FA_PREC_F32 ? sizeof(float) : sizeof(double);
  int rc0 = check_columns(out32, out64, local, epi->v, ve);
  if (rc0) return rc0;
  if (!epi->v) return fail(FA_ERR_ARG, "apply needs v");
  fa_epilogue local_epi = *epi;
  local_epi.prev = local;
  const int64_t blocks = (n + kThreads * 4 - 1) / (kThreads * 4);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc;
#define FA_APPLY(T, OPV)                                                                        \
  hipLaunchKernelGGL((apply_kernel<T, OPV>), dim3((unsigned)blocks), dim3(kThreads), 0, s, local, \
                     static_cast<const T*>(glob), n, e)
  if (prec == FA_PREC_F64) {
    Epi<double> e;
    if ((rc = make_epi<double>(&local_epi, 1.0, out32, out64, &e))) return rc;
    switch (epi->op) {
      case FA_OP_AVGM: FA_APPLY(double, FA_OP_AVGM); break;
      case FA_OP_ADAGRAD: FA_APPLY(double, FA_OP_ADAGRAD); break;
      case FA_OP_YOGI: FA_APPLY(double, FA_OP_YOGI); break;
      default: FA_APPLY(double, FA_OP_ADAM); break;
    }
  } else if (prec == FA_PREC_F32) {
    Epi<float> e;
    if ((rc = make_epi<float>(&local_epi, 1.0, out32, out64, &e))) return rc;
    switch (epi->op) {
      case FA_OP_AVGM: FA_APPLY(float, FA_OP_AVGM); break;
      case FA_OP_ADAGRAD: FA_APPLY(float, FA_OP_ADAGRAD); break;
      case FA_OP_YOGI: FA_APPLY(float, FA_OP_YOGI); break;
      default: FA_APPLY(float, FA_OP_ADAM); break;
    }
  } else {
    return fail(FA_ERR_ARG, "unknown precision");
  }
#undef FA_APPLY
  return launch_check();
}

int fa_fill_uniform_f32(float* dst, int64_t row_stride, int32_t n_rows, int64_t n_cols,
                        uint64_t seed, int64_t row_begin, int64_t col_global_begin, void* stream) {
  if (!dst || n_rows < 0 || n_cols < 0 || row_stride < n_cols) return fail(FA_ERR_ARG, "bad fill");
  if (n_rows == 0 || n_cols == 0) return FA_OK;
  if (n_rows > 65535) return fail(FA_ERR_ARG, "too many rows for one fill");
  int64_t bx = (n_cols + kThreads - 1) / kThreads;
  if (bx > 4096) bx = 4096;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3((unsigned)bx, (unsigned)n_rows), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), dst, row_stride, n_cols, seed, row_begin,
                     col_global_begin);
  return launch_check();
}

}  // extern "C"
