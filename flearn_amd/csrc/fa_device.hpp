// fa_device.hpp — device code of the FedAVG-family aggregation engine (gfx950).
//
// Included by fa_reduce.hip (the product C ABI) and by tools/tune_reduce.hip (the geometry
// sweep).  Everything here is header-only templates in namespace fa.
//
// Hot path: Strategy.server_ensemble (flearn/common/strategy/strategy.py:102-130), i.e. for
// every element p of the flattened model bucket
//     acc = a0*x[0][p];  acc += a_n*x[n][p]  (n = 1..N-1, in list order);  w = acc / sum(a)
// optionally followed by the AVGM / FedOPT update (avgm.py:19-36, opt.py:23-65).
//
// Mapping (HBM-bound streaming reduce, 0.5 flop/B, no MFMA):
//   * a TILE is kThreads*V quads (4 contiguous fp32 = one 16-B global_load_dwordx4) of every
//     client row; thread t owns quads t, t+kThreads, ... so each wave instruction reads 1 KiB
//     contiguous of one row;
//   * the client loop walks the rows in list order (the bit-exact sequential fp32 sum numpy
//     does) unrolled U deep: U*V independent 16-B loads in flight per thread hide HBM latency
//     behind a running sum that depends only on already-arrived data;
//   * every client value is read exactly once per launch (NT: non-temporal loads);
//   * the epilogue (divide, optional momentum/adaptive update, f32/f64 stores) is fused: the only
//     HBM traffic is N*P*4 bytes of client reads plus O(P) output/state bytes.
// Compile with -ffp-contract=off: a fused a*x+acc changes fp32 rounding and breaks bit-parity.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flearn_amd.h"

namespace fa {

constexpr int kThreads = 256;

template <typename T>
struct vec4 {
  typedef T type __attribute__((ext_vector_type(4)));
};

template <typename T, bool NT>
__device__ __forceinline__ typename vec4<T>::type load_quad(const T* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const typename vec4<T>::type*>(p));
  else
    return *reinterpret_cast<const typename vec4<T>::type*>(p);
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
// type against the tensor dtype (resolved on the host: flearn_amd/semantics.py).
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
  T beta, eta, tau, beta2, c;  // c = 1 - beta2 (evaluated in double on the host, as Python does);
                               // FA_OP_DYN: c = alpha / N (a Python float, cast to T by numpy)
  float* h;                    // FA_OP_DYN: fp32 h; v holds theta
  T n;                         // FA_OP_DYN: len(w_local_lst)
  float alpha32;               // FA_OP_DYN: fl32(alpha) — alpha * (fp32 h) stays fp32
  float* out32;
  double* out64;
  unsigned long long* trace;  // tuning only (reduce_kernel_rowmajor<..., TR = true>): phase timestamps
  T* v_out;                   // where the updated v goes; NULL: back into v (in place)
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
    const float* ls = OP == FA_OP_DYN ? e.h : e.prev;  // the fp32 per-column operand
    if (valid == 4) {
      l = *reinterpret_cast<const typename vec4<float>::type*>(ls + c);
      vv = *reinterpret_cast<const typename vec4<T>::type*>(e.v + c);
    } else {
      l = load_quad_guarded(ls + c, valid);
      vv = load_quad_guarded(e.v + c, valid);
    }
  }
  if constexpr (OP == FA_OP_DYN) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const T g = (T)acc[j] / e.denom;
      const T d = g * e.n - vv[j];                // delta_theta = w_glob*N - theta   dyn.py:20-21
      const float hn = (float)((T)l[j] - e.c * d);  // h -= alpha/N * delta (fp32 h)    dyn.py:26
      const float ah = e.alpha32 * hn;            // alpha * h stays fp32              dyn.py:33
      w[j] = g - (T)ah;                           // w_glob - alpha*h                  dyn.py:33
      l[j] = hn;
      vv[j] = w[j];                               // theta = w_glob                    dyn.py:34
    }
    store_quad<float>(e.h + c, l, valid);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const T g = (T)acc[j] / e.denom;  // np.divide(w_glob, np.sum(a))  strategy.py:127-129
      T vj = vv[j];
      w[j] = update<T, OP>(e, g, (T)l[j], vj);
      vv[j] = vj;
    }
  }
  if constexpr (OP != FA_OP_MEAN) store_quad<T>((e.v_out ? e.v_out : e.v) + c, vv, valid);
  if (e.out32) {
    typename vec4<float>::type o = {(float)w[0], (float)w[1], (float)w[2], (float)w[3]};
    store_quad<float>(e.out32 + c, o, valid);
  }
  if (e.out64) {
    typename vec4<double>::type o = {(double)w[0], (double)w[1], (double)w[2], (double)w[3]};
    store_quad<double>(e.out64 + c, o, valid);
  }
}

// Sub-tile kinds for reduce_subtile.
enum Part : int {
  kFull = 0,   // all V quads of every thread complete and inside the window (the hot path)
  kMasked = 1  // only slots v < nv are this block's; nv is WAVE-uniform (scalar branches)
};

// One sub-tile of the client stack for this thread: quads q0 + v*kThreads (v < V) of every row,
// all N rows in list order, then the fused epilogue.
// kMasked: slots v >= nv are outside this block's range.  Their loads are NOT skipped (an `if`
// around a load becomes exec-masked control flow and the compiler drains vmcnt at every join,
// serialising the row's loads); they re-read slot nv-1's address instead — an L1/L2 hit inside
// the same wave, no extra HBM traffic — and only the final stores are predicated.
template <class P, typename T, int OP, int V, int U, bool NT, int PART>
__device__ __forceinline__ void reduce_subtile(const typename P::x_t* __restrict__ base,
                                               int64_t stride, int n,
                                               const typename P::w_t* __restrict__ w, int64_t q0,
                                               int nv, const Epi<T>& e) {
  typedef typename P::x_t X;
  typedef typename P::acc_t A;
  typedef typename vec4<X>::type XV;
  typedef typename vec4<A>::type AV;
  // this lane's quad in slot 0, and each slot's offset from it (wave-uniform: nv is uniform)
  const X* lane = base + q0 * 4;
  int off[V];
#pragma unroll
  for (int v = 0; v < V; ++v) off[v] = ((PART == kFull || v < nv) ? v : nv - 1) * kThreads * 4;
  AV acc[V];
  {
    const typename P::w_t w0 = w[0];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const XV x = load_quad<X, NT>(lane + off[v]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[v][j] = P::mul(w0, x[j]);
    }
  }
  int i = 1;
  for (; i + U <= n; i += U) {
    XV x[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const X* row = lane + (int64_t)(i + u) * stride;
#pragma unroll
      for (int v = 0; v < V; ++v) x[u][v] = load_quad<X, NT>(row + off[v]);
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
    const X* row = lane + (int64_t)i * stride;
    const typename P::w_t wi = w[i];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const XV x = load_quad<X, NT>(row + off[v]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[v][j] = add<A>(acc[v][j], P::mul(wi, x[j]));
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v)
    if (PART == kFull || v < nv) finish_quad<T, OP, A>(e, (q0 + (int64_t)v * kThreads) * 4, 4, acc[v]);
}

// Buffer-descriptor form of a sub-tile (4-byte elements).  Per client row the block builds a
// buffer resource whose base is the row's first quad of this sub-tile and whose num_records is
// the sub-tile's valid byte count; lane offsets (VGPR) are the same for every row and slot v's
// 4-KiB step rides in soffset.  Slots past the valid range are dropped by the hardware range
// check (they return 0, generate no memory request and need no branch), so a partial sub-tile
// issues exactly the loads of its valid quads with the same instruction stream as a full one.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <bool NT>
__device__ __forceinline__ vec4<float>::type buf_load_quad(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, NT ? 2 : 0);
  return __builtin_bit_cast(vec4<float>::type, u);
}

// ---------------------------------------------------------------------------------------------
// Piece epilogue through buffer descriptors.  A lane's slots of a piece are quads
// q = threadIdx.x + v*STEP; the state operands (prev or h, v) are loaded for B slots at once,
// UNCONDITIONALLY, through descriptors whose range is the piece's valid columns — the raw-buffer
// range check is per dword on gfx950 (tools/probe_oob.py), so lanes past the end read 0 and their
// stores are dropped, with no branch — then the B results are computed and stored.  With one
// guarded generic load per quad (finish_quad) the compiler waited for each quad's loads, and for
// the previous quad's stores, before the next: 24 serial HBM round trips at every piece-group end
// of the fused FedAVGM kernel.
// ---------------------------------------------------------------------------------------------
// Cache policy bits of the epilogue's state loads and result / state stores (2 = non-temporal).
// Non-temporal stores: +1.6% on 100 x 25.6 M mean, +1.2% AVGM, +-0.1% Adagrad 100 x 86.6 M (5
// interleaved passes each, tools/gpu_epi_aux2.sh, profiles/r02/tune_epiaux/); non-temporal state
// loads were mixed (-1..-5% Adagrad) and stay cached.
#ifndef FA_EPI_LOAD_AUX
#define FA_EPI_LOAD_AUX 0
#endif
#ifndef FA_EPI_STORE_AUX
#define FA_EPI_STORE_AUX 2
#endif
// 8-byte elements (v_t / theta state in f64, the f64 result) are stored as two 16-B halves per
// quad, each instruction covering every other 16 B of a wave's 2 KiB: partial 128-B lines.
#ifndef FA_EPI_STORE64_AUX
#define FA_EPI_STORE64_AUX FA_EPI_STORE_AUX
#endif
template <typename T>
__device__ __forceinline__ typename vec4<T>::type buf_load_tquad(__amdgpu_buffer_rsrc_t r, int q) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(typename vec4<T>::type, __builtin_amdgcn_raw_buffer_load_b128(r, q * 16, 0, FA_EPI_LOAD_AUX));
  } else {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 lo = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, q * 32, 0, FA_EPI_LOAD_AUX));
    const d2 hi = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, q * 32 + 16, 0, FA_EPI_LOAD_AUX));
    return typename vec4<T>::type{lo[0], lo[1], hi[0], hi[1]};
  }
}

// XL (whole-line f64 stores): the wave's 64 consecutive f64 quads (2 KiB) are regrouped through
// LDS so that each of the two store instructions writes 1 KiB contiguous (eight whole 128-B
// lines) instead of every other 16 B of the 2 KiB (DESIGN.md §4 finding 22).  Callers run it
// wave-convergent with q = (the wave's first quad) + lane (finish_piece's slots).  The product
// enables it where it does not make the kernel spill (rowmajor_group); FA_EPI_STORE64_LDS=1
// forces it everywhere (tuning builds).
#ifndef FA_EPI_STORE64_LDS
#define FA_EPI_STORE64_LDS 0
#endif
template <typename T, bool XL = false>
__device__ __forceinline__ void buf_store_tquad(__amdgpu_buffer_rsrc_t r, int q, typename vec4<T>::type v) {
  if constexpr (sizeof(T) == 4) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, q * 16, 0, FA_EPI_STORE_AUX);
  } else if constexpr (XL || FA_EPI_STORE64_LDS != 0) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    __shared__ d2 xch[8][128];  // 2 KiB per wave, up to 8 waves per block
    // the thread index made opaque HERE: otherwise the lane-dependent LDS and store addresses
    // are hoisted out of the group sweep and held in VGPRs through it (KG = 4: the sweep is at
    // 256 + 256 registers already, and those few more spilled it to scratch)
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    d2* s = xch[tid >> 6];
    s[2 * lane] = d2{v[0], v[1]};
    s[2 * lane + 1] = d2{v[2], v[3]};
    // lane l reads what lanes l/2 and 32 + l/2 wrote: a cross-lane dependency the compiler does
    // not see, so pin the order (one wave's LDS operations complete in order)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
    const d2 a = s[lane], b = s[64 + lane];
    const int base = (q - lane) * 32;  // the wave's first byte
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), r, base + lane * 16, 0, FA_EPI_STORE64_AUX);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), r, base + 1024 + lane * 16, 0,
                                           FA_EPI_STORE64_AUX);
    __builtin_amdgcn_wave_barrier();  // the next slot's writes come after these reads
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  } else {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), r, q * 32, 0, FA_EPI_STORE64_AUX);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), r, q * 32 + 16, 0, FA_EPI_STORE64_AUX);
  }
}

template <typename E>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t col_rsrc(E* base, int64_t qbase, int cols) {
  // a null array (no out32 / out64) gets an empty range: every access is dropped.  Scalar
  // arithmetic only (a select between two descriptors is lowered to VGPRs, and every access
  // through a VGPR descriptor becomes a readfirstlane loop)
  // through readfirstlane: the Epi fields may have been reloaded from the private copy the kernel
  // makes for the noinline ragged path, and the compiler then cannot prove them wave-uniform
  const uint64_t a = (uint64_t)(uintptr_t)base + (uint64_t)(qbase * 4 * (int64_t)sizeof(E));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane(base ? cols * (int)sizeof(E) : 0);
  return row_rsrc(reinterpret_cast<const void*>((uintptr_t)(((uint64_t)hi << 32) | lo)), n);
}

// The four descriptors of one piece's epilogue (state operands, results); a null array or, for
// the plain mean, the state gets an empty range.
template <typename T, int OP>
struct EpiRsrc {
  __amdgpu_buffer_rsrc_t rl, rv, rvo, r32, r64;
  __device__ __forceinline__ EpiRsrc(const Epi<T>& e, int64_t qbase, int cols)
      : rl(col_rsrc<const float>(OP == FA_OP_DYN ? e.h : e.prev, qbase, OP == FA_OP_MEAN ? 0 : cols)),
        rv(col_rsrc<T>(e.v, qbase, OP == FA_OP_MEAN ? 0 : cols)),
        rvo(col_rsrc<T>(e.v_out ? e.v_out : e.v, qbase, OP == FA_OP_MEAN ? 0 : cols)),
        r32(col_rsrc<float>(e.out32, qbase, cols)),
        r64(col_rsrc<double>(e.out64, qbase, cols)) {}
};

// state operands of quad q (zeros for the plain mean, which has none)
template <typename T, int OP>
__device__ __forceinline__ void epi_load(const EpiRsrc<T, OP>& r, int q, typename vec4<float>::type& l,
                                         typename vec4<T>::type& vv) {
  if constexpr (OP != FA_OP_MEAN) {
    l = buf_load_tquad<float>(r.rl, q);
    vv = buf_load_tquad<T>(r.rv, q);
  } else {
    l = typename vec4<float>::type{0.f, 0.f, 0.f, 0.f};
    vv = typename vec4<T>::type{T(0), T(0), T(0), T(0)};
  }
}

// divide and update one quad: a = its sums, l / vv = its loaded state in, updated state out (l:
// FedDyn's h), w = the new global values
template <typename T, int OP, typename A>
__device__ __forceinline__ void epi_compute(const Epi<T>& e, const typename vec4<A>::type a,
                                            typename vec4<float>::type& l, typename vec4<T>::type& vv,
                                            typename vec4<T>::type& w) {
  if constexpr (OP == FA_OP_DYN) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const T g = (T)a[j] / e.denom;
      const T d = g * e.n - vv[j];                  // delta_theta = w_glob*N - theta   dyn.py:20-21
      const float hn = (float)((T)l[j] - e.c * d);  // h -= alpha/N * delta (fp32 h)    dyn.py:26
      const float ah = e.alpha32 * hn;              // alpha * h stays fp32              dyn.py:33
      w[j] = g - (T)ah;                             // w_glob - alpha*h                  dyn.py:33
      l[j] = hn;
      vv[j] = w[j];                                 // theta = w_glob                    dyn.py:34
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const T g = (T)a[j] / e.denom;  // np.divide(w_glob, np.sum(a))  strategy.py:127-129
      T vj = vv[j];
      w[j] = update<T, OP>(e, g, (T)l[j], vj);
      vv[j] = vj;
    }
  }
}

// store quad q's updated state and results.  GUARD = false: the result stores are issued
// unconditionally (a null out32 / out64 has an empty descriptor range, so they are dropped) and
// the quad is one basic block.
template <typename T, int OP, bool GUARD = true, bool XL = false>
__device__ __forceinline__ void epi_store(const Epi<T>& e, const EpiRsrc<T, OP>& r, int q,
                                          const typename vec4<float>::type l, const typename vec4<T>::type vv,
                                          const typename vec4<T>::type w) {
  if constexpr (OP == FA_OP_DYN) buf_store_tquad<float>(r.rl, q, l);
  if constexpr (OP != FA_OP_MEAN) buf_store_tquad<T, XL>(r.rvo, q, vv);
  if (!GUARD || e.out32) buf_store_tquad<float>(r.r32, q, typename vec4<float>::type{(float)w[0], (float)w[1], (float)w[2], (float)w[3]});
  if (!GUARD || e.out64) buf_store_tquad<double, XL>(r.r64, q, typename vec4<double>::type{(double)w[0], (double)w[1], (double)w[2], (double)w[3]});
}

template <typename T, int OP, typename A, bool GUARD = true, bool XL = false>
__device__ __forceinline__ void epi_quad(const Epi<T>& e, const EpiRsrc<T, OP>& r, int q,
                                         const typename vec4<A>::type a, typename vec4<float>::type l,
                                         typename vec4<T>::type vv) {
  typename vec4<T>::type w;
  epi_compute<T, OP, A>(e, a, l, vv, w);
  epi_store<T, OP, GUARD, XL>(e, r, q, l, vv, w);
}

template <typename T, int OP, typename A, int V, int STEP, int B, bool XL = false>
__device__ __forceinline__ void finish_piece(const Epi<T>& e, int64_t qbase, int cols,
                                             const typename vec4<A>::type (&acc)[V]) {
  static_assert(V % B == 0, "batch must divide the slots");
  if (cols <= 0) return;
  const EpiRsrc<T, OP> r(e, qbase, cols);
#pragma unroll
  for (int b0 = 0; b0 < V; b0 += B) {
    typename vec4<float>::type l[B];
    typename vec4<T>::type vv[B];
#pragma unroll
    for (int b = 0; b < B; ++b) epi_load<T, OP>(r, (int)threadIdx.x + (b0 + b) * STEP, l[b], vv[b]);
#pragma unroll
    for (int b = 0; b < B; ++b)
      epi_quad<T, OP, A, true, XL>(e, r, (int)threadIdx.x + (b0 + b) * STEP, acc[b0 + b], l[b], vv[b]);
  }
}

template <class P, typename T, int OP, int V, int U, bool NT>
__device__ __forceinline__ void reduce_subtile_buf(const float* __restrict__ base, int64_t stride,
                                                   int n, const typename P::w_t* __restrict__ w,
                                                   int64_t qt, int nvalid_quads, const Epi<T>& e) {
  typedef typename P::acc_t A;
  typedef typename vec4<float>::type XV;
  typedef typename vec4<A>::type AV;
  const char* tile0 = reinterpret_cast<const char*>(base + qt * 4);
  const uint32_t bytes = (uint32_t)nvalid_quads * 16u;
  const int64_t row_bytes = stride * 4;
  const int voff = (int)threadIdx.x * 16;
  AV acc[V];
  {
    const __amdgpu_buffer_rsrc_t r = row_rsrc(tile0, bytes);
    const typename P::w_t w0 = w[0];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const XV x = buf_load_quad<NT>(r, voff, v * kThreads * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[v][j] = P::mul(w0, x[j]);
    }
  }
  int i = 1;
  for (; i + U <= n; i += U) {
    XV x[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const __amdgpu_buffer_rsrc_t r = row_rsrc(tile0 + (int64_t)(i + u) * row_bytes, bytes);
#pragma unroll
      for (int v = 0; v < V; ++v) x[u][v] = buf_load_quad<NT>(r, voff, v * kThreads * 16);
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
    const __amdgpu_buffer_rsrc_t r = row_rsrc(tile0 + (int64_t)i * row_bytes, bytes);
    const typename P::w_t wi = w[i];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const XV x = buf_load_quad<NT>(r, voff, v * kThreads * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[v][j] = add<A>(acc[v][j], P::mul(wi, x[j]));
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v)
    if (v * kThreads + (int)threadIdx.x < nvalid_quads)
      finish_quad<T, OP, A>(e, (qt + (int64_t)v * kThreads + threadIdx.x) * 4, 4, acc[v]);
}

// The window's ragged end (at most one wave per launch): one quad at a time, element-guarded.
template <class P, typename T, int OP>
__device__ __attribute__((noinline)) void reduce_ragged(const typename P::x_t* __restrict__ base,
                                                        int64_t stride, int n,
                                                        const typename P::w_t* __restrict__ w,
                                                        int64_t q0, int64_t qlim, int64_t ncols,
                                                        const Epi<T>& e) {
  typedef typename P::x_t X;
  typedef typename vec4<typename P::acc_t>::type AV;
#pragma unroll 1
  for (int64_t q = q0; q < qlim; q += kThreads) {
    const int64_t c = q * 4;
    const int valid = (int)((ncols - c) < 4 ? (ncols - c) : 4);
    AV acc;
    {
      const typename vec4<X>::type x = load_quad_guarded(base + c, valid);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = P::mul(w[0], x[j]);
    }
#pragma unroll 1
    for (int i = 1; i < n; ++i) {
      const typename vec4<X>::type x = load_quad_guarded(base + (int64_t)i * stride + c, valid);
      const typename P::w_t wi = w[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = add<typename P::acc_t>(acc[j], P::mul(wi, x[j]));
    }
    finish_quad<T, OP, typename P::acc_t>(e, c, valid, acc);
  }
}

// Sub-tile starting at quad qt, limited to quads < qlim (the block's range, <= the window).
template <class P, typename T, int OP, int V, int U, bool NT, bool BUF = false>
__device__ __forceinline__ void reduce_range_subtile(const typename P::x_t* __restrict__ base,
                                                     int64_t stride, int n,
                                                     const typename P::w_t* __restrict__ w,
                                                     int64_t qt, int64_t qlim, int64_t ncols,
                                                     const Epi<T>& e) {
  constexpr int kSub = kThreads * V;
  const int64_t q0 = qt + threadIdx.x;
  const int64_t qfull = ncols / 4;  // complete quads in the window
  if constexpr (BUF) {
    static_assert(sizeof(typename P::x_t) == 4, "buffer path is for 4-byte elements");
    const int64_t end = qt + kSub < qlim ? qt + kSub : qlim;  // this sub-tile's quads [qt, end)
    const int64_t full_end = end < qfull ? end : qfull;
    if (full_end > qt) reduce_subtile_buf<P, T, OP, V, U, NT>(base, stride, n, w, qt, (int)(full_end - qt), e);
    // the window's ragged last quad (ncols % 4 != 0), if it falls in this sub-tile
    if (qfull < end && qfull >= qt && q0 == qt + (qfull - qt) % kThreads)
      reduce_ragged<P, T, OP>(base, stride, n, w, qfull, qfull + 1, ncols, e);
    return;
  }
  if (qt + kSub <= qlim && qt + kSub <= qfull) {
    reduce_subtile<P, T, OP, V, U, NT, kFull>(base, stride, n, w, q0, V, e);
    return;
  }
  // slot v of wave wv covers quads [qt + v*kThreads + 64*wv, +64): count the complete ones
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x) / 64;
  const int64_t wbase = qt + 64 * wv;
  const int64_t lim = qlim < qfull ? qlim : qfull;
  int nv = 0;
  while (nv < V && wbase + (int64_t)nv * kThreads + 64 <= lim) ++nv;
  if (nv > 0) reduce_subtile<P, T, OP, V, U, NT, kMasked>(base, stride, n, w, q0, nv, e);
  // the rest of this wave's slots (only at the window's ragged end: lim < qlim)
  const int64_t qr = q0 + (int64_t)nv * kThreads;
  if (qr < qlim) reduce_ragged<P, T, OP>(base, stride, n, w, qr, qlim, ncols, e);
}

// Balanced grid.  Work unit: a CHUNK of 64 quads (1 KiB of one fp32 row = one wave-wide dwordx4
// instruction).  The host sizes the grid as k full waves of resident blocks (k = rounds) so that
// every block owns an equal share +-1 chunk of the window, preferably <= one sub-tile: all
// blocks of a round finish together (no tail of late blocks) and, because neighbouring blocks own
// neighbouring column ranges and sweep the rows in lockstep, the chip streams each client row
// almost sequentially — the access pattern of a plain linear read.
template <class P, typename T, int OP, int V, int U, bool NT, bool BUF = false>
__global__ __launch_bounds__(kThreads) void reduce_kernel_balanced(
    const typename P::x_t* __restrict__ stack, int64_t stride, int n,
    const typename P::w_t* __restrict__ w, int64_t col0, int64_t ncols, Epi<T> e) {
  const int64_t nquads = (ncols + 3) / 4;
  const int64_t nchunks = (nquads + 63) / 64;
  const int64_t b = blockIdx.x, g = gridDim.x;
  const int64_t per = nchunks / g, extra = nchunks % g;
  const int64_t c0 = b * per + (b < extra ? b : extra);
  const int64_t c1 = c0 + per + (b < extra ? 1 : 0);
  const int64_t qlim = c1 * 64 < nquads ? c1 * 64 : nquads;
  const typename P::x_t* base = stack + col0;
  for (int64_t qt = c0 * 64; qt < qlim; qt += kThreads * V)
    reduce_range_subtile<P, T, OP, V, U, NT, BUF>(base, stride, n, w, qt, qlim, ncols, e);
}

// One sub-tile per block (grid = number of sub-tiles): the simple mapping.
template <class P, typename T, int OP, int V, int U, bool NT, bool BUF = false>
__global__ __launch_bounds__(kThreads) void reduce_kernel(
    const typename P::x_t* __restrict__ stack, int64_t stride, int n,
    const typename P::w_t* __restrict__ w, int64_t col0, int64_t ncols, Epi<T> e) {
  const int64_t qt = (int64_t)blockIdx.x * (kThreads * V);
  const int64_t nquads = (ncols + 3) / 4;
  reduce_range_subtile<P, T, OP, V, U, NT, BUF>(stack + col0, stride, n, w, qt,
                                           qt + kThreads * V < nquads ? qt + kThreads * V : nquads,
                                           ncols, e);
}

// acc + w*x on whole quads, written as <4 x T> IR operations: per-element scalar code gets packed
// by the SLP vectorizer, which re-places the packed products after the pipeline's scheduling
// barriers.  Elementwise identical to P::mul / add (no contraction under -ffp-contract=off).
template <class P>
__device__ __forceinline__ typename vec4<typename P::acc_t>::type quad_axpy(
    typename vec4<typename P::acc_t>::type acc, typename P::w_t w, typename vec4<float>::type x) {
  typedef typename vec4<typename P::acc_t>::type AV;
  if constexpr (sizeof(typename P::acc_t) == 4)
    return acc + w * x;
  else
    return acc + (AV)(typename P::acc_t)w * __builtin_convertvector(x, AV);
}
template <class P>
__device__ __forceinline__ typename vec4<typename P::acc_t>::type quad_mul(
    typename P::w_t w, typename vec4<float>::type x) {
  typedef typename vec4<typename P::acc_t>::type AV;
  if constexpr (sizeof(typename P::acc_t) == 4)
    return w * x;
  else
    return (AV)(typename P::acc_t)w * __builtin_convertvector(x, AV);
}

// Row addressing of the pipeline: a contiguous client stack (row i at tile0 + i*row_bytes), or a
// table of per-client device pointers (row i at ptr[i] + off: uploads read where they lie).
struct StackRows {
  const char* tile0;
  int64_t row_bytes;
  __device__ __forceinline__ const char* operator()(int i) const { return tile0 + (int64_t)i * row_bytes; }
};
struct PtrRows {
  const float* const* __restrict__ ptr;  // wave-uniform index: scalar loads
  int64_t off_bytes;
  __device__ __forceinline__ const char* operator()(int i) const {
    return reinterpret_cast<const char*>(ptr[i]) + off_bytes;
  }
};

// The rolling register pipeline over rows 0..n-1 of one piece (nq full quads, `bytes` = nq*16
// per row; lane l owns quads l, l+64W, ...): acc[v] = sum_i w[i]*x[i] in list order.
template <class P, int V, int D, int W, bool NT, class R>
__device__ __forceinline__ void rows_sweep(const R& row, uint32_t bytes, int n,
                                           const typename P::w_t* __restrict__ w,
                                           typename vec4<typename P::acc_t>::type (&acc)[V],
                                           int voff = (int)threadIdx.x * 16) {
  typedef typename vec4<float>::type XV;
  XV x[D][V];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (1 + d < n) {
      const __amdgpu_buffer_rsrc_t r = row_rsrc(row(1 + d), bytes);
#pragma unroll
      for (int v = 0; v < V; ++v) x[d][v] = buf_load_quad<NT>(r, voff + v * 64 * W * 16, 0);
    }
  {
    const __amdgpu_buffer_rsrc_t r = row_rsrc(row(0), bytes);
    const typename P::w_t w0 = w[0];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = quad_mul<P>(w0, buf_load_quad<NT>(r, voff + v * 64 * W * 16, 0));
  }
  // rows 1..n-1: slot d holds row i+d; consume it, refill it with row i+d+D (steady state:
  // every refill is a real row, so no branch)
  int i = 1;
  for (; i + 2 * D <= n; i += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const typename P::w_t wi = w[i + d];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = quad_axpy<P>(acc[v], wi, x[d][v]);
      // pin the order "consume slot d, then refill it": if the scheduler hoists the refill
      // (or the products of later slots) the old values need copies, and the copies wait for
      // every in-flight row — the pipeline collapses into batches
      __builtin_amdgcn_sched_barrier(0);
      const __amdgpu_buffer_rsrc_t r = row_rsrc(row(i + d + D), bytes);
#pragma unroll
      for (int v = 0; v < V; ++v) x[d][v] = buf_load_quad<NT>(r, voff + v * 64 * W * 16, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // drain: fewer than 2*D rows left (wave-uniform branches)
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (i + d < n) {
      const typename P::w_t wi = w[i + d];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = quad_axpy<P>(acc[v], wi, x[d][v]);
      if (i + d + D < n) {
        const __amdgpu_buffer_rsrc_t r = row_rsrc(row(i + d + D), bytes);
#pragma unroll
        for (int v = 0; v < V; ++v) x[d][v] = buf_load_quad<NT>(r, voff + v * 64 * W * 16, 0);
      }
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (i + D + d < n) {
      const typename P::w_t wi = w[i + D + d];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = quad_axpy<P>(acc[v], wi, x[d][v]);
    }
  }
}

// Row-pipelined grid.  Built for deep, narrow windows (many clients, few columns: the per-rank
// column shards of a multi-GPU aggregation, e.g. 800 clients x 365 K columns), where the
// sub-tile kernels run out of column parallelism and a batch of rows that is issued, drained
// and re-issued keeps only half its bytes in flight on average.  Here:
//   * a block is W waves; lane l owns quads l, l+64W, ..., l+(V-1)*64W of the block's piece of
//     every row (V*W KiB contiguous per row), so each wave instruction reads 1 KiB of one row;
//   * rows are a rolling register pipeline D rows deep (rows_sweep): row i+D is loaded right
//     after row i is consumed, so D*V loads stay in flight per lane for the whole sweep
//     (s_waitcnt vmcnt((D-1)*V) in the steady state, no drain per batch);
//   * loads go through per-row buffer descriptors whose range check covers the window's end, so
//     a partial last piece needs no per-lane branches (the slot offset rides in voffset, which
//     the range check always covers) and the window's ragged last quad (ncols % 4) is read in
//     the same instructions (the range check is per dword).
// The summation order (client list order, first product initialises the sum) is unchanged.
template <class P, typename T, int OP, int V, int D, int W, bool NT>
__device__ __forceinline__ void rows_piece(const float* __restrict__ stack, int64_t stride, int n,
                                           const typename P::w_t* __restrict__ w, int64_t col0,
                                           int64_t ncols, const Epi<T>& e, int64_t qb,
                                           int64_t qend) {
  // the piece is quads [qb, qend), qend - qb <= 64*W*V; its columns, the window's ragged last
  // quad (ncols % 4 != 0) included: the raw-buffer range check is per dword on gfx950
  // (tools/probe_oob.py), so the missing elements of that quad load as 0 and are never stored
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  const int64_t cend = qend * 4 < ncols ? qend * 4 : ncols;
  const int cols = cend > qb * 4 ? (int)(cend - qb * 4) : 0;
  if (cols > 0) {
    AV acc[V];
    rows_sweep<P, V, D, W, NT>(StackRows{reinterpret_cast<const char*>(stack + col0 + qb * 4), stride * 4},
                               (uint32_t)cols * 4u, n, w, acc);
    finish_piece<T, OP, A, V, 64 * W, (V >= 2 ? 2 : V)>(e, qb, cols, acc);
  }
}

// Segmented row-pointer reduce (fa_reduce_f32_rows): uploads that are separate device tensors
// per (client, key) are read where they lie — no pack copy.  Work = pieces (fa_rows_plan): each
// is a column range of ONE segment, so every row of a piece is one contiguous range of one
// tensor and gets one buffer descriptor; client order and epilogue are the row pipeline's.
//   * scheduling: pieces come largest first; block b starts with piece b and then claims the
//     next unclaimed one from a device counter.  Blocks finish within about one small piece of
//     each other whatever the mix of tensor sizes — a static split of 100 ResNet-sized uploads
//     left a ~10% tail (tools/tune_rows.py);
//   * narrow pieces (<= W KiB of a row: BN vectors, biases) are latency-bound, not
//     bandwidth-bound: they take a one-quad-per-lane sweep V*D rows deep instead of D, so a
//     64-element tensor of 100 clients costs ~7 HBM round trips instead of ~50.
// The counter must be 0 at launch (the host clears it on the stream before each launch).
template <class P, typename T, int OP, int V, int D, int W, bool NT>
__global__ __launch_bounds__(64 * W) void reduce_kernel_segrows(const float* const* __restrict__ rows, int n,
                                                                const typename P::w_t* __restrict__ w,
                                                                const fa_piece* __restrict__ pieces,
                                                                int64_t npieces, int* __restrict__ next, Epi<T> e) {
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  __shared__ int s_next;
  int64_t p = blockIdx.x;
  while (p < npieces) {
    int claimed = 0;
    if (threadIdx.x == 0) claimed = (int)gridDim.x + atomicAdd(next, 1);
    const fa_piece pc = pieces[p];
    const float* const* rp = rows + (int64_t)pc.seg * n;
    // a segment's ragged last quad rides in the vector path: the range check is per dword
    // (`bytes` = exactly the piece's columns), its missing elements load as 0 and are not stored
    const int nq = (pc.n_cols + 3) >> 2;
    const uint32_t bytes = (uint32_t)pc.n_cols * 4u;
    const PtrRows row{rp, pc.seg_off * 4};
    if (nq > 64 * W) {
      AV acc[V];
      rows_sweep<P, V, D, W, NT>(row, bytes, n, w, acc);
      finish_piece<T, OP, A, V, 64 * W, (V >= 2 ? 2 : V)>(e, pc.col / 4, pc.n_cols, acc);
    } else if (nq > 0) {
      AV acc[1];
      rows_sweep<P, 1, V * D, W, NT>(row, bytes, n, w, acc);
      finish_piece<T, OP, A, 1, 64 * W, 1>(e, pc.col / 4, pc.n_cols, acc);
    }
    if (threadIdx.x == 0) s_next = claimed;
    __syncthreads();
    p = s_next;
    __syncthreads();  // s_next is rewritten in the next iteration
  }
}

// Split-N reduce (fa_reduce_f32_splitn) for windows too narrow to fill the chip with one
// sequential sweep per column (LeNet5-sized models of many clients: 44 K columns x 1000 rows is
// 174 one-KiB row chunks for 256 CUs, each walking 1000 rows).  Here the CLIENTS are split too:
//   * a block owns one 1-KiB chunk of the window (64 quads) and W client splits: wave v sums the
//     contiguous rows [v*n/W, (v+1)*n/W) in list order (the split's first product initialises its
//     sum) through the row pipeline (rows_sweep, D rows in flight; the split index is made
//     wave-uniform with readfirstlane so every row keeps ONE scalar buffer descriptor);
//   * the W partial sums of a quad are staged in LDS and combined by a FIXED binary tree in
//     split order, ((p0+p1)+(p2+p3))+..., one barrier per level;
//   * then the epilogue of the row pipeline (divide, optional optimizer update, stores).
// Deterministic (the tree does not depend on scheduling) but NOT the reference's sequential
// order: opt-in, checked at <= 1e-6 normwise relative error per tensor (tests/test_gpu_splitn.py)
// — except columns whose terms nearly cancel (sum of |products| > 2 |sum|, or a non-finite
// sum): those are re-summed in list order by wave 0 (the cancellation guard below), bit-exact.
// oracle.c_reduce_splitn restates this exact order and guard (the tests pin it bit for bit).
// Needs n >= W (every split non-empty; the host falls back to the sequential kernel otherwise).
template <class P, typename T, int OP, int W, int D, bool NT, bool STRIDED = false>
__global__ __launch_bounds__(64 * W) void reduce_kernel_splitn(const float* __restrict__ stack, int64_t stride, int n,
                                                               const typename P::w_t* __restrict__ w, int64_t col0,
                                                               int64_t ncols, Epi<T> e) {
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  __shared__ AV part[W][64];
  __shared__ AV apart[W][64];  // the splits' sums of |product|: the cancellation guard
  const int lane = (int)threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);  // the split: wave-uniform
  // the chunk's columns, its last quad possibly partial: the raw buffer range check is per dword
  // on gfx950 (tools/probe_oob.py, profiles/r02/oob.json), so `bytes` = exactly the chunk's
  // columns and the missing elements of a ragged last quad load as 0 and are never stored
  const int64_t qb = (int64_t)blockIdx.x * 64;  // first quad of the chunk
  const int64_t cleft = ncols - qb * 4;
  const int tcols = cleft <= 0 ? 0 : (cleft < 256 ? (int)cleft : 256);
  const int nq = (tcols + 3) / 4;  // quads, the last possibly partial
  // split wv: contiguous rows [r0, r1), or (STRIDED) rows wv, wv+W, wv+2W, ... so that all
  // splits read neighbouring rows at the same time
  const int r0 = STRIDED ? wv : (int)((int64_t)wv * n / W);
  const int r1 = STRIDED ? n : (int)((int64_t)(wv + 1) * n / W);
  constexpr int RS = STRIDED ? W : 1;  // row step of a split
  typedef typename vec4<float>::type XV;
  const char* tile00 = reinterpret_cast<const char*>(stack + col0 + qb * 4);
  const uint32_t bytes = (uint32_t)tcols * 4u;
  const int voff = lane * 16;
  AV acc = {A(0), A(0), A(0), A(0)}, aacc = {A(0), A(0), A(0), A(0)};
  auto absq = [](AV v) { return AV{v[0] < A(0) ? -v[0] : v[0], v[1] < A(0) ? -v[1] : v[1],
                                   v[2] < A(0) ? -v[2] : v[2], v[3] < A(0) ? -v[3] : v[3]}; };
  if (nq > 0) {
    // this split's rows through a D-deep rolling pipeline with NO guarded loads: a slot past the
    // split's end re-reads its last row (a cache hit) and the product is discarded by a select,
    // so the loads stay unconditional and the ramp is not serialised by waitcnt merges.  Each
    // product p = fl(w*x) feeds the running sum (acc + p: the same rounding as acc + w*x, no
    // contraction) and the running sum of |p|
    const char* tile0 = tile00 + (int64_t)r0 * stride * 4;
    const int64_t row_bytes = stride * 4 * RS;
    const int cnt = (r1 - r0 + RS - 1) / RS;  // >= 1
    const typename P::w_t* ws = w + r0;
    XV x[D];
#pragma unroll
    for (int d = 0; d < D; ++d)
      x[d] = buf_load_quad<NT>(row_rsrc(tile0 + (int64_t)(d < cnt ? d : cnt - 1) * row_bytes, bytes), voff, 0);
    acc = quad_mul<P>(ws[0], x[0]);
    aacc = absq(acc);
    {
      const int r = D < cnt ? D : cnt - 1;
      x[0] = buf_load_quad<NT>(row_rsrc(tile0 + (int64_t)r * row_bytes, bytes), voff, 0);
    }
#pragma unroll
    for (int d = 1; d < D; ++d) {  // rows 1..D-1
      const AV p = quad_mul<P>(ws[(d < cnt ? d : 0) * RS], x[d]);
      acc = d < cnt ? acc + p : acc;
      aacc = d < cnt ? aacc + absq(p) : aacc;
      __builtin_amdgcn_sched_barrier(0);
      const int r = d + D < cnt ? d + D : cnt - 1;
      x[d] = buf_load_quad<NT>(row_rsrc(tile0 + (int64_t)r * row_bytes, bytes), voff, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int base = D; base < cnt; base += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int i = base + d;
        const AV p = quad_mul<P>(ws[(i < cnt ? i : 0) * RS], x[d]);
        acc = i < cnt ? acc + p : acc;
        aacc = i < cnt ? aacc + absq(p) : aacc;
        __builtin_amdgcn_sched_barrier(0);
        const int r = i + D < cnt ? i + D : cnt - 1;
        x[d] = buf_load_quad<NT>(row_rsrc(tile0 + (int64_t)r * row_bytes, bytes), voff, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  part[wv][lane] = acc;
  apart[wv][lane] = aacc;
  __syncthreads();
#pragma unroll
  for (int h = 1; h < W; h *= 2) {  // fixed tree over the splits, one level per barrier
    if ((wv % (2 * h)) == 0 && wv + h < W) {
      part[wv][lane] = part[wv][lane] + part[wv + h][lane];
      apart[wv][lane] = apart[wv][lane] + apart[wv + h][lane];
    }
    __syncthreads();
  }
  if (wv == 0) {
    // cancellation guard: a column whose sum is not at least half its sum of |products|
    // (!(S_abs <= 2|S|): also NaN / inf) takes the reference's sequential sum instead — a
    // reordered sum of nearly cancelling terms can lie arbitrarily far (relatively) from the
    // sequential one; every other column is within the reordering's rounding error of it
    AV r = part[0][lane];
    const AV aa = apart[0][lane];
    bool flag[4], any = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const A ab = r[k] < A(0) ? -r[k] : r[k];
      flag[k] = !(aa[k] <= A(2) * ab) || !(ab <= A(3.0e38));
      any |= flag[k];
    }
    if (__builtin_amdgcn_ballot_w64(any && lane < nq) != 0) {  // (wave-uniform)
      AV seq[1];
      rows_sweep<P, 1, 16, 1, NT>(StackRows{tile00, stride * 4}, bytes, n, w, seq);
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = flag[k] ? seq[0][k] : r[k];
    }
    const AV rr[1] = {r};
    finish_piece<T, OP, A, 1, 64, 1>(e, qb, tcols, rr);
  }
}

// Row-major form of the row-pointer reduce.  A claim is a GROUP of KG wide pieces (the leading
// pieces[0].aux entries of the largest-first table) swept together row by row — step (row i,
// piece j), j fastest, one step (V*W KiB) in flight, like reduce_kernel_rowmajor — so the blocks
// stay on neighbouring client rows as the stack kernel's do; the row pointer of the step after
// the next one is fetched while the next is in flight (every index is static: j is unrolled).
// Claims past the groups are the narrow pieces, one at a time, through the deep one-quad sweep.
// TR (tools/tune_rows.hip): wave 0 of every block stamps the 100-MHz wall clock at each claim it
// starts (e.trace[block * 32 + 1 + c], c < 30) and at its exit (slot 0), claim count in slot 31.
// DS: steps in flight (1, or any divisor of KG: step s = (i, j) lives in slot j % DS).
// PFA > 0 (tuning, tools/tune_rows.hip): translation prefetch — after each refill every wave also
// loads ONE dword (all lanes the same address) of the step PFA steps past the next one, so the
// page translation of that upload row is resolved before its 64-KiB step is issued (the
// row-pointer kernel takes 2.4x the UTCL1 translation misses of the stack kernel on per-tensor
// allocations: profiles/r04/rows_pmc/).  The dword is consumed one row later (xor into a sink
// kept alive by an empty asm), when it has long arrived.
// LT > 0 (n <= LT clients, the host's choice): the group's KG x n row pointers are copied into LDS
// at its claim (one coalesced vector load per wave, one barrier) and every step's pointer comes
// from there (a ds_read, made wave-uniform with readfirstlane) instead of a scalar load from the
// rows table in L2: 8 waves x 2 pointer loads per step, each a scalar-cache miss on a table of
// S x N pointers, left the waves waiting on SMEM before their vector loads (SQ_INSTS_SMEM 9.2x,
// SQ_WAIT_INST_ANY 3-4x the stack kernel's: profiles/r04/rows_pmc/).
template <int LT>
__device__ __forceinline__ const float* srm_row_ptr(const float* const* lds_row, const float* const* g_row, int i) {
  if constexpr (LT > 0) {
    const uint64_t p = reinterpret_cast<uint64_t>(lds_row[i]);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
  } else {
    return g_row[i];
  }
}

// XLS: the epilogue's f64 stores as whole cache lines (buf_store_tquad XL, 2 KiB of LDS per wave),
// as rowmajor_group does for fused epilogues at KG <= 3 (DESIGN.md §4 finding 22).
template <class P, typename T, int OP, int V, int W, int KG, int DN, bool NT, bool TR = false, int DS = 1,
          bool SG = false, int PFA = 0, int LT = 0, bool XLS = false>
__global__ __launch_bounds__(64 * W) void reduce_kernel_segrows_rm(const float* const* __restrict__ rows, int n,
                                                                   const typename P::w_t* __restrict__ w,
                                                                   const fa_piece* __restrict__ pieces,
                                                                   int64_t npieces, int* __restrict__ next, Epi<T> e) {
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  typedef typename vec4<float>::type XV;
  __shared__ int s_next;
  const int64_t nwide = npieces > 0 ? pieces[0].aux : 0;
  const int64_t groups = (nwide + KG - 1) / KG;
  const int64_t claims = groups + (npieces - nwide);
  const int voff = (int)threadIdx.x * 16;
  int64_t t = blockIdx.x;
  int nclaim = 0;
  // SG (static groups, tuning): block b takes groups b, b + grid, ... in lockstep and claims only
  // the narrow pieces, numbered from max(groups, grid)
  const int64_t nbase = SG && groups > (int64_t)gridDim.x ? groups : (int64_t)gridDim.x;
#define FA_SRM_CLAIM() \
  ((SG && t < groups && t + (int64_t)gridDim.x < groups) ? (int)(t + gridDim.x) : (int)nbase + atomicAdd(next, 1))
  while (t < claims) {
    // the next claim: a group (hundreds of us) claims during its last row, so an idle block can
    // take what is left meanwhile (claiming at the start reserved work behind a long group while
    // blocks that had drawn short pieces ran dry: tools/tune_rows.py --trace); a narrow piece
    // claims at its start, which hides the atomic behind its short sweep
    int claimed = 0;
    if (t >= groups && threadIdx.x == 0) claimed = FA_SRM_CLAIM();
    if constexpr (TR) {
      if (threadIdx.x == 0 && nclaim < 30) e.trace[blockIdx.x * 32 + 1 + nclaim] = wall_clock64();
      ++nclaim;
    }
    if (t < groups) {
      const float* const* rp[KG];
      int64_t ob[KG], col[KG];
      int cols[KG];
      uint32_t bytes[KG];
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        const int64_t pi = t * KG + j;
        const fa_piece pc = pi < nwide ? pieces[pi] : fa_piece{0, 0, 0, 0, 0};
        rp[j] = rows + (int64_t)pc.seg * n;  // a missing piece keeps segment 0's pointers, 0 bytes
        ob[j] = pc.seg_off * 4;
        col[j] = pc.col;
        cols[j] = pc.n_cols;
        bytes[j] = (uint32_t)pc.n_cols * 4u;
      }
      __shared__ const float* s_tab[KG][LT > 0 ? LT : 1];
      if constexpr (LT > 0) {  // the previous claim's readers are past the loop-end barriers
#pragma unroll
        for (int j = 0; j < KG; ++j)
          for (int k = (int)threadIdx.x; k < n; k += 64 * W) s_tab[j][k] = rp[j][k];
        __syncthreads();
      }
      // row pointer of step (i, j); rows clamped (a step past the end is never loaded)
#define FA_SRM_PTR(i, j) (reinterpret_cast<const char*>(srm_row_ptr<LT>(s_tab[j], rp[j], (i) < n ? (i) : n - 1)) + ob[j])
#define FA_SRM_LOAD(p, j, slot)                                                                              \
  {                                                                                                          \
    const __amdgpu_buffer_rsrc_t r_ = row_rsrc((p), bytes[j]);                                               \
    _Pragma("unroll") for (int v = 0; v < V; ++v) x[slot][v] = buf_load_quad<NT>(r_, voff + v * 64 * W * 16, 0); \
  }
      static_assert(KG % DS == 0, "steps in flight must divide the group");
      AV acc[KG][V];
      XV x[DS][V];
      uint32_t pf[KG > 0 ? KG : 1];
      uint32_t sink = 0;
#pragma unroll
      for (int j = 0; j < KG; ++j) pf[j] = 0;
#pragma unroll
      for (int d = 0; d < DS; ++d) FA_SRM_LOAD(FA_SRM_PTR(d / KG, d % KG), d % KG, d);
      const char* pn = FA_SRM_PTR(DS / KG, DS % KG);  // the pointer of the next step to load
      // after consuming step (i, j): refill its slot with step (i, j) + DS, then fetch the pointer
      // of the step after that one
#define FA_SRM_REFILL(i, j)                                                                          \
  __builtin_amdgcn_sched_barrier(0);                                                                 \
  if ((i) + ((j) + DS) / KG < n) {                                                                   \
    FA_SRM_LOAD(pn, ((j) + DS) % KG, (j) % DS);                                                      \
    pn = FA_SRM_PTR((i) + ((j) + DS + 1) / KG, ((j) + DS + 1) % KG);                                \
    if constexpr (PFA > 0) {                                                                         \
      sink ^= pf[j];                                                                                 \
      pf[j] = __builtin_amdgcn_raw_buffer_load_b32(                                                  \
          row_rsrc(FA_SRM_PTR((i) + ((j) + DS + 1 + PFA) / KG, ((j) + DS + 1 + PFA) % KG), 4u), 0, 0, 0); \
    }                                                                                                \
  }                                                                                                  \
  __builtin_amdgcn_sched_barrier(0);
      {  // row 0: the products initialise the sums (peeled: a select between the first product
         // and the running sum kept both alive for every slot and spilled KG >= 3)
        const typename P::w_t w0 = w[0];
        if (n == 1 && threadIdx.x == 0) claimed = FA_SRM_CLAIM();
#pragma unroll
        for (int j = 0; j < KG; ++j) {
#pragma unroll
          for (int v = 0; v < V; ++v) acc[j][v] = quad_mul<P>(w0, x[j % DS][v]);
          FA_SRM_REFILL(0, j)
        }
      }
      for (int i = 1; i < n; ++i) {
        if (i == n - 1 && threadIdx.x == 0) claimed = FA_SRM_CLAIM();
        const typename P::w_t wi = w[i];
#pragma unroll
        for (int j = 0; j < KG; ++j) {
#pragma unroll
          for (int v = 0; v < V; ++v) acc[j][v] = quad_axpy<P>(acc[j][v], wi, x[j % DS][v]);
          FA_SRM_REFILL(i, j)
        }
      }
#undef FA_SRM_REFILL
#undef FA_SRM_LOAD
#undef FA_SRM_PTR
      if constexpr (PFA > 0) {
#pragma unroll
        for (int j = 0; j < KG; ++j) sink ^= pf[j];
        asm volatile("" ::"v"(sink));
      }
#pragma unroll
      for (int j = 0; j < KG; ++j) finish_piece<T, OP, A, V, 64 * W, (V >= 2 ? 2 : V), XLS>(e, col[j] / 4, cols[j], acc[j]);
    } else {
      const fa_piece pc = pieces[nwide + (t - groups)];
      const float* const* rp = rows + (int64_t)pc.seg * n;
      const uint32_t bytes = (uint32_t)pc.n_cols * 4u;
      const PtrRows row{rp, pc.seg_off * 4};
      if (((pc.n_cols + 3) >> 2) > 64 * W) {  // a wide piece the groups did not take
        AV acc[V];
        rows_sweep<P, V, 1, W, NT>(row, bytes, n, w, acc);
        finish_piece<T, OP, A, V, 64 * W, (V >= 2 ? 2 : V), XLS>(e, pc.col / 4, pc.n_cols, acc);
      } else if (pc.n_cols > 0) {
        AV acc[1];
        rows_sweep<P, 1, DN, W, NT>(row, bytes, n, w, acc);
        finish_piece<T, OP, A, 1, 64 * W, 1, XLS>(e, pc.col / 4, pc.n_cols, acc);
      }
    }
    if (threadIdx.x == 0) s_next = claimed;
    __syncthreads();
    t = s_next;
    __syncthreads();
  }
#undef FA_SRM_CLAIM
  if constexpr (TR) {
    if (threadIdx.x == 0) {
      e.trace[blockIdx.x * 32] = wall_clock64();
      e.trace[blockIdx.x * 32 + 31] = (unsigned long long)nclaim;
    }
  }
}

// fa_gather_rows: block (s, i) copies client i's tensor of segment s into its stack row.
template <typename E>
__global__ __launch_bounds__(kThreads) void gather_rows_kernel(E* __restrict__ stack, int64_t stride, int n,
                                                               const E* const* __restrict__ rows,
                                                               const int64_t* __restrict__ segs, int nseg, int i0) {
  const int s = blockIdx.x, i = i0 + (int)blockIdx.y;  // i0: client tile (grid.y <= 65535)
  const int64_t col = segs[s], len = segs[nseg + s];
  const E* src = rows[(int64_t)s * n + i];
  E* dst = stack + (int64_t)i * stride + col;
  for (int64_t k = threadIdx.x; k < len; k += kThreads) dst[k] = src[k];
}

// fa_gather_rows_f64: the same into a float64 stack, segment s's source converted by kind
// (segs[2*nseg + s]: FA_SRC_F64 copy, FA_SRC_I64 int64 -> double rounded to nearest, FA_SRC_F32).
__global__ __launch_bounds__(kThreads) void gather_rows_f64_kernel(double* __restrict__ stack, int64_t stride, int n,
                                                                   const void* const* __restrict__ rows,
                                                                   const int64_t* __restrict__ segs, int nseg, int i0) {
  const int s = blockIdx.x, i = i0 + (int)blockIdx.y;
  const int64_t col = segs[s], len = segs[nseg + s], kind = segs[2 * nseg + s];
  const void* src = rows[(int64_t)s * n + i];
  double* dst = stack + (int64_t)i * stride + col;
  if (kind == FA_SRC_I64) {
    const int64_t* x = static_cast<const int64_t*>(src);
    for (int64_t k = threadIdx.x; k < len; k += kThreads) dst[k] = (double)x[k];
  } else if (kind == FA_SRC_F32) {
    const float* x = static_cast<const float*>(src);
    for (int64_t k = threadIdx.x; k < len; k += kThreads) dst[k] = (double)x[k];
  } else {
    const double* x = static_cast<const double*>(src);
    for (int64_t k = threadIdx.x; k < len; k += kThreads) dst[k] = x[k];
  }
}

// Work split: the window's 1-KiB chunks are cut into equal pieces of pc <= W*V chunks, as many
// as make k whole rounds of the grid (pc = ceil(chunks / (k * grid))), so every block sweeps k
// pieces (the last one or two blocks one fewer) and the launch has no tail round.
//   INTERLEAVE: block b takes pieces b, b+grid, b+2*grid, ...: at any moment the grid's pieces
//               form one contiguous stretch of each row (a linear-read access pattern);
//   otherwise:  block b takes k consecutive pieces (one contiguous share of the window).
template <class P, typename T, int OP, int V, int D, int W, bool NT, bool INTERLEAVE = true,
          bool XCDMAP = false>
__global__ __launch_bounds__(64 * W) void reduce_kernel_rows(const float* __restrict__ stack,
                                                             int64_t stride, int n,
                                                             const typename P::w_t* __restrict__ w,
                                                             int64_t col0, int64_t ncols, Epi<T> e) {
  static_assert(sizeof(typename P::x_t) == 4, "row pipeline is for 4-byte elements");
  const int64_t nquads = (ncols + 3) / 4;
  const int64_t chunks = (nquads + 63) / 64;
  const int64_t g = gridDim.x;
  const int64_t k = (chunks + g * W * V - 1) / (g * W * V);  // rounds
  const int64_t pc = (chunks + g * k - 1) / (g * k);         // chunks per piece (<= W*V)
  const int64_t pieces = (chunks + pc - 1) / pc;
  const int64_t step = INTERLEAVE ? g : 1;
  // XCDMAP (tuning): blocks b, b+8, b+16, ... share an XCD under round-robin placement; give
  // them consecutive piece slots so each XCD streams one contiguous stretch per round
  const int64_t slot = (XCDMAP && g % 8 == 0) ? (blockIdx.x % 8) * (g / 8) + blockIdx.x / 8 : blockIdx.x;
  const int64_t first = INTERLEAVE ? slot : slot * k;
  const int64_t last = INTERLEAVE ? pieces : (first + k < pieces ? first + k : pieces);
  for (int64_t p = first; p < last; p += step) {
    const int64_t qs = p * pc * 64;
    rows_piece<P, T, OP, V, D, W, NT>(stack, stride, n, w, col0, ncols, e, qs,
                                      qs + pc * 64 < nquads ? qs + pc * 64 : nquads);
  }
}

// Narrow windows, deep pipeline (at most two 1-KiB row chunks per block: LeNet-sized models, deep
// client stacks).  Block b owns chunks [b*W, b*W + W), one per wave, lane l one quad.  Only D rows
// per wave bound the bytes in flight here (a wave's vmcnt counts at most 63 loads), so D goes up
// to 60 and the pipeline has no drain code: the sweep runs whole D-row rounds; in the last two a
// refill past the last row re-loads row n-1 (an L2 hit) and a product past it is dropped by a
// select.  The row address
// advances by the stride through one running scalar pointer (opaque to the compiler: written as
// row(i + d) in the unrolled loop, every d * stride was kept in a scalar register pair and
// spilled).  Same sums, same order as reduce_kernel_rows.
template <class P, typename T, int OP, int D, int W, bool NT>
__global__ __launch_bounds__(64 * W) void reduce_kernel_narrow(const float* __restrict__ stack, int64_t stride,
                                                               int n, const typename P::w_t* __restrict__ w,
                                                               int64_t col0, int64_t ncols, Epi<T> e) {
  static_assert(sizeof(typename P::x_t) == 4 && D <= 63, "4-byte rows; vmcnt counts 63 loads");
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  typedef typename vec4<float>::type XV;
  const int64_t nquads = (ncols + 3) / 4;
  const int64_t qb = (int64_t)blockIdx.x * 64 * W;
  const int64_t qe = qb + 64 * W < nquads ? qb + 64 * W : nquads;
  const int64_t cend = qe * 4 < ncols ? qe * 4 : ncols;
  if (cend <= qb * 4) return;
  const int cols = (int)(cend - qb * 4);
  const uint32_t bytes = (uint32_t)cols * 4u;
  const int voff = (int)threadIdx.x * 16;
  const int64_t rb = stride * 4;
  const char* base = reinterpret_cast<const char*>(stack + col0 + qb * 4);
  const char* lastp = base + (int64_t)(n - 1) * rb;
  const char* p = base + rb;  // the next row to load (row 1)
#define FA_NW_LOAD(dst, CLAMP)                                                         \
  {                                                                                      \
    const char* q_ = p;                                                                  \
    if (CLAMP) q_ = p <= lastp ? p : lastp;                                              \
    dst = buf_load_quad<NT>(row_rsrc(q_, bytes), voff, 0);                               \
    p += rb;                                                                             \
    asm volatile("" : "+s"(p));                                                          \
  }
  // the weights of a round ride in one VGPR (lane l: row i + l), loaded a round ahead through a
  // range-checked descriptor and broadcast with readlane: a scalar load per row, waited for right
  // before its product, put a scalar-cache round trip on every row of the serial chain
  typedef typename P::w_t WT;
  const __amdgpu_buffer_rsrc_t wr = row_rsrc(w, (uint32_t)n * (uint32_t)sizeof(WT));
  const int lane = (int)threadIdx.x & 63;
  auto wload = [&](int first) {  // lane l of every wave: w[first + l] (0 past the end)
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
  for (int d = 0; d < D; ++d) FA_NW_LOAD(x[d], true);
  AV acc = quad_mul<P>(w[0], buf_load_quad<NT>(row_rsrc(base, bytes), voff, 0));
  int i = 1;
  // steady rounds: every consumed row and every refill row is real
  for (; i + 2 * D <= n; i += D) {
    const WT wnext = wload(i + D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc = quad_axpy<P>(acc, wlane(wcur, d), x[d]);
      __builtin_amdgcn_sched_barrier(0);
      FA_NW_LOAD(x[d], false);
      __builtin_amdgcn_sched_barrier(0);
    }
    wcur = wnext;
  }
  // the last (at most two) rounds: refills clamped to row n-1, products past it dropped
  for (; i < n; i += D) {
    const WT wnext = wload(i + D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const AV t = quad_axpy<P>(acc, wlane(wcur, d), x[d]);
      acc = i + d < n ? t : acc;
      __builtin_amdgcn_sched_barrier(0);
      FA_NW_LOAD(x[d], true);
      __builtin_amdgcn_sched_barrier(0);
    }
    wcur = wnext;
  }
#undef FA_NW_LOAD
  const AV accs[1] = {acc};
  finish_piece<T, OP, A, 1, 64 * W, 1>(e, qb, cols, accs);
}

// piece j of the group starting at slot g0: quads [qb, qb + bytes/16) of every row (interleaved
// over the grid as in reduce_kernel_rows); the window's ragged last quad included (per-dword range
// check: its missing elements load as 0 and are never stored); bytes 0: every access dropped
__device__ __forceinline__ void rowmajor_piece_geom(int64_t g0, int j, int64_t k, int64_t pc, int64_t pieces,
                                                    int64_t nquads, int64_t ncols, int64_t* qb, uint32_t* bytes) {
  const int64_t pj = blockIdx.x + (g0 + j) * (int64_t)gridDim.x;
  int64_t q = pj * pc * 64;
  const int64_t qe = q + pc * 64 < nquads ? q + pc * 64 : nquads;
  const int64_t ce = qe * 4 < ncols ? qe * 4 : ncols;
  const int64_t left = ce - q * 4;
  const uint32_t b = (pj < pieces && g0 + j < k && left > 0) ? (uint32_t)left * 4u : 0u;
  *qb = b ? q : 0;
  *bytes = b;
}

// One group of a row-major block: KG of the block's pieces (slots g0 .. g0+KG-1, interleaved
// over the grid as in reduce_kernel_rows), all rows swept once, then the group epilogue.
// PFG (cross-group prefetch): x arrives holding this group's first D steps (issued by the previous
// group, or by the kernel for the first), and after this group's last row the first D steps of the
// NEXT group (slot g0 + KG) are issued into x BEFORE this group's epilogue — so its result stores
// are younger than those loads, and the next group's first wait (vmcnt counts loads and stores in
// order) does not wait for them; without PFG every group end drained the stores before the next
// group's first product (NS: the result stores cost ~2.3x their bytes, profiles/r04/nostore).
template <class P, typename T, int OP, int V, int D, int W, int KG, bool NT, int EPIB, bool TR, int XLM = -1,
          bool PFG = false>
__device__ __forceinline__ void rowmajor_group(const char* __restrict__ base, int64_t row_bytes, int n,
                                               const typename P::w_t* __restrict__ w, int64_t g0, int64_t k,
                                               int64_t pc, int64_t pieces, int64_t nquads, int64_t ncols,
                                               int gi, const Epi<T>& e,
                                               typename vec4<float>::type (&x)[D][V]) {
  static_assert(KG % D == 0, "pipeline depth must divide the group size");
  typedef typename P::acc_t A;
  typedef typename vec4<A>::type AV;
  const int voff = (int)threadIdx.x * 16;
  int64_t qb[KG];
  uint32_t bytes[KG];  // 4 x the piece's columns; 0: every access of this slot is dropped
#pragma unroll
  for (int j = 0; j < KG; ++j) rowmajor_piece_geom(g0, j, k, pc, pieces, nquads, ncols, &qb[j], &bytes[j]);
  AV acc[KG][V];
  // step s = (i, j), i = s / KG, j = s % KG; slot = j % D
#define FA_RM_LOAD(slot, row, j)                                                                      \
  {                                                                                                   \
    const __amdgpu_buffer_rsrc_t r_ = row_rsrc(base + qb[j] * 16 + (int64_t)(row) * row_bytes, bytes[j]); \
    _Pragma("unroll") for (int v = 0; v < V; ++v) x[slot][v] = buf_load_quad<NT>(r_, voff + v * 64 * W * 16, 0); \
  }
  if constexpr (!PFG) {
#pragma unroll
    for (int d = 0; d < D; ++d) FA_RM_LOAD(d, 0, d);
  }
  // row 0: products initialise the sums
#pragma unroll
  for (int j = 0; j < KG; ++j) {
    const typename P::w_t w0 = w[0];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[j][v] = quad_mul<P>(w0, x[j % D][v]);
    __builtin_amdgcn_sched_barrier(0);
    if (j + D < KG) {
      FA_RM_LOAD(j % D, 0, j + D);
    } else if (n > 1) {
      FA_RM_LOAD(j % D, 1, j + D - KG);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  int i = 1;
  for (; i + 1 < n; ++i) {  // rows with a successor: every refill is a real step
    const typename P::w_t wi = w[i];
#pragma unroll
    for (int j = 0; j < KG; ++j) {
#pragma unroll
      for (int v = 0; v < V; ++v) acc[j][v] = quad_axpy<P>(acc[j][v], wi, x[j % D][v]);
      __builtin_amdgcn_sched_barrier(0);
      if (j + D < KG) {
        FA_RM_LOAD(j % D, i, j + D);
      } else {
        FA_RM_LOAD(j % D, i + 1, j + D - KG);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (i < n) {  // last row: refills only inside the row
    const typename P::w_t wi = w[i];
#pragma unroll
    for (int j = 0; j < KG; ++j) {
#pragma unroll
      for (int v = 0; v < V; ++v) acc[j][v] = quad_axpy<P>(acc[j][v], wi, x[j % D][v]);
      if (j + D < KG) FA_RM_LOAD(j % D, i, j + D);
    }
  }
#undef FA_RM_LOAD
  if constexpr (PFG) {  // the next group's first D steps, before this group's epilogue stores
    if (g0 + KG < k) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        int64_t qn;
        uint32_t bn;
        rowmajor_piece_geom(g0 + KG, d, k, pc, pieces, nquads, ncols, &qn, &bn);
        const __amdgpu_buffer_rsrc_t r_ = row_rsrc(base + qn * 16, bn);
#pragma unroll
        for (int v = 0; v < V; ++v) x[d][v] = buf_load_quad<NT>(r_, voff + v * 64 * W * 16, 0);
      }
    }
  }
  if constexpr (TR) {
    if (threadIdx.x == 0 && gi < 7) e.trace[blockIdx.x * 16 + 1 + 2 * gi] = wall_clock64();
  }
  if constexpr (EPIB == 0) {  // per-quad epilogue (tuning reference: tools/tune_reduce.hip set "epib")
#pragma unroll
    for (int j = 0; j < KG; ++j) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int q = v * 64 * W + (int)threadIdx.x;
        const int valid = (int)(bytes[j] / 4) - q * 4;
        if (valid > 0) finish_quad<T, OP, A>(e, (qb[j] + q) * 4, valid < 4 ? valid : 4, acc[j][v]);
      }
    }
  } else {
    // whole-line f64 state / result stores where they cost no spills: the fused ops at KG <= 3
    // (at KG = 4 the LDS regrouping pushes the kernel past 256 + 256 registers; finding 22)
    // (XLM: -1 this rule, 0 / 1 forced off / on by the tuner; 2: on, with the last KG/2 pieces'
    // sums parked in LDS while the first ones finish, so the regrouping has registers to use)
    constexpr bool XL = XLM >= 0 ? XLM >= 1 : (sizeof(T) == 8 && OP != FA_OP_MEAN && KG <= 3);
    if constexpr (XLM == 2 && KG >= 2) {
      constexpr int KP = KG / 2;  // pieces parked
      // lane-private slots, [piece][slot][thread]: consecutive lanes, consecutive 16 B (no bank
      // conflicts); a wave reads only what its own lanes wrote, in program order (no barrier)
      __shared__ AV park[KP][V][64 * W];
#pragma unroll
      for (int j = 0; j < KP; ++j)
#pragma unroll
        for (int v = 0; v < V; ++v) park[j][v][threadIdx.x] = acc[KG - KP + j][v];
      // the compiler must not forward the stored values (that would keep them in registers)
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < KG - KP; ++j) finish_piece<T, OP, A, V, 64 * W, EPIB, XL>(e, qb[j], (int)(bytes[j] / 4), acc[j]);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        AV a2[V];
#pragma unroll
        for (int v = 0; v < V; ++v) a2[v] = park[j][v][threadIdx.x];
        finish_piece<T, OP, A, V, 64 * W, EPIB, XL>(e, qb[KG - KP + j], (int)(bytes[KG - KP + j] / 4), a2);
      }
    } else {
#pragma unroll
      for (int j = 0; j < KG; ++j) finish_piece<T, OP, A, V, 64 * W, EPIB, XL>(e, qb[j], (int)(bytes[j] / 4), acc[j]);
    }
  }
  if constexpr (TR) {
    if (threadIdx.x == 0 && gi < 7) e.trace[blockIdx.x * 16 + 2 + 2 * gi] = wall_clock64();
  }
}

// Row-major variant for blocks that own several pieces (k > 1: C2-C5-sized buckets).  The
// column-major walk (reduce_kernel_rows: piece after piece, all rows each) starts every round of
// pieces with the blocks out of step, and rounds after the first measured ~8% slower per row on
// 100-client buckets (tune/trace_*).  Here a block sweeps the rows ONCE for a group of up to KG
// pieces: step s = (row i, piece j) with j fastest, KG accumulators per lane, and the same
// rolling register pipeline D steps deep (D divides KG, so every slot index is static).  The
// whole grid then moves through the client rows together.  Per element the sum is still rows
// 0..N-1 in order.
// TR (tools/tune_reduce.hip set "timeline"): wave 0 of every block stamps the 100-MHz wall clock
// at its start and at each group's sweep end and epilogue end into e.trace[block * 16 + slot].
template <class P, typename T, int OP, int V, int D, int W, int KG, bool NT, int EPIB = (V >= 2 ? 2 : V),
          bool TR = false, int XLM = -1, bool PFG = false>
__global__ __launch_bounds__(64 * W) void reduce_kernel_rowmajor(const float* __restrict__ stack,
                                                                 int64_t stride, int n,
                                                                 const typename P::w_t* __restrict__ w,
                                                                 int64_t col0, int64_t ncols, Epi<T> e) {
  static_assert(sizeof(typename P::x_t) == 4, "row pipeline is for 4-byte elements");
  const int64_t nquads = (ncols + 3) / 4;
  const int64_t chunks = (nquads + 63) / 64;
  const int64_t g = gridDim.x;
  const int64_t k = (chunks + g * W * V - 1) / (g * W * V);  // pieces per block
  const int64_t pc = (chunks + g * k - 1) / (g * k);         // chunks per piece (<= W*V)
  const int64_t pieces = (chunks + pc - 1) / pc;
  const int64_t row_bytes = stride * 4;
  const char* base = reinterpret_cast<const char*>(stack + col0);
  if constexpr (TR) {
    if (threadIdx.x == 0) e.trace[blockIdx.x * 16] = wall_clock64();
  }
  typename vec4<float>::type x[D][V];
  if constexpr (PFG) {  // the first group's first D steps (later groups get theirs from the previous one)
    const int voff = (int)threadIdx.x * 16;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      int64_t q0;
      uint32_t b0;
      rowmajor_piece_geom(0, d, k, pc, pieces, nquads, ncols, &q0, &b0);
      const __amdgpu_buffer_rsrc_t r_ = row_rsrc(base + q0 * 16, b0);
#pragma unroll
      for (int v = 0; v < V; ++v) x[d][v] = buf_load_quad<NT>(r_, voff + v * 64 * W * 16, 0);
    }
  }
#define FA_RM_GROUP(KGX, G0, GI) \
  rowmajor_group<P, T, OP, V, D, W, KGX, NT, EPIB, TR, XLM, PFG>(base, row_bytes, n, w, G0, k, pc, pieces, nquads, ncols, \
                                                                 GI, e, x)
  int gi = 0;
  for (int64_t g0 = 0; g0 < k; g0 += KG) FA_RM_GROUP(KG, g0, gi++);
#undef FA_RM_GROUP
}

// Column-blocked client stack: element (n, c) lives at ((c / B) * N + n) * B + c % B with
// B = kThreads*V*4 columns (one tile).  Tile b's N rows are one contiguous N*B*4-byte region, so
// a block streams its whole tile linearly (rows B*4 bytes apart) — the access pattern of a plain
// streaming read.  One tile per block; the window is the whole (padded) bucket.
template <class P, typename T, int OP, int V, int U, bool NT>
__global__ __launch_bounds__(kThreads) void reduce_kernel_blocked(
    const typename P::x_t* __restrict__ stack, int n, const typename P::w_t* __restrict__ w,
    int64_t ncols, Epi<T> e) {
  constexpr int64_t B = (int64_t)kThreads * V * 4;
  const int64_t tile = blockIdx.x;
  const typename P::x_t* base = stack + tile * (int64_t)n * B;
  Epi<T> et = e;
  if (et.out32) et.out32 += tile * B;
  if (et.out64) et.out64 += tile * B;
  if constexpr (OP != FA_OP_MEAN) {
    if (et.prev) et.prev += tile * B;
    if (et.h) et.h += tile * B;
    et.v += tile * B;
  }
  const int64_t cols = ncols - tile * B < B ? ncols - tile * B : B;
  reduce_range_subtile<P, T, OP, V, U, NT, (sizeof(typename P::x_t) == 4)>(
      base, B, n, w, 0, (cols + 3) / 4, cols, et);
}

// Standalone update (client_receive form): g read from memory instead of reduced.
template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void apply_kernel(const T* __restrict__ glob, int64_t n,
                                                         Epi<T> e) {
  const int64_t c = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 4;
  if (c >= n) return;
  const int valid = (int)((n - c) < 4 ? (n - c) : 4);
  typename vec4<T>::type g = load_quad_guarded(glob + c, valid);
  finish_quad<T, OP, T>(e, c, valid, g);  // denom == 1: T(g)/1 == g exactly
}

// Plain copy (fa_copy): 16-B non-temporal loads and stores, grid-stride; the last nbytes % 16
// bytes by the first block's lanes.  Pointers 16-byte aligned (checked on the host).
__global__ __launch_bounds__(kThreads) void copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                        int64_t nbytes) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const int64_t quads = nbytes >> 4;
  const u4* s = reinterpret_cast<const u4*>(src);
  u4* d = reinterpret_cast<u4*>(dst);
  for (int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x; q < quads; q += (int64_t)gridDim.x * kThreads)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + q), d + q);
  const int64_t tail = nbytes - (quads << 4);
  if (blockIdx.x == 0 && threadIdx.x < tail) dst[(quads << 4) + threadIdx.x] = src[(quads << 4) + threadIdx.x];
}

// One-shot all-gather leg (fa_push): each lane loads 16 B of the local stripe once and stores it
// into every destination (the peers' receive buffers over their xGMI links, and the local one);
// the closing system-scope fence makes the peer stores visible once the kernel has completed.
// Paced: every wave drains its stores (vmcnt(0): on gfx9 the counter covers stores) before its
// next round's loads, so at most U x n_dsts KiB per wave is in flight and the grid sets the total.
// Stores queued beyond a link's bandwidth-delay product back up into the data fabric the reduce
// beside them streams through: on one GPU's PCIe stand-in, 8 blocks reach 52 GB/s either way and
// slow the reduce 1.27-1.32x paced, 1.27-2.08x unpaced (2.08 in the same run as the paced 1.27;
// tools/overlap_probe.py paced<U>x<B> / pushhost<B>).
struct PushDsts {
  uint8_t* p[8];
};

// One system-scope cache fence per wave: RELEASE (K = 0) writes the L2 back to HBM, ACQUIRE
// (K = 1) invalidates it, so that a copy engine (which reads and writes HBM behind the L2) and the
// kernels around it see each other's data (fa_cache_fence).  Each XCD has its own L2: the launch
// spreads one wave over every XCD, several times over.
template <int K>
__global__ __launch_bounds__(64) void cache_fence_kernel() {
  if (K == 0)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__global__ __launch_bounds__(kThreads) void push_kernel(const uint8_t* __restrict__ src, int64_t quads, PushDsts d,
                                                        int n_dsts) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  constexpr int U = 4;  // quads per lane per round: U loads, then U stores to every destination
  const u4* s = reinterpret_cast<const u4*>(src);
  const int64_t G = (int64_t)gridDim.x * kThreads;
  for (int64_t q0 = (int64_t)blockIdx.x * kThreads + threadIdx.x; q0 < quads; q0 += U * G) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = q0 + u * G;
      v[u] = q < quads ? __builtin_nontemporal_load(s + q) : u4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i >= n_dsts) break;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + u * G;
        if (q < quads) reinterpret_cast<u4*>(d.p[i])[q] = v[u];
      }
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // pace: this round's stores done first
  }
  __threadfence_system();
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

}  // namespace fa
