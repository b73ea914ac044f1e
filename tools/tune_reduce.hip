// tune_reduce.hip — geometry sweep of the fused reduce kernel on the MI355X.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iflearn_amd/csrc \
//         tools/tune_reduce.hip -o tools/tune_reduce
//   tools/tune_reduce [n_clients=100] [n_cols=11699136] [rounds=7] [op=mean|avgm]
//
// Times every variant (quads/thread V, client unroll U, non-temporal loads, one-shot vs
// persistent grid) with hipEvents in interleaved rounds (one process, same data), checks each
// variant's output bitwise against the first, and brackets them with two roofs measured on the
// same buffers: a pure streaming read of the N x P stack and a float4 copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
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

// read roof: stream the whole stack once, 16-B loads, keep the data alive with one store/thread
__global__ __launch_bounds__(256) void read_roof(const float* __restrict__ x, int64_t quads,
                                                 float* __restrict__ sink) {
  typedef vec4<float>::type f4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < quads; q += (int64_t)gridDim.x * 256) {
    f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + q);
    acc += v;
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.678f) sink[threadIdx.x] = acc[0];
}

__global__ __launch_bounds__(256) void copy_roof(const float* __restrict__ x, float* __restrict__ y,
                                                 int64_t quads) {
  typedef vec4<float>::type f4;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < quads; q += (int64_t)gridDim.x * 256)
    reinterpret_cast<f4*>(y)[q] = reinterpret_cast<const f4*>(x)[q];
}

// roof in the reduce's access shape: tiles of 256*B quads read as B 1-KiB-per-wave bursts, tile
// after tile (grid-stride), LDS used only to cap occupancy; no row jumps, no arithmetic chain
template <int B>
__global__ __launch_bounds__(256) void roof_burst(const float* __restrict__ x, int64_t quads,
                                                  float* __restrict__ sink) {
  extern __shared__ float lds_cap[];
  typedef vec4<float>::type f4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t tiles = quads / (256 * B);
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    f4 v[B];
#pragma unroll
    for (int b = 0; b < B; ++b)
      v[b] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + t * 256 * B + b * 256 + threadIdx.x);
#pragma unroll
    for (int b = 0; b < B; ++b) acc += v[b];
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.678f) {
    lds_cap[threadIdx.x] = acc[0];
    sink[threadIdx.x] = lds_cap[(threadIdx.x + 1) & 255];
  }
}

namespace fa {
// ---------------------------------------------------------------------------------------------
// Tuning-only kernel (set "dfr", profiles/r02/tune_dfr/, DESIGN.md §4 finding 14 — measured slower
// than the product's group-end epilogue, so it stays here and not in fa_device.hpp).
// Row-major groups with DEFERRED epilogues (reduce_kernel_rowmajor_dfr).  In reduce_kernel_rowmajor
// every block reaches its group end at the same moment (the grid moves through the client rows
// together), so each group epilogue is a chip-wide burst of mixed state reads and result writes
// at the copy rate (~5 TB/s, DESIGN.md §4 finding 11) with no client reads left to overlap.
// Here a group's sums go to LDS instead (KG x 64 KiB per block: KG <= 2 within the CU's 160 KiB)
// and its epilogue is spread over the NEXT group's sweep: in each of its first rows a lane finishes one quad
// (state loads issued one unit ahead, then divide / update / store), so the state traffic rides
// inside the client stream.  Only the last group's epilogue runs at the end.  Each lane reads
// back only the LDS slots it wrote: no barrier.  Sums and epilogue arithmetic are those of
// reduce_kernel_rowmajor, element for element.
// ---------------------------------------------------------------------------------------------
struct RmGeom {  // the interleaved piece plan of reduce_kernel_rowmajor
  int64_t g, k, pc, pieces, nquads, ncols;
  // slot s of this block: piece blockIdx.x + s*g, columns [qb*4, qb*4 + bytes/4)
  __device__ __forceinline__ void piece(int64_t s, int64_t& qb, uint32_t& bytes) const {
    const int64_t pj = blockIdx.x + s * g;
    qb = pj * pc * 64;
    const int64_t qe = qb + pc * 64 < nquads ? qb + pc * 64 : nquads;
    const int64_t ce = qe * 4 < ncols ? qe * 4 : ncols;
    const int64_t left = ce - qb * 4;
    bytes = (s >= 0 && pj < pieces && s < k && left > 0) ? (uint32_t)left * 4u : 0u;
    if (bytes == 0) qb = 0;
  }
};

template <class P, typename T, int OP, int V, int W, int KGX, bool NT, int EPIB, int TM>
__device__ __forceinline__ void dfr_group(const char* __restrict__ base, int64_t row_bytes, int n,
                                          const typename P::w_t* __restrict__ w, const RmGeom& G,
                                          int64_t g0, int64_t pg0, int pkg, bool last, const Epi<T>& e,
                                          typename vec4<float>::type* stash) {
  typedef typename P::acc_t A;
  typedef typename vec4<float>::type XV;
  typedef typename vec4<T>::type TV;
  typedef typename vec4<A>::type AV;
  constexpr int STEP = 64 * W;
  const int voff = (int)threadIdx.x * 16;
  int64_t qb[KGX];
  uint32_t bytes[KGX];
#pragma unroll
  for (int j = 0; j < KGX; ++j) G.piece(g0 + j, qb[j], bytes[j]);
  // the pending group (pkg pieces from slot pg0; pkg = 0: none): unit u = its piece u / V, slot u % V
  int64_t pq0, pq1;
  uint32_t pb0, pb1;
  G.piece(pkg > 0 ? pg0 : -1, pq0, pb0);
  G.piece(pkg > 1 ? pg0 + 1 : -1, pq1, pb1);
  const int U = TM == 0 ? 0 : pkg * V;  // TM 0 (timing probe only): deferred epilogues dropped
  XV tl, ta, rl;
  TV tv, rv, rw;
#define FA_DFR_ISSUE(uu)                                                          \
  {                                                                               \
    const int j_ = (uu) >= V;                                                     \
    const int q_ = (int)threadIdx.x + ((uu) - j_ * V) * STEP;                     \
    const EpiRsrc<T, OP> r_(e, j_ ? pq1 : pq0, (int)((j_ ? pb1 : pb0) / 4));      \
    epi_load<T, OP>(r_, q_, tl, tv);                                              \
    ta = stash[(uu) * STEP + (int)threadIdx.x];                                   \
  }
#define FA_DFR_FINISH(uu)                                                         \
  {                                                                               \
    const int j_ = (uu) >= V;                                                     \
    const int q_ = (int)threadIdx.x + ((uu) - j_ * V) * STEP;                     \
    const EpiRsrc<T, OP> r_(e, j_ ? pq1 : pq0, (int)((j_ ? pb1 : pb0) / 4));      \
    epi_quad<T, OP, A, false>(e, r_, q_, ta, tl, tv);                             \
  }
#define FA_DFR_STORE(uu)  /* TM 2: the results of unit uu, computed a row earlier (uu < 0: none) */ \
  {                                                                                         \
    const int us_ = (uu) > 0 ? (uu) : 0;                                                    \
    const int j_ = us_ >= V;                                                                \
    const int q_ = (int)threadIdx.x + (us_ - j_ * V) * STEP;                                \
    const EpiRsrc<T, OP> r_(e, j_ ? pq1 : pq0, (uu) < 0 ? 0 : (int)((j_ ? pb1 : pb0) / 4)); \
    epi_store<T, OP, false>(e, r_, q_, rl, rv, rw);                                         \
  }
#define FA_DFR_LOAD(row, j)                                                                           \
  {                                                                                                   \
    const __amdgpu_buffer_rsrc_t r_ = row_rsrc(base + qb[j] * 16 + (int64_t)(row) * row_bytes, bytes[j]); \
    _Pragma("unroll") for (int v = 0; v < V; ++v) x[v] = buf_load_quad<NT>(r_, voff + v * STEP * 16, 0); \
  }
  XV x[V];
  AV acc[KGX][V];
  int u = 0;
  FA_DFR_LOAD(0, 0);
  if (U > 0) FA_DFR_ISSUE(0);
  // row 0: products initialise the sums
#pragma unroll
  for (int j = 0; j < KGX; ++j) {
    const typename P::w_t w0 = w[0];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[j][v] = quad_mul<P>(w0, x[v]);
    __builtin_amdgcn_sched_barrier(0);
    if (j + 1 < KGX) {
      FA_DFR_LOAD(0, j + 1);
    } else if (n > 1) {
      FA_DFR_LOAD(1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // rows 1 .. U finish one pending unit each, between the row's last step and the next row's
  // first refill (one basic block: the scheduling barriers keep that order; a unit's state loads
  // were issued a row earlier and its stores go out before the refill, so no wait for the next
  // step covers them); the remaining rows are the plain sweep
#define FA_DFR_ROW(TRICKLE)                                                                    \
  {                                                                                            \
    const typename P::w_t wi = w[i];                                                           \
    _Pragma("unroll") for (int j = 0; j < KGX; ++j) {                                          \
      _Pragma("unroll") for (int v = 0; v < V; ++v) acc[j][v] = quad_axpy<P>(acc[j][v], wi, x[v]); \
      __builtin_amdgcn_sched_barrier(0);                                                       \
      if (j + 1 < KGX) {                                                                       \
        FA_DFR_LOAD(i, j + 1);                                                                 \
      } else {                                                                                 \
        if (TRICKLE && TM == 1) {                                                              \
          FA_DFR_FINISH(u);                                                                    \
          ++u;                                                                                 \
          FA_DFR_ISSUE(u < U ? u : U - 1);                                                     \
          __builtin_amdgcn_sched_barrier(0);                                                   \
        }                                                                                      \
        if (TRICKLE && TM == 2) {                                                              \
          FA_DFR_STORE(u - 1);                                                                 \
          __builtin_amdgcn_sched_barrier(0);                                                   \
        }                                                                                      \
        FA_DFR_LOAD(i + 1, 0);                                                                 \
        if (TRICKLE && TM == 2) {                                                              \
          __builtin_amdgcn_sched_barrier(0);                                                   \
          rl = tl;                                                                             \
          rv = tv;                                                                             \
          epi_compute<T, OP, A>(e, ta, rl, rv, rw);                                            \
          ++u;                                                                                 \
          FA_DFR_ISSUE(u < U ? u : U - 1);                                                     \
        }                                                                                      \
      }                                                                                        \
      __builtin_amdgcn_sched_barrier(0);                                                       \
    }                                                                                          \
  }
  int i = 1;
  if (U > 0) {
    for (; i + 1 < n && u < U; ++i) FA_DFR_ROW(true);
  }
  for (; i + 1 < n; ++i) FA_DFR_ROW(false);
#undef FA_DFR_ROW
  if (i < n) {  // last row: refills only inside the row
    const typename P::w_t wi = w[i];
#pragma unroll
    for (int j = 0; j < KGX; ++j) {
#pragma unroll
      for (int v = 0; v < V; ++v) acc[j][v] = quad_axpy<P>(acc[j][v], wi, x[v]);
      if (j + 1 < KGX) FA_DFR_LOAD(i, j + 1);
    }
  }
  if (TM == 2 && u > 0) FA_DFR_STORE(u - 1);
  // units the sweep had no rows left for (few clients)
  while (u < U) {
    FA_DFR_FINISH(u);
    ++u;
    if (u < U) FA_DFR_ISSUE(u);
  }
#undef FA_DFR_ISSUE
#undef FA_DFR_FINISH
#undef FA_DFR_STORE
#undef FA_DFR_LOAD
  if (last) {
#pragma unroll
    for (int j = 0; j < KGX; ++j) finish_piece<T, OP, A, V, STEP, EPIB>(e, qb[j], (int)(bytes[j] / 4), acc[j]);
  } else {
#pragma unroll
    for (int j = 0; j < KGX; ++j) {
#pragma unroll
      for (int v = 0; v < V; ++v) stash[(j * V + v) * STEP + (int)threadIdx.x] = acc[j][v];
    }
  }
}

template <class P, typename T, int OP, int V, int W, int KG, bool NT, int TM = 2, int EPIB = 2>
__global__ __launch_bounds__(64 * W) void reduce_kernel_rowmajor_dfr(const float* __restrict__ stack,
                                                                     int64_t stride, int n,
                                                                     const typename P::w_t* __restrict__ w,
                                                                     int64_t col0, int64_t ncols, Epi<T> e) {
  static_assert(sizeof(typename P::x_t) == 4 && sizeof(typename P::acc_t) == 4, "fp32 sums only");
  static_assert(KG == 1 || KG == 2, "KG x 64 KiB of sums must fit the CU's LDS");
  static_assert(V * W == 64, "64-KiB pieces");
  __shared__ typename vec4<float>::type stash[KG * V * 64 * W];
  RmGeom G;
  G.nquads = (ncols + 3) / 4;
  const int64_t chunks = (G.nquads + 63) / 64;
  G.g = gridDim.x;
  G.k = (chunks + G.g * W * V - 1) / (G.g * W * V);
  G.pc = (chunks + G.g * G.k - 1) / (G.g * G.k);
  G.pieces = (chunks + G.pc - 1) / G.pc;
  G.ncols = ncols;
  const char* base = reinterpret_cast<const char*>(stack + col0);
  const int64_t row_bytes = stride * 4;
  int64_t pg0 = 0;
  int pkg = 0;
  for (int64_t g0 = 0; g0 < G.k; g0 += KG) {
    const bool last = g0 + KG >= G.k;
    if (G.k - g0 >= KG) {
      dfr_group<P, T, OP, V, W, KG, NT, EPIB, TM>(base, row_bytes, n, w, G, g0, pg0, pkg, last, e, stash);
      pkg = KG;
    } else {
      dfr_group<P, T, OP, V, W, 1, NT, EPIB, TM>(base, row_bytes, n, w, G, g0, pg0, pkg, last, e, stash);
      pkg = 1;
    }
    pg0 = g0;
  }
}

// ---- tuning-only kernels measured in round 3 and NOT adopted (DESIGN.md §4 findings 17, 18) ----

// [tuning only, not adopted: slower than reduce_kernel_narrow on every shape] LDS-staged narrow reduce (deep, narrow windows: LeNet-sized models of many clients), bit-exact.
// reduce_kernel_narrow gives each 1-KiB chunk of the window ONE wave, and a wave's vmcnt caps its
// loads in flight at 63 — so 1000 LeNet5 uploads (174 chunks) keep only ~7 MB in flight on the
// whole chip and stream at ~74% of spec.  Splitting the CLIENTS over waves (split-N) gets more
// loads in flight but changes the summation order.  Here the LOADING is split and the SUMMING
// is not:
//   * a block owns one chunk (256 columns) and W waves; rows go in STAGES of R = W*DW rows, wave
//     v loading rows [s*R + v*DW, +DW) of stage s (whole 1-KiB rows, one buffer descriptor each)
//     L stages ahead, so W*L*DW KiB stay in flight per block (e.g. 4 x 3 x 8 = 96 KiB);
//   * at stage s every wave writes its landed rows into an LDS row buffer (double-buffered,
//     2 x R KiB), one barrier, and then EVERY wave sums its own 64 columns over all R rows of the
//     stage in row order — lane l of wave v owns column 64v + l, reads it from LDS (a 256-B
//     conflict-free ds_read_b32 row slice) and runs the reference's sequential chain:
//     acc = fl(w0*x0), acc = fl(acc + fl(w_i*x_i)) for i = 1..N-1 in list order;
//   * the stage's weights are loaded with its rows (one VGPR of wave 0, lane j: w[s*R + j]) and
//     ride through LDS with them (a broadcast read; no scalar-cache round trip in the chain);
//   * the per-column sums meet in LDS and wave 0 applies the usual piece epilogue.
// The double buffer needs one barrier per stage: buffer s&1 is rewritten at stage s+2, after the
// barrier of stage s+1, which no wave passes before it has finished consuming stage s.
template <class P, typename T, int OP, int W, int DW, int L, bool NT>
__global__ __launch_bounds__(64 * W) void reduce_kernel_lds(const float* __restrict__ stack, int64_t stride, int n,
                                                            const typename P::w_t* __restrict__ w, int64_t col0,
                                                            int64_t ncols, Epi<T> e) {
  typedef typename P::acc_t A;
  typedef typename P::w_t WT;
  typedef typename vec4<float>::type XV;
  typedef typename vec4<A>::type AV;
  constexpr int R = W * DW;  // rows per stage
  static_assert(sizeof(typename P::x_t) == 4 && R <= 64 && L * (DW + 1) <= 63, "stage geometry");
  static_assert(W == 4, "4 waves x 64 lanes = the chunk's 256 columns, one per lane");
  __shared__ XV rowbuf[2][R][64];
  __shared__ WT wbuf[2][R];
  __shared__ A accbuf[256];
  const int lane = (int)threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int64_t qb = (int64_t)blockIdx.x * 64;  // the chunk's first quad
  const int64_t cleft = ncols - qb * 4;
  if (cleft <= 0) return;  // (uniform over the block)
  const int tcols = cleft < 256 ? (int)cleft : 256;
  const uint32_t bytes = (uint32_t)tcols * 4u;
  const char* base = reinterpret_cast<const char*>(stack + col0 + qb * 4);
  const int64_t rb = stride * 4;
  const int stages = (n + R - 1) / R;
  const int voff = lane * 16;
  const __amdgpu_buffer_rsrc_t wrs = row_rsrc(w, (uint32_t)n * (uint32_t)sizeof(WT));
  auto wload = [&](int first) {  // lane j: w[first + j] (0 past the end)
    if constexpr (sizeof(WT) == 4)
      return __builtin_bit_cast(WT, __builtin_amdgcn_raw_buffer_load_b32(wrs, (lane + first) * 4, 0, 0));
    else
      return __builtin_bit_cast(WT, __builtin_amdgcn_raw_buffer_load_b64(wrs, (lane + first) * 8, 0, 0));
  };

  XV x[L][DW];
  WT ws[L];
  // stage s into slot t: this wave's DW rows (clamped to the last row: the refills of the at most
  // L-1 padding stages past the end re-read row n-1, an L2 hit) and the stage's weights.  No
  // branch around any load: the compiler's vmcnt bookkeeping then sees the same L*(DW+1) loads
  // in flight at every stage and waits only for the oldest stage's
#define FA_LDS_ISSUE(t, s)                                                                           \
  {                                                                                                  \
    const int r0_ = (s) * R + wv * DW;                                                               \
    _Pragma("unroll") for (int i = 0; i < DW; ++i) {                                                 \
      const int r_ = r0_ + i < n ? r0_ + i : n - 1;                                                  \
      x[t][i] = buf_load_quad<NT>(row_rsrc(base + (int64_t)r_ * rb, bytes), voff, 0);                \
    }                                                                                                \
    ws[t] = wload((s) * R);                                                                          \
  }
#pragma unroll
  for (int t = 0; t < L; ++t) FA_LDS_ISSUE(t, t);
  const float* lrow = reinterpret_cast<const float*>(&rowbuf[0][0][0]);
  const int c = wv * 64 + lane;  // this lane's column of the chunk
  A acc = A(0);
  for (int s0 = 0; s0 < stages; s0 += L) {
#pragma unroll
    for (int t = 0; t < L; ++t) {
      const int s = s0 + t;  // may be a padding stage past the end (its rows are not summed)
      const int buf = s & 1;
#pragma unroll
      for (int i = 0; i < DW; ++i) rowbuf[buf][wv * DW + i][lane] = x[t][i];
      if (wv == 0 && lane < R) wbuf[buf][lane] = ws[t];  // the stage's weights ride along
      // LDS-only barrier: this wave's row writes are done (lgkmcnt(0)); the global loads in
      // flight are NOT waited for (__syncthreads() would drain vmcnt and serialise the stages)
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      FA_LDS_ISSUE(t, s + L);
      __builtin_amdgcn_sched_barrier(0);
      const float* lb = lrow + buf * R * 256 + c;
      const int rows = n - s * R;  // rows of this stage to sum (<= 0: padding)
      // all R row values first (one LDS round trip per stage, not one per row pair), then the chain
      float xs[R];
      WT wj[R];
#pragma unroll
      for (int j = 0; j < R; ++j) xs[j] = lb[j * 256];
#pragma unroll
      for (int j = 0; j < R; ++j) wj[j] = wbuf[buf][j];  // (a broadcast read)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const A p = P::mul(wj[j], xs[j]);
        const A a2 = (s == 0 && j == 0) ? p : add<A>(acc, p);
        acc = j < rows ? a2 : acc;
      }
    }
  }
#undef FA_LDS_ISSUE
  accbuf[c] = acc;
  __syncthreads();  // (after the last stage: draining the padding refills costs nothing here)
  if (wv == 0) {
    const AV r[1] = {AV{accbuf[lane * 4], accbuf[lane * 4 + 1], accbuf[lane * 4 + 2], accbuf[lane * 4 + 3]}};
    finish_piece<T, OP, A, 1, 64, 1>(e, qb, tcols, r);
  }
}

// [tuning only, not adopted: slower than reduce_kernel_rowmajor on NS / C3 / C5] Row-major groups with a dynamically claimed tail.  The blocks of reduce_kernel_rowmajor end
// their last group over a spread of ~60 us (C3: 4% of the launch; the per-block stream rate
// differs with its XCD and HBM channels, DESIGN §4 finding 11), and a static split cannot know
// which blocks will be late.  Here the window's first `ncols_static` columns are the static
// row-major groups, and the rest is cut into STRIPS of W KiB of every row (one quad per lane),
// claimed one at a time from a device counter by whichever block is free: a strip sweeps all N
// rows TD deep (TD*W KiB in flight, like a group step) and applies the epilogue to its columns.
// A strip is short (100 rows x 8 KiB ~ 20 us), so the blocks finish within about one strip of
// each other.  Per element the sum is still rows 0..N-1 in list order (bit-exact): a column is
// summed by exactly one block, static or strip.  *work must be 0 at launch.
template <class P, typename T, int OP, int V, int D, int W, int KG, bool NT, int TD, int EPIB = (V >= 2 ? 2 : V)>
__global__ __launch_bounds__(64 * W) void reduce_kernel_rowmajor_tail(const float* __restrict__ stack,
                                                                      int64_t stride, int n,
                                                                      const typename P::w_t* __restrict__ w,
                                                                      int64_t col0, int64_t ncols_static,
                                                                      int64_t ncols, Epi<T> e,
                                                                      int* __restrict__ work) {
  static_assert(sizeof(typename P::x_t) == 4, "row pipeline is for 4-byte elements");
  const int64_t g = gridDim.x;
  const int64_t row_bytes = stride * 4;
  const char* base = reinterpret_cast<const char*>(stack + col0);
  if (ncols_static > 0) {
    const int64_t nquads_s = (ncols_static + 3) / 4;
    const int64_t chunks_s = (nquads_s + 63) / 64;
    const int64_t k = (chunks_s + g * W * V - 1) / (g * W * V);
    const int64_t pc = (chunks_s + g * k - 1) / (g * k);
    const int64_t pieces = (chunks_s + pc - 1) / pc;
    int gi = 0;
    typename vec4<float>::type x[D][V];
    for (int64_t g0 = 0; g0 < k; g0 += KG)
      rowmajor_group<P, T, OP, V, D, W, KG, NT, EPIB, false>(base, row_bytes, n, w, g0, k, pc, pieces, nquads_s,
                                                            ncols_static, gi++, e, x);
  }
  // the tail: strips of 64*W quads from quad ncols_static/4 (ncols_static is a multiple of 4)
  const int64_t nquads = (ncols + 3) / 4;
  const int64_t qt0 = ncols_static / 4;
  const int64_t strips = (nquads - qt0 + 64 * W - 1) / (64 * W);
  __shared__ int s_claim;
  if (threadIdx.x == 0) s_claim = atomicAdd(work, 1);
  __syncthreads();
  int s = s_claim;
  while (s < strips) {
    const int64_t qs = qt0 + (int64_t)s * 64 * W;
    const int64_t qe = qs + 64 * W < nquads ? qs + 64 * W : nquads;
    rows_piece<P, T, OP, 1, TD, W, NT>(stack, stride, n, w, col0, ncols, e, qs, qe);
    __syncthreads();  // every wave is done with s_claim and its strip
    if (threadIdx.x == 0) s_claim = atomicAdd(work, 1);
    __syncthreads();
    s = s_claim;
  }
}

// [tuning] The narrow-window kernel with narrower strips per wave: lane l reads LB bytes (one
// dword, a dword pair or a quad) of every row, so a single-wave block owns a 64*LB-byte strip of
// the window.  With LB = 4 a row slot costs one VGPR instead of four, so the same vmcnt budget
// (63 loads) is reached with a quarter of the registers, and a LeNet-wide window is 4x as many
// waves (695 instead of 174 for 44,426 columns), spread over every CU instead of 174 of the 256.
// Same pipeline as reduce_kernel_narrow (no drain code, weights broadcast by readlane), same sums,
// same order.  The epilogue regroups the strip into quads with cross-lane reads (lane q gets the
// columns 4q..4q+3) and applies the usual piece epilogue; lanes past the strip's quads are dropped
// by the descriptor range.
template <int LB>
struct LaneCols;
template <>
struct LaneCols<4> {
  static constexpr int C = 1;
  template <bool NT>
  static __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int voff, float (&x)[1]) {
    x[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, NT ? 2 : 0));
  }
};
template <>
struct LaneCols<8> {
  static constexpr int C = 2;
  template <bool NT>
  static __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int voff, float (&x)[2]) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, NT ? 2 : 0));
    x[0] = v[0];
    x[1] = v[1];
  }
};

template <class P, typename T, int OP, int LB, int D, bool NT>
__global__ __launch_bounds__(64) void reduce_kernel_narrow_lb(const float* __restrict__ stack, int64_t stride, int n,
                                                              const typename P::w_t* __restrict__ w, int64_t col0,
                                                              int64_t ncols, Epi<T> e) {
  static_assert(sizeof(typename P::x_t) == 4 && D <= 62, "4-byte rows; vmcnt counts 63 loads (+ the weights)");
  typedef LaneCols<LB> LC;
  constexpr int C = LC::C;
  constexpr int SC = 64 * C;  // columns of the strip
  typedef typename P::acc_t A;
  typedef typename P::w_t WT;
  const int64_t cb = (int64_t)blockIdx.x * SC;
  if (cb >= ncols) return;
  const int cols = ncols - cb < SC ? (int)(ncols - cb) : SC;
  const uint32_t bytes = (uint32_t)cols * 4u;
  const int lane = (int)threadIdx.x & 63;
  const int voff = lane * LB;
  const int64_t rb = stride * 4;
  const char* base = reinterpret_cast<const char*>(stack + col0 + cb);
  const char* lastp = base + (int64_t)(n - 1) * rb;
  const char* p = base + rb;
#define FA_NL_LOAD(dst, CLAMP)                                  \
  {                                                             \
    const char* q_ = p;                                         \
    if (CLAMP) q_ = p <= lastp ? p : lastp;                     \
    LC::template load<NT>(row_rsrc(q_, bytes), voff, dst);      \
    p += rb;                                                    \
    asm volatile("" : "+s"(p));                                 \
  }
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
  float x[D][C];
#pragma unroll
  for (int d = 0; d < D; ++d) FA_NL_LOAD(x[d], true);
  A acc[C];
  {
    float x0[C];
    LC::template load<NT>(row_rsrc(base, bytes), voff, x0);
    const WT w0 = w[0];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = P::mul(w0, x0[c]);
  }
  int i = 1;
  for (; i + 2 * D <= n; i += D) {
    const WT wnext = wload(i + D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const WT wd = wlane(wcur, d);
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = add<A>(acc[c], P::mul(wd, x[d][c]));
      __builtin_amdgcn_sched_barrier(0);
      FA_NL_LOAD(x[d], false);
      __builtin_amdgcn_sched_barrier(0);
    }
    wcur = wnext;
  }
  for (; i < n; i += D) {
    const WT wnext = wload(i + D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const WT wd = wlane(wcur, d);
      const bool live = i + d < n;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const A t = add<A>(acc[c], P::mul(wd, x[d][c]));
        acc[c] = live ? t : acc[c];
      }
      __builtin_amdgcn_sched_barrier(0);
      FA_NL_LOAD(x[d], true);
      __builtin_amdgcn_sched_barrier(0);
    }
    wcur = wnext;
  }
#undef FA_NL_LOAD
  // regroup into quads: lane q takes columns 4q + j = lane (4q + j) / C, element (4q + j) % C
  typename vec4<A>::type q;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    A v = acc[0];
#pragma unroll
    for (int c = 1; c < C; ++c) v = (j % C == c) ? acc[c] : v;
    q[j] = __shfl(v, (4 * lane + j) / C);
  }
  const typename vec4<A>::type accs[1] = {q};
  finish_piece<T, OP, A, 1, 64, 1>(e, cb / 4, cols, accs);
}

}  // namespace fa

struct Variant {
  std::string name;
  double bytes;
  std::function<void()> launch;
  bool checks_output;
  std::vector<float> times;
};

template <int V, int U, bool NT, int OP, typename T, bool BUF = false>
Variant make_oneshot(const float* stack, int64_t stride, int n, const float* w, int64_t ncols,
                     Epi<T> e, double bytes) {
  const int64_t tiles = (ncols + 256 * V * 4 - 1) / (256 * V * 4);
  char name[96];
  snprintf(name, sizeof name, "oneshot%s V%d U%d NT%d", BUF ? "-buf" : "", V, U, (int)NT);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel<AccF32, T, OP, V, U, NT, BUF>), dim3((unsigned)tiles), dim3(256),
                               0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

// rounds_extra: grid = (k + rounds_extra) * CUs * occupancy, k = the fewest rounds for which
// every block's share fits one sub-tile
template <int V, int U, bool NT, int OP, typename T, bool BUF = false>
Variant make_balanced(const float* stack, int64_t stride, int n, const float* w, int64_t ncols,
                      Epi<T> e, double bytes, int cus, int rounds_extra) {
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reduce_kernel_balanced<AccF32, T, OP, V, U, NT, BUF>,
                                                  256, 0));
  const int64_t slots = (int64_t)cus * occ;
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  const int64_t k = (chunks + slots * 4 * V - 1) / (slots * 4 * V) + rounds_extra;
  const int grid = (int)std::min<int64_t>(std::max<int64_t>(1, k * slots), chunks);
  char name[96];
  snprintf(name, sizeof name, "balanced%s V%d U%d occ%d g%d", BUF ? "-buf" : "", V, U, occ, grid);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_balanced<AccF32, T, OP, V, U, NT, BUF>), dim3(grid), dim3(256), 0, 0,
                               stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

template <int V, int D, int W, int OP, typename T, bool IL = true, bool XM = false, bool NTL = true>
Variant make_rows(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                  double bytes, int64_t max_grid = 0) {
  int64_t grid = ((ncols + 3) / 4 + 64 * W * V - 1) / (64 * W * V);
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (max_grid > 0) grid = max_grid < chunks ? max_grid : chunks;
  char name[96];
  snprintf(name, sizeof name, "rows%s%s%s V%d D%d W%d g%lld", IL ? "-il" : "-ct", XM ? "-xcd" : "",
           NTL ? "" : "-temporal", V, D, W, (long long)grid);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_rows<AccF32, T, OP, V, D, W, NTL, IL, XM>), dim3((unsigned)grid),
                               dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

template <int D, int W, int OP, typename T>
Variant make_narrow(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                    double bytes) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  const int64_t grid = (chunks + W - 1) / W;
  char name[96];
  snprintf(name, sizeof name, "narrow D%d W%d g%lld", D, W, (long long)grid);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_narrow<AccF32, T, OP, D, W, true>), dim3((unsigned)grid),
                               dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

template <int LB, int D, int OP, typename T>
Variant make_narrow_lb(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                       double bytes) {
  const int64_t sc = 16 * LB;  // columns per single-wave strip
  const int64_t grid = (ncols + sc - 1) / sc;
  char name[96];
  snprintf(name, sizeof name, "narrow-lb LB%d D%d g%lld", LB, D, (long long)grid);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_narrow_lb<AccF32, T, OP, LB, D, true>), dim3((unsigned)grid), dim3(64),
                               0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

template <int V, int D, int W, int KG, int OP, typename T, int EPIB, int XLM>
Variant make_rowmajor_xl(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                         double bytes, int64_t grid) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (grid > chunks) grid = chunks;
  char name[96];
  snprintf(name, sizeof name, "rowmajor V%d W%d KG%d g%lld epib%d xl%d", V, W, KG, (long long)grid, EPIB, XLM);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_rowmajor<AccF32, T, OP, V, D, W, KG, true, EPIB, false, XLM>),
                               dim3((unsigned)grid), dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

template <int V, int D, int W, int KG, int OP, typename T, int EPIB, int XLM, bool PFG>
Variant make_rowmajor_pfg(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                          double bytes, int64_t grid) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (grid > chunks) grid = chunks;
  char name[112];
  snprintf(name, sizeof name, "rowmajor V%d W%d KG%d g%lld epib%d xl%d pfg%d", V, W, KG, (long long)grid, EPIB, XLM,
           (int)PFG);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_rowmajor<AccF32, T, OP, V, D, W, KG, true, EPIB, false, XLM, PFG>),
                               dim3((unsigned)grid), dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

template <int V, int D, int W, int KG, int OP, typename T, int EPIB = (V >= 2 ? 2 : V)>
Variant make_rowmajor(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                      double bytes, int64_t grid) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (grid > chunks) grid = chunks;
  char name[96];
  snprintf(name, sizeof name, "rowmajor V%d D%d W%d KG%d g%lld epib%d", V, D, W, KG, (long long)grid, EPIB);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_rowmajor<AccF32, T, OP, V, D, W, KG, true, EPIB>), dim3((unsigned)grid),
                               dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

// row-major groups over the first (1 - tail) of the window, then W-KiB strips claimed from a
// device counter (reduce_kernel_rowmajor_tail); the counter is cleared on the stream before every
// launch (part of the timed work, as in the product)
template <int V, int D, int W, int KG, int TD, int OP, typename T>
Variant make_rmtail(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                    double bytes, int64_t grid, double tail, int* work) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (grid > chunks) grid = chunks;
  const int64_t ns = (int64_t)((double)ncols * (1.0 - tail)) / 256 * 256;
  char name[96];
  snprintf(name, sizeof name, "rmtail V%d W%d KG%d TD%d g%lld t%.3f", V, W, KG, TD, (long long)grid, tail);
  return {name, bytes,
          [=] {
            CK(hipMemsetAsync(work, 0, sizeof(int), 0));
            hipLaunchKernelGGL((reduce_kernel_rowmajor_tail<AccF32, T, OP, V, D, W, KG, true, TD>), dim3((unsigned)grid),
                               dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ns, ncols, e, work);
          },
          true, {}};
}

template <int W, int DW, int L, int OP, typename T>
Variant make_lds(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e, double bytes) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  char name[96];
  snprintf(name, sizeof name, "lds W%d DW%d L%d g%lld", W, DW, L, (long long)chunks);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_lds<AccF32, T, OP, W, DW, L, true>), dim3((unsigned)chunks), dim3(64 * W), 0,
                               0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          true, {}};
}

// the opt-in split-N kernel (reordered sum: not bit-checked here)
template <int OP, typename T>
Variant make_splitn(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e, double bytes) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  return {"splitn W4 D8 (reordered)", bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_splitn<AccF32, T, OP, 4, 8, true>), dim3((unsigned)chunks), dim3(256), 0, 0,
                               stack, stride, n, w, (int64_t)0, ncols, e);
          },
          false, {}};
}

template <int V, int W, int KG, int OP, typename T, int TM>
Variant make_dfr(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e,
                 double bytes, int64_t grid) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (grid > chunks) grid = chunks;
  char name[96];
  snprintf(name, sizeof name, "rm-dfr V%d W%d KG%d g%lld tm%d", V, W, KG, (long long)grid, TM);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_rowmajor_dfr<AccF32, T, OP, V, W, KG, true, TM>), dim3((unsigned)grid),
                               dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
          },
          TM != 0, {}};
}

// one traced launch of reduce_kernel_rowmajor<..., TR = true>: per group, the spread over blocks
// of the sweep end and the epilogue end (us from the first block's start), and the epilogue length
template <int V, int D, int W, int KG, int OP, typename T, int EB = 2>
void timeline(const float* stack, int64_t stride, int n, const float* w, int64_t ncols, Epi<T> e, int64_t grid) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (grid > chunks) grid = chunks;
  const int64_t k = (chunks + grid * W * V - 1) / (grid * W * V);
  const int groups = (int)std::min<int64_t>((k + KG - 1) / KG, 7);
  unsigned long long* tr;
  CK(hipMalloc(&tr, grid * 16 * 8));
  std::vector<unsigned long long> h(grid * 16);
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipMemset(tr, 0, grid * 16 * 8));
    e.trace = tr;
    hipLaunchKernelGGL((reduce_kernel_rowmajor<AccF32, T, OP, V, D, W, KG, true, EB, true>),
                       dim3((unsigned)grid), dim3(64 * W), 0, 0, stack, stride, n, w, (int64_t)0, ncols, e);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), tr, grid * 16 * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (int64_t b = 0; b < grid; ++b) t0 = std::min(t0, h[b * 16]);
    auto stat = [&](int slot, const char* what) {
      std::vector<double> us;
      for (int64_t b = 0; b < grid; ++b)
        if (h[b * 16 + slot]) us.push_back((h[b * 16 + slot] - t0) / 100.0);  // 100 MHz
      if (us.empty()) return;
      std::sort(us.begin(), us.end());
      printf("  %-12s min %8.1f  p10 %8.1f  med %8.1f  p90 %8.1f  max %8.1f us\n", what, us[0],
             us[us.size() / 10], us[us.size() / 2], us[us.size() * 9 / 10], us.back());
    };
    printf("timeline V%d D%d W%d KG%d g%lld k%lld op%d epib%d rep %d\n", V, D, W, KG, (long long)grid, (long long)k,
           OP, EB, rep);
    stat(0, "start");
    {  // the last epilogue end per XCD (blocks are dispatched to the 8 XCDs round-robin)
      const int last = 2 + 2 * (groups - 1);
      printf("  end by XCD  ");
      for (int x = 0; x < 8; ++x) {
        double s = 0;
        int c = 0;
        for (int64_t b = x; b < grid; b += 8)
          if (h[b * 16 + last]) s += (h[b * 16 + last] - t0) / 100.0, ++c;
        printf(" %7.1f", c ? s / c : 0.0);
      }
      printf(" us (mean)\n");
    }
    for (int gi = 0; gi < groups; ++gi) {
      char a[32], b2[32];
      snprintf(a, sizeof a, "g%d sweep", gi);
      snprintf(b2, sizeof b2, "g%d epi", gi);
      stat(1 + 2 * gi, a);
      stat(2 + 2 * gi, b2);
      std::vector<double> d;
      for (int64_t b = 0; b < grid; ++b)
        if (h[b * 16 + 2 + 2 * gi]) d.push_back((h[b * 16 + 2 + 2 * gi] - h[b * 16 + 1 + 2 * gi]) / 100.0);
      if (d.empty()) continue;
      std::sort(d.begin(), d.end());
      printf("  g%d epi len   min %8.1f  med %8.1f  max %8.1f us\n", gi, d[0], d[d.size() / 2], d.back());
    }
  }
  CK(hipFree(tr));
}

template <int V, int U, int OP, typename T>
Variant make_blocked(const float* stack, int n, const float* w, int64_t ncols, Epi<T> e, double bytes) {
  const int64_t B = 256 * V * 4;
  const int64_t tiles = (ncols + B - 1) / B;
  char name[96];
  snprintf(name, sizeof name, "blocked-buf V%d U%d", V, U);
  return {name, bytes,
          [=] {
            hipLaunchKernelGGL((reduce_kernel_blocked<AccF32, T, OP, V, U, true>), dim3((unsigned)tiles), dim3(256),
                               0, 0, stack, n, w, ncols, e);
          },
          false, {}};
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 100;
  const int64_t ncols = argc > 2 ? atoll(argv[2]) : 11699136;
  const int rounds = argc > 3 ? atoi(argv[3]) : 7;
  const char* opname = argc > 4 ? argv[4] : "mean";
  const int op = !strcmp(opname, "avgm") ? FA_OP_AVGM : !strcmp(opname, "adagrad") ? FA_OP_ADAGRAD : FA_OP_MEAN;
  const bool avgm = op != FA_OP_MEAN;  // any fused epilogue
  const int64_t pad = argc > 5 ? atoll(argv[5]) : 0;  // extra row-stride elements (bank-conflict probe)
  const int64_t stride = (ncols + 63) / 64 * 64 + pad;

  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("# device %s  CUs %d  n=%d ncols=%lld op=%s stride=%lld\n", prop.gcnArchName,
         prop.multiProcessorCount, n, (long long)ncols, opname, (long long)stride);

  float *stack, *w, *out32, *prev, *sink, *copy_dst;
  double* v;
  // room for the column-blocked layout too: every tile (up to 16384 columns) holds N full rows
  const int64_t blocked_cols = (ncols + 16383) / 16384 * 16384;
  const size_t stack_elems = (size_t)n * (size_t)(stride > blocked_cols ? stride : blocked_cols);
  CK(hipMalloc(&stack, stack_elems * 4));
  CK(hipMemset(stack, 0, stack_elems * 4));
  CK(hipMalloc(&w, n * 4));
  CK(hipMalloc(&out32, stride * 4));
  CK(hipMalloc(&prev, stride * 4));
  CK(hipMalloc(&v, stride * 8));
  CK(hipMalloc(&sink, 4096));
  int* work;
  CK(hipMalloc(&work, 256));
  const int64_t copy_quads = (int64_t)n * stride / 8;  // copy half the stack into the other half
  copy_dst = stack + copy_quads * 4;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(4096, n), dim3(256), 0, 0, stack, stride, stride, 2024ull,
                     (int64_t)0, (int64_t)0);
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(4096, 1), dim3(256), 0, 0, prev, stride, stride, 1ull,
                     (int64_t)0, (int64_t)0);
  std::vector<float> ones(n, 1.0f);
  CK(hipMemcpy(w, ones.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(v, 0, stride * 8));
  CK(hipDeviceSynchronize());

  Epi<double> e{};
  e.denom = (double)n;
  e.out32 = out32;
  e.beta = 0.9;
  e.eta = 0.1;
  e.tau = 1e-9;
  if (avgm) {
    e.prev = prev;
    e.v = v;
  }
  if (avgm && getenv("TUNE_V2") && atoi(getenv("TUNE_V2"))) {  // double-buffered v_t (the product's form)
    double* vdb;
    CK(hipMalloc(&vdb, stride * 8));
    e.v_out = vdb;
  }
  const double bytes = (double)n * ncols * 4 + ncols * 4 + (avgm ? ncols * (4.0 + 16.0) : 0.0);

  std::vector<Variant> vs;
  const int cus = prop.multiProcessorCount;
#define ONESHOT(V, U, NT)                                                                             \
  vs.push_back(op == FA_OP_AVGM      ? make_oneshot<V, U, NT, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes) \
               : op == FA_OP_ADAGRAD ? make_oneshot<V, U, NT, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes) \
                                     : make_oneshot<V, U, NT, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes))
#define BAL(V, U, G4)                                                                                     \
  vs.push_back(op == FA_OP_AVGM      ? make_balanced<V, U, true, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes, cus, G4) \
               : op == FA_OP_ADAGRAD ? make_balanced<V, U, true, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes, cus, G4) \
                                     : make_balanced<V, U, true, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes, cus, G4))
  const char* set = getenv("TUNE_SET") ? getenv("TUNE_SET") : "main";
  ONESHOT(2, 8, true);  // previous product geometry first: the bitwise reference for the others
  ONESHOT(8, 4, true);
  if (!strcmp(set, "roof")) {
    const int64_t q = (int64_t)n * stride / 4;
    auto add_roof = [&](auto kern, int B, int waves_per_simd) {
      // blocks per CU = waves_per_simd (4 waves per 256-thread block, one per SIMD)
      const int lds = waves_per_simd >= 8 ? 0 : (160 * 1024) / waves_per_simd - 64;
      const int grid = cus * waves_per_simd;
      char name[96];
      snprintf(name, sizeof name, "roof burst B%d occ%d", B, waves_per_simd);
      vs.push_back({name, (double)(q / (256 * B)) * 256 * B * 16,
                    [=] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, stack, q, sink); }, false, {}});
    };
    for (int occ : {8, 4, 3, 2}) {
      add_roof(roof_burst<1>, 1, occ);
      add_roof(roof_burst<4>, 4, occ);
      add_roof(roof_burst<16>, 16, occ);
    }
  }
#define ONESHOTB(V, U)                                                                                       \
  vs.push_back(op == FA_OP_AVGM      ? make_oneshot<V, U, true, FA_OP_AVGM, double, true>(stack, stride, n, w, ncols, e, bytes) \
               : op == FA_OP_ADAGRAD ? make_oneshot<V, U, true, FA_OP_ADAGRAD, double, true>(stack, stride, n, w, ncols, e, bytes) \
                                     : make_oneshot<V, U, true, FA_OP_MEAN, double, true>(stack, stride, n, w, ncols, e, bytes))
#define BALB(V, U, G4)                                                                                    \
  vs.push_back(op == FA_OP_AVGM      ? make_balanced<V, U, true, FA_OP_AVGM, double, true>(stack, stride, n, w, ncols, e, bytes, cus, G4) \
               : op == FA_OP_ADAGRAD ? make_balanced<V, U, true, FA_OP_ADAGRAD, double, true>(stack, stride, n, w, ncols, e, bytes, cus, G4) \
                                     : make_balanced<V, U, true, FA_OP_MEAN, double, true>(stack, stride, n, w, ncols, e, bytes, cus, G4))
#define BLOCKED(V, U)                                                                                    \
  vs.push_back(op == FA_OP_AVGM      ? make_blocked<V, U, FA_OP_AVGM, double>(stack, n, w, ncols, e, bytes)   \
               : op == FA_OP_ADAGRAD ? make_blocked<V, U, FA_OP_ADAGRAD, double>(stack, n, w, ncols, e, bytes) \
                                     : make_blocked<V, U, FA_OP_MEAN, double>(stack, n, w, ncols, e, bytes))
  if (!strcmp(set, "blocked")) {
    ONESHOT(16, 1, true);
    ONESHOTB(16, 1);
    BALB(16, 1, 0);
    BLOCKED(16, 1);
    BLOCKED(16, 2);
    BLOCKED(8, 1);
    BLOCKED(8, 2);
    BLOCKED(4, 4);
    BLOCKED(4, 8);
    BLOCKED(2, 8);
    BLOCKED(1, 16);
  }
  if (!strcmp(set, "buf")) {
    ONESHOT(16, 1, true);
    ONESHOTB(16, 1);
    ONESHOTB(12, 1);
    ONESHOTB(8, 1);
    BAL(16, 1, 0);
    BALB(16, 1, 0);
    BALB(16, 1, 1);
    BALB(12, 1, 0);
    BALB(8, 1, 0);
    BALB(8, 2, 0);
    BALB(4, 4, 0);
  }
  if (!strcmp(set, "balance")) {
    ONESHOT(16, 1, true);
    ONESHOT(15, 1, true);
    ONESHOT(14, 1, true);
    ONESHOT(12, 1, true);
    ONESHOT(10, 1, true);
    BAL(16, 1, 0);
    BAL(12, 1, 0);
  }
#define ROWSG(V, D, W, G)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rows<V, D, W, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_rows<V, D, W, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_rows<V, D, W, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes, G))
#define ROWS(V, D, W) ROWSG(V, D, W, 0)
#define ROWSC(V, D, W, G)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rows<V, D, W, FA_OP_AVGM, double, false>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_rows<V, D, W, FA_OP_ADAGRAD, double, false>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_rows<V, D, W, FA_OP_MEAN, double, false>(stack, stride, n, w, ncols, e, bytes, G))
#define ROWSX(V, D, W, G, XM, NTL)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rows<V, D, W, FA_OP_AVGM, double, true, XM, NTL>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_rows<V, D, W, FA_OP_ADAGRAD, double, true, XM, NTL>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_rows<V, D, W, FA_OP_MEAN, double, true, XM, NTL>(stack, stride, n, w, ncols, e, bytes, G))
#define RM(V, D, W, KG, G)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rowmajor<V, D, W, KG, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_rowmajor<V, D, W, KG, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_rowmajor<V, D, W, KG, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes, G))
#define RME(V, D, W, KG, G, EB)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rowmajor<V, D, W, KG, FA_OP_AVGM, double, EB>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_rowmajor<V, D, W, KG, FA_OP_ADAGRAD, double, EB>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_rowmajor<V, D, W, KG, FA_OP_MEAN, double, EB>(stack, stride, n, w, ncols, e, bytes, G))
#define DFR(V, W, KG, G, TM)                                                                               \
  vs.push_back(op == FA_OP_AVGM      ? make_dfr<V, W, KG, FA_OP_AVGM, double, TM>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_dfr<V, W, KG, FA_OP_ADAGRAD, double, TM>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_dfr<V, W, KG, FA_OP_MEAN, double, TM>(stack, stride, n, w, ncols, e, bytes, G))
#define NARROW(D, W)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_narrow<D, W, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes)   \
               : op == FA_OP_ADAGRAD ? make_narrow<D, W, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes) \
                                     : make_narrow<D, W, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes))
  if (!strcmp(set, "deep3")) {  // wider windows (3..30 chunks per block): row kernel vs one-wave narrow blocks
    ROWSG(1, 16, 4, 192);
    ROWSG(2, 8, 4, 192);
    ROWSG(4, 4, 4, 192);
    ROWSG(8, 2, 4, 192);
    NARROW(16, 1);
    NARROW(32, 1);
    NARROW(40, 1);
  }
#define NARROWLB(LB, D)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_narrow_lb<LB, D, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes)   \
               : op == FA_OP_ADAGRAD ? make_narrow_lb<LB, D, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes) \
                                     : make_narrow_lb<LB, D, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes))
#define RMXL(KG, EB, XLM)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rowmajor_xl<16, 1, 4, KG, FA_OP_AVGM, double, EB, XLM>(stack, stride, n, w, ncols, e, bytes, 192)   \
               : op == FA_OP_ADAGRAD ? make_rowmajor_xl<16, 1, 4, KG, FA_OP_ADAGRAD, double, EB, XLM>(stack, stride, n, w, ncols, e, bytes, 192) \
                                     : make_rowmajor_xl<16, 1, 4, KG, FA_OP_MEAN, double, EB, XLM>(stack, stride, n, w, ncols, e, bytes, 192))
#define RMXLG(KG, EB, XLM, G)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_rowmajor_xl<16, 1, 4, KG, FA_OP_AVGM, double, EB, XLM>(stack, stride, n, w, ncols, e, bytes, G)   \
               : op == FA_OP_ADAGRAD ? make_rowmajor_xl<16, 1, 4, KG, FA_OP_ADAGRAD, double, EB, XLM>(stack, stride, n, w, ncols, e, bytes, G) \
                                     : make_rowmajor_xl<16, 1, 4, KG, FA_OP_MEAN, double, EB, XLM>(stack, stride, n, w, ncols, e, bytes, G))
  if (!strcmp(set, "xlg")) {  // KG = 4 shapes: the product (KG 4, no XL) vs KG 3 with XL on a grid whose k splits in 3s
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    int64_t g3 = 192;
    for (int64_t gg = 184; gg <= 216; ++gg) {
      const int64_t kk = (chunks + gg * 64 - 1) / (gg * 64);
      if (kk % 3 == 0) { g3 = gg; break; }
    }
    printf("# KG 3 grid %lld\n", (long long)g3);
    for (int rep = 0; rep < 2; ++rep) {
      RMXL(4, 4, 0);
      if (g3 == 192) { RMXLG(3, 4, 1, 192); RMXLG(3, 4, 0, 192); }
      else if (g3 == 196) { RMXLG(3, 4, 1, 196); RMXLG(3, 4, 0, 196); }
      else if (g3 == 200) { RMXLG(3, 4, 1, 200); RMXLG(3, 4, 0, 200); }
      else if (g3 == 204) { RMXLG(3, 4, 1, 204); RMXLG(3, 4, 0, 204); }
      else { RMXLG(3, 4, 1, 208); RMXLG(3, 4, 0, 208); }
    }
  }
  if (!strcmp(set, "xl")) {  // whole-line f64 stores (LDS regrouping) off / on, the product geometry, each twice
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + 192 * 64 - 1) / (192 * 64);
    if (k % 3 == 0) {
      RMXL(3, 4, 0);
      RMXL(3, 4, 1);
      RMXL(3, 4, 0);
      RMXL(3, 4, 1);
    } else {
      RMXL(4, 4, 0);
      RMXL(4, 4, 1);
      RMXL(4, 4, 0);
      RMXL(4, 4, 1);
    }
  }
  if (!strcmp(set, "pfg")) {  // cross-group prefetch (the next group's first step before the epilogue stores)
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + 192 * 64 - 1) / (192 * 64);
    const int kg = k % 3 == 0 ? 3 : 4;
    printf("# k %lld KG %d\n", (long long)k, kg);
#define PFGV(KG, EB, PF)                                                                                           \
  vs.push_back(op == FA_OP_AVGM      ? make_rowmajor_pfg<16, 1, 4, KG, FA_OP_AVGM, double, EB, -1, PF>(stack, stride, n, w, ncols, e, bytes, 192) \
               : op == FA_OP_ADAGRAD ? make_rowmajor_pfg<16, 1, 4, KG, FA_OP_ADAGRAD, double, EB, -1, PF>(stack, stride, n, w, ncols, e, bytes, 192) \
                                     : make_rowmajor_pfg<16, 1, 4, KG, FA_OP_MEAN, double, EB, -1, PF>(stack, stride, n, w, ncols, e, bytes, 192))
    for (int rep = 0; rep < 2; ++rep) {
      if (kg == 3) {
        if (op == FA_OP_MEAN) { PFGV(3, 2, false); PFGV(3, 2, true); } else { PFGV(3, 4, false); PFGV(3, 4, true); }
      } else {
        if (op == FA_OP_MEAN) { PFGV(4, 2, false); PFGV(4, 2, true); } else { PFGV(4, 4, false); PFGV(4, 4, true); }
      }
    }
#undef PFGV
  }
  if (!strcmp(set, "nostore")) {  // NS product geometry (KG 3) with and without its fp32 result stores
    for (int rep = 0; rep < 3; ++rep) {
      RMXL(3, 2, -1);
      Epi<double> e2 = e;
      e2.out32 = nullptr;  // every result store dropped by the descriptor's empty range
      Variant v = make_rowmajor_xl<16, 1, 4, 3, FA_OP_MEAN, double, 2, -1>(stack, stride, n, w, ncols, e2, bytes, 192);
      v.name += " NOSTORE";
      v.checks_output = false;
      vs.push_back(v);
    }
  }
  if (!strcmp(set, "xl4")) {  // KG = 4 (C5): whole-line f64 stores at epilogue batch 1 / 2 (no scratch) vs the product
    for (int rep = 0; rep < 2; ++rep) {
      RMXL(4, 4, 0);
      RMXL(4, 1, 1);
      RMXL(4, 2, 1);
      RMXL(4, 1, 0);
      vs.push_back(op == FA_OP_AVGM ? make_rowmajor_xl<8, 1, 8, 4, FA_OP_AVGM, double, 4, 1>(stack, stride, n, w, ncols, e, bytes, 192)
                                    : make_rowmajor_xl<8, 1, 8, 4, FA_OP_ADAGRAD, double, 4, 1>(stack, stride, n, w, ncols, e, bytes, 192));
    }
  }
  if (!strcmp(set, "nlb")) {  // narrow strips per wave (LB bytes per lane) vs the product's narrow kernel
    NARROW(40, 1);
    NARROW(32, 1);
    NARROWLB(4, 16);
    NARROWLB(4, 32);
    NARROWLB(4, 48);
    NARROWLB(4, 60);
    NARROWLB(8, 16);
    NARROWLB(8, 32);
    NARROWLB(8, 48);
    NARROWLB(8, 60);
  }
  if (!strcmp(set, "deep2")) {  // the narrow-window kernel: depth, waves per block
    ROWSG(1, 32, 1, 192);
    NARROW(16, 1);
    NARROW(32, 1);
    NARROW(40, 1);
    NARROW(48, 1);
    NARROW(56, 1);
    NARROW(60, 1);
    NARROW(32, 2);
    NARROW(60, 2);
  }
  if (!strcmp(set, "deep")) {  // windows of ~1 chunk per block (small P, deep N): pipeline depth per wave
    ROWSG(1, 16, 4, 192);
    ROWSG(1, 16, 1, 192);
    ROWSG(1, 32, 1, 192);
    ROWSG(1, 48, 1, 192);
    ROWSG(1, 60, 1, 192);
    ROWSG(2, 24, 1, 192);
    ROWSG(1, 32, 2, 192);
    ROWSG(1, 16, 1, 256);
    ROWSG(1, 48, 1, 256);
  }
  if (!strcmp(set, "dfr")) {  // deferred group epilogues (LDS-stashed sums) vs the product geometries
    RM(16, 1, 4, 3, 192);
    RM(16, 1, 4, 4, 192);
    RM(8, 1, 8, 4, 192);
    RM(16, 1, 4, 4, 196);
    RM(16, 1, 4, 2, 196);
    RM(8, 1, 8, 2, 196);
    DFR(16, 4, 2, 196, 2);
    DFR(16, 4, 2, 196, 0);
    DFR(8, 8, 2, 196, 2);
    DFR(8, 8, 2, 196, 0);
    DFR(8, 8, 1, 192, 2);
    DFR(8, 8, 1, 192, 0);
  }
#define RMT(V, D, W, KG, TD, G, TAIL)                                                                            \
  vs.push_back(op == FA_OP_AVGM      ? make_rmtail<V, D, W, KG, TD, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes, G, TAIL, work)   \
               : op == FA_OP_ADAGRAD ? make_rmtail<V, D, W, KG, TD, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes, G, TAIL, work) \
                                     : make_rmtail<V, D, W, KG, TD, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes, G, TAIL, work))
  if (!strcmp(set, "tail")) {  // row-major groups + a dynamically claimed tail of W-KiB strips
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + 192 * 64 - 1) / (192 * 64);
    if (k % 3 == 0) {
      RM(16, 1, 4, 3, 192);  // the product geometry of NS / C3 (first: the bitwise reference)
    } else {
      RM(16, 1, 4, 4, 192);  // C5 (k = 28)
    }
    RM(8, 1, 8, 4, 192);
    RMT(16, 1, 4, 4, 16, 192, 0.11);  // 8 pieces of ~58 chunks static (2 groups of 4) + ~11% strips
    RMT(16, 1, 4, 4, 16, 192, 0.06);
    RMT(16, 1, 4, 4, 16, 192, 0.16);
    RMT(8, 1, 8, 4, 8, 192, 0.11);
    RMT(16, 1, 4, 3, 16, 192, 0.11);
    RMT(16, 1, 4, 2, 16, 192, 0.11);
    RMT(16, 1, 4, 4, 16, 208, 0.11);
    RMT(16, 1, 4, 4, 8, 192, 0.11);
  }
#define LDSK(W, DW, L)                                                                                      \
  vs.push_back(op == FA_OP_AVGM      ? make_lds<W, DW, L, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes)   \
               : op == FA_OP_ADAGRAD ? make_lds<W, DW, L, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes) \
                                     : make_lds<W, DW, L, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes))
  if (!strcmp(set, "lds")) {  // LDS-staged bit-exact narrow kernel vs the one-wave narrow kernel and split-N
    NARROW(40, 1);
    NARROW(32, 1);
    LDSK(4, 8, 3);
    LDSK(4, 8, 4);
    LDSK(4, 8, 5);
    LDSK(4, 4, 6);
    LDSK(4, 4, 10);
    LDSK(4, 16, 2);
    LDSK(4, 16, 3);
    LDSK(4, 12, 4);
    vs.push_back(op == FA_OP_AVGM      ? make_splitn<FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, bytes)
                 : op == FA_OP_ADAGRAD ? make_splitn<FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, bytes)
                                       : make_splitn<FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, bytes));
  }
  if (!strcmp(set, "nsgrid")) {  // north-star shape: group size / grid / piece width
    RM(8, 1, 8, 3, 192);
    RM(8, 1, 8, 3, 208);
    RM(8, 1, 8, 3, 240);
    RM(8, 1, 8, 4, 192);
    RM(8, 1, 8, 5, 176);
    RM(8, 1, 8, 2, 192);
    RM(16, 1, 4, 3, 192);
    RM(16, 1, 4, 4, 192);
    RM(16, 1, 4, 2, 192);
    RM(16, 1, 4, 5, 176);
    RM(16, 1, 4, 3, 208);
    RM(16, 1, 4, 4, 224);
    RM(16, 1, 4, 3, 176);
  }
  if (!strcmp(set, "timeline")) {  // phase timestamps of the product geometry (printed after the timing)
    RM(16, 1, 4, 3, 192);
    RM(16, 1, 4, 4, 192);
  }
  if (!strcmp(set, "epinT")) {  // product geometry; built twice (-DFA_EPI_STORE_AUX / LOAD_AUX) for the A/B
    RM(16, 1, 4, 3, 192);
    RM(16, 1, 4, 4, 192);
    RM(8, 1, 8, 4, 192);
  }
  if (!strcmp(set, "kgrid")) {  // fewer, larger groups from a grid a few blocks off 192 (k = 8 / KG 4 at 196)
    RM(16, 1, 4, 3, 192);
    RM(16, 1, 4, 4, 196);
    RM(16, 1, 4, 4, 200);
    RM(16, 1, 4, 4, 208);
    RM(16, 1, 4, 2, 192);
    RM(8, 1, 8, 4, 196);
  }
  if (!strcmp(set, "epiw")) {  // fused epilogues: 8 waves x 8 KiB vs 4 waves x 16 KiB steps
    RME(8, 1, 8, 4, 192, 2);
    RME(8, 1, 8, 3, 192, 2);
    RME(16, 1, 4, 4, 192, 2);
    RME(16, 1, 4, 3, 192, 2);
    RME(16, 1, 4, 2, 192, 2);
    RME(16, 1, 4, 4, 192, 1);
    RME(16, 1, 4, 3, 192, 1);
  }
  if (!strcmp(set, "inplace")) {  // product geometry, separate out32 vs out32 == prev (bench.py's in-place step)
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + 192 * 64 - 1) / (192 * 64);
    const int kg = k % 3 == 0 ? 3 : 4;
    double* v2 = nullptr;
    if (avgm) CK(hipMalloc(&v2, stride * 8));
    for (int rep = 0; rep < 2; ++rep) {
      for (int mode = 0; mode < 4; ++mode) {  // bit 0: out32 == prev; bit 1: v_out = a second v
        const int inpl = mode & 1;
        if (!avgm && mode) continue;
        Epi<double> e2 = e;
        if (inpl && avgm) e2.out32 = prev;
        if (mode & 2) e2.v_out = v2;
        Variant v = kg == 3 ? (op == FA_OP_AVGM      ? make_rowmajor<16, 1, 4, 3, FA_OP_AVGM, double, 4>(stack, stride, n, w, ncols, e2, bytes, 192)
                               : op == FA_OP_ADAGRAD ? make_rowmajor<16, 1, 4, 3, FA_OP_ADAGRAD, double, 4>(stack, stride, n, w, ncols, e2, bytes, 192)
                                                     : make_rowmajor<16, 1, 4, 3, FA_OP_MEAN, double, 4>(stack, stride, n, w, ncols, e2, bytes, 192))
                            : (op == FA_OP_AVGM      ? make_rowmajor<16, 1, 4, 4, FA_OP_AVGM, double, 4>(stack, stride, n, w, ncols, e2, bytes, 192)
                               : op == FA_OP_ADAGRAD ? make_rowmajor<16, 1, 4, 4, FA_OP_ADAGRAD, double, 4>(stack, stride, n, w, ncols, e2, bytes, 192)
                                                     : make_rowmajor<16, 1, 4, 4, FA_OP_MEAN, double, 4>(stack, stride, n, w, ncols, e2, bytes, 192));
        if (mode & 2) v.name += " v2";
        if (inpl && avgm) {
          v.name += " inplace";
          v.checks_output = false;
        }
        vs.push_back(v);
      }
    }
  }
  if (!strcmp(set, "epib4")) {  // product EPIB 2 vs 4, each twice (the duplicates gauge the noise)
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + 192 * 64 - 1) / (192 * 64);
    if (k % 3 == 0) {
      RME(16, 1, 4, 3, 192, 2);
      RME(16, 1, 4, 3, 192, 4);
      RME(16, 1, 4, 3, 192, 2);
      RME(16, 1, 4, 3, 192, 4);
    } else {
      RME(16, 1, 4, 4, 192, 2);
      RME(16, 1, 4, 4, 192, 4);
      RME(16, 1, 4, 4, 192, 2);
      RME(16, 1, 4, 4, 192, 4);
    }
  }
  if (!strcmp(set, "epib16")) {  // the product's 4-wave x 16 KiB geometry: epilogue batch size B
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + 192 * 64 - 1) / (192 * 64);
    if (k % 3 == 0) {
      RME(16, 1, 4, 3, 192, 2);  // product (first: the bitwise reference)
      RME(16, 1, 4, 3, 192, 1);
      RME(16, 1, 4, 3, 192, 4);
      RME(16, 1, 4, 3, 192, 8);
    } else {
      RME(16, 1, 4, 4, 192, 2);  // product
      RME(16, 1, 4, 4, 192, 1);
      RME(16, 1, 4, 4, 192, 4);
      RME(16, 1, 4, 4, 192, 8);
    }
    RME(16, 1, 4, 2, 192, 2);  // half the accumulators: no AGPR traffic in the sweep
    RME(8, 1, 8, 2, 192, 2);
    RME(8, 1, 8, 4, 192, 2);
  }
  if (!strcmp(set, "epib")) {  // piece epilogue: per-quad guarded loads (0) vs batched buffer loads of B slots
    RME(8, 1, 8, 4, 192, 0);
    RME(8, 1, 8, 4, 192, 2);
    RME(8, 1, 8, 4, 192, 4);
    RME(8, 1, 8, 4, 192, 8);
    RME(8, 1, 8, 3, 192, 0);
    RME(8, 1, 8, 3, 192, 4);
    RME(8, 1, 8, 2, 192, 4);
  }
  if (!strcmp(set, "rmgrid")) {  // row-major: grid / group size around the product's choice
    RM(8, 1, 8, 5, 176);
    RM(8, 1, 8, 4, 192);
    RM(8, 1, 8, 4, 208);
    RM(8, 1, 8, 4, 224);
    RM(8, 1, 8, 3, 240);
    RM(8, 1, 8, 3, 192);
    RM(8, 1, 8, 2, 208);
    RM(8, 1, 8, 3, 256);
  }
  if (!strcmp(set, "rm")) {  // row-major multi-piece sweep vs the column-major product geometry
    ROWSG(16, 1, 4, 192);
    ROWSG(8, 1, 8, 192);
    RM(8, 1, 8, 4, 192);
    RM(4, 2, 8, 8, 192);
    RM(4, 2, 8, 4, 192);
    RM(8, 2, 4, 4, 192);
    RM(4, 4, 4, 4, 192);
    RM(8, 1, 8, 4, 224);
  }
  if (!strcmp(set, "epi")) {  // fused-epilogue geometry: 4 vs 8 waves per block
    ROWSG(16, 1, 4, 224);
    ROWSG(16, 1, 4, 192);
    ROWSG(8, 1, 8, 160);
    ROWSG(8, 1, 8, 192);
    ROWSG(8, 1, 8, 224);
    ROWSG(8, 1, 8, 256);
    ROWSG(4, 2, 8, 192);
    ROWSG(2, 4, 8, 192);
    ROWSG(1, 8, 8, 192);
  }
  if (!strcmp(set, "misc")) {
    ROWSX(16, 1, 4, 192, false, true);
    ROWSX(16, 1, 4, 192, true, true);
    ROWSX(16, 1, 4, 192, false, false);
    ROWSX(8, 1, 8, 192, false, true);
    ROWSX(8, 2, 8, 192, false, true);
    ROWSX(4, 4, 8, 192, false, true);
    ROWSX(16, 1, 4, 256, true, true);
  }
  if (!strcmp(set, "one")) {  // the product geometry against the roofs
    ONESHOTB(16, 1);
    ROWSG(16, 1, 4, 192);
    ROWSG(16, 1, 4, 224);
    ROWSG(16, 1, 4, 256);
    ROWSG(32, 1, 4, 192);
  }
  if (!strcmp(set, "il")) {  // interleaved vs contiguous piece assignment
    ONESHOTB(16, 1);
    for (int g : {160, 192, 224, 256}) {
      ROWSG(16, 1, 4, g);
      ROWSC(16, 1, 4, g);
      ROWSG(8, 2, 4, g);
      ROWSC(8, 2, 4, g);
    }
    ROWSG(4, 4, 4, 192);
    ROWSC(4, 4, 4, 192);
    ROWSG(16, 2, 4, 192);
  }
  if (!strcmp(set, "inflight")) {  // blocks vs bytes in flight per block
    ONESHOTB(16, 1);
    ROWSG(16, 1, 4, 192);
    ROWSG(16, 1, 4, 160);
    ROWSG(16, 1, 4, 176);
    ROWSG(16, 1, 4, 208);
    ROWSG(12, 1, 4, 256);
    ROWSG(12, 1, 4, 192);
    ROWSG(8, 1, 4, 384);
    ROWSG(8, 1, 4, 256);
    ROWSG(16, 1, 3, 256);
    ROWSG(16, 1, 2, 384);
    ROWSG(16, 1, 2, 512);
    ROWSG(8, 2, 4, 192);
    ROWSG(4, 4, 4, 192);
    ROWSG(4, 3, 4, 256);
  }
  if (!strcmp(set, "grid")) {  // balanced row pipeline: how many resident blocks stream best
    ONESHOTB(16, 1);
    for (int g : {128, 192, 224, 256, 384, 512}) {
      ROWSG(16, 1, 4, g);
      ROWSG(8, 2, 4, g);
      ROWSG(4, 4, 4, g);
    }
    ROWSG(16, 2, 4, 256);
    ROWSG(2, 8, 4, 256);
    ROWSG(1, 16, 4, 256);
  }
  if (!strcmp(set, "rows")) {  // row-pipelined grid vs the product geometries
    ONESHOTB(16, 1);
    BALB(16, 1, 0);
    BALB(4, 8, 0);
    ROWS(1, 16, 1);
    ROWS(2, 8, 1);
    ROWS(4, 4, 1);
    ROWS(4, 8, 1);
    ROWS(2, 8, 4);
    ROWS(4, 4, 4);
    ROWS(4, 8, 4);
    ROWS(8, 2, 4);
    ROWS(8, 4, 4);
    ROWS(16, 1, 4);
    ROWS(16, 2, 4);
  }
  if (!strcmp(set, "narrow")) {  // many rows x few columns: per-rank shards of the multi-GPU runs
    BAL(4, 4, 0);
    BAL(4, 8, 0);
    BAL(2, 8, 0);
    BAL(2, 16, 0);
    BAL(1, 16, 0);
    BAL(4, 4, 1);
    BALB(4, 4, 0);
    BALB(4, 8, 0);
    BALB(8, 4, 0);
    BALB(16, 1, 0);
    ONESHOTB(16, 1);
  }
  if (!strcmp(set, "main")) {
    ONESHOT(4, 1, true);
    ONESHOT(8, 1, true);
    ONESHOT(16, 1, true);
    BAL(4, 1, 0);
    BAL(4, 1, 1);
    BAL(8, 1, 0);
    BAL(8, 1, 1);
    BAL(16, 1, 0);
    BAL(16, 1, 1);
    BAL(4, 4, 0);
    BAL(8, 2, 0);
  }
  const int64_t quads = (int64_t)n * stride / 4;
  vs.push_back({"roof: stream read N*P", (double)n * stride * 4,
                [=] { hipLaunchKernelGGL(read_roof, dim3(cus * 8), dim3(256), 0, 0, stack, quads, sink); },
                false, {}});
  vs.push_back({"roof: float4 copy (R+W)", (double)copy_quads * 32,
                [=] {
                  hipLaunchKernelGGL(copy_roof, dim3(cus * 8), dim3(256), 0, 0, stack, copy_dst, copy_quads);
                },
                false, {}});

  // reference output of the product geometry
  std::vector<float> ref(ncols), got(ncols);
  std::vector<double> v_save;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // warm up + correctness (state-free for mean; for avgm reset v before each checked launch)
  for (size_t i = 0; i < vs.size(); ++i) {
    if (!vs[i].checks_output) continue;
    CK(hipMemset(v, 0, stride * 8));
    vs[i].launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(i == 0 ? ref.data() : got.data(), out32, ncols * 4, hipMemcpyDeviceToHost));
    if (i > 0 && memcmp(ref.data(), got.data(), ncols * 4) != 0) {
      printf("MISMATCH %s\n", vs[i].name.c_str());
      return 2;
    }
  }
  // copy_roof overwrites the second half of the stack: run the roofs after the checks, and the
  // reduce variants only read, so timings stay valid.
  // TUNE_FLUSH=1: every timed launch starts from cold caches (a 1-GiB memset between launches
  // evicts L2 and the 256-MiB Infinity Cache), each launch timed alone
  const bool flush = getenv("TUNE_FLUSH") && atoi(getenv("TUNE_FLUSH"));
  void* flush_buf = nullptr;
  if (flush) CK(hipMalloc(&flush_buf, (size_t)1 << 30));
  for (int r = 0; r < rounds; ++r) {
    for (auto& var : vs) {
      var.launch();  // warm
      const int reps = 5;
      float ms = 0.f;
      if (flush) {
        for (int k = 0; k < reps; ++k) {
          CK(hipMemsetAsync(flush_buf, k & 0xff, (size_t)1 << 30, 0));
          CK(hipEventRecord(a, 0));
          var.launch();
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float t;
          CK(hipEventElapsedTime(&t, a, b));
          ms += t;
        }
      } else {
        CK(hipEventRecord(a, 0));
        for (int k = 0; k < reps; ++k) var.launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
      }
      var.times.push_back(ms / reps);
    }
  }
  printf("%-28s %10s %10s %10s %8s\n", "variant", "med_us", "min_us", "GB/s(med)", "%8TB/s");
  for (auto& var : vs) {
    std::sort(var.times.begin(), var.times.end());
    const double med = var.times[var.times.size() / 2], mn = var.times[0];
    const double gbs = var.bytes / 1e9 / (med / 1e3);
    printf("%-28s %10.1f %10.1f %10.1f %8.2f\n", var.name.c_str(), med * 1e3, mn * 1e3, gbs, gbs / 80.0);
  }
  if (!strcmp(set, "timeline")) {
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t kk = (chunks + 192 * 64 - 1) / (192 * 64);
    if (op == FA_OP_AVGM) {
      timeline<16, 1, 4, 3, FA_OP_AVGM, double>(stack, stride, n, w, ncols, e, 192);
    } else if (op == FA_OP_ADAGRAD) {
      timeline<16, 1, 4, 4, FA_OP_ADAGRAD, double>(stack, stride, n, w, ncols, e, 192);
    } else if (kk % 3 == 0) {
      timeline<16, 1, 4, 3, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, 192);
    } else {
      timeline<16, 1, 4, 4, FA_OP_MEAN, double>(stack, stride, n, w, ncols, e, 192);
    }
  }
  return 0;
}
