// fa_reduce.hip — C ABI of the FedAVG-family aggregation engine (include/flearn_amd.h).
//
// Host side only: argument validation, dtype/mode dispatch and launches of the gfx950 kernels in
// fa_device.hpp on the caller's stream.  No allocation, no synchronisation, no host copies.
// Geometry (measured with tools/tune_reduce.hip on MI355X):
//   * fp32 client stacks (every configuration of the hot path): the row-pipelined kernel on
//     192 blocks (0.75 per CU) with equal interleaved pieces of the window; each block sweeps its
//     pieces (V KiB x W waves wide; W = 4 for the mean, 8 with a fused optimizer epilogue), rows
//     pipelined D = 64/(V*W) deep through per-row buffer descriptors (~64 KiB of client rows in
//     flight per block, whatever the window's width or depth);
//   * 8-byte kinds (f64 / i64 buckets, small): 4 quads per thread, one row at a time.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <string>
#include <vector>

#include "fa_device.hpp"
#include "flearn_amd.h"

namespace {

using namespace fa;

thread_local std::string g_last_error;

int fail(int code, const char* what) {
  g_last_error = what;
  return code;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
constexpr bool kNT = true;  // client bytes are read once: non-temporal

template <class P>
struct Geometry;  // 8-byte kinds only; fp32 stacks use the row pipeline
template <>
struct Geometry<AccF64> {
  static constexpr int kSmallV = 4, kSmallU = 1;
};
template <>
struct Geometry<AccI64> {
  static constexpr int kSmallV = 4, kSmallU = 1;
};

int device_cus() {
  static thread_local int dev = -1, cus = 0;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 256;
  if (d != dev) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || cus <= 0)
      cus = 256;
    dev = d;
  }
  return cus;
}

template <typename K>
int resident_blocks_per_cu(K kernel) {
  static int occ = 0;  // per kernel instantiation
  if (occ == 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kernel, kThreads, 0) != hipSuccess || o <= 0) o = 1;
    occ = o;
  }
  return occ;
}

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

// fp32 client stacks.  Fewer blocks than CUs stream best: ~192 blocks on 256 CUs,
// each keeping ~64 KiB of client rows in flight, equal interleaved pieces of the window.
//   * several pieces per block (k >= 2): reduce_kernel_rowmajor, 8 waves x 8 KiB per piece,
//     rows swept once per group of KG pieces (fp32 sums only: f64 sums need 2x the registers);
//   * one piece per block: reduce_kernel_rows; the piece width and pipeline depth follow the
//     share s (KiB of every row per block): the narrowest piece that covers s, D = 64/(V*W) rows
//     deep.  Plain mean: 4 waves x up to 16 KiB per row; fused optimizer epilogues: 8 waves x up
//     to 8 KiB (half the per-lane state work at every piece end, twice the waves to overlap it).
constexpr double kRowsBlocksPerCU = 0.75;
constexpr int kPieceChunks = 64;  // max KiB of a row per block and piece (= W * Vmax)

template <class P, typename T, int OP, int V, int W>
int launch_rows(const float* stack, int64_t stride, int n, const typename P::w_t* w, int64_t col0,
                int64_t ncols, const Epi<T>& e, int64_t grid, hipStream_t s) {
  static_assert(V * W <= kPieceChunks, "piece wider than the in-flight budget");
  hipLaunchKernelGGL((reduce_kernel_rows<P, T, OP, V, kPieceChunks / (V * W), W, kNT>), dim3((unsigned)grid),
                     dim3(64 * W), 0, s, stack, stride, n, w, col0, ncols, e);
  return launch_check();
}

template <class P, typename T, int OP, int D>
int launch_narrow(const float* stack, int64_t stride, int n, const typename P::w_t* w, int64_t col0,
                  int64_t ncols, const Epi<T>& e, int64_t grid, hipStream_t s) {
  hipLaunchKernelGGL((reduce_kernel_narrow<P, T, OP, D, 1, kNT>), dim3((unsigned)grid), dim3(64), 0, s, stack, stride,
                     n, w, col0, ncols, e);
  return launch_check();
}

template <class P, typename T, int OP, int KG>
int launch_rowmajor(const float* stack, int64_t stride, int n, const typename P::w_t* w, int64_t col0,
                    int64_t ncols, const Epi<T>& e, int64_t grid, hipStream_t s) {
  // The same 64-KiB pieces either as 8 waves x 8 KiB or as 4 waves x 16 KiB.  With several groups
  // per block (k >= 6) 4 waves stream ~1% faster — plain mean 100 x 25.6 M: 86.6 vs 85.8% and
  // 85.1 vs 83.7% on two boxes, 100 x 86.6 M: 83.2 vs 82.3% (profiles/r02/tune_nsgrid); fused
  // AVGM 100 x 25.6 M: 85.7 vs 84.4%, Adagrad 100 x 86.6 M: 85.1 vs 84.1% (profiles/r02/tune_epiw)
  // — with one group (C2, C4) they do not (84.2 vs 85.0%, 89.7 vs 89.8%, AVGM 83.2 vs 83.4%).
  // Yogi's f64 epilogue does not fit 4 x 16 quads of sums (144 spilled VGPRs)
  if constexpr (KG <= 3 || (KG == 4 && !(OP == FA_OP_YOGI && sizeof(T) == 8))) {
    const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
    const int64_t k = (chunks + grid * kPieceChunks - 1) / (grid * kPieceChunks);
    if (k >= 6) {
      // fused epilogues batch the state of 4 slots per lane (EPIB 4) instead of 2: one process,
      // 9 interleaved rounds, each variant twice (tools/tune_reduce.hip set "epib4",
      // profiles/r03/tune_epib4/): Adagrad 100 x 86.6 M 5315 -> 5272 us, AVGM 100 x 25.6 M
      // 1599 -> 1595 us, AVGM 100 x 11.7 M 711 -> 707 us; the plain mean has no state (+-0.1%)
      constexpr int EB = OP == FA_OP_MEAN ? 2 : 4;
      hipLaunchKernelGGL((reduce_kernel_rowmajor<P, T, OP, 16, 1, 4, KG, kNT, EB>), dim3((unsigned)grid), dim3(256), 0,
                         s, stack, stride, n, w, col0, ncols, e);
      return launch_check();
    }
  }
  hipLaunchKernelGGL((reduce_kernel_rowmajor<P, T, OP, 8, 1, 8, KG, kNT>), dim3((unsigned)grid), dim3(512), 0, s,
                     stack, stride, n, w, col0, ncols, e);
  return launch_check();
}

// Row-major geometry for windows of several 64-KiB pieces per block (k >= 2): a grid near 192
// blocks whose k splits into equal groups of KG in {4, 3, 2} pieces (every step of a group is
// a real piece).  Returns false when no grid in [160, cus] gives such a k.
bool rowmajor_geometry(int64_t chunks, int cus, int64_t target, int64_t* grid, int* kg) {
  const int64_t lo = 160 < cus ? 160 : cus, hi = cus;
  for (int64_t d = 0; d <= hi - lo; ++d) {
    for (int sgn = 0; sgn < 2; ++sgn) {
      const int64_t g = sgn ? target - d : target + d;
      if (g < lo || g > hi || (d == 0 && sgn)) continue;
      const int64_t k = (chunks + g * kPieceChunks - 1) / (g * kPieceChunks);
      if (k < 2) return false;  // one piece per block: the column-major kernel
      for (int c : {4, 3, 2}) {  // (5 x 8 quads of sums + the pipeline do not fit 256 VGPRs)
        if (k % c == 0) {
          *grid = g;
          *kg = c;
          return true;
        }
      }
    }
  }
  return false;
}

// The widest grid of one-piece blocks (reduce_kernel_rows) the geometry below uses: 13/16 of the
// CUs (100 x 3.2 M columns on 196 blocks 89.7-90.1%, 100 x 3.5 M on 214 blocks 88.6%)
int64_t rows_grid_max(int cus) { return (int64_t)cus * 13 / 16; }

// fa_set_reduce_grid: 0 = the geometry below chooses the grid
std::atomic<int> g_reduce_grid{0};

// KG for a forced grid: the group size in {4, 3, 2} that wastes the fewest group slots
int kg_for(int64_t k) {
  int best = 4;
  int64_t waste = (k + 3) / 4 * 4 - k;
  for (int c : {3, 2}) {
    const int64_t wc = (k + c - 1) / c * c - k;
    if (wc < waste) {
      waste = wc;
      best = c;
    }
  }
  return best;
}

template <class P, typename T, int OP>
int launch_reduce_window(const typename P::x_t* stack, int64_t stride, int n, const void* w, int64_t col0,
                         int64_t ncols, const Epi<T>& e, hipStream_t s) {
  const typename P::w_t* wt = static_cast<const typename P::w_t*>(w);
  const int cus = device_cus();
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;  // 1-KiB row pieces
  const int forced = g_reduce_grid.load(std::memory_order_relaxed);
  if constexpr (sizeof(typename P::x_t) == 4) {
    if constexpr (sizeof(typename P::acc_t) == 4) {  // fp32 sums (every flearn weight type but f64)
      int64_t g = 0;
      int kg = 0;
      if (forced > 0 && chunks > (int64_t)forced * kPieceChunks) {
        g = forced;
        kg = kg_for((chunks + g * kPieceChunks - 1) / (g * kPieceChunks));
        switch (kg) {
          case 2: return launch_rowmajor<P, T, OP, 2>(stack, stride, n, wt, col0, ncols, e, g, s);
          case 3: return launch_rowmajor<P, T, OP, 3>(stack, stride, n, wt, col0, ncols, e, g, s);
          default: return launch_rowmajor<P, T, OP, 4>(stack, stride, n, wt, col0, ncols, e, g, s);
        }
      }
      // Past one round of the grid: row-major groups.  So also where one piece per block would
      // take more than rows_grid_max blocks — two pieces per block on a grid near 13/16 of the
      // CUs instead (100 x 4.19 M columns: 256 one-piece blocks 246 us = 86.0%, 208 blocks x 2
      // pieces 235 us = 90.2%; tools/width_sweep.py, profiles/r06/width/)
      const bool past = chunks > (int64_t)cus * kPieceChunks;
      if (forced <= 0 && chunks > rows_grid_max(cus) * kPieceChunks &&
          rowmajor_geometry(chunks, cus, past ? (int64_t)(cus * kRowsBlocksPerCU + 0.5) : (int64_t)cus * 13 / 16, &g,
                            &kg)) {
        switch (kg) {
          case 2: return launch_rowmajor<P, T, OP, 2>(stack, stride, n, wt, col0, ncols, e, g, s);
          case 3: return launch_rowmajor<P, T, OP, 3>(stack, stride, n, wt, col0, ncols, e, g, s);
          default: return launch_rowmajor<P, T, OP, 4>(stack, stride, n, wt, col0, ncols, e, g, s);
        }
      }
    }
    int64_t grid = forced > 0 ? forced : (int64_t)(cus * kRowsBlocksPerCU + 0.5);
    // a window just wider than one round of full pieces: a few more blocks (up to one per CU)
    // instead of a second, nearly empty round
    if (forced <= 0 && chunks > grid * kPieceChunks && chunks <= (int64_t)cus * kPieceChunks)
      grid = (chunks + kPieceChunks - 1) / kPieceChunks;
    if (grid < 1) grid = 1;
    if (grid > chunks) grid = chunks;
    int64_t share = (chunks + grid - 1) / grid;  // chunks per block
    if (share <= 2) {
      // narrow windows (at most two 1-KiB chunks of every row per block: LeNet-sized models, deep
      // client stacks): reduce_kernel_narrow, one single-wave block per chunk, a D-deep pipeline
      // with no drain code and the round's weights broadcast from one VGPR.  A 4- or 8-wave
      // block had work for one or two waves (8-16 KiB in flight per block).  1000 x LeNet5 51.1
      // -> 31.8 us, 2000 clients 98.3 -> 55.6 us, 400 clients 27.5 -> 15.7 us, 100 clients
      // 9.8 -> 7.4 us, 300 x 70,001 -> 17.2 us (tools/tune_reduce.hip sets "deep", "deep2";
      // profiles/r02/tune_deep/).  D: 16 rows below 350 clients (the ramp of a deeper pipeline
      // does not pay off), 32 below 700, else 40 (48-60 lose: fewer waves' worth of latency
      // hiding per row than the issue cost of the extra slots).  Same sums, same order.
      const int64_t g1 = chunks;
      if (n < 350) return launch_narrow<P, T, OP, 16>(stack, stride, n, wt, col0, ncols, e, g1, s);
      if (n < 700) return launch_narrow<P, T, OP, 32>(stack, stride, n, wt, col0, ncols, e, g1, s);
      return launch_narrow<P, T, OP, 40>(stack, stride, n, wt, col0, ncols, e, g1, s);
    }
    if constexpr (OP == FA_OP_MEAN) {
      constexpr int W = 4;
      // A share just past a power of two leaves about half of every pipeline slot empty (the
      // piece is V*W KiB wide, `share` KiB of it real, D = 64/(V*W) rows deep).  Where a grid of
      // at most rows_grid_max blocks makes the share a whole power of two, take that grid: plain
      // mean 100 x 1.6 M columns 95.1 -> 90.3-90.8 us, 100 x 800 K 48.6 -> 46.5 us; shares >= 60% full
      // (100 x 2.4 M, 1.2 M, 600 K, 200 K) lose with it, and so do the fused epilogues
      // (tools/width_sweep.py, profiles/r06/width/)
      if (forced <= 0) {
        int64_t cap = W;
        while (cap < share) cap *= 2;
        const int64_t g2 = (chunks + cap / 2 - 1) / (cap / 2);
        if (cap > W && share * 5 < cap * 3 && g2 <= rows_grid_max(cus)) {
          grid = g2;
          share = (chunks + grid - 1) / grid;
        }
      }
      if (share <= 1 * W) return launch_rows<P, T, OP, 1, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
      if (share <= 2 * W) return launch_rows<P, T, OP, 2, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
      if (share <= 4 * W) return launch_rows<P, T, OP, 4, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
      if (share <= 8 * W) return launch_rows<P, T, OP, 8, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
      return launch_rows<P, T, OP, 16, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
    } else {
      constexpr int W = 8;
      // shares of at most 8 KiB on 4 waves: with 8 waves one quad per lane (V = 1, 8 rows deep)
      // compiles into register copies — 240 VGPRs, scratch spills and ~1,290 v_mov_b64 per
      // kernel, for every epilogue — and 100 x 200 K FedAVGM took 45 us, 3x the plain mean
      if (share <= 4) return launch_rows<P, T, OP, 1, 4>(stack, stride, n, wt, col0, ncols, e, grid, s);
      if (share <= 8) return launch_rows<P, T, OP, 2, 4>(stack, stride, n, wt, col0, ncols, e, grid, s);
      // a share just past 16 or 32 KiB: the grid that makes it a whole 16 / 32 KiB piece, on 4
      // waves (the mean's rule; 8 waves lose there): FedAVGM 100 x 1.6 M 85.0 -> 88.4-88.6%,
      // 100 x 800 K 83.0 -> 85.8-86.0%; shares of 9-16 KiB stay on 8 waves (100 x 400 K: 77.9%
      // against 75.6-75.9% filled on 4; tools/width_sweep.py, profiles/r06/width/fused_*)
      if (forced <= 0 && share > 16) {
        const int64_t cap = share <= 32 ? 32 : 64;
        const int64_t g2 = (chunks + cap / 2 - 1) / (cap / 2);
        if (share * 5 < cap * 3 && g2 <= rows_grid_max(cus)) {
          grid = g2;
          share = (chunks + grid - 1) / grid;
          if (share <= 16) return launch_rows<P, T, OP, 4, 4>(stack, stride, n, wt, col0, ncols, e, grid, s);
          return launch_rows<P, T, OP, 8, 4>(stack, stride, n, wt, col0, ncols, e, grid, s);
        }
      }
      if (share <= 2 * W) return launch_rows<P, T, OP, 2, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
      if (share <= 4 * W) return launch_rows<P, T, OP, 4, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
      return launch_rows<P, T, OP, 8, W>(stack, stride, n, wt, col0, ncols, e, grid, s);
    }
  } else {
    // 8-byte kinds (f64 / i64 buckets: BN counters, float64 state; small): 4 quads per thread,
    // one row at a time, round-balanced grid
    typedef Geometry<P> G;
    auto kern = reduce_kernel_balanced<P, T, OP, G::kSmallV, G::kSmallU, kNT>;
    const int64_t slots = (int64_t)cus * resident_blocks_per_cu(kern);
    const int64_t grid = chunks < slots ? chunks : slots;
    hipLaunchKernelGGL(kern, dim3((unsigned)(grid > 0 ? grid : 1)), dim3(kThreads), 0, s, stack, stride, n, wt,
                       col0, ncols, e);
    return launch_check();
  }
}

// Wide fp32 windows as several launches over consecutive column windows of the same stack
// (round 5, tools/probe_slabs.py --windows, profiles/r05/c5/: same stack, same allocation,
// interleaved rounds, two allocations each).  Each window gets its own row-major geometry (grid,
// KG, groups per block), and these splits measured faster than one launch: fused epilogues at
// 16 M+ columns in 3 windows — FedOPT-Adagrad 100 x 86.6 M 5282/5270 -> 5190/5211 us, FedAVGM
// 100 x 86.6 M 5260/5249 -> 5177/5183, FedAVGM 100 x 25.6 M 1561/1564 -> 1542/1544 (2 windows:
// 1574/1572, slower); plain means of 8-16 M columns in 2 — 100 x 11.7 M 666/665 -> 660/661,
// 1000 x 11.7 M 6481/6486 -> 6441/6437 (3 windows: 6545).  The plain mean of 25.6 M (NS) stays
// one launch (2 windows 0.2-0.4% slower), as does 86.6 M (no consistent gain).  Per column the
// sums and epilogue are unchanged: bit-identical results.  Not with a forced grid (ABI 7).
template <int OP>
int window_count(int64_t ncols) {
  if (OP != FA_OP_MEAN) return ncols >= ((int64_t)16 << 20) ? 3 : 1;
  return (ncols >= ((int64_t)8 << 20) && ncols < ((int64_t)16 << 20)) ? 2 : 1;
}

template <typename T>
Epi<T> epi_at(const Epi<T>& e, int64_t c) {  // the epilogue's per-column arrays from column c on
  Epi<T> o = e;
  if (o.prev) o.prev += c;
  if (o.v) o.v += c;
  if (o.v_out) o.v_out += c;
  if (o.h) o.h += c;
  if (o.out32) o.out32 += c;
  if (o.out64) o.out64 += c;
  return o;
}

template <class P, typename T, int OP>
int launch_reduce(const typename P::x_t* stack, int64_t stride, int n, const void* w, int64_t col0,
                  int64_t ncols, const Epi<T>& e, hipStream_t s) {
  int S = 1;
  if constexpr (sizeof(typename P::x_t) == 4 && sizeof(typename P::acc_t) == 4)
    if (g_reduce_grid.load(std::memory_order_relaxed) <= 0) S = window_count<OP>(ncols);
  if (S <= 1) return launch_reduce_window<P, T, OP>(stack, stride, n, w, col0, ncols, e, s);
  const int64_t width = (ncols + S - 1) / S / 256 * 256 + 256;  // 1-KiB chunks of a row: 16-B aligned
  for (int64_t c = 0; c < ncols; c += width) {
    const int64_t wc = ncols - c < width ? ncols - c : width;
    if (int rc = launch_reduce_window<P, T, OP>(stack, stride, n, w, col0 + c, wc, epi_at(e, c), s)) return rc;
  }
  return FA_OK;
}

// Segmented row-pointer reduce (fa_reduce_f32_rows): reduce_kernel_segrows_rm — blocks claim
// groups of kSegKG wide pieces (at most kSegPieceChunks KiB of a row each) and sweep them row by
// row, one 64-KiB step (8 waves x 8 KiB) in flight like the stack kernel's row-major groups; then
// the narrow pieces one by one through a 16-deep one-quad sweep.  192 blocks (tools/tune_rows.py,
// profiles/r02/tune_rows/: grouped 100 x ResNet-18 85.7% = the stack kernel's, against 81-84% for
// one claimed piece at a time).  Plain mean: 4 waves x 8 KiB, D = 2; fused epilogues: 8 waves
// x 4 KiB, D = 2.
constexpr int kSegPieceChunks = 64;
constexpr double kSegBlocksPerCU = 0.75;
constexpr int kSegW = 8, kSegV = 8, kSegKG = 2;                // row-major groups of 2 pieces, 8 x 8 KiB
constexpr int64_t kSegWideCols = (int64_t)64 * kSegW * 4;      // wider pieces go into groups

template <class P, typename T, int OP>
int launch_segrows(const float* const* rows, int n, const void* w, const fa_piece* pieces, int64_t npieces,
                   int grid, int32_t* work, const Epi<T>& e, hipStream_t s) {
  const typename P::w_t* wt = static_cast<const typename P::w_t*>(w);
  // f64 sums (np.float64 weights) need twice the accumulator registers: one piece per group
  constexpr int KG = sizeof(typename P::acc_t) == 8 ? 1 : kSegKG;
  // fused f64 state: whole-line stores (FedAVGM 100 x ResNet-50 uploads in place 1647.6 -> 1633.8 us,
  // bit-identical: tools/probe_rows_xl.py, profiles/r05/rows_xl/)
  constexpr bool XLS = sizeof(T) == 8 && OP != FA_OP_MEAN;
  hipLaunchKernelGGL((reduce_kernel_segrows_rm<P, T, OP, kSegV, kSegW, KG, 16, kNT, false, 1, false, 0, 0, XLS>),
                     dim3((unsigned)grid), dim3(64 * kSegW), 0, s, rows, n, wt, pieces, npieces, work, e);
  return launch_check();
}

template <class P, typename T>
int dispatch_segrows(int op, const float* const* rows, int n, const void* w, const fa_piece* pieces,
                     int64_t npieces, int grid, int32_t* work, const Epi<T>& e, hipStream_t s) {
  switch (op) {
    case FA_OP_MEAN: return launch_segrows<P, T, FA_OP_MEAN>(rows, n, w, pieces, npieces, grid, work, e, s);
    case FA_OP_AVGM: return launch_segrows<P, T, FA_OP_AVGM>(rows, n, w, pieces, npieces, grid, work, e, s);
    case FA_OP_ADAGRAD: return launch_segrows<P, T, FA_OP_ADAGRAD>(rows, n, w, pieces, npieces, grid, work, e, s);
    case FA_OP_YOGI: return launch_segrows<P, T, FA_OP_YOGI>(rows, n, w, pieces, npieces, grid, work, e, s);
    case FA_OP_ADAM: return launch_segrows<P, T, FA_OP_ADAM>(rows, n, w, pieces, npieces, grid, work, e, s);
    case FA_OP_DYN: return launch_segrows<P, T, FA_OP_DYN>(rows, n, w, pieces, npieces, grid, work, e, s);
    default: return fail(FA_ERR_ARG, "unknown epilogue op");
  }
}

// Split-N geometry (tools/tune_splitn.py, profiles/r02/tune_splitn): one 1-KiB chunk of every row
// per block, kSplitW client splits (one per wave), each a rolling pipeline kSplitD rows deep.
// 1000 x 44,416 fp32: 28.7 us vs 50.2 us sequential; 4000 x 44,416: 111 vs 184 us; but
// 1000 x 1 M (3907 chunks): 738 vs 572 us — so the split form is used only for windows of fewer
// 1-KiB chunks than CUs, and with at least 2 * kSplitW clients.  And at most kSplitMaxN clients:
// a reordered fp32 sum differs from the sequential one by about the sequential sum's own rounding
// error, which grows like sqrt(N), and the contract is <= 1e-6 per tensor.  The exact CPU
// restatement of both orders (tests/splitn_error.py, profiles/r03/splitn_error.json; LeNet5
// tensors, 3 seeds x 3 weight kinds x 2 data kinds) puts the worst tensor at 6.2e-7 for N = 256,
// 7.4e-7 at 512, 2.5e-6 at 1024 (a 6-element bias, MOON weights), 1.3e-6 at 2048 — so 256.
// Columns whose terms nearly cancel are re-summed in order by the kernel's guard.
constexpr int kSplitW = 4, kSplitD = 8, kSplitMaxN = 256;
constexpr int kSplitS = kSplitW;

template <class P, typename T, int OP>
int launch_splitn(const float* stack, int64_t stride, int n, const void* w, int64_t col0, int64_t ncols,
                  const Epi<T>& e, hipStream_t s) {
  const int64_t chunks = ((ncols + 3) / 4 + 63) / 64;
  if (n < 2 * kSplitS || n > kSplitMaxN || chunks >= device_cus())  // see kSplitMaxN
    return launch_reduce<P, T, OP>(stack, stride, n, w, col0, ncols, e, s);
  hipLaunchKernelGGL((reduce_kernel_splitn<P, T, OP, kSplitW, kSplitD, kNT>), dim3((unsigned)chunks),
                     dim3(64 * kSplitW), 0, s, stack, stride, n, static_cast<const typename P::w_t*>(w), col0, ncols, e);
  return launch_check();
}

template <class P, typename T>
int dispatch_splitn(int op, const float* stack, int64_t stride, int n, const void* w, int64_t col0, int64_t ncols,
                    const Epi<T>& e, hipStream_t s) {
  switch (op) {
    case FA_OP_MEAN: return launch_splitn<P, T, FA_OP_MEAN>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_AVGM: return launch_splitn<P, T, FA_OP_AVGM>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_ADAGRAD: return launch_splitn<P, T, FA_OP_ADAGRAD>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_YOGI: return launch_splitn<P, T, FA_OP_YOGI>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_ADAM: return launch_splitn<P, T, FA_OP_ADAM>(stack, stride, n, w, col0, ncols, e, s);
    case FA_OP_DYN: return launch_splitn<P, T, FA_OP_DYN>(stack, stride, n, w, col0, ncols, e, s);
    default: return fail(FA_ERR_ARG, "unknown epilogue op");
  }
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
    case FA_OP_DYN: return launch_reduce<P, T, FA_OP_DYN>(stack, stride, n, w, col0, ncols, e, s);
    default: return fail(FA_ERR_ARG, "unknown epilogue op");
  }
}

bool aligned_to(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

// [a, a + bytes) and [b, b + bytes) share a byte
bool overlaps(const void* a, const void* b, size_t bytes) {
  const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
  return x < y + bytes && y < x + bytes;
}

// ncols: the columns the launch touches (0: unknown — only the exact-alias check applies)
template <typename T>
int make_epi(const fa_epilogue* in, double denom, int n_reduced, float* out32, double* out64, Epi<T>* e,
             int64_t ncols = 0) {
  e->denom = (T)denom;
  e->prev = nullptr;
  e->v = nullptr;
  e->h = nullptr;
  e->trace = nullptr;
  e->v_out = nullptr;
  e->beta = e->eta = e->tau = e->beta2 = e->c = e->n = T(0);
  e->alpha32 = 0.f;
  e->out32 = out32;
  e->out64 = out64;
  if (!in || in->op == FA_OP_MEAN) return FA_OK;
  if (in->op < FA_OP_AVGM || in->op > FA_OP_DYN) return fail(FA_ERR_ARG, "unknown epilogue op");
  if (!in->v) return fail(FA_ERR_ARG, "epilogue needs v");
  e->v = static_cast<T*>(in->v);
  if (in->v_out) {
    if (!aligned_to(in->v_out, 4 * sizeof(T))) return fail(FA_ERR_ALIGN, "v_out must be 4-element aligned");
    if (in->v_out == in->v || (ncols > 0 && overlaps(in->v_out, in->v, (size_t)ncols * sizeof(T))))
      return fail(FA_ERR_ARG, "v_out must be NULL (in place) or an array not overlapping v");
    e->v_out = static_cast<T*>(in->v_out);
  }
  if (in->op == FA_OP_DYN) {
    if (!in->h) return fail(FA_ERR_ARG, "FedDyn epilogue needs h");
    const double nc = in->n_clients > 0 ? in->n_clients : (double)n_reduced;
    if (!(nc >= 1)) return fail(FA_ERR_ARG, "FedDyn epilogue needs n_clients >= 1");
    e->h = in->h;
    e->n = (T)nc;
    e->c = (T)(in->alpha / nc);  // self.alpha / len(w_local_lst): a Python float   dyn.py:26
    e->alpha32 = (float)in->alpha;
    return FA_OK;
  }
  if (!in->prev) return fail(FA_ERR_ARG, "epilogue needs prev and v");
  e->prev = in->prev;
  e->beta = (T)in->beta;
  e->eta = (T)in->eta;
  e->tau = (T)in->tau;
  e->beta2 = (T)in->beta2;
  e->c = (T)(1.0 - in->beta2);  // Python evaluates (1 - self.beta2) in double
  return FA_OK;
}


// per-column arrays are accessed with 4-element vector loads/stores
int check_columns(const float* out32, const double* out64, const void* prev, const void* v,
                  size_t v_elem, const float* h = nullptr) {
  if (!aligned_to(out32, 16) || !aligned_to(out64, 32) || !aligned_to(prev, 16) ||
      !aligned_to(v, 4 * v_elem) || !aligned_to(h, 16))
    return fail(FA_ERR_ALIGN, "output / prev / v / h arrays must be 4-element aligned");
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

namespace {
// Piece cut of one segment: `pc` chunks at most, equal pieces (the last one takes the remainder)
template <typename F>
void cut_segment(int64_t len, int64_t pc, F&& emit) {
  const int64_t chunks = (len + 255) / 256;
  if (chunks == 0) return;
  const int64_t np = (chunks + pc - 1) / pc;
  const int64_t per = (chunks + np - 1) / np * 256;  // columns per piece, whole 1-KiB chunks
  for (int64_t off = 0; off < len; off += per) emit(off, len - off < per ? len - off : per);
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
                          mode == FA_MODE_W32_DIV32 ? sizeof(float) : sizeof(double),
                          epi ? epi->h : nullptr)))
    return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == FA_MODE_W32_DIV64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, n_clients, out32, out64, &e, n_cols))) return rc;
    return dispatch_op<AccF32, double>(op, stack, row_stride, n_clients, weights, col_begin, n_cols,
                                       e, s);
  }
  if (mode == FA_MODE_W32_DIV32) {
    Epi<float> e;
    if ((rc = make_epi<float>(epi, denom, n_clients, out32, out64, &e, n_cols))) return rc;
    return dispatch_op<AccF32, float>(op, stack, row_stride, n_clients, weights, col_begin, n_cols,
                                      e, s);
  }
  if (mode == FA_MODE_W64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, n_clients, out32, out64, &e, n_cols))) return rc;
    return dispatch_op<AccF32W64, double>(op, stack, row_stride, n_clients, weights, col_begin,
                                          n_cols, e, s);
  }
  return fail(FA_ERR_ARG, "unknown reduce mode");
}

int fa_reduce_f32_splitn(const float* stack, int64_t row_stride, int32_t n_clients, int32_t mode,
                         const void* weights, double denom, int64_t col_begin, int64_t n_cols,
                         const fa_epilogue* epi, float* out32, double* out64, void* stream) {
  int rc = check_common(stack, row_stride, n_clients, weights, col_begin, n_cols, out32, out64);
  if (rc) return rc;
  if (n_cols == 0) return FA_OK;
  const int op = epi ? epi->op : FA_OP_MEAN;
  if ((rc = check_columns(out32, out64, epi ? epi->prev : nullptr, epi ? epi->v : nullptr,
                          mode == FA_MODE_W32_DIV32 ? sizeof(float) : sizeof(double), epi ? epi->h : nullptr)))
    return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == FA_MODE_W32_DIV64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, n_clients, out32, out64, &e, n_cols))) return rc;
    return dispatch_splitn<AccF32, double>(op, stack, row_stride, n_clients, weights, col_begin, n_cols, e, s);
  }
  if (mode == FA_MODE_W32_DIV32) {
    Epi<float> e;
    if ((rc = make_epi<float>(epi, denom, n_clients, out32, out64, &e, n_cols))) return rc;
    return dispatch_splitn<AccF32, float>(op, stack, row_stride, n_clients, weights, col_begin, n_cols, e, s);
  }
  if (mode == FA_MODE_W64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, n_clients, out32, out64, &e, n_cols))) return rc;
    return dispatch_splitn<AccF32W64, double>(op, stack, row_stride, n_clients, weights, col_begin, n_cols, e, s);
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
  make_epi<double>(nullptr, denom, n_clients, nullptr, out64, &e);
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
  make_epi<double>(nullptr, denom, n_clients, nullptr, out64, &e);
  return launch_reduce<AccI64, double, FA_OP_MEAN>(stack, row_stride, n_clients, weights, col_begin,
                                                   n_cols, e, static_cast<hipStream_t>(stream));
}

int fa_opt_apply(int32_t prec, const fa_epilogue* epi, const float* local, const void* glob,
                 int64_t n, float* out32, double* out64, void* stream) {
  if (!epi || !glob || n < 0) return fail(FA_ERR_ARG, "bad apply arguments");
  if (!local && epi->op != FA_OP_DYN) return fail(FA_ERR_ARG, "apply needs local");
  if (!out32 && !out64) return fail(FA_ERR_ARG, "no output");
  if (n == 0) return FA_OK;
  if (epi->op == FA_OP_MEAN) return fail(FA_ERR_ARG, "apply needs an optimizer op");
  if (epi->op == FA_OP_DYN && !(epi->n_clients >= 1))
    return fail(FA_ERR_ARG, "FedDyn apply needs n_clients >= 1");
  const size_t ve = prec == FA_PREC_F32 ? sizeof(float) : sizeof(double);
  int rc0 = check_columns(out32, out64, local, epi->v, ve, epi->h);
  if (rc0) return rc0;
  if (!epi->v) return fail(FA_ERR_ARG, "apply needs v");
  fa_epilogue local_epi = *epi;
  if (epi->op != FA_OP_DYN) local_epi.prev = local;
  const int64_t blocks = (n + kThreads * 4 - 1) / (kThreads * 4);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc;
#define FA_APPLY(T, OPV)                                                                   \
  hipLaunchKernelGGL((apply_kernel<T, OPV>), dim3((unsigned)blocks), dim3(kThreads), 0, s, \
                     static_cast<const T*>(glob), n, e)
  if (prec == FA_PREC_F64) {
    Epi<double> e;
    if ((rc = make_epi<double>(&local_epi, 1.0, 1, out32, out64, &e, n))) return rc;
    switch (epi->op) {
      case FA_OP_AVGM: FA_APPLY(double, FA_OP_AVGM); break;
      case FA_OP_ADAGRAD: FA_APPLY(double, FA_OP_ADAGRAD); break;
      case FA_OP_YOGI: FA_APPLY(double, FA_OP_YOGI); break;
      case FA_OP_DYN: FA_APPLY(double, FA_OP_DYN); break;
      default: FA_APPLY(double, FA_OP_ADAM); break;
    }
  } else if (prec == FA_PREC_F32) {
    Epi<float> e;
    if ((rc = make_epi<float>(&local_epi, 1.0, 1, out32, out64, &e, n))) return rc;
    switch (epi->op) {
      case FA_OP_AVGM: FA_APPLY(float, FA_OP_AVGM); break;
      case FA_OP_ADAGRAD: FA_APPLY(float, FA_OP_ADAGRAD); break;
      case FA_OP_YOGI: FA_APPLY(float, FA_OP_YOGI); break;
      case FA_OP_DYN: FA_APPLY(float, FA_OP_DYN); break;
      default: FA_APPLY(float, FA_OP_ADAM); break;
    }
  } else {
    return fail(FA_ERR_ARG, "unknown precision");
  }
#undef FA_APPLY
  return launch_check();
}


int fa_rows_plan(int32_t n_segments, const int64_t* seg_col, const int64_t* seg_len, int32_t op,
                 int32_t grid_hint, fa_piece* pieces, int64_t cap, int64_t* n_pieces, int32_t* grid) {
  if (n_segments < 0 || (n_segments > 0 && (!seg_col || !seg_len)) || !n_pieces || !grid)
    return fail(FA_ERR_ARG, "bad rows plan arguments");
  if (op < FA_OP_MEAN || op > FA_OP_DYN) return fail(FA_ERR_ARG, "unknown epilogue op");
  for (int32_t s = 0; s < n_segments; ++s)
    if (seg_len[s] < 0 || seg_col[s] < 0 || seg_col[s] % 4 != 0)
      return fail(FA_ERR_ARG, "segment columns must be >= 0 and 4-aligned");
  const int64_t target = grid_hint > 0 ? grid_hint : (int64_t)(device_cus() * kSegBlocksPerCU + 0.5);
  // Piece width and grid: the widest pieces (<= kSegPieceChunks) and a grid near the target
  // whose KG-piece groups fill whole rounds — a group is the unit a block claims, and every slot
  // of the last round left empty is a block idling through a whole group sweep (92% fill left
  // 15 of 192 blocks idle for half of a 100 x ResNet-18 launch: tools/tune_rows.py --trace).
  // A grid hint is taken as given.
  auto count = [&](int64_t pc, int64_t* nwide) {
    int64_t all = 0, wide = 0;
    for (int32_t s = 0; s < n_segments; ++s)
      cut_segment(seg_len[s], pc, [&](int64_t, int64_t cols) {
        ++all;
        wide += cols > kSegWideCols;
      });
    *nwide = wide;
    return all;
  };
  const int64_t glo = grid_hint > 0 ? target : target - target / 8, ghi = target;
  int64_t best_pc = kSegPieceChunks, g = target, best_fill = -1;
  for (int64_t pc = kSegPieceChunks; pc >= kSegPieceChunks * 5 / 8 && best_fill < 1000; --pc) {
    int64_t nwide = 0;
    count(pc, &nwide);
    const int64_t groups = (nwide + kSegKG - 1) / kSegKG;
    for (int64_t gg = ghi; gg >= glo && gg >= 1; --gg) {
      const int64_t rounds = (groups + gg - 1) / gg;
      const int64_t fill = groups == 0 ? 1000 : groups * 1000 / (rounds * gg);  // busy share of the slots
      if (fill > best_fill) {
        best_fill = fill;
        best_pc = pc;
        g = gg;
      }
      if (fill >= 1000) break;
    }
  }
  int64_t nwide = 0;
  const int64_t total = count(best_pc, &nwide);
  const int64_t claims = (nwide + kSegKG - 1) / kSegKG + (total - nwide);
  if (g > claims) g = claims;
  *grid = (int32_t)g;
  *n_pieces = total;
  if (!pieces) return FA_OK;
  if (cap < total) return fail(FA_ERR_SIZE, "piece array too small");
  int64_t k = 0;
  for (int32_t s = 0; s < n_segments; ++s)
    cut_segment(seg_len[s], best_pc, [&](int64_t off, int64_t cols) {
      fa_piece& p = pieces[k++];
      p.col = seg_col[s] + off;
      p.seg_off = off;
      p.seg = s;
      p.n_cols = (int32_t)cols;
      p.aux = 0;
    });
  // largest first (stable: equal pieces keep bucket order): the wide pieces lead and pair into
  // groups of similar size, the narrow ones are claimed last, one at a time
  std::stable_sort(pieces, pieces + k, [](const fa_piece& a, const fa_piece& b) { return a.n_cols > b.n_cols; });
  if (k > 0) pieces[0].aux = nwide;
  return FA_OK;
}

int fa_reduce_f32_rows(const float* const* rows, int32_t n_clients, int32_t mode, const void* weights,
                       double denom, const fa_piece* pieces, int64_t n_pieces, int32_t grid, int32_t* work,
                       const fa_epilogue* epi, float* out32, double* out64, void* stream) {
  if (n_clients <= 0) return fail(FA_ERR_ARG, "n_clients must be >= 1");
  if (n_pieces < 0 || (n_pieces > 0 && (!rows || !pieces || !work))) return fail(FA_ERR_ARG, "null rows, pieces or work");
  if (n_pieces > 0 && (grid <= 0 || grid > n_pieces)) return fail(FA_ERR_ARG, "grid must be in [1, n_pieces]");
  if (!weights) return fail(FA_ERR_ARG, "null weights");
  if (!out32 && !out64) return fail(FA_ERR_ARG, "no output");
  if (n_pieces == 0) return FA_OK;
  const int op = epi ? epi->op : FA_OP_MEAN;
  int rc;
  if ((rc = check_columns(out32, out64, epi ? epi->prev : nullptr, epi ? epi->v : nullptr,
                          mode == FA_MODE_W32_DIV32 ? sizeof(float) : sizeof(double), epi ? epi->h : nullptr)))
    return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(work, 0, sizeof(int32_t), s) != hipSuccess) return fail(FA_ERR_LAUNCH, "clearing the piece counter");
  if (mode == FA_MODE_W32_DIV64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, n_clients, out32, out64, &e))) return rc;
    return dispatch_segrows<AccF32, double>(op, rows, n_clients, weights, pieces, n_pieces, grid, work, e, s);
  }
  if (mode == FA_MODE_W32_DIV32) {
    Epi<float> e;
    if ((rc = make_epi<float>(epi, denom, n_clients, out32, out64, &e))) return rc;
    return dispatch_segrows<AccF32, float>(op, rows, n_clients, weights, pieces, n_pieces, grid, work, e, s);
  }
  if (mode == FA_MODE_W64) {
    Epi<double> e;
    if ((rc = make_epi<double>(epi, denom, n_clients, out32, out64, &e))) return rc;
    return dispatch_segrows<AccF32W64, double>(op, rows, n_clients, weights, pieces, n_pieces, grid, work, e, s);
  }
  return fail(FA_ERR_ARG, "unknown reduce mode");
}

int fa_gather_rows(void* stack, int64_t row_stride, int32_t n_clients, int32_t elem_size,
                   const void* const* rows, const int64_t* segs, int32_t n_segments, void* stream) {
  if (n_clients < 0 || n_segments < 0 || row_stride < 0) return fail(FA_ERR_ARG, "bad gather sizes");
  if (n_clients == 0 || n_segments == 0) return FA_OK;
  if (!stack || !rows || !segs) return fail(FA_ERR_ARG, "null gather pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (elem_size != 4 && elem_size != 8) return fail(FA_ERR_ARG, "elem_size must be 4 or 8");
  // one launch per tile of up to 65535 clients (the grid's y limit)
  for (int32_t i0 = 0; i0 < n_clients; i0 += 65535) {
    const dim3 grid((unsigned)n_segments, (unsigned)std::min<int32_t>(65535, n_clients - i0));
    if (elem_size == 4)
      hipLaunchKernelGGL(gather_rows_kernel<uint32_t>, grid, dim3(kThreads), 0, s, static_cast<uint32_t*>(stack),
                         row_stride, n_clients, reinterpret_cast<const uint32_t* const*>(rows), segs, n_segments, i0);
    else
      hipLaunchKernelGGL(gather_rows_kernel<uint64_t>, grid, dim3(kThreads), 0, s, static_cast<uint64_t*>(stack),
                         row_stride, n_clients, reinterpret_cast<const uint64_t* const*>(rows), segs, n_segments, i0);
    if (int rc = launch_check()) return rc;
  }
  return FA_OK;
}

int fa_gather_rows_f64(double* stack, int64_t row_stride, int32_t n_clients, const void* const* rows,
                       const int64_t* segs, int32_t n_segments, void* stream) {
  if (n_clients < 0 || n_segments < 0 || row_stride < 0) return fail(FA_ERR_ARG, "bad gather sizes");
  if (n_clients == 0 || n_segments == 0) return FA_OK;
  if (!stack || !rows || !segs) return fail(FA_ERR_ARG, "null gather pointer");
  for (int32_t i0 = 0; i0 < n_clients; i0 += 65535) {
    hipLaunchKernelGGL(gather_rows_f64_kernel, dim3((unsigned)n_segments, (unsigned)std::min<int32_t>(65535, n_clients - i0)),
                       dim3(kThreads), 0, static_cast<hipStream_t>(stream), stack, row_stride, n_clients, rows, segs,
                       n_segments, i0);
    if (int rc = launch_check()) return rc;
  }
  return FA_OK;
}

int fa_reduce_windows(int32_t op, int64_t n_cols) {
  if (n_cols < 0) return fail(FA_ERR_ARG, "negative n_cols");
  if (g_reduce_grid.load(std::memory_order_relaxed) > 0) return 1;
  switch (op) {
    case FA_OP_MEAN: return window_count<FA_OP_MEAN>(n_cols);
    case FA_OP_AVGM: case FA_OP_ADAGRAD: case FA_OP_YOGI: case FA_OP_ADAM: case FA_OP_DYN:
      return window_count<FA_OP_AVGM>(n_cols);
    default: return fail(FA_ERR_ARG, "unknown epilogue op");
  }
}

int fa_set_reduce_grid(int32_t grid) {
  if (grid < 0) return fail(FA_ERR_ARG, "grid must be >= 0");
  return g_reduce_grid.exchange(grid);
}

int fa_copy(void* dst, const void* src, int64_t nbytes, void* stream) {
  if ((!dst || !src) && nbytes > 0) return fail(FA_ERR_ARG, "null copy pointer");
  if (nbytes < 0) return fail(FA_ERR_ARG, "negative copy size");
  if (nbytes == 0) return FA_OK;
  if (((uintptr_t)dst | (uintptr_t)src) & 15) return fail(FA_ERR_ALIGN, "copy pointers must be 16-byte aligned");
  // 512 blocks of 256 lanes, grid-stride: enough 16-B stores in flight for PCIe (tools/probe_zc.cpp)
  const int64_t quads = nbytes / 16;
  int64_t blocks = (quads + kThreads - 1) / kThreads;
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(copy_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), nbytes);
  return launch_check();
}

// fa_push's default grid.  The kernel is paced (each wave drains its stores per round): a block
// keeps 4 waves x 4 quads x 1 KiB = 16 KiB in flight per destination link, so 16 blocks keep
// ~256 KiB per link — about an xGMI link's bandwidth-delay product (64-153 GB/s x 1-2 us), more
// only queues in the fabric and slows a reduce beside the push.  Provisional:
// no multi-GPU run has measured it against seven xGMI links; bench.py's calibration picks the grid
// on the node and records every grid's push-beside-reduce pair, 16 included
constexpr int64_t kPushGrid = 16;

int fa_ipc_handle(const void* ptr, void* handle, int64_t* offset) {
  if (!ptr || !handle || !offset) return fail(FA_ERR_ARG, "null ipc argument");
  static_assert(sizeof(hipIpcMemHandle_t) == FA_IPC_HANDLE_BYTES, "IPC handle size");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(ptr)));
  if (e != hipSuccess) return fail(FA_ERR_ARG, hipGetErrorString(e));
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base));
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  memcpy(handle, &h, sizeof h);
  *offset = (int64_t)((const char*)ptr - (const char*)base);
  return FA_OK;
}

int fa_ipc_open(const void* handle, void** base) {
  if (!handle || !base) return fail(FA_ERR_ARG, "null ipc argument");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof h);
  const hipError_t e = hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  return FA_OK;
}

int fa_ipc_close(void* base) {
  if (!base) return fail(FA_ERR_ARG, "null ipc base");
  const hipError_t e = hipIpcCloseMemHandle(base);
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  return FA_OK;
}

int fa_dev_alloc(int64_t nbytes, void** ptr) {
  if (!ptr || nbytes <= 0) return fail(FA_ERR_ARG, "bad device allocation request");
  *ptr = nullptr;
  const hipError_t e = hipMalloc(ptr, (size_t)nbytes);
  if (e != hipSuccess) {
    *ptr = nullptr;
    return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  }
  return FA_OK;
}

int fa_dev_free(void* ptr) {
  if (!ptr) return FA_OK;
  const hipError_t e = hipFree(ptr);
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  return FA_OK;
}

int fa_mem_range(const void* ptr, void** base, int64_t* size) {
  if (!ptr || !base || !size) return fail(FA_ERR_ARG, "null range argument");
  hipDeviceptr_t b = nullptr;
  size_t n = 0;
  const hipError_t e = hipMemGetAddressRange(&b, &n, reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(ptr)));
  if (e != hipSuccess) return fail(FA_ERR_ARG, hipGetErrorString(e));
  *base = reinterpret_cast<void*>(b);
  *size = (int64_t)n;
  return FA_OK;
}

int fa_push(const void* src, int64_t nbytes, void* const* dsts, int32_t n_dsts, int32_t grid, void* stream) {
  if (nbytes < 0 || n_dsts < 0 || n_dsts > 8 || grid < 0) return fail(FA_ERR_ARG, "bad push size, destination count or grid");
  if (nbytes == 0 || n_dsts == 0) return FA_OK;
  if (!src || !dsts) return fail(FA_ERR_ARG, "null push pointer");
  PushDsts d{};
  uintptr_t any = (uintptr_t)src;
  for (int i = 0; i < n_dsts; ++i) {
    if (!dsts[i]) return fail(FA_ERR_ARG, "null push destination");
    d.p[i] = static_cast<uint8_t*>(dsts[i]);
    any |= (uintptr_t)dsts[i];
  }
  if ((any & 15) || (nbytes & 15)) return fail(FA_ERR_ALIGN, "push pointers and size must be 16-byte multiples");
  const int64_t quads = nbytes / 16;
  int64_t blocks = (quads + kThreads - 1) / kThreads;
  const int64_t cap = grid > 0 ? grid : kPushGrid;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(push_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(src), quads, d, n_dsts);
  return launch_check();
}

constexpr hipMemcpyKind kCopyEngine = hipMemcpyDeviceToDeviceNoCU;

int fa_copy_dma(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (nbytes < 0) return fail(FA_ERR_ARG, "negative copy size");
  if (nbytes == 0) return FA_OK;
  if (!dst || !src) return fail(FA_ERR_ARG, "null copy pointer");
  // NoCU: a copy engine, not the runtime's blit kernel.  With hipMemcpyDeviceToDevice the runtime
  // ran every leg as __amd_rocclr_copyBuffer kernels on the compute queues (rocprofv3, round 5:
  // profiles/r05/push_dma_trace/) — the CUs and memory pipelines the "copy-engine" push was meant
  // to leave to the reduce
  const hipError_t e = hipMemcpyAsync(dst, src, (size_t)nbytes, kCopyEngine, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  return FA_OK;
}

// one event recorded on `from`, waited for by `to` (destroyed at once: HIP releases it when done)
static int stream_after(hipStream_t to, hipStream_t from) {
  hipEvent_t ev;
  hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(ev, from);
  if (e == hipSuccess) e = hipStreamWaitEvent(to, ev, 0);
  (void)hipEventDestroy(ev);
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  return FA_OK;
}

int fa_push_dma(const void* src, int64_t nbytes, void* const* dsts, int32_t n_dsts, void* const* streams,
                void* stream) {
  if (nbytes < 0 || n_dsts < 0 || n_dsts > 8) return fail(FA_ERR_ARG, "bad push size or destination count");
  if (nbytes == 0 || n_dsts == 0) return FA_OK;
  if (!src || !dsts || !streams) return fail(FA_ERR_ARG, "null push pointer");
  for (int i = 0; i < n_dsts; ++i)
    if (!dsts[i] || !streams[i]) return fail(FA_ERR_ARG, "null push destination or stream");
  hipEvent_t ev;
  hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(ev, static_cast<hipStream_t>(stream));
  for (int i = 0; i < n_dsts && e == hipSuccess; ++i) {
    hipStream_t s = static_cast<hipStream_t>(streams[i]);
    e = hipStreamWaitEvent(s, ev, 0);
    if (e == hipSuccess) e = hipMemcpyAsync(dsts[i], src, (size_t)nbytes, kCopyEngine, s);
  }
  (void)hipEventDestroy(ev);
  if (e != hipSuccess) return fail(FA_ERR_LAUNCH, hipGetErrorString(e));
  return FA_OK;
}

int fa_cache_fence(int32_t kind, void* stream) {
  // 64 one-wave blocks: workgroups are dealt round-robin over the 8 XCDs, so every XCD's L2 gets
  // the fence from several waves
  if (kind == FA_FENCE_RELEASE)
    hipLaunchKernelGGL(cache_fence_kernel<0>, dim3(64), dim3(64), 0, static_cast<hipStream_t>(stream));
  else if (kind == FA_FENCE_ACQUIRE)
    hipLaunchKernelGGL(cache_fence_kernel<1>, dim3(64), dim3(64), 0, static_cast<hipStream_t>(stream));
  else
    return fail(FA_ERR_ARG, "unknown cache fence kind");
  return launch_check();
}

int fa_stream_join(void* stream, void* const* streams, int32_t n) {
  if (n < 0 || n > 16 || (n > 0 && !streams)) return fail(FA_ERR_ARG, "bad stream list");
  for (int i = 0; i < n; ++i) {
    const int rc = stream_after(static_cast<hipStream_t>(stream), static_cast<hipStream_t>(streams[i]));
    if (rc) return rc;
  }
  return FA_OK;
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

