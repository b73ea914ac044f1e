/*
 * flearn_amd.h — C ABI of the MI355X FedAVG-family aggregation engine.
 *
 * The reference (wnma3mz/flearn v0.0.5) is pure Python and has no FFI; every entry point below
 * replaces a numpy expression sequence inside the reference's Strategy plugins.  The reference
 * interface each function stands in for is cited (paths relative to the flearn repo root).
 *
 * Conventions (all functions):
 *   - every data pointer is a DEVICE pointer (hipMalloc / torch CUDA tensor storage) on the
 *     current HIP device, except where noted;
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream); launches are
 *     asynchronous, nothing here synchronises, allocates or frees;
 *   - a client stack is a row-major [n_clients][row_stride] array: row r holds client r's
 *     flattened bucket; the functions read the column window [col_begin, col_begin + n_cols)
 *     of every row, and index every per-column array (out32, out64, prev, v) from 0 at col_begin;
 *   - vector paths need `stack`, `col_begin` and `row_stride` aligned so that each row window
 *     starts on 16 bytes (FA_ERR_ALIGN otherwise); n_cols may be any value >= 0.  For full
 *     speed make row_stride a multiple of 64 floats (256 B, what the Python side lays out):
 *     100 x 25.6 M fp32 with a 16-B-aligned pitch streams at 85.1% of 8 TB/s, with the pitch
 *     rounded up to 64 floats at 90.1% (profiles/r06/width/pitch_unaligned_vs_aligned.jsonl);
 *   - return FA_OK (0) or a negative FA_ERR_*; fa_last_error() gives a thread-local message.
 *   - client order is the list order: client 0's product initialises the sum and clients
 *     1..n-1 are added strictly in order, with no fused multiply-add, which is what makes the
 *     fp32 path bit-identical to the reference's numpy loop.
 */
#ifndef FLEARN_AMD_H_
#define FLEARN_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_ABI_VERSION 14

/* return codes */
#define FA_OK 0
#define FA_ERR_ARG (-1)    /* bad size / null pointer / unknown enum */
#define FA_ERR_ALIGN (-2)  /* row window not 16-byte aligned */
#define FA_ERR_LAUNCH (-3) /* HIP launch error */
#define FA_ERR_SIZE (-4)        /* output buffer too small (the needed size is reported)      */
#define FA_ERR_UNSUPPORTED (-5) /* wire codec: pickle content outside the supported subset   */
#define FA_ERR_DATA (-6)        /* wire codec: malformed / non-canonical base64 or pickle     */

/* Reduce modes: how numpy (NEP 50, numpy >= 2) evaluates
 *   w = a0*x0; w += a_n*x_n; w = np.divide(w, np.sum(a))          strategy.py:123-129
 * for fp32 client tensors, by the Python type of the weights a_n.                               */
#define FA_MODE_W32_DIV64 0 /* Python float/int weights: fl32(a)*x, fp32 sum, f64 divide by the
                               f64/int64 np.sum -> float64 result (flearn default, Client.py:157) */
#define FA_MODE_W32_DIV32 1 /* np.float32 weights: fp32 product/sum, fp32 divide by the fp32
                               np.sum -> float32 result                                           */
#define FA_MODE_W64 2       /* np.float64 / np.int64 weights: f64 product, f64 sum, f64 divide   */

/* Server-side epilogues fused after the mean (the reference runs the same formulas in
 * client_receive with w_local = the client's weights; the fused server form uses
 * w_local = prev = the previous global model).                                                  */
#define FA_OP_MEAN 0    /* w = mean                                                  avg.py:25-33 */
#define FA_OP_AVGM 1    /* d = g - l; v = d + beta*v; w = l + v                    avgm.py:19-36 */
#define FA_OP_ADAGRAD 2 /* d = g - l; v = v + d*d; w = l + (eta*d)/(sqrt(v)+tau)   opt.py:52-63 */
#define FA_OP_YOGI 3    /* v = v - (c*d*d)*sign(v - d*d), c = 1-beta2               opt.py:54-58 */
#define FA_OP_ADAM 4    /* v = beta2*v + c*d*d                                      opt.py:59-60 */
#define FA_OP_DYN 5     /* FedDyn, state h (fp32) and theta (in v):                dyn.py:17-36
                           d = g*N - theta; h = fl32(h - (alpha/N)*d); w = g - fl32(alpha)*h;
                           theta = w.  In precision T (F64/F32 below) except h and alpha*h,
                           which numpy keeps fp32 (h is the model's fp32 state_dict).        */

/* Precision of the epilogue state / the mean (FA_PREC_F64 for modes DIV64 and W64,
 * FA_PREC_F32 for mode DIV32 — the dtype numpy gives w_glob in that mode).                      */
#define FA_PREC_F32 0
#define FA_PREC_F64 1

typedef struct fa_epilogue {
  int32_t op;        /* FA_OP_*                                                         */
  int32_t reserved;  /* must be 0                                                       */
  const float* prev; /* [n_cols] fp32 previous global model (AVGM/OPT), else NULL       */
  void* v;           /* [n_cols] optimizer state v_t: double* (F64) or float* (F32)     */
  double beta;       /* AVGM momentum beta (reference default 0.9, avgm.py:38)          */
  double eta;        /* OPT step size 1e-1 (opt.py:24)                                  */
  double tau;        /* OPT epsilon 1e-9 (opt.py:25)                                    */
  double beta2;      /* OPT beta2 0.99 (opt.py:27); kernels use c = 1 - beta2 and beta2 */
  float* h;          /* FA_OP_DYN: [n_cols] fp32 h, updated in place; else NULL          */
  double alpha;      /* FA_OP_DYN alpha (dyn.py:15, 0.01)                                */
  double n_clients;  /* FA_OP_DYN len(w_local_lst) (dyn.py:21,26); 0 = the reduce's N    */
  void* v_out;       /* NULL: the updated v_t / theta is written back into v (in place);
                        else [n_cols] of v's element type, not overlapping v: the updated
                        state goes here and v is only read (ABI 6)                          */
} fa_epilogue;
/* FA_OP_DYN: v is theta (double* / float*, updated to w); prev is unused.  out32 / out64 may
 * alias v or prev when they have its element type (each element is read before written).
 * Double-buffered state (out32 != prev, v_out != v, the caller swapping the pairs each round)
 * is the fast form: in place, the epilogue's stores land on the lines it has just loaded and
 * the fused launch runs 1-3% slower (DESIGN.md §4 finding 20).                                */

int fa_abi_version(void);
const char* fa_last_error(void);

/* Weighted mean of fp32 client tensors (+ optional fused epilogue).
 * Replaces Strategy.server_ensemble (flearn/common/strategy/strategy.py:102-130) for the
 * fp32 keys of the bucket, and — with epi->op != FA_OP_MEAN — the AVGM/OPT update math of
 * flearn/common/strategy/avgm.py:19-36 / opt.py:23-65.
 *   weights : device array of n_clients values, already cast the way numpy casts them:
 *             float (fp32) for FA_MODE_W32_*, double for FA_MODE_W64.
 *   denom   : np.sum(agg_weight_lst) as a double (exact for every dtype numpy produces here).
 *   out32   : [n_cols] fp32 result (what load_state_dict ends up with), may be NULL.
 *   out64   : [n_cols] f64 result (the reference's w_glob dtype for DIV64/W64), may be NULL.
 *   epi     : host pointer, NULL == FA_OP_MEAN.                                                */
int fa_reduce_f32(const float* stack, int64_t row_stride, int32_t n_clients, int32_t mode,
                  const void* weights, double denom, int64_t col_begin, int64_t n_cols,
                  const fa_epilogue* epi, float* out32, double* out64, void* stream);

/* Split-N form of fa_reduce_f32 for windows too narrow to fill the GPU with one sequential sweep
 * per column (few parameters, many clients: e.g. 1000 LeNet5 uploads, 44 K columns).  Each
 * column's clients are cut into 4 contiguous splits summed in list order, and the partial sums
 * are combined by a fixed binary tree in split order (staged in LDS).  Deterministic, but NOT
 * the reference's sequential order: results agree with strategy.py:123-129 to rounding
 * (normwise relative error <= 1e-6 per tensor), not bit for bit; the caller opts in.  A column
 * whose terms nearly cancel (sum of |w*x| > 2 |sum of w*x|, or a non-finite sum) is re-summed in
 * list order, bit-exact.  Used only where it is faster and within the tolerance — a window of
 * fewer 1-KiB row chunks than the GPU has CUs and 8..256 clients; otherwise this runs
 * fa_reduce_f32's bit-exact sequential kernel.  Same arguments, modes and epilogues as
 * fa_reduce_f32.                                                                               */
int fa_reduce_f32_splitn(const float* stack, int64_t row_stride, int32_t n_clients, int32_t mode,
                         const void* weights, double denom, int64_t col_begin, int64_t n_cols,
                         const fa_epilogue* epi, float* out32, double* out64, void* stream);

/* Weighted mean of f64 client tensors (float64 buffers, and int64 buffers the host has cast to
 * f64 — numpy promotes int64 * Python-float to float64).  f64 product and sum, f64 divide.
 * Replaces server_ensemble for those keys (strategy.py:123-129).                              */
int fa_reduce_f64(const double* stack, int64_t row_stride, int32_t n_clients,
                  const double* weights, double denom, int64_t col_begin, int64_t n_cols,
                  double* out64, void* stream);

/* Weighted sum of int64 client tensors with int64 weights (Python-int weights times int64
 * buffers stay int64 in numpy, wrapping on overflow), then true division in f64.
 * Replaces server_ensemble for int64 keys with integer weights (strategy.py:123-129).         */
int fa_reduce_i64(const int64_t* stack, int64_t row_stride, int32_t n_clients,
                  const int64_t* weights, double denom, int64_t col_begin, int64_t n_cols,
                  double* out64, void* stream);

/* Standalone AVGM/OPT update of a received global model (no reduce): the reference location
 * of this math, AVGM.client_receive (avgm.py:38-45) / OPT.client_receive (opt.py:67-76).
 *   prec   : FA_PREC_F64 (glob is double*, v is double*) or FA_PREC_F32 (float*, float*).
 *   local  : [n] fp32 w_local; glob : [n] the received w_glob.                                */
int fa_opt_apply(int32_t prec, const fa_epilogue* epi, const float* local, const void* glob,
                 int64_t n, float* out32, double* out64, void* stream);

/* ---- device-resident uploads read in place (row-pointer form) --------------------------------
 * flearn's simulator path hands the server torch tensors (run2, flearn/server/Communicator.py:
 * 287-292, then Server.ensemble -> strategy.server, flearn/server/Server.py:140): on the GPU
 * every (client, key) tensor is its own allocation.  Instead of packing N*K tensors into a
 * stack, these read them where they lie.  A SEGMENT is one key: columns [seg_col, +seg_len) of
 * the logical bucket (the index of out32 / out64 / prev / v / h), stored for client i at
 * rows[s * n_clients + i] (a device pointer to seg_len contiguous elements).                    */

/* One unit of work of fa_reduce_f32_rows: logical columns [col, col + n_cols) = elements
 * [seg_off, seg_off + n_cols) of segment seg.  Built by fa_rows_plan.                          */
typedef struct fa_piece {
  int64_t col;
  int64_t seg_off;
  int32_t seg;
  int32_t n_cols;
  int64_t aux; /* set by fa_rows_plan (pieces[0].aux: how many leading pieces are swept in
                  row-major groups); pass the plan through unchanged                          */
} fa_piece;

/* HOST function: the work plan of fa_reduce_f32_rows: every segment cut into equal pieces of at
 * most 64 KiB of a row (the width chosen so the wide pieces fill whole rounds of the grid),
 * largest first, and the grid to launch (grid_hint <= 0: the library's default for the current
 * device, never more than the work items).  seg_col[s] must be a multiple of 4.
 * pieces == NULL or cap too small: *n_pieces / *grid report the sizes (FA_ERR_SIZE when
 * pieces != NULL).                                                                             */
int fa_rows_plan(int32_t n_segments, const int64_t* seg_col, const int64_t* seg_len, int32_t op,
                 int32_t grid_hint, fa_piece* pieces, int64_t cap, int64_t* n_pieces, int32_t* grid);

/* fa_reduce_f32 over row pointers: same modes, weights, epilogues and bit-exact client order,
 * one launch, HBM traffic = the uploads once + the outputs / state.  Replaces server_ensemble
 * (strategy.py:102-130) for device-resident fp32 uploads.
 *   rows   : device array [n_segments * n_clients] of device pointers, each 16-byte aligned;
 *   pieces : device copy of fa_rows_plan's n_pieces pieces (same op), launched on its grid;
 *   work   : device int32 scratch (1 element): the blocks' piece counter, cleared on the stream
 *            before the launch; one launch at a time may use it.
 * Columns outside every segment (alignment gaps of the bucket) are not written.               */
int fa_reduce_f32_rows(const float* const* rows, int32_t n_clients, int32_t mode, const void* weights,
                       double denom, const fa_piece* pieces, int64_t n_pieces, int32_t grid, int32_t* work,
                       const fa_epilogue* epi, float* out32, double* out64, void* stream);

/* One-launch gather of device tensors into a client stack (elem_size 4 or 8):
 *   stack[i * row_stride + seg_col[s] + e] = rows[s * n_clients + i][e],  e < seg_len[s].
 * For the small kinds (int64 / float64 buffers: BN num_batches_tracked) and fp32 tensors that
 * are not 16-byte aligned.  segs: device int64 array [2 * n_segments] = seg_col..., seg_len....
 * Any alignment (element-wise copies).                                                         */
int fa_gather_rows(void* stack, int64_t row_stride, int32_t n_clients, int32_t elem_size,
                   const void* const* rows, const int64_t* segs, int32_t n_segments, void* stream);

/* The same gather into a float64 stack, converting each segment's source elements as numpy's
 * astype(np.float64) does (what np.multiply(w_local[k], agg_weight) does to an int64 or float32
 * value before the float64 sum, strategy.py:124-126): segs = device int64 [3 * n_segments] =
 * seg_col..., seg_len..., seg_src... with seg_src[s] one of FA_SRC_F64 (copied), FA_SRC_I64
 * (rounded to nearest, as a C cast), FA_SRC_F32 (exact).  For BN num_batches_tracked (int64)
 * of device uploads.                                                                          */
#define FA_SRC_F64 0
#define FA_SRC_I64 1
#define FA_SRC_F32 2
int fa_gather_rows_f64(double* stack, int64_t row_stride, int32_t n_clients, const void* const* rows,
                       const int64_t* segs, int32_t n_segments, void* stream);

/* Synthetic client data: dst[r*row_stride + c] = U(-1,1) from splitmix64 of
 * (seed, row_begin + r, col_global_begin + c) — the bench/test generator; the CPU oracle
 * regenerates any element.  Not a reference interface.                                        */
int fa_fill_uniform_f32(float* dst, int64_t row_stride, int32_t n_rows, int64_t n_cols,
                        uint64_t seed, int64_t row_begin, int64_t col_global_begin, void* stream);

/* Process-wide grid of the fp32 stack reduce (fa_reduce_f32 / _splitn's fallback): the number
 * of blocks the row-pipelined kernels are launched with.  0 (the default) = the library's own
 * choice (~0.75 blocks per CU, one block per CU at most: DESIGN.md section 4).  A smaller grid
 * leaves CUs free for kernels that run beside the reduce — RCCL's all-gather of the previous
 * stripe in the multi-GPU pipeline (flearn_amd.dist; DESIGN.md section 6 measures the
 * contention).  Results do not depend on the grid (every column is still summed in client
 * order).  Returns the previous value; grid < 0 -> FA_ERR_ARG.  No reference counterpart: a
 * scheduling knob of this engine (the reference has one CPU thread).                         */
int fa_set_reduce_grid(int32_t grid);

/* How many launches fa_reduce_f32 makes for an fp32-sum window (modes FA_MODE_W32_DIV64 /
 * _DIV32; FA_MODE_W64 is always one) of n_cols columns with epilogue `op` (FA_OP_*): wide windows run as consecutive column windows, each with its own geometry
 * (fused epilogues at >= 16 Mi columns in 3, plain means of 8-16 Mi columns in 2; 1 with a
 * forced grid) — measured faster, bit-identical (DESIGN.md section 4 finding 26).  For callers
 * that time or profile per launch.  FA_ERR_ARG for an unknown op.  ABI 13.                    */
int fa_reduce_windows(int32_t op, int64_t n_cols);

/* Copy nbytes from src to dst with a kernel on `stream` (both 16-byte aligned; either may be
 * pinned host memory mapped into the GPU's address space).  For a device result going to a
 * pinned host buffer the kernel's stores cross PCIe at ~53 GB/s where the copy engine's D2H
 * runs at ~30 GB/s on the MI355X hosts measured (PCIe).  Replaces the
 * D2H of the reduced bucket that ends Strategy.server's round (the result handed back to
 * flearn as numpy arrays, strategy.py:123-129).  FA_ERR_ALIGN when a pointer is not 16-byte
 * aligned (the caller then uses the copy engine).                                             */
int fa_copy(void* dst, const void* src, int64_t nbytes, void* stream);

/* ---- one-shot all-gather over xGMI (multi-GPU reassembly) -----------------
 * The reference has no multi-GPU path; these replace the all-gather that reassembles the
 * column-sharded global model (the north star's "RCCL all-gather over xGMI") with direct peer
 * stores: every rank maps its peers' receive buffers once (IPC handles exchanged by the caller)
 * and pushes each reduced stripe straight into all of them, one xGMI link per peer, with no
 * forwarding and no re-read of received data.  The caller orders pushes and reads with barriers
 * (flearn_amd.dist.PushGather). */
#define FA_IPC_HANDLE_BYTES 64

/* The IPC handle of the device allocation holding `ptr` (handle: FA_IPC_HANDLE_BYTES bytes) and
 * ptr's byte offset in it.                                                                   */
int fa_ipc_handle(const void* ptr, void* handle, int64_t* offset);

/* Map a peer process's allocation (its fa_ipc_handle) into this process: *base = its start.   */
int fa_ipc_open(const void* handle, void** base);

/* Unmap a base returned by fa_ipc_open.                                                      */
int fa_ipc_close(void* base);

/* A receive bucket of its own: hipMalloc(nbytes) into *ptr (exceptions to "nothing here
 * allocates or frees").  An IPC export of a caching-allocator tensor names the whole segment
 * that holds it, shared with and recycled for other tensors; a bucket from fa_dev_alloc is
 * exactly one export.  fa_dev_free (NULL is a no-op; synchronises the device as hipFree does) is
 * for buckets that were never exported: on this runtime, freeing memory a peer has imported
 * makes 13-34% of later imports map the wrong allocation, so flearn_amd.dist keeps exported
 * buckets for the process's lifetime and re-exports them.  ABI 13.      */
int fa_dev_alloc(int64_t nbytes, void** ptr);
int fa_dev_free(void* ptr);


/* The device allocation holding ptr: *base and *size (hipMemGetAddressRange) — what
 * fa_ipc_handle exports for ptr.  ABI 13.                                                     */
int fa_mem_range(const void* ptr, void** base, int64_t* size);

/* Copy nbytes from src to each of dsts[0..n_dsts) (n_dsts <= 8; every pointer 16-byte aligned;
 * dsts: a HOST array of device pointers, local or peer-mapped) in one kernel of `grid` blocks
 * (0: the library's choice) on `stream`; every lane ends with a system-scope release so the
 * stores are visible to the peers once the kernel has completed.  Paced: each wave drains its
 * stores before its next loads, so a block keeps ~16 KiB in flight per destination and the grid
 * sets the total; a small grid fills a link, and stores queued beyond a link's bandwidth-delay
 * product slow a reduce running beside the push (the data fabric backs up: DESIGN.md section 6).
 * Default (grid 0) 16 blocks — PROVISIONAL: sized from one GPU's PCIe stand-in and a
 * bandwidth-delay estimate, never measured against seven xGMI links; bench.py calibrates the grid
 * on the node (push_calibration.pair_us_by_grid, 16 among the grids it times).  ABI 10 adds `grid`. */
int fa_push(const void* src, int64_t nbytes, void* const* dsts, int32_t n_dsts, int32_t grid, void* stream);

/* hipMemcpyAsync(dst, src, nbytes, hipMemcpyDeviceToDeviceNoCU) on `stream`: a copy-engine
 * transfer, so a push leg costs the reduce no CUs (the copy-engine form of the one-shot
 * all-gather: one stream per peer).  Round 5: with plain hipMemcpyDeviceToDevice the runtime ran
 * these copies as blit kernels on the compute queues (rocprofv3).  ABI 11. */
int fa_copy_dma(void* dst, const void* src, int64_t nbytes, void* stream);

/* The copy-engine push leg of one stripe in one call: after the work queued so far on `stream`
 * (the stream that wrote src),
 * copy nbytes from src to dsts[i] on streams[i] (i < n_dsts <= 8; one copy engine per peer
 * stream).  What eight Python-level event records / waits / copies cost in host time per stripe
 * (~80 us) this does in a few.  ABI 12.  The ordering is a device-side cross-queue event wait:
 * with eight processes sharing a GPU and the legs' streams on hardware queues of their own, legs
 * ordered this way copied stripes before their reduce had finished.
 * flearn_amd.dist issues its legs in HOST order instead — fa_copy_dma per leg once the host has
 * seen the reduce complete — and keeps this entry for C callers and the probe's A/B.            */
int fa_push_dma(const void* src, int64_t nbytes, void* const* dsts, int32_t n_dsts, void* const* streams,
                void* stream);


/* `stream` waits for the work queued so far on streams[0..n) (n <= 16).  ABI 12.             */
int fa_stream_join(void* stream, void* const* streams, int32_t n);

/* A system-scope cache fence on every XCD's L2, queued on `stream`: FA_FENCE_RELEASE writes the
 * L2 back to HBM (before a copy engine reads what kernels wrote), FA_FENCE_ACQUIRE invalidates it
 * (before kernels read what a copy engine or a peer wrote).  ABI 14.                          */
#define FA_FENCE_RELEASE 0
#define FA_FENCE_ACQUIRE 1
int fa_cache_fence(int32_t kind, void* stream);

/* ---- wire codec (HOST functions: every pointer below is host memory) -------------------------
 * flearn's HTTP mode ships uploads and global models as base64(pickle.dumps(obj))
 * (flearn/common/Encrypt.py:17-44, Encrypt.encode / Encrypt.decode; decoded per upload in
 * Server.ensemble, flearn/server/Server.py:126-131).  These replace base64.b64encode /
 * base64.b64decode / pickle.loads on that path.  `threads` <= 0 picks a default (<= 16). */

/* Decoded length of canonical base64 text (length % 4 == 0, '=' only as final padding), or
 * FA_ERR_DATA.  Non-canonical text is left to the caller (Python's lenient b64decode).       */
int64_t fa_b64_decoded_size(const char* src, int64_t n);

/* base64.b64decode(src) -> dst (cap bytes).  FA_ERR_DATA on a non-alphabet character.      */
int fa_b64_decode(const char* src, int64_t n, uint8_t* dst, int64_t cap, int32_t threads);

/* Decode only the decoded-byte ranges [offsets[r], offsets[r] + lengths[r]) of the base64
 * text, each straight into dsts[r] — how array payloads land in pinned staging without an
 * intermediate bytes object.  Ranges need no alignment.                                      */
int fa_b64_decode_ranges(const char* src, int64_t n, int32_t count, const int64_t* offsets,
                         const int64_t* lengths, void* const* dsts, int32_t threads);

/* base64.b64encode(src) -> dst (4*ceil(n/3) characters, no terminator).                     */
int fa_b64_encode(const uint8_t* src, int64_t n, char* dst, int64_t cap, int32_t threads);

/* base64.b64encode(srcs[0] + srcs[1] + ... + srcs[count-1]) -> dst: the encode of a byte
 * stream held in pieces (the chunks a pickler streamed out, large payloads by reference), so
 * Encrypt.encode (Encrypt.py:17-30) never joins them into one pickle bytes object.           */
int fa_b64_encode_gather(int32_t count, const uint8_t* const* srcs, const int64_t* lens, char* dst,
                         int64_t cap, int32_t threads);

/* Restricted pickle scan (pickle.loads replacement for the structure check): walk the pickle
 * inside base64 text WITHOUT decoding array payloads and write a JSON manifest of the object:
 *   null/true/false/ints/"str"; {"__f":"<C99 hex float>"}; {"__b":[off,len]} bytes;
 *   {"__t":[...]} tuple; [...] list; {"__d":[[k,v],...]} dict; {"__od":[...]} OrderedDict;
 *   {"__nd":[dtype,[shape],fortran,off,len,setstate]} numpy array (setstate=1: rebuilt by
 *   ndarray.__setstate__, which returns native byte order; 0: numpy's protocol-5 _frombuffer); {"__sc":[dtype,off,len]} numpy
 *   scalar; {"__dt":dtype} numpy dtype — off/len are decoded-byte ranges of the payload.
 * Accepts protocol 2-5 opcodes for dicts/lists/tuples/str/bytes/ints/floats/bools/None and the
 * numpy reconstructors only; anything else (other globals, torch tensors) -> FA_ERR_UNSUPPORTED.
 * FA_ERR_SIZE when cap is too small (*out_len = needed).                                     */
int fa_pickle_scan_b64(const char* src, int64_t n, char* out, int64_t cap, int64_t* out_len);
/* Same over already-decoded pickle bytes. */
int fa_pickle_scan(const uint8_t* buf, int64_t n, char* out, int64_t cap, int64_t* out_len);
/* Thread-local message of the last failing wire-codec call. */
const char* fa_wire_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* FLEARN_AMD_H_ */
