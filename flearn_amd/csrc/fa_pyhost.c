// Host-side pack helper for the Python strategy mirror (flearn_amd/bucket.py).  NOT part of the C
// ABI in include/: it takes Python objects and is loaded with ctypes.PyDLL (called with the GIL
// held; Python symbols resolve against the running interpreter, nothing is linked).
//
// flearn's loopback server hands Strategy.server one dict of host arrays per client
// (Server.py:126-140); packing them into the pinned bucket rows from Python costs ~1 us of
// interpreter work per (client, key) on top of the copy, which is most of a LeNet-sized round.
// This walks the dicts natively: every value is taken through the buffer protocol (numpy arrays
// and numpy scalars export one), checked against the plan (C-contiguous, element format and byte
// size), and the copies run with the GIL released.  Anything else (torch tensors, Python scalars,
// a missing key, another format) returns FA_PY_FALLBACK with no exception set and nothing
// copied, and the caller packs those rows the Python way, which reports real errors the way the
// reference does.
//
// numpy arrays are read through numpy's C API (type number, byte order, flags, dims, data: a few
// nanoseconds each) — the buffer protocol costs ~0.15 us per value (numpy builds a format string
// per export), which for 100 LeNet5-sized values was half the native pack time and more than
// the Python signature check it replaced.  Values that are not ndarrays (numpy scalars, other
// buffer exporters) still go through the buffer protocol.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#define PY_ARRAY_UNIQUE_SYMBOL fa_pyhost_ARRAY_API
#include <numpy/arrayobject.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { FA_PY_OK = 0, FA_PY_FALLBACK = 1, FA_PY_NOMEM = 2 };

// numpy's C-API table, imported on first use (this library is not a Python module)
static int np_ready(void) {
  static int state = 0;  // 0 not tried, 1 ready, -1 unavailable
  if (state == 0) {
    if (_import_array() < 0) {
      PyErr_Clear();
      state = -1;
    } else {
      state = 1;
    }
  }
  return state == 1;
}

// format class of an ndarray: 'f' f32, 'd' f64, 'i' int64, native byte order; 0 otherwise
static char array_class(PyArrayObject *a) {
  PyArray_Descr *d = PyArray_DESCR(a);
  if (PyDataType_ISBYTESWAPPED(d)) return 0;
  switch (d->type_num) {
    case NPY_FLOAT32: return 'f';
    case NPY_FLOAT64: return 'd';
    case NPY_INT64: return 'i';
    default: return 0;
  }
}

// One value's bytes: an ndarray read directly (a new reference kept in *owner), anything else
// through the buffer protocol (the view kept in *view, *owner = NULL).  0 on success.
typedef struct {
  const char *buf;
  int64_t len;
  char fmt;
  PyObject *owner;
  Py_buffer view;
  int has_view;
} Val;

// format class of a buffer: 'f' f32, 'd' f64, 'i' 8-byte signed integer; 0 otherwise
static char format_class(const Py_buffer *v) {
  const char *f = v->format ? v->format : "B";
  if (*f == '@' || *f == '=' || *f == '<') f++;
  if (f[0] == 0 || f[1] != 0) return 0;
  switch (f[0]) {
    case 'f': return v->itemsize == 4 ? 'f' : 0;
    case 'd': return v->itemsize == 8 ? 'd' : 0;
    case 'l': case 'q': return v->itemsize == 8 ? 'i' : 0;
    default: return 0;
  }
}

// clients: list of dicts.  keys: tuple, one key per piece (a key split over shards appears once
// per piece).  desc: int64 table, 7 rows of npieces then one row of len(clients):
//   total[p]    the value's whole size in bytes
//   src_lo[p]   first byte of the value copied
//   nbytes[p]   bytes copied
//   fmt[p]      format class ('f', 'd' or 'i', see format_class)
//   dst_base[p] address of the staging row 0 the piece lands in
//   dst_row[p]  bytes between staging rows
//   dst_off[p]  byte offset of the piece in its staging row
//   skip[r]     nonzero: row r is not packed (its upload already sits in a pinned row)
// Rows [r0, r1) are packed.  All-or-nothing: either every copy of the call is done or none.
static char format_class(const Py_buffer *v);

static int val_get(PyObject *v, Val *out) {
  out->has_view = 0;
  out->owner = NULL;
  if (np_ready() && PyArray_Check(v)) {
    PyArrayObject *a = (PyArrayObject *)v;
    if (!PyArray_IS_C_CONTIGUOUS(a)) return -1;
    out->buf = (const char *)PyArray_DATA(a);
    out->len = (int64_t)PyArray_NBYTES(a);
    out->fmt = array_class(a);
    Py_INCREF(v);
    out->owner = v;
    return 0;
  }
  if (PyObject_GetBuffer(v, &out->view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
    PyErr_Clear();
    return -1;
  }
  out->has_view = 1;
  out->buf = (const char *)out->view.buf;
  out->len = (int64_t)out->view.len;
  out->fmt = format_class(&out->view);
  return 0;
}

static void val_release(Val *v) {
  if (v->has_view) PyBuffer_Release(&v->view);
  Py_XDECREF(v->owner);
}

int fa_py_pack_rows(PyObject *clients, PyObject *keys, int64_t npieces, const int64_t *desc,
                    int64_t r0, int64_t r1) {
  const int64_t *total = desc, *src_lo = desc + npieces, *nbytes = desc + 2 * npieces,
                *fmt = desc + 3 * npieces, *dst_base = desc + 4 * npieces, *dst_row = desc + 5 * npieces,
                *dst_off = desc + 6 * npieces, *skip = desc + 7 * npieces;
  if (!PyList_Check(clients) || !PyTuple_Check(keys) || PyTuple_GET_SIZE(keys) != npieces ||
      r0 < 0 || r1 > PyList_GET_SIZE(clients) || r0 > r1)
    return FA_PY_FALLBACK;
  int64_t nrows = r1 - r0;
  Val *views = (Val *)calloc((size_t)(nrows * npieces > 0 ? nrows * npieces : 1), sizeof(Val));
  if (!views) return FA_PY_NOMEM;
  int64_t held = 0;
  int rc = FA_PY_OK;
  for (int64_t r = r0; r < r1 && rc == FA_PY_OK; r++) {
    if (skip[r]) continue;
    PyObject *d = PyList_GET_ITEM(clients, r);
    if (!PyDict_Check(d)) { rc = FA_PY_FALLBACK; break; }
    for (int64_t p = 0; p < npieces; p++) {
      PyObject *v = PyDict_GetItemWithError(d, PyTuple_GET_ITEM(keys, p));  // borrowed
      if (!v) { PyErr_Clear(); rc = FA_PY_FALLBACK; break; }
      Val *b = &views[held];
      if (val_get(v, b) != 0) { rc = FA_PY_FALLBACK; break; }
      held++;
      if (b->len != total[p] || b->fmt != fmt[p] || src_lo[p] < 0 || src_lo[p] + nbytes[p] > b->len) {
        rc = FA_PY_FALLBACK; break;
      }
    }
  }
  if (rc == FA_PY_OK) {
    Py_BEGIN_ALLOW_THREADS
    int64_t i = 0;
    for (int64_t r = r0; r < r1; r++) {
      if (skip[r]) continue;
      for (int64_t p = 0; p < npieces; p++, i++) {
        if (nbytes[p] == 0) continue;
        memcpy((char *)(intptr_t)dst_base[p] + r * dst_row[p] + dst_off[p], views[i].buf + src_lo[p],
               (size_t)nbytes[p]);
      }
    }
    Py_END_ALLOW_THREADS
  }
  for (int64_t i = 0; i < held; i++) val_release(&views[i]);
  free(views);
  return rc;
}

// 1: every client's value for every key has client 0's Python type, element format, item size
// and shape (what bucket.py _raw_signature compares for numpy uploads: type, dtype, shape;
// numpy's buffer export carries the dtype as format + itemsize); 0: some value differs; -1:
// cannot tell (not a list of dicts, a missing key, a value without a plain buffer) — the caller
// compares in Python.  No exception is left set.
int fa_py_same_signature(PyObject *clients, PyObject *keys) {
  if (!PyList_Check(clients) || !PyTuple_Check(keys)) return -1;
  const Py_ssize_t n = PyList_GET_SIZE(clients), nk = PyTuple_GET_SIZE(keys);
  if (n == 0) return -1;
  for (Py_ssize_t c = 0; c < n; ++c)
    if (!PyDict_Check(PyList_GET_ITEM(clients, c))) return -1;
  PyObject *d0 = PyList_GET_ITEM(clients, 0);
  int result = 1;
  if (np_ready()) {  // all-ndarray fast path: type, dtype (identity of the descriptor's type and
                     // byte order) and dims compared through the C API
    int all_arrays = 1;
    for (Py_ssize_t k = 0; k < nk && result == 1 && all_arrays; ++k) {
      PyObject *key = PyTuple_GET_ITEM(keys, k);
      PyObject *v0 = PyDict_GetItemWithError(d0, key);
      if (!v0 || !PyArray_Check(v0)) { PyErr_Clear(); all_arrays = 0; break; }
      PyArrayObject *a0 = (PyArrayObject *)v0;
      const int nd = PyArray_NDIM(a0);
      const npy_intp *dims0 = PyArray_DIMS(a0);
      PyArray_Descr *t0 = PyArray_DESCR(a0);
      for (Py_ssize_t c = 1; c < n; ++c) {
        PyObject *v = PyDict_GetItemWithError(PyList_GET_ITEM(clients, c), key);
        if (!v || !PyArray_Check(v)) { PyErr_Clear(); all_arrays = 0; break; }
        PyArrayObject *a = (PyArrayObject *)v;
        PyArray_Descr *t = PyArray_DESCR(a);
        int same = Py_TYPE(v) == Py_TYPE(v0) && PyArray_NDIM(a) == nd &&
                   (t == t0 || (t->type_num == t0->type_num && t->byteorder == t0->byteorder &&
                                PyDataType_ELSIZE(t) == PyDataType_ELSIZE(t0)));
        for (int i = 0; same && i < nd; ++i) same = PyArray_DIMS(a)[i] == dims0[i];
        if (!same) { result = 0; break; }
      }
    }
    if (all_arrays) return result;
    result = 1;
  }
  for (Py_ssize_t k = 0; k < nk && result >= 0; ++k) {
    PyObject *key = PyTuple_GET_ITEM(keys, k);
    PyObject *v0 = PyDict_GetItemWithError(d0, key);
    Py_buffer b0;
    if (!v0 || PyObject_GetBuffer(v0, &b0, PyBUF_STRIDES | PyBUF_FORMAT) != 0) {
      PyErr_Clear();
      return -1;
    }
    for (Py_ssize_t c = 1; c < n; ++c) {
      PyObject *v = PyDict_GetItemWithError(PyList_GET_ITEM(clients, c), key);
      Py_buffer b;
      if (!v || PyObject_GetBuffer(v, &b, PyBUF_STRIDES | PyBUF_FORMAT) != 0) {
        PyErr_Clear();
        result = -1;
        break;
      }
      int same = Py_TYPE(v) == Py_TYPE(v0) && b.itemsize == b0.itemsize && b.ndim == b0.ndim &&
                 strcmp(b.format ? b.format : "B", b0.format ? b0.format : "B") == 0;
      for (int i = 0; same && i < b.ndim; ++i) same = b.shape[i] == b0.shape[i];
      PyBuffer_Release(&b);
      if (!same) result = 0;
    }
    PyBuffer_Release(&b0);
  }
  return result;
}

// ---- asynchronous pack (the client-side update's chunked pipeline, strategy/_update.py) -------
// fa_py_pack_start resolves every piece's source under the GIL (all-or-nothing: one value that is
// not a C-contiguous array of the planned format and size and nothing is queued), splits the
// copies into jobs of at most split_bytes in chunk order and hands them to a persistent pool of
// native threads; fa_pack_wait(h, c) — called through ctypes.CDLL, so without the GIL — returns
// once chunk c's copies are done, copying jobs of chunks <= c itself while it waits;
// fa_py_pack_end waits for every copy and releases the values.  Python-side pool tasks (one GIL
// hand-off per 4 MiB part, ~16 threads contending for it) kept the first chunk ~0.5-0.9 ms from
// its launch; this path has no per-job interpreter work.
#include <pthread.h>
#include <stdatomic.h>
#include <unistd.h>

typedef struct {
  char *dst;
  const char *src;
  int64_t n;
  int64_t chunk;
} PackJob;

typedef struct Pack {
  PackJob *jobs;
  int64_t njobs;
  atomic_llong next;  // next unclaimed job
  atomic_llong *left; // per chunk: jobs not yet copied
  int64_t nchunks;
  Val *vals;
  int64_t nvals;
  pthread_mutex_t mu;  // chunk completion
  pthread_cond_t cv;
  int refs;            // workers inside this pack (g_mu)
  int max_workers;     // at most this many workers copy for this pack at once
  int queued;          // still on the pool's queue (g_mu)
  struct Pack *qnext;
} Pack;

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_work = PTHREAD_COND_INITIALIZER;  // a pack was queued
static pthread_cond_t g_idle = PTHREAD_COND_INITIALIZER;  // a worker left a pack
static Pack *g_head = NULL, *g_tail = NULL;
static int g_workers = 0;
static pid_t g_pid = 0;

static void pack_done_job(Pack *p, int64_t chunk) {
  if (atomic_fetch_sub(&p->left[chunk], 1) == 1) {
    pthread_mutex_lock(&p->mu);
    pthread_cond_broadcast(&p->cv);
    pthread_mutex_unlock(&p->mu);
  }
}

static void unqueue_locked(Pack *p) {  // g_mu held
  if (!p->queued) return;
  Pack **pp = &g_head, *prev = NULL;
  while (*pp && *pp != p) { prev = *pp; pp = &(*pp)->qnext; }
  if (*pp) {
    *pp = p->qnext;
    if (g_tail == p) g_tail = prev;
  }
  p->queued = 0;
}

static void *pack_worker(void *arg) {
  (void)arg;
  for (;;) {
    pthread_mutex_lock(&g_mu);
    Pack *p;
    for (;;) {  // the oldest queued pack that still takes another worker
      for (p = g_head; p && p->refs >= p->max_workers; p = p->qnext) {
      }
      if (p) break;
      pthread_cond_wait(&g_work, &g_mu);
    }
    p->refs++;
    pthread_mutex_unlock(&g_mu);
    for (;;) {
      const int64_t i = atomic_fetch_add(&p->next, 1);
      if (i >= p->njobs) break;
      memcpy(p->jobs[i].dst, p->jobs[i].src, (size_t)p->jobs[i].n);
      pack_done_job(p, p->jobs[i].chunk);
    }
    pthread_mutex_lock(&g_mu);
    unqueue_locked(p);  // every job is claimed: nothing left for the other workers
    p->refs--;
    pthread_cond_broadcast(&g_idle);
    pthread_cond_broadcast(&g_work);  // a worker slot of some queued pack may have opened
    pthread_mutex_unlock(&g_mu);
  }
  return NULL;
}

// GIL held.  dicts: a tuple or list of dicts.  keys: tuple, one per piece.  desc: int64 table,
// 7 rows of npieces:
//   src[p]    index into dicts of the dict holding the piece's value
//   total[p]  the value's size in bytes
//   fmt[p]    format class ('f', 'd' or 'i')
//   dst[p]    destination address
//   chunk[p]  chunk index, non-decreasing in p, < nchunks
//   lo[p]     first byte of the value copied
//   nbytes[p] bytes copied (lo + nbytes <= total)
// At most `threads` pool workers copy for this pack at once (the pool grows to the largest
// `threads` asked for).  Returns a handle, or NULL with *status FA_PY_FALLBACK (a value off the plan; nothing queued,
// no exception set) or FA_PY_NOMEM.
void *fa_py_pack_start(PyObject *dicts, PyObject *keys, int64_t npieces, const int64_t *desc,
                       int64_t nchunks, int64_t split_bytes, int32_t threads, int32_t *status) {
  const int64_t *src = desc, *total = desc + npieces, *fmt = desc + 2 * npieces, *dst = desc + 3 * npieces,
                *chunk = desc + 4 * npieces, *lo = desc + 5 * npieces, *nbytes = desc + 6 * npieces;
  *status = FA_PY_FALLBACK;
  if (!PySequence_Check(dicts) || !PyTuple_Check(keys) || PyTuple_GET_SIZE(keys) != npieces || nchunks < 1 ||
      split_bytes < 4096)
    return NULL;
  PyObject *seq = PySequence_Fast(dicts, "dicts");
  if (!seq) { PyErr_Clear(); return NULL; }
  const Py_ssize_t nd = PySequence_Fast_GET_SIZE(seq);
  Pack *p = (Pack *)calloc(1, sizeof(Pack));
  Val *vals = (Val *)calloc((size_t)(npieces > 0 ? npieces : 1), sizeof(Val));
  atomic_llong *left = (atomic_llong *)calloc((size_t)nchunks, sizeof(atomic_llong));
  int64_t held = 0, njobs = 0;
  int rc = (p && vals && left) ? FA_PY_OK : FA_PY_NOMEM;
  for (int64_t i = 0; i < npieces && rc == FA_PY_OK; i++) {
    if (src[i] < 0 || src[i] >= nd || chunk[i] < 0 || chunk[i] >= nchunks || (i && chunk[i] < chunk[i - 1])) {
      rc = FA_PY_FALLBACK;
      break;
    }
    PyObject *d = PySequence_Fast_GET_ITEM(seq, src[i]);
    // plain dict / OrderedDict only: their item lookup is the C one; a subclass may override it
    if (!PyDict_CheckExact(d) && strcmp(Py_TYPE(d)->tp_name, "collections.OrderedDict") != 0) {
      rc = FA_PY_FALLBACK;
      break;
    }
    PyObject *v = PyDict_GetItemWithError(d, PyTuple_GET_ITEM(keys, i));  // borrowed
    if (!v) { PyErr_Clear(); rc = FA_PY_FALLBACK; break; }
    if (val_get(v, &vals[held]) != 0) { rc = FA_PY_FALLBACK; break; }
    held++;
    if (vals[i].len != total[i] || vals[i].fmt != fmt[i] || lo[i] < 0 || nbytes[i] < 0 ||
        lo[i] + nbytes[i] > total[i]) {
      rc = FA_PY_FALLBACK;
      break;
    }
    njobs += (nbytes[i] + split_bytes - 1) / split_bytes;
  }
  Py_DECREF(seq);
  PackJob *jobs = NULL;
  if (rc == FA_PY_OK) {
    jobs = (PackJob *)malloc((size_t)(njobs > 0 ? njobs : 1) * sizeof(PackJob));
    if (!jobs) rc = FA_PY_NOMEM;
  }
  if (rc != FA_PY_OK) {
    for (int64_t i = 0; i < held; i++) val_release(&vals[i]);
    free(vals);
    free(left);
    free(p);
    *status = rc;
    return NULL;
  }
  int64_t j = 0;
  for (int64_t i = 0; i < npieces; i++)
    for (int64_t o = 0; o < nbytes[i]; o += split_bytes) {
      const int64_t n = nbytes[i] - o < split_bytes ? nbytes[i] - o : split_bytes;
      jobs[j++] = (PackJob){(char *)(intptr_t)dst[i] + o, vals[i].buf + lo[i] + o, n, chunk[i]};
      atomic_fetch_add(&left[chunk[i]], 1);
    }
  p->jobs = jobs;
  p->njobs = njobs;
  atomic_init(&p->next, 0);
  p->left = left;
  p->nchunks = nchunks;
  p->vals = vals;
  p->nvals = held;
  pthread_mutex_init(&p->mu, NULL);
  pthread_cond_init(&p->cv, NULL);
  *status = FA_PY_OK;
  if (njobs == 0) return p;
  const int want = threads < 1 ? 1 : threads > 64 ? 64 : threads;
  p->max_workers = want;
  pthread_mutex_lock(&g_mu);
  if (g_pid != getpid()) {  // first use, or a forked child (its parent's workers do not exist here)
    g_pid = getpid();
    g_workers = 0;
    g_head = g_tail = NULL;
  }
  while (g_workers < want) {
    pthread_t t;
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    const int ok = pthread_create(&t, &at, pack_worker, NULL) == 0;
    pthread_attr_destroy(&at);
    if (!ok) break;  // fewer workers: the waiting caller copies the rest itself
    g_workers++;
  }
  p->queued = 1;
  if (g_tail) g_tail->qnext = p; else g_head = p;
  g_tail = p;
  pthread_cond_broadcast(&g_work);
  pthread_mutex_unlock(&g_mu);
  return p;
}

// No GIL needed (call through ctypes.CDLL).  0 once chunk c's copies are done; -1 bad arguments.
int fa_pack_wait(void *h, int64_t c) {
  Pack *p = (Pack *)h;
  if (!p || c < 0 || c >= p->nchunks) return -1;
  for (;;) {  // help: copy unclaimed jobs of chunks <= c
    int64_t i = atomic_load(&p->next);
    if (i >= p->njobs || p->jobs[i].chunk > c) break;
    if (!atomic_compare_exchange_weak(&p->next, &i, i + 1)) continue;
    memcpy(p->jobs[i].dst, p->jobs[i].src, (size_t)p->jobs[i].n);
    pack_done_job(p, p->jobs[i].chunk);
  }
  pthread_mutex_lock(&p->mu);
  while (atomic_load(&p->left[c]) > 0) pthread_cond_wait(&p->cv, &p->mu);
  pthread_mutex_unlock(&p->mu);
  return 0;
}

// GIL held.  Waits for every copy (and for the workers to leave the pack), releases the values,
// frees the handle.  0, or -1 for a NULL handle.
int fa_py_pack_end(void *h) {
  Pack *p = (Pack *)h;
  if (!p) return -1;
  Py_BEGIN_ALLOW_THREADS
  for (int64_t c = 0; c < p->nchunks; c++) fa_pack_wait(p, c);
  pthread_mutex_lock(&g_mu);
  unqueue_locked(p);
  while (p->refs > 0) pthread_cond_wait(&g_idle, &g_mu);
  pthread_mutex_unlock(&g_mu);
  Py_END_ALLOW_THREADS
  for (int64_t i = 0; i < p->nvals; i++) val_release(&p->vals[i]);
  pthread_mutex_destroy(&p->mu);
  pthread_cond_destroy(&p->cv);
  free(p->vals);
  free(p->left);
  free(p->jobs);
  free(p);
  return 0;
}
