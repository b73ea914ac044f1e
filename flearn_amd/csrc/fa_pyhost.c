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
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { FA_PY_OK = 0, FA_PY_FALLBACK = 1, FA_PY_NOMEM = 2 };

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
int fa_py_pack_rows(PyObject *clients, PyObject *keys, int64_t npieces, const int64_t *desc,
                    int64_t r0, int64_t r1) {
  const int64_t *total = desc, *src_lo = desc + npieces, *nbytes = desc + 2 * npieces,
                *fmt = desc + 3 * npieces, *dst_base = desc + 4 * npieces, *dst_row = desc + 5 * npieces,
                *dst_off = desc + 6 * npieces, *skip = desc + 7 * npieces;
  if (!PyList_Check(clients) || !PyTuple_Check(keys) || PyTuple_GET_SIZE(keys) != npieces ||
      r0 < 0 || r1 > PyList_GET_SIZE(clients) || r0 > r1)
    return FA_PY_FALLBACK;
  int64_t nrows = r1 - r0;
  Py_buffer *views = (Py_buffer *)calloc((size_t)(nrows * npieces > 0 ? nrows * npieces : 1), sizeof(Py_buffer));
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
      Py_buffer *b = &views[held];
      if (PyObject_GetBuffer(v, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) {
        PyErr_Clear(); rc = FA_PY_FALLBACK; break;
      }
      held++;
      if (b->len != total[p] || format_class(b) != fmt[p] || src_lo[p] < 0 || src_lo[p] + nbytes[p] > b->len) {
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
        memcpy((char *)(intptr_t)dst_base[p] + r * dst_row[p] + dst_off[p],
               (const char *)views[i].buf + src_lo[p], (size_t)nbytes[p]);
      }
    }
    Py_END_ALLOW_THREADS
  }
  for (int64_t i = 0; i < held; i++) PyBuffer_Release(&views[i]);
  free(views);
  return rc;
}
