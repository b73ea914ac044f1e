// Tensor metadata walks for the device-upload path (flearn's run2 mode hands Strategy.server one
// dict of torch tensors per client: Communicator.py:287-292).  NOT part of the C ABI in include/:
// the functions take Python objects, are loaded with ctypes.PyDLL (GIL held) and read each
// tensor's TensorImpl directly (torch's own headers, linked against the libtorch of this image).
//
// Why native: a ResNet-50 round of 100 clients is 26,700 fp32 tensors plus 5,400 BN counters.
// Through Python every tensor costs ~1-2 us of torch method dispatch (`.shape`, `.data_ptr()`,
// `.get_device()`, `.is_contiguous()` each go through the argument parser) — ~10 ms per server()
// call on the box against a 1.6 ms reduce.  Read from the TensorImpl they cost nanoseconds.
//
// Neither function raises or leaves an exception set: a value that is not a tensor, a missing
// key, or any other surprise answers "cannot tell" / "fallback", and the caller takes its Python
// path (flearn_amd/bucket.py), which reports real errors the reference's way.
#include <Python.h>

#include <torch/csrc/Dtype.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>

namespace {

enum { kSame = 1, kDiffer = 0, kUnknown = -1 };
enum { kOk = 0, kFallback = 1 };

const at::Tensor* tensor_of(PyObject* v) {
  if (!v || !THPVariable_Check(v)) return nullptr;
  return &THPVariable_Unpack(v);
}

}  // namespace

extern "C" {

// 1: every client's value for every key has client 0's Python type, dtype, shape and layout
// (what bucket.py _raw_signature compares); 0: some value differs; -1: cannot tell (a value is not a
// torch tensor, a key is missing, an upload is not a dict) — the caller compares in Python.
static int same_signature(PyObject* clients, PyObject* keys) {
  if (!PyList_Check(clients) || !PyTuple_Check(keys)) return kUnknown;
  const Py_ssize_t n = PyList_GET_SIZE(clients), nk = PyTuple_GET_SIZE(keys);
  if (n == 0) return kUnknown;
  for (Py_ssize_t c = 0; c < n; ++c)
    if (!PyDict_Check(PyList_GET_ITEM(clients, c))) return kUnknown;
  PyObject* d0 = PyList_GET_ITEM(clients, 0);
  int result = kSame;
  for (Py_ssize_t k = 0; k < nk; ++k) {
    PyObject* key = PyTuple_GET_ITEM(keys, k);
    PyObject* v0 = PyDict_GetItemWithError(d0, key);  // borrowed
    const at::Tensor* t0 = tensor_of(v0);
    if (!t0) {
      PyErr_Clear();
      return kUnknown;
    }
    const auto dt0 = t0->scalar_type();
    const auto sz0 = t0->sizes();
    for (Py_ssize_t c = 1; c < n; ++c) {
      PyObject* v = PyDict_GetItemWithError(PyList_GET_ITEM(clients, c), key);
      const at::Tensor* t = tensor_of(v);
      if (!t) {
        PyErr_Clear();
        return kUnknown;
      }
      if (Py_TYPE(v) != Py_TYPE(v0) || t->scalar_type() != dt0 || t->sizes() != sz0 || t->layout() != t0->layout())
        result = kDiffer;
    }
  }
  return result;
}

// out[k * n + c] = data pointer of clients[c][keys[k]] when every such value is a contiguous
// tensor of dtype dtypes[k] (a tuple of torch.dtype objects, one per key) on CUDA/HIP device
// `device`; each value is also stored in keep[k * n + c] (a list of that length made by the
// caller) so the tensors outlive the kernel that reads them.  Returns 0, or 1 (nothing reliable
// written) at the first value that does not qualify.
static int tensor_ptrs(PyObject* clients, PyObject* keys, PyObject* dtypes, int64_t device, int64_t* out,
                       PyObject* keep) {
  if (!PyList_Check(clients) || !PyTuple_Check(keys) || !PyList_Check(keep) || !PyTuple_Check(dtypes))
    return kFallback;
  const Py_ssize_t n = PyList_GET_SIZE(clients), nk = PyTuple_GET_SIZE(keys);
  if (PyList_GET_SIZE(keep) != n * nk || PyTuple_GET_SIZE(dtypes) != nk) return kFallback;
  for (Py_ssize_t c = 0; c < n; ++c)
    if (!PyDict_Check(PyList_GET_ITEM(clients, c))) return kFallback;
  for (Py_ssize_t k = 0; k < nk; ++k) {
    PyObject* key = PyTuple_GET_ITEM(keys, k);
    PyObject* dt = PyTuple_GET_ITEM(dtypes, k);
    if (!THPDtype_Check(dt)) return kFallback;
    const auto want = reinterpret_cast<THPDtype*>(dt)->scalar_type;
    for (Py_ssize_t c = 0; c < n; ++c) {
      PyObject* v = PyDict_GetItemWithError(PyList_GET_ITEM(clients, c), key);  // borrowed
      const at::Tensor* t = tensor_of(v);
      if (!t) {
        PyErr_Clear();
        return kFallback;
      }
      const c10::Device dv = t->device();
      // strided layout with storage first: is_contiguous / data_ptr throw on sparse or
      // storage-less tensors
      if (t->scalar_type() != want || !dv.is_cuda() || dv.index() != device || t->layout() != c10::kStrided ||
          !t->has_storage() || !t->is_contiguous())
        return kFallback;
      out[k * n + c] = reinterpret_cast<int64_t>(t->data_ptr());
      Py_INCREF(v);
      PyList_SetItem(keep, k * n + c, v);  // steals the new reference, drops the old item
    }
  }
  return kOk;
}

#ifndef FA_TM_STAMP
#error "build with -DFA_TM_STAMP=\"<torch version>|cxx11abi=<0|1>\"" (flearn_amd/_build.py)
#endif
// The torch build this library's TensorImpl reads were compiled against (checked at load time).
const char* fa_tm_stamp() { return FA_TM_STAMP; }

// C++ exceptions must not cross the ctypes boundary: any one answers "cannot tell" / "fallback"
int fa_tm_same_signature(PyObject* clients, PyObject* keys) {
  try {
    return same_signature(clients, keys);
  } catch (...) {
    PyErr_Clear();
    return kUnknown;
  }
}

int fa_tm_tensor_ptrs(PyObject* clients, PyObject* keys, PyObject* dtypes, int64_t device, int64_t* out,
                      PyObject* keep) {
  try {
    return tensor_ptrs(clients, keys, dtypes, device, out, keep);
  } catch (...) {
    PyErr_Clear();
    return kFallback;
  }
}

}  // extern "C"
