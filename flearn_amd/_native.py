"""ctypes binding of the C ABI in include/flearn_amd.h (libflearn_amd.so, built for gfx950).

torch is imported first on purpose: torch ships its own ROCm runtime whose soname
(libamdhip64.so.7) is the same as the system one, so loading torch first makes the dynamic
linker bind libflearn_amd.so to the runtime torch already initialised — one HIP runtime per
process, and device pointers from torch tensors are valid in our kernels.

There is no fallback: if the library is missing or the process has no GPU, every entry point
raises NativeUnavailable.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libflearn_amd.so"
ABI_VERSION = 14
FENCE_RELEASE, FENCE_ACQUIRE = 0, 1  # fa_cache_fence kinds

FA_OK = 0
FA_ERR_ARG, FA_ERR_ALIGN, FA_ERR_LAUNCH = -1, -2, -3
FA_ERR_SIZE, FA_ERR_UNSUPPORTED, FA_ERR_DATA = -4, -5, -6
MODE_W32_DIV64, MODE_W32_DIV32, MODE_W64 = 0, 1, 2
OP_MEAN, OP_AVGM, OP_ADAGRAD, OP_YOGI, OP_ADAM, OP_DYN = 0, 1, 2, 3, 4, 5
SRC_F64, SRC_I64, SRC_F32 = 0, 1, 2  # fa_gather_rows_f64 source kinds
PREC_F32, PREC_F64 = 0, 1
OP_BY_NAME = {"mean": OP_MEAN, "avgm": OP_AVGM, "adagrad": OP_ADAGRAD, "yogi": OP_YOGI, "adam": OP_ADAM, "dyn": OP_DYN}

#: every symbol include/flearn_amd.h declares (checked by tests/test_cabi.py)
EXPORTS = (
    "fa_abi_version",
    "fa_last_error",
    "fa_reduce_f32",
    "fa_reduce_f32_splitn",
    "fa_reduce_f64",
    "fa_reduce_i64",
    "fa_opt_apply",
    "fa_rows_plan",
    "fa_reduce_f32_rows",
    "fa_gather_rows",
    "fa_gather_rows_f64",
    "fa_fill_uniform_f32",
    "fa_copy",
    "fa_ipc_handle",
    "fa_ipc_open",
    "fa_ipc_close",
    "fa_dev_alloc",
    "fa_dev_free",
    "fa_mem_range",
    "fa_push",
    "fa_copy_dma",
    "fa_push_dma",
    "fa_stream_join",
    "fa_cache_fence",
    "fa_set_reduce_grid",
    "fa_reduce_windows",
    "fa_b64_decoded_size",
    "fa_b64_decode",
    "fa_b64_decode_ranges",
    "fa_b64_encode",
    "fa_b64_encode_gather",
    "fa_pickle_scan_b64",
    "fa_pickle_scan",
    "fa_wire_last_error",
)


class NativeUnavailable(RuntimeError):
    """The HIP library or a GPU is missing: the aggregation path cannot run."""


class NativeError(RuntimeError):
    """A C-ABI call returned an error code."""


class Piece(ctypes.Structure):
    """struct fa_piece (include/flearn_amd.h)."""

    _fields_ = [("col", ctypes.c_int64), ("seg_off", ctypes.c_int64), ("seg", ctypes.c_int32),
                ("n_cols", ctypes.c_int32), ("aux", ctypes.c_int64)]


class Epilogue(ctypes.Structure):
    """struct fa_epilogue (include/flearn_amd.h)."""

    _fields_ = [
        ("op", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("prev", ctypes.c_void_p),
        ("v", ctypes.c_void_p),
        ("beta", ctypes.c_double),
        ("eta", ctypes.c_double),
        ("tau", ctypes.c_double),
        ("beta2", ctypes.c_double),
        ("h", ctypes.c_void_p),
        ("alpha", ctypes.c_double),
        ("n_clients", ctypes.c_double),
        ("v_out", ctypes.c_void_p),
    ]


_lock = threading.Lock()
_lib = None
_pyhost = None
PYHOST_PATH = LIB_PATH.parent / "libfa_pyhost.so"


def load_pyhost():
    """The Python-object pack helper (csrc/fa_pyhost.c fa_py_pack_rows), loaded with
    ctypes.PyDLL so it runs with the GIL held (it releases it around its copies).  Raises
    NativeUnavailable."""
    global _pyhost
    with _lock:
        if _pyhost is None:
            if not PYHOST_PATH.exists():
                raise NativeUnavailable(
                    f"{PYHOST_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
                )
            L = ctypes.PyDLL(str(PYHOST_PATH))
            P, I64, O = ctypes.c_void_p, ctypes.c_int64, ctypes.py_object
            L.fa_py_pack_rows.argtypes = [O, O, I64, P, I64, I64]
            L.fa_py_pack_rows.restype = ctypes.c_int
            L.fa_py_same_signature.argtypes = [O, O]
            L.fa_py_same_signature.restype = ctypes.c_int
            L.fa_py_pack_start.argtypes = [O, O, I64, P, I64, I64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
            L.fa_py_pack_start.restype = P
            L.fa_py_pack_end.argtypes = [P]
            L.fa_py_pack_end.restype = ctypes.c_int
            # fa_pack_wait blocks on native copies: the same library through CDLL, so the call
            # releases the GIL while it waits
            W = ctypes.CDLL(str(PYHOST_PATH))
            W.fa_pack_wait.argtypes = [P, I64]
            W.fa_pack_wait.restype = ctypes.c_int
            L.fa_pack_wait = W.fa_pack_wait
            _pyhost = L
    return _pyhost


_torchmeta = None
TORCHMETA_PATH = LIB_PATH.parent / "libfa_torchmeta.so"


def load_torchmeta():
    """The tensor-metadata walks (csrc/fa_torchmeta.cpp: fa_tm_same_signature,
    fa_tm_tensor_ptrs), loaded with ctypes.PyDLL (GIL held), or None when the library is not
    built or was built for another torch (its fa_tm_stamp differs) — they only speed up checks
    the callers can also do in Python."""
    global _torchmeta
    with _lock:
        if _torchmeta is None:
            if not TORCHMETA_PATH.exists():
                _torchmeta = False
            else:
                from ._build import read_torchmeta_stamp, torch_stamp

                try:
                    L = ctypes.PyDLL(str(TORCHMETA_PATH))
                except OSError:
                    _torchmeta = False
                else:
                    if read_torchmeta_stamp(TORCHMETA_PATH) != torch_stamp():
                        # built against another torch: its TensorImpl reads would be undefined
                        _torchmeta = False
                        return None
                    O, P, I64 = ctypes.py_object, ctypes.c_void_p, ctypes.c_int64
                    L.fa_tm_same_signature.argtypes = [O, O]
                    L.fa_tm_same_signature.restype = ctypes.c_int
                    L.fa_tm_tensor_ptrs.argtypes = [O, O, O, I64, P, O]
                    L.fa_tm_tensor_ptrs.restype = ctypes.c_int
                    _torchmeta = L
    return _torchmeta or None


def load(require_gpu: bool = False):
    """Load and type the library (no GPU needed just to load).  Raises NativeUnavailable."""
    global _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise NativeUnavailable(
                    f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
                )
            L = ctypes.CDLL(str(LIB_PATH))
            P, I32, I64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
            sig = {
                "fa_abi_version": ([], ctypes.c_int),
                "fa_last_error": ([], ctypes.c_char_p),
                "fa_reduce_f32": ([P, I64, I32, I32, P, D, I64, I64, ctypes.POINTER(Epilogue), P, P, P],
                                  ctypes.c_int),
                "fa_reduce_f32_splitn": ([P, I64, I32, I32, P, D, I64, I64, ctypes.POINTER(Epilogue), P, P, P],
                                         ctypes.c_int),
                "fa_reduce_f64": ([P, I64, I32, P, D, I64, I64, P, P], ctypes.c_int),
                "fa_reduce_i64": ([P, I64, I32, P, D, I64, I64, P, P], ctypes.c_int),
                "fa_opt_apply": ([I32, ctypes.POINTER(Epilogue), P, P, I64, P, P, P], ctypes.c_int),
                "fa_rows_plan": ([I32, P, P, I32, I32, P, I64, ctypes.POINTER(I64), ctypes.POINTER(I32)],
                                 ctypes.c_int),
                "fa_reduce_f32_rows": ([P, I32, I32, P, D, P, I64, I32, P, ctypes.POINTER(Epilogue), P, P, P],
                                       ctypes.c_int),
                "fa_gather_rows": ([P, I64, I32, I32, P, P, I32, P], ctypes.c_int),
                "fa_gather_rows_f64": ([P, I64, I32, P, P, I32, P], ctypes.c_int),
                "fa_fill_uniform_f32": ([P, I64, I32, I64, ctypes.c_uint64, I64, I64, P], ctypes.c_int),
                "fa_copy": ([P, P, I64, P], ctypes.c_int),
                "fa_ipc_handle": ([P, P, ctypes.POINTER(I64)], ctypes.c_int),
                "fa_ipc_open": ([P, ctypes.POINTER(P)], ctypes.c_int),
                "fa_ipc_close": ([P], ctypes.c_int),
                "fa_dev_alloc": ([I64, ctypes.POINTER(P)], ctypes.c_int),
                "fa_dev_free": ([P], ctypes.c_int),
                "fa_mem_range": ([P, ctypes.POINTER(P), ctypes.POINTER(I64)], ctypes.c_int),
                "fa_push": ([P, I64, ctypes.POINTER(P), I32, I32, P], ctypes.c_int),
                "fa_copy_dma": ([P, P, I64, P], ctypes.c_int),
                "fa_push_dma": ([P, I64, ctypes.POINTER(P), I32, ctypes.POINTER(P), P], ctypes.c_int),
                "fa_stream_join": ([P, ctypes.POINTER(P), I32], ctypes.c_int),
                "fa_cache_fence": ([I32, P], ctypes.c_int),
                "fa_set_reduce_grid": ([I32], ctypes.c_int),
                "fa_reduce_windows": ([I32, I64], ctypes.c_int),
                "fa_b64_decoded_size": ([P, I64], I64),
                "fa_b64_decode": ([P, I64, P, I64, I32], ctypes.c_int),
                "fa_b64_decode_ranges": ([P, I64, I32, P, P, P, I32], ctypes.c_int),
                "fa_b64_encode": ([P, I64, P, I64, I32], ctypes.c_int),
                "fa_b64_encode_gather": ([I32, P, P, P, I64, I32], ctypes.c_int),
                "fa_pickle_scan_b64": ([P, I64, P, I64, ctypes.POINTER(I64)], ctypes.c_int),
                "fa_pickle_scan": ([P, I64, P, I64, ctypes.POINTER(I64)], ctypes.c_int),
                "fa_wire_last_error": ([], ctypes.c_char_p),
            }
            for name, (args, res) in sig.items():
                try:
                    fn = getattr(L, name)
                except AttributeError:  # a library built from older sources: an environment error
                    raise NativeUnavailable(f"{LIB_PATH} does not export {name}: rebuild it "
                                            "(__graft_entry__.build())") from None
                fn.argtypes = args
                fn.restype = res
            v = L.fa_abi_version()
            if v != ABI_VERSION:
                raise NativeUnavailable(f"libflearn_amd ABI {v}, expected {ABI_VERSION}")
            _lib = L
    if require_gpu and not torch.cuda.is_available():
        raise NativeUnavailable("no HIP device visible: the aggregation kernels need an MI355X")
    return _lib


def lib():
    """The library, with a GPU required (the product path)."""
    return load(require_gpu=True)


def check(rc: int, what: str) -> None:
    if rc != FA_OK:
        msg = _lib.fa_last_error().decode(errors="replace") if _lib is not None else "?"
        raise NativeError(f"{what} failed with code {rc}: {msg}")


def stream_handle(device) -> int:
    """hipStream_t of torch's current stream on `device` (what every launch is queued on)."""
    return torch.cuda.current_stream(device).cuda_stream
