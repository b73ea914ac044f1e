"""CPU oracle for the FedAVG-family aggregation path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the timed CPU baseline.  The product (``flearn_amd``)
never imports it; the product fails loudly when its HIP library is missing.

Two restatements of the reference (wnma3mz/flearn v0.0.5) arithmetic:

* ``server_ensemble`` / ``mean_momentum`` / ``adaptive_opt`` / ``dyn_f`` / ``logits_mean`` — numpy
  op-sequence restatements of ``flearn/common/strategy/strategy.py:102-130``, ``avgm.py:19-36``,
  ``opt.py:23-65``, ``dyn.py:17-36`` and ``distill.py:42-46``: the
  same ufunc calls in the same order, so numpy applies the same (NEP 50) promotions.  This is
  "flearn's CPU path" timed by bench.py.
* ``c_reduce`` / ``c_update`` — the per-element C restatement (``fa_oracle.c``, strict IEEE, no
  contraction) of the same arithmetic with the dtypes spelled out; the GPU kernels are checked
  against it at sizes too big for fixtures.

Both are pinned bit-for-bit to golden vectors captured from the reference itself
(``tests/golden/make_golden.py`` → ``tests/golden/*.npz``; see tests/test_oracle_golden.py).
"""
from __future__ import annotations

import copy
import ctypes
from functools import reduce
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None

# ---------------------------------------------------------------------------------------------
# numpy op-sequence restatement
# ---------------------------------------------------------------------------------------------


def intersect_keys(w_local_lst, key_lst=None):
    """Key selection of strategy.py:119-121 (set intersection), returned in the first client's
    insertion order so results are deterministic (the reference's order is hash-random)."""
    if key_lst is not None:
        return list(key_lst)
    common = reduce(lambda a, b: a & b, [set(w.keys()) for w in w_local_lst])
    return [k for k in w_local_lst[0].keys() if k in common]


def server_ensemble(agg_weight_lst, w_local_lst, key_lst=None):
    """strategy.py:102-130: w = a0*x0; w += a_n*x_n in list order; w = np.divide(w, np.sum(a))."""
    keys = intersect_keys(w_local_lst, key_lst)
    glob = {}
    for k in keys:
        glob[k] = agg_weight_lst[0] * w_local_lst[0][k]  # strategy.py:123
    for a, w_local in zip(agg_weight_lst[1:], w_local_lst[1:]):  # strategy.py:124-126
        for k in keys:
            glob[k] += a * w_local[k]
    denom = np.sum(agg_weight_lst)  # strategy.py:127
    for k in keys:  # strategy.py:128-129
        glob[k] = np.divide(glob[k], denom)
    return glob


def mean_momentum(w_local, w_glob, v_t, beta=0.9):
    """avgm.py:19-36 with the state passed explicitly (v_t dict or None on the first call).
    Returns (new w_local dict, new v_t dict)."""
    delta = copy.deepcopy(w_glob)
    for k in w_glob.keys():
        delta[k] = delta[k] - w_local[k]
    if v_t is None:
        v_t = {k: np.zeros_like(delta[k]) for k in delta.keys()}
    v_t = dict(v_t)
    for k in w_glob.keys():
        v_t[k] = delta[k] + beta * v_t[k]
    w_local = dict(w_local)
    for k in w_glob.keys():
        w_local[k] = w_local[k] + v_t[k]
    return w_local, v_t


def adaptive_opt(w_local, w_glob, v_t, method, eta=1e-1, tau=1e-9, beta2=0.99):
    """opt.py:23-65 (simplified delta_t = delta_w, as the reference ships it), state explicit."""
    delta = {k: w_glob[k] - w_local[k] for k in w_glob.keys()}
    if v_t is None:
        v_t = {k: np.zeros_like(delta[k]) for k in delta.keys()}
    sq = {k: np.multiply(delta[k], delta[k]) for k in delta.keys()}
    if method == "adagrad":
        v_t = {k: v_t[k] + sq[k] for k in delta.keys()}
    elif method == "yogi":
        v_t = {k: v_t[k] - (1 - beta2) * sq[k] * np.sign(v_t[k] - sq[k]) for k in delta.keys()}
    elif method == "adam":
        v_t = {k: beta2 * v_t[k] + (1 - beta2) * sq[k] for k in delta.keys()}
    else:
        raise ValueError(method)
    w_local = dict(w_local)
    for k in w_glob.keys():
        w_local[k] = w_local[k] + eta * delta[k] / (np.sqrt(v_t[k]) + tau)
    return w_local, v_t


def dyn_f(w_glob, h, theta, n_clients, alpha=0.01):
    """dyn.py:17-36 with the state passed explicitly: h is updated IN PLACE (keys whose in-place
    float update numpy refuses, e.g. int64 BN counters, are skipped, dyn.py:24-29); returns
    (new w_glob, new theta) — theta becomes w_glob (dyn.py:35)."""
    delta = {k: w_glob[k] * n_clients - theta[k] for k in h.keys()}
    skipped = []
    for k in h.keys():
        try:
            h[k] -= alpha / n_clients * delta[k]
        except Exception:
            skipped.append(k)
    w_glob = dict(w_glob)
    for k in h.keys():
        if k in skipped:
            continue
        w_glob[k] = w_glob[k] - alpha * h[k]
    return w_glob, w_glob


def logits_mean(logits_lst):
    """Distill.aggregate_logits (distill.py:42-46): user_logits = 0; user_logits += item for each
    table in list order (0 + t0 makes a fresh array: -0.0 becomes +0.0); / len(logits_lst) in the
    tables' dtype.  torch tensors are restated through numpy (same IEEE fp32/f64 ops, and torch's
    CPU true-divide by a Python int is the correctly rounded division, checked by the fixtures)."""
    arrs = [np.asarray(t.numpy() if hasattr(t, "numpy") else t) for t in logits_lst]
    acc = 0
    for a in arrs:
        acc += a
    return acc / len(arrs)


# ---------------------------------------------------------------------------------------------
# C restatement (liboracle.so)
# ---------------------------------------------------------------------------------------------

MODE_W32_DIV64, MODE_W32_DIV32, MODE_W64 = 0, 1, 2
OPS = {"avgm": 1, "adagrad": 2, "yogi": 3, "adam": 4}


def build():
    """Compile liboracle.so with the committed Makefile (gcc, -ffp-contract=off)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = _HERE / "liboracle.so"
        src = _HERE / "fa_oracle.c"
        if not path.exists() or path.stat().st_mtime < src.stat().st_mtime:
            build()
        L = ctypes.CDLL(str(path))
        P, I64, I32, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        for name, args in {
            "ora_reduce_w32_div64": [P, I64, I32, P, D, I64, P],
            "ora_reduce_w32_div32": [P, I64, I32, P, ctypes.c_float, I64, P],
            "ora_reduce_w64": [P, I64, I32, P, D, I64, P],
            "ora_sum_w32_splitn": [P, I64, I32, P, I32, I64, P, I32],
            "ora_reduce_f64": [P, I64, I32, P, D, I64, P],
            "ora_reduce_i64": [P, I64, I32, P, D, I64, P],
            "ora_update_f64": [I32, P, P, P, D, D, D, D, I64, P],
            "ora_update_f32": [I32, P, P, P, D, D, D, D, I64, P],
            "ora_fill_uniform": [P, I64, I32, I64, ctypes.c_uint64, I64, I64],
            "ora_update_dyn_f64": [P, P, P, D, D, I64, P],
            "ora_update_dyn_f32": [P, P, P, D, D, I64, P],
        }.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = None
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def c_reduce(mode, stack, weights, denom):
    """Per-element sequential reduce of a [N, P] stack.  mode: MODE_* (fp32 stack), or 'f64' /
    'i64' for float64 / int64 stacks.  Returns the f64 (or f32 for DIV32) mean [P]."""
    L = lib()
    n, p = stack.shape
    if mode == "f64":
        stack = np.ascontiguousarray(stack, np.float64)
        w = np.ascontiguousarray(weights, np.float64)
        out = np.empty(p, np.float64)
        L.ora_reduce_f64(_ptr(stack), p, n, _ptr(w), float(denom), p, _ptr(out))
        return out
    if mode == "i64":
        stack = np.ascontiguousarray(stack, np.int64)
        w = np.ascontiguousarray(weights, np.int64)
        out = np.empty(p, np.float64)
        L.ora_reduce_i64(_ptr(stack), p, n, _ptr(w), float(denom), p, _ptr(out))
        return out
    stack = np.ascontiguousarray(stack, np.float32)
    if mode == MODE_W32_DIV64:
        w = np.ascontiguousarray(weights, np.float32)
        out = np.empty(p, np.float64)
        L.ora_reduce_w32_div64(_ptr(stack), p, n, _ptr(w), float(denom), p, _ptr(out))
    elif mode == MODE_W32_DIV32:
        w = np.ascontiguousarray(weights, np.float32)
        out = np.empty(p, np.float32)
        L.ora_reduce_w32_div32(_ptr(stack), p, n, _ptr(w), float(denom), p, _ptr(out))
    elif mode == MODE_W64:
        w = np.ascontiguousarray(weights, np.float64)
        out = np.empty(p, np.float64)
        L.ora_reduce_w64(_ptr(stack), p, n, _ptr(w), float(denom), p, _ptr(out))
    else:
        raise ValueError(mode)
    return out


def c_reduce_splitn(mode, stack, weights, denom, splits=4, guard=True):
    """The split-N kernel's order and cancellation guard (ora_sum_w32_splitn) for the fp32-weight
    modes, then the mode's divide: f64 [P] for MODE_W32_DIV64, fp32 for MODE_W32_DIV32 — as
    c_reduce returns them.  guard=False: the bare reordered sum (to measure the reordering)."""
    L = lib()
    n, p = stack.shape
    stack = np.ascontiguousarray(stack, np.float32)
    w = np.ascontiguousarray(weights, np.float32)
    acc = np.empty(p, np.float32)
    L.ora_sum_w32_splitn(_ptr(stack), p, n, _ptr(w), int(splits), p, _ptr(acc), int(bool(guard)))
    if mode == MODE_W32_DIV64:
        return acc.astype(np.float64) / float(denom)
    if mode == MODE_W32_DIV32:
        return acc / np.float32(denom)
    raise ValueError("split-N order is defined here for the fp32-weight modes")


def c_update(op, g, local32, v, beta=0.9, eta=1e-1, tau=1e-9, beta2=0.99):
    """AVGM / OPT update: returns new w (dtype of g); v (same dtype as g) is updated in place."""
    L = lib()
    opi = OPS[op]
    local32 = np.ascontiguousarray(local32, np.float32)
    n = local32.size
    if g.dtype == np.float64:
        assert v.dtype == np.float64 and v.flags.c_contiguous
        g = np.ascontiguousarray(g)
        out = np.empty(n, np.float64)
        L.ora_update_f64(opi, _ptr(g), _ptr(local32), _ptr(v), beta, eta, tau, beta2, n, _ptr(out))
    else:
        assert g.dtype == np.float32 and v.dtype == np.float32 and v.flags.c_contiguous
        g = np.ascontiguousarray(g)
        out = np.empty(n, np.float32)
        L.ora_update_f32(opi, _ptr(g), _ptr(local32), _ptr(v), beta, eta, tau, beta2, n, _ptr(out))
    return out


def c_update_dyn(g, h32, theta, n_clients, alpha=0.01):
    """FedDyn update per element (dyn.py:17-36): h32 (fp32) and theta (dtype of g) are updated in
    place; returns the new w_glob (dtype of g)."""
    L = lib()
    assert h32.dtype == np.float32 and h32.flags.c_contiguous and theta.flags.c_contiguous
    g = np.ascontiguousarray(g)
    out = np.empty_like(g)
    if g.dtype == np.float64:
        assert theta.dtype == np.float64
        L.ora_update_dyn_f64(_ptr(g), _ptr(h32), _ptr(theta), float(n_clients), alpha, g.size, _ptr(out))
    else:
        assert g.dtype == np.float32 and theta.dtype == np.float32
        L.ora_update_dyn_f32(_ptr(g), _ptr(h32), _ptr(theta), float(n_clients), alpha, g.size, _ptr(out))
    return out


def fill_uniform(n_rows, n_cols, seed, row0=0, col0=0):
    """Host copy of the device generator (fa_fill_uniform_f32): [n_rows, n_cols] fp32."""
    out = np.empty((n_rows, n_cols), np.float32)
    if out.size:
        lib().ora_fill_uniform(_ptr(out), n_cols, n_rows, n_cols, seed, row0, col0)
    return out
