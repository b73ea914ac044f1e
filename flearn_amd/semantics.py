"""Which arithmetic the reference performs, decided from the weight objects and tensor dtype.

The reference reduce (flearn/common/strategy/strategy.py:123-129) is plain numpy:

    w = a0 * x0;  w += a_n * x_n;  w = np.divide(w, np.sum(agg_weight_lst))

so its precision is whatever numpy's promotion (NEP 50, numpy >= 2) gives each step:

* product/sum dtype  = np.result_type(a_n, x.dtype): Python float/int weights are "weak" and keep
  fp32 tensors in fp32 (the weight is rounded to fp32 first); np.float64/np.int64 weights are
  "strong" and promote to float64;
* denominator        = np.sum(agg_weight_lst), a numpy scalar (float64 for Python floats, int64
  for Python ints, float32 for np.float32 weights);
* result dtype       = promotion of the sum dtype with that (strong) scalar; integer sums are
  true-divided into float64.

This module reproduces that decision table without touching tensor data, and returns the weights
cast exactly the way numpy casts them, so the device kernels can run the same arithmetic.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _native as na

KIND_F32 = "f32"  # fp32 tensors -> fa_reduce_f32 (modes W32_DIV64 / W32_DIV32 / W64)
KIND_F64 = "f64"  # float64 tensors, or int64 tensors promoted to f64 -> fa_reduce_f64
KIND_I64 = "i64"  # int64 tensors with integer weights -> fa_reduce_i64

_F32, _F64, _I64 = np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int64)


@dataclass(frozen=True)
class Numerics:
    kind: str  # KIND_*
    mode: int  # fa_reduce_f32 mode (KIND_F32 only)
    weights: np.ndarray  # per-client weights, cast like numpy casts them (fp32 / f64 / int64)
    denom: float  # np.sum(agg_weight_lst) as an exact double
    acc_dtype: np.dtype  # dtype of the running sum
    out_dtype: np.dtype  # dtype of the reference's w_glob[k]

    @property
    def prec(self) -> int:
        return na.PREC_F32 if self.out_dtype == _F32 else na.PREC_F64


def _is_weight(w) -> bool:
    return isinstance(w, (bool, int, float, np.integer, np.floating))


def denominator(agg_weight_lst):
    """strategy.py:127 — np.sum over the weight list (pairwise), kept as numpy computes it."""
    return np.sum(agg_weight_lst)


def resolve(agg_weight_lst, x_dtype) -> Numerics:
    """Decide the arithmetic for tensors of dtype `x_dtype` under these weights (see module doc).
    Raises TypeError for combinations the engine does not reproduce (mixed promotion, fp16...)."""
    if len(agg_weight_lst) == 0:
        raise IndexError("list index out of range")  # what agg_weight_lst[0] raises (strategy.py:123)
    for w in agg_weight_lst:
        if not _is_weight(w):
            raise TypeError(f"agg_weight must be a real scalar, got {type(w).__name__}")
    x_dtype = np.dtype(x_dtype)
    if x_dtype not in (_F32, _F64, _I64):
        raise TypeError(f"tensor dtype {x_dtype} is not supported by the aggregation kernels")
    prods = {np.result_type(w, x_dtype) for w in agg_weight_lst}
    if len(prods) != 1:
        raise TypeError(
            "agg_weight types promote differently (" + ", ".join(sorted(map(str, prods))) + "); "
            "the reference would mix precisions per client — use one weight type"
        )
    acc = prods.pop()
    denom = denominator(agg_weight_lst)
    out = np.result_type(acc, denom)
    if out.kind in "iub":
        out = _F64  # np.divide on integers is true division
    if out not in (_F32, _F64):
        raise TypeError(f"result dtype {out} is not supported")

    if acc == _F32:
        weights = np.array([np.float32(w) for w in agg_weight_lst], dtype=np.float32)
        mode = na.MODE_W32_DIV64 if out == _F64 else na.MODE_W32_DIV32
        return Numerics(KIND_F32, mode, weights, float(denom), acc, out)
    if acc == _F64:
        weights = np.array([np.float64(w) for w in agg_weight_lst], dtype=np.float64)
        kind = KIND_F32 if x_dtype == _F32 else KIND_F64
        return Numerics(kind, na.MODE_W64, weights, float(denom), acc, out)
    if acc == _I64:
        weights = np.array([int(w) for w in agg_weight_lst], dtype=np.int64)
        return Numerics(KIND_I64, -1, weights, float(denom), acc, out)
    raise TypeError(f"accumulation dtype {acc} is not supported")
