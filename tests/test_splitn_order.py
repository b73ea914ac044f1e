"""The opt-in split-N order against the reference's, on the CPU, exactly: oracle.c_reduce (the
reference's sequential fp32 sum, pinned to its fixtures) vs oracle.c_reduce_splitn (the split-N
kernel's splits, tree and cancellation guard — tests/test_gpu_splitn.py pins the kernel to it bit
for bit).  At the selection limit (kSplitMaxN clients) every LeNet5 tensor must be within the
north star's 1e-6, for zero-mean, near-common and nearly cancelling uploads and for Python-float,
int (MOON) and unit weights; unguarded, cancelling tensors are not (why the guard exists)."""
import re
from pathlib import Path

import numpy as np
import pytest

import oracle
from flearn_amd import layouts
from splitn_error import data, tensors, weights

TOL = 1e-6
HIP = Path(__file__).resolve().parent.parent / "flearn_amd" / "csrc" / "fa_reduce.hip"


def split_max_n():
    m = re.search(r"kSplitMaxN\s*=\s*(\d+)", HIP.read_text())
    return int(m.group(1))


def _worst(n, dk, wk, guard, seeds=(1, 2)):
    lay, p = tensors(layouts.get("lenet5"))
    rng = np.random.default_rng(0)
    worst = 0.0
    for seed in seeds:
        x = data(dk, n, p, seed + n)
        w = weights(wk, n, rng)
        w32 = np.asarray(w, np.float64).astype(np.float32)
        denom = float(np.sum(w))
        a = oracle.c_reduce(oracle.MODE_W32_DIV64, x, w32, denom)
        b = oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, x, w32, denom, guard=guard)
        for _, off, m in lay:
            ra, rb = a[off : off + m], b[off : off + m]
            nrm = np.linalg.norm(ra)
            worst = max(worst, float(np.linalg.norm(ra - rb) / nrm) if nrm else 0.0)
    return worst


def test_limit_is_what_the_sweep_supports():
    assert split_max_n() == 256


@pytest.mark.parametrize("dk", ["zero_mean", "near_common", "cancelling"])
@pytest.mark.parametrize("wk", ["ones", "moon_int", "float"])
def test_guarded_split_order_within_tolerance_at_the_limit(dk, wk):
    assert _worst(split_max_n(), dk, wk, guard=True) <= TOL


def test_unguarded_order_fails_on_cancelling_tensors():
    assert _worst(64, "cancelling", "ones", guard=False, seeds=(1,)) > 10 * TOL


def test_split_order_restatement_basics():
    x = oracle.fill_uniform(37, 1000, 5)
    w = np.linspace(0.5, 2, 37).astype(np.float32)
    seq = oracle.c_reduce(oracle.MODE_W32_DIV64, x, w, 3.0)
    # one split, no guard: the sequential sum itself
    assert np.array_equal(oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, x, w, 3.0, splits=1, guard=False), seq)
    # the guard only ever swaps in the sequential value
    g = oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, x, w, 3.0)
    u = oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, x, w, 3.0, guard=False)
    assert np.all((g == seq) | (g == u))
