"""GPU: property test of the stack kernel's geometry selection (fa_reduce.hip launch_reduce) —
random window widths drawn around every boundary where the host picks another kernel, grid or
piece (the narrow kernel, one-piece shares just past a power of two, the 13/16-of-the-CUs band,
row-major groups, the wide windows split into launches), random client counts, weights, column
offsets and epilogues (mean, AVGM, Adagrad, Yogi, Adam) — against the C oracle, bit for bit.
The geometry may change how the columns are cut, never a column's sum or update."""
import os

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle
from flearn_amd import _native as na
from flearn_amd import aggregator as agg
from golden_io import bitwise_equal

pytestmark = pytest.mark.gpu

CUS = 256  # MI355X; other CU counts move the boundaries, the property holds anyway
# 1-KiB row chunks at which the selection changes (share = ceil(chunks / grid), grid 192 or
# more): shares 2 / 4 / 8 / 16 / 32 / 64 on 192 blocks, the fill rule's 3/5 points, the
# 13/16 and 16/16 bands
EDGES = sorted({c for s in (2, 4, 8, 16, 32, 64) for c in (192 * s, 192 * s + 1, 192 * s * 3 // 5 * 2)}
               | {CUS * 13 // 16 * 64, CUS * 13 // 16 * 64 + 1, CUS * 64, CUS * 64 + 1})
MAX_ELEMS = 40_000_000  # clients x columns: the C oracle's share of a test stays in seconds


@st.composite
def window(draw):
    if draw(st.booleans()):
        chunks = draw(st.sampled_from(EDGES)) + draw(st.integers(-2, 2))
        ncols = max(1, chunks * 256 - draw(st.integers(0, 255)))  # ragged ends included
    else:
        ncols = int(10 ** draw(st.floats(0.0, 6.65)))
    n_max = max(1, min(130, MAX_ELEMS // ncols))
    n = draw(st.sampled_from(sorted({1, 2, 3, 5, min(17, n_max), n_max})))
    n = min(n, n_max)
    op = draw(st.sampled_from(["mean", "mean", "avgm", "adagrad", "yogi", "adam"]))
    col0 = draw(st.sampled_from([0, 0, 4, 64, 1028]))
    seed = draw(st.integers(0, 2**31 - 1))
    return n, ncols, op, col0, seed


@settings(max_examples=int(os.environ.get("FA_PROP_EXAMPLES", "40")), deadline=None,
          suppress_health_check=list(HealthCheck))
@given(c=window())
def test_window_geometry_matches_oracle(c, cuda):
    n, ncols, op, col0, seed = c
    stride = -(-(col0 + ncols) // 64) * 64
    x = torch.empty((n, stride), dtype=torch.float32, device=cuda)
    agg.fill_uniform(x, seed)
    rng = np.random.default_rng(seed)
    w = rng.uniform(0.25, 3.0, n).astype(np.float32)
    denom = float(np.sum([float(v) for v in w]))
    wd = torch.from_numpy(w).to(cuda)
    xs = x[:, col0:col0 + ncols].cpu().numpy()
    g = oracle.c_reduce(oracle.MODE_W32_DIV64, xs, w, denom)
    if op == "mean":
        out64 = torch.empty(ncols, dtype=torch.float64, device=cuda)
        agg.reduce_stack(x, wd, na.MODE_W32_DIV64, denom, col_begin=col0, n_cols=ncols, out64=out64)
        assert bitwise_equal(out64.cpu().numpy(), g), (n, ncols, col0)
        return
    prev = torch.empty((1, ncols), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed ^ 0x5A5A)
    prev = prev[0]
    v = torch.from_numpy(rng.uniform(0.0, 0.5, ncols)).to(cuda)
    prev_h, v_h = prev.cpu().numpy().copy(), v.cpu().numpy().copy()
    out32 = torch.empty(ncols, dtype=torch.float32, device=cuda)
    v_out = torch.empty_like(v)
    agg.reduce_stack(x, wd, na.MODE_W32_DIV64, denom, col_begin=col0, n_cols=ncols, out32=out32,
                     op=na.OP_BY_NAME[op], prev=prev, v=v, v_out=v_out)
    want = oracle.c_update(op, g, prev_h, v_h)  # updates v_h in place
    assert bitwise_equal(out32.cpu().numpy(), want.astype(np.float32)), (n, ncols, op, col0)
    assert bitwise_equal(v_out.cpu().numpy(), v_h), (n, ncols, op, col0)
