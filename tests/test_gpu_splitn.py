"""GPU: the opt-in split-N kernel (fa_reduce_f32_splitn) for narrow models with many clients.

Not the reference's summation order (each column's clients are cut into contiguous splits summed in
list order, combined by a fixed tree; columns whose terms nearly cancel are re-summed in list order
by the kernel's guard), so the bar against the reference is the north star's tolerance: normwise
relative error <= 1e-6 per fp32 tensor against the C oracle (the reference's sequential arithmetic,
pinned to its fixtures).  The kernel itself is pinned bit for bit to the oracle's restatement of
its own order and guard (oracle.c_reduce_splitn), so every number the tolerance is argued from
(tests/test_splitn_order.py, profiles/r03/splitn_error*.json) is what the GPU computes; where the
library falls back to the sequential kernel (few or many clients, wide windows) results are
bit-exact to the reference."""
import numpy as np
import pytest
import torch

import oracle
from flearn_amd import AVG, AVGM
from flearn_amd import _native as na
from flearn_amd import aggregator as agg
from flearn_amd import layouts
from golden_io import bitwise_equal

pytestmark = pytest.mark.gpu

TOL = 1e-6  # north star: "within 1e-6 relative per fp32 tensor"
SPLIT_MAX_N = 256  # kSplitMaxN (flearn_amd/csrc/fa_reduce.hip)


def _uses_split(n, p):
    chunks = ((p + 3) // 4 + 63) // 64
    return 8 <= n <= SPLIT_MAX_N and chunks < torch.cuda.get_device_properties(0).multi_processor_count


def _rel(got, want):
    want = np.asarray(want, np.float64)
    d = np.linalg.norm(np.asarray(got, np.float64) - want)
    n = np.linalg.norm(want)
    return d / n if n else d


def _stack(n, p, seed):
    stride = -(-p // 64) * 64
    x = torch.empty((n, stride), dtype=torch.float32, device="cuda")
    agg.fill_uniform(x, seed=seed, n_cols=p)
    return x


def _cancelling_stack(n, p, seed):
    """Client pairs that nearly cancel (the mean is ~1e-4 of the values), plus a zero-mean tail."""
    h = oracle.fill_uniform(n, p, seed)
    y = np.empty_like(h)
    y[0::2] = h[: y[0::2].shape[0]]
    y[1::2] = -h[: y[1::2].shape[0]] + np.float32(1e-4) * oracle.fill_uniform(n // 2, p, seed + 7)
    stride = -(-p // 64) * 64
    x = torch.zeros((n, stride), dtype=torch.float32, device="cuda")
    x[:, :p] = torch.from_numpy(y).cuda()
    return x, y


@pytest.mark.parametrize("n,p", [(1000, 44_426), (64, 44_426), (200, 4_099), (256, 44_426), (257, 44_426),
                                 (4000, 44_416), (9, 70_001), (33, 3)])
@pytest.mark.parametrize("op", ["mean", "avgm", "adagrad"])
def test_splitn_within_tolerance_and_deterministic(n, p, op, cuda):
    x = _stack(n, p, seed=n + p)
    wh = (np.arange(1, n + 1) % 7 + 0.5).astype(np.float32)
    w = torch.from_numpy(wh).to(cuda)
    denom = float(np.sum([float(v) for v in wh]))
    kw, prev_h = {}, None
    if op != "mean":
        prev = torch.empty((1, x.shape[1]), dtype=torch.float32, device=cuda)
        agg.fill_uniform(prev, seed=3)
        prev_h = prev[0, :p].cpu().numpy().copy()
    outs = []
    for _ in range(2):
        out = torch.empty(x.shape[1], dtype=torch.float64, device=cuda)
        if op != "mean":
            kw = dict(op=na.OP_BY_NAME[op], prev=prev[0].clone(), v=torch.zeros(x.shape[1], dtype=torch.float64, device=cuda))
        agg.reduce_stack(x, w, na.MODE_W32_DIV64, denom, n_cols=p, out64=out, reorder=True, **kw)
        outs.append(out[:p].cpu().numpy())
    assert bitwise_equal(outs[0], outs[1])  # deterministic
    xh = oracle.fill_uniform(n, p, n + p)
    want = oracle.c_reduce(oracle.MODE_W32_DIV64, xh, wh, denom)
    split = oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, xh, wh, denom)
    if op != "mean":
        want = oracle.c_update(op, want, prev_h, np.zeros(p))
        split = oracle.c_update(op, split, prev_h, np.zeros(p))
    assert _rel(outs[0], want) <= TOL
    if _uses_split(n, p):
        assert bitwise_equal(outs[0], split)  # the kernel's own order and guard, bit for bit
    else:
        assert bitwise_equal(outs[0], want)  # the library kept the sequential kernel


@pytest.mark.parametrize("n", [16, 100, 256])
def test_splitn_cancellation_guard(n, cuda):
    """Near-cancelling tensors: every column whose terms nearly cancel is re-summed in
    the reference's order by the kernel's guard, so the result is bit-equal to the reference
    there; unguarded, the reordered sum lies ~1e-4 away (relative) on this data."""
    p = 44_426
    x, xh = _cancelling_stack(n, p, seed=n)
    wh = np.ones(n, np.float32)
    out = torch.empty(x.shape[1], dtype=torch.float64, device=cuda)
    agg.reduce_stack(x, torch.from_numpy(wh).to(cuda), na.MODE_W32_DIV64, float(n), n_cols=p, out64=out, reorder=True)
    got = out[:p].cpu().numpy()
    want = oracle.c_reduce(oracle.MODE_W32_DIV64, xh, wh, float(n))
    assert bitwise_equal(got, oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, xh, wh, float(n)))
    assert _rel(got, want) <= TOL
    assert _rel(oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, xh, wh, float(n), guard=False), want) > 10 * TOL


def test_splitn_at_the_limit_moon_weights(cuda):
    """N = kSplitMaxN (256) with MOON-style integer weights (MOONClient.py:19, len(trainloader)):
    per LeNet5 tensor within 1e-6 of the reference, through the Strategy API."""
    layout = layouts.get("lenet5")
    p = layouts.fp32_elems(layout)
    flat = oracle.fill_uniform(SPLIT_MAX_N, p, seed=11)
    clients = [layouts.synthetic_state_dict(layout, flat[i]) for i in range(SPLIT_MAX_N)]
    weights = [int(v) for v in np.random.default_rng(3).integers(1, 601, SPLIT_MAX_N)]
    s = AVG()
    s.reorder = True
    got = s.server([{"agg_weight": a, "params": c} for a, c in zip(weights, clients)], 0)["w_glob"]
    want = oracle.server_ensemble(weights, clients)
    for k in want:
        assert _rel(got[k], want[k]) <= TOL, k


def test_strategy_reorder_lenet5_1000_clients(cuda):
    """AVG with reorder on 1000 LeNet5 uploads (the small-P / deep-N shape): every tensor within
    1e-6 normwise of the reference's numpy result; dtypes and keys as the reference's."""
    layout = layouts.get("lenet5")
    p = layouts.fp32_elems(layout)
    flat = oracle.fill_uniform(1000, p, seed=5)
    clients = [layouts.synthetic_state_dict(layout, flat[i]) for i in range(1000)]
    weights = [float(1 + i % 5) for i in range(1000)]
    s = AVG()
    s.reorder = True
    got = s.server([{"agg_weight": a, "params": c} for a, c in zip(weights, clients)], 0)["w_glob"]
    want = oracle.server_ensemble(weights, clients)
    assert set(got) == set(want)
    for k in want:
        assert np.asarray(got[k]).dtype == np.asarray(want[k]).dtype
        assert _rel(got[k], want[k]) <= TOL, k


def test_strategy_reorder_keeps_wide_models_bit_exact(cuda):
    layout = [x for x in layouts.get("resnet18") if x[2] == "f32"]
    p = layouts.fp32_elems(layout)
    flat = oracle.fill_uniform(12, p, seed=9)
    clients = [layouts.synthetic_state_dict(layout, flat[i]) for i in range(12)]
    s = AVGM(server_side=True)
    s.reorder = True
    got = s.server([{"agg_weight": 1.0, "params": c} for c in clients], 0)["w_glob"]
    want = oracle.server_ensemble([1.0] * 12, clients)
    for k in want:
        assert bitwise_equal(np.asarray(got[k]), np.asarray(want[k])), k
