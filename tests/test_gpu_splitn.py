"""GPU: the opt-in split-N kernel (fa_reduce_f32_splitn) for narrow models with many clients.

Not the reference's summation order (each column's clients are cut into contiguous splits summed in
list order, combined by a fixed tree), so the bar is the north star's tolerance instead of bit
equality: normwise relative error <= 1e-6 per fp32 tensor against the C oracle (the reference's
sequential arithmetic, pinned to its fixtures), deterministic run to run; and where the library
falls back to the sequential kernel (few clients, wide windows) results stay bit-exact."""
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


@pytest.mark.parametrize("n,p", [(1000, 44_426), (64, 44_426), (200, 4_099), (4000, 44_416), (9, 70_001), (33, 3)])
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
    want = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, n + p), wh, denom)
    if op != "mean":
        want = oracle.c_update(op, want, prev_h, np.zeros(p))
    assert _rel(outs[0], want) <= TOL
    if n < 8 or n > 2048 or ((p + 3) // 4 + 63) // 64 >= torch.cuda.get_device_properties(0).multi_processor_count:
        assert bitwise_equal(outs[0], want)  # the library kept the sequential kernel


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
