"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors and the
C oracle.  Bar: bit-exact (every output dtype, NaN position and sign of zero) — the kernels run
the reference's fp32/f64 operation sequence with no contraction."""
import math
import os

import numpy as np
import pytest
import torch

import oracle
from flearn_amd import AVG, AVGM, BN, LG, LG_R, OPT
from flearn_amd import _native as na
from flearn_amd import aggregator as agg
from flearn_amd import layouts
from golden_io import Golden, assert_dict_bitwise, bitwise_equal, cases

pytestmark = pytest.mark.gpu

REDUCE_CASES = [c for c in cases() if c.startswith(("avg_", "bn_", "lg_", "trace_"))]
ROUND_CASES = [c for c in cases() if c.endswith("_rounds3") and not c.startswith("dyn_")]


def upload(clients, weights):
    return [{"agg_weight": w, "params": c} for w, c in zip(weights, clients)]


def strategy_for(g: Golden):
    call = g.meta["call"]
    if call.startswith("BN()"):
        return BN()
    if call.startswith("LG_R("):
        return LG_R(g.meta["shared_key_layers"])
    if call.startswith("LG("):
        return LG(g.meta["shared_key_layers"])
    return AVG()


# ---------------------------------------------------------------------------------------------
# golden vectors from the reference
# ---------------------------------------------------------------------------------------------


@pytest.mark.parametrize("name", REDUCE_CASES)
def test_strategy_server_matches_reference(name, cuda):
    g = Golden(name)
    s = strategy_for(g)
    got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
    want = g.output()
    assert_dict_bitwise(got, want, name)
    kinds = g.output_kinds()
    for k, v in got.items():  # value types as the reference returns them
        if kinds[k].startswith("scalar:"):
            assert type(v).__name__ == kinds[k].split(":")[1], k
        elif kinds[k].startswith("torch:"):
            assert isinstance(v, torch.Tensor) and str(v.dtype) == kinds[k][6:], k
        else:
            assert isinstance(v, np.ndarray), k


@pytest.mark.parametrize("name", REDUCE_CASES)
def test_float32_output_is_cast_of_reference(name, cuda):
    """output='float32' returns fl32(w_glob) — what load_state_dict stores."""
    g = Golden(name)
    if g.meta.get("input_kind") == "torch":
        pytest.skip("torch uploads keep torch outputs")
    s = strategy_for(g)
    s.output = "float32"
    got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
    for k, w in g.output().items():
        w = np.asarray(w)
        if w.dtype == np.float64 and g.meta["in_dtypes"][k] == "float32":
            assert bitwise_equal(np.asarray(got[k]), w.astype(np.float32)), k


def _round_inputs(g, r):
    from golden_io import decode_weight, regenerate

    layout = [(k, tuple(s)) for k, s in g.meta["gen"]["layout"]]
    clients = regenerate(layout, 6, g.meta["gen"]["seeds"][r])
    return clients, [decode_weight(e) for e in g.meta["round_weights"][r]]


@pytest.mark.parametrize("name", ROUND_CASES)
def test_server_side_fused_optimizer_matches_reference(name, cuda):
    """Server-fused FedAVGM / FedOPT: round r = mean of fresh uploads, then the reference update
    with w_local = previous global (fp32); 3 rounds, state carried in HBM."""
    g = Golden(name)
    op = g.meta["op"]
    s = AVGM(server_side=True) if op == "avgm" else OPT(server_side=True, method=op)
    s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
    for r in range(g.meta["rounds"]):
        clients, weights = _round_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        assert_dict_bitwise(got, g.output(f"w{r}"), f"{name} w{r}")
        v = s.server_opt.v_t(s.engine.last_plan)
        assert_dict_bitwise(v, g.output(f"v{r}"), f"{name} v{r}")


@pytest.mark.parametrize("source", ["returned", "state_dict"])
@pytest.mark.parametrize("name", ROUND_CASES)
def test_server_optimizer_state_restores_on_a_fresh_strategy(name, source, cuda):
    """A server restart between rounds: round 0 on one strategy, its state saved (the w_glob the
    server returned + v_t(), or ServerOptimizer.state_dict()), then a FRESH AVGM / OPT(server_side)
    restores it (load_state) and runs rounds 1-2 — bit-identical to the reference's 3 rounds
    (avgm.py:28-35, opt.py:45-63 keep v_t across rounds; without the restore the momentum or
    Adagrad state would silently restart from zero)."""
    g = Golden(name)
    op = g.meta["op"]

    def fresh():
        return AVGM(server_side=True) if op == "avgm" else OPT(server_side=True, method=op)

    s = fresh()
    s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
    clients, weights = _round_inputs(g, 0)
    got = s.server(upload(clients, weights), 0)["w_glob"]
    assert_dict_bitwise(got, g.output("w0"), f"{name} w0")
    if source == "returned":
        saved = {"w_glob": {k: np.array(v, copy=True) for k, v in got.items()}, "v_t": s.server_opt.v_t()}
    else:
        saved = s.server_opt.state_dict()
    del s
    s = fresh()
    s.server_opt.load_state(saved)
    for r in range(1, g.meta["rounds"]):
        clients, weights = _round_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        assert_dict_bitwise(got, g.output(f"w{r}"), f"{name} w{r} after restore")
        assert_dict_bitwise(s.server_opt.v_t(), g.output(f"v{r}"), f"{name} v{r} after restore")


def test_server_optimizer_restore_refuses_a_foreign_v_t(cuda):
    """v_t restored for another model: a missing key raises KeyError, a wrong shape ValueError —
    at the next round, before anything is launched."""
    name = next(n for n in ROUND_CASES if Golden(n).meta["op"] == "adagrad")
    g = Golden(name)
    prev0 = {k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")}
    clients, weights = _round_inputs(g, 0)
    v0 = {k: np.zeros(np.shape(v)) for k, v in prev0.items()}
    missing = dict(v0)
    missing.pop(next(iter(missing)))
    wrong = {k: (np.zeros(3) if i == 0 else v) for i, (k, v) in enumerate(v0.items())}
    for bad, exc in ((missing, SystemExit), (wrong, SystemExit)):
        s = OPT(server_side=True, method="adagrad")
        s.server_opt.load_state({"w_glob": prev0, "v_t": bad})
        with pytest.raises(exc):  # a client/config data error: server_exception, as the reference's
            s.server(upload(clients, weights), 0)


def test_fused_round_refused_keeps_optimizer_state(cuda, monkeypatch):
    """A fused step whose launch is refused (here: reduce_stack raising before it queues anything)
    leaves the double-buffered state on the pair it had, so the rounds after it still match the
    reference (ServerOptimizer.swap_buffers / unswap)."""
    from flearn_amd import aggregator

    name = next(n for n in ROUND_CASES if Golden(n).meta["op"] == "avgm")
    g = Golden(name)
    s = AVGM(server_side=True)
    s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
    real = aggregator.reduce_stack
    for r in range(g.meta["rounds"]):
        clients, weights = _round_inputs(g, r)
        if r == 1:  # one refused attempt of round 1 first
            def refuse(*a, **k):
                if k.get("v_out") is not None:
                    raise ValueError("refused launch")
                return real(*a, **k)

            monkeypatch.setattr(aggregator, "reduce_stack", refuse)
            with pytest.raises(SystemExit):  # client/config data errors take server_exception
                s.server(upload(clients, weights), r)
            monkeypatch.setattr(aggregator, "reduce_stack", real)
        got = s.server(upload(clients, weights), r)["w_glob"]
        assert_dict_bitwise(got, g.output(f"w{r}"), f"{name} w{r}")
        assert_dict_bitwise(s.server_opt.v_t(s.engine.last_plan), g.output(f"v{r}"), f"{name} v{r}")


@pytest.mark.parametrize("name", ROUND_CASES)
def test_client_side_update_matches_reference(name, cuda):
    """AVGM.mean_momentum / OPT.adaptive_opt on the GPU (the reference's client_receive math)."""
    g = Golden(name)
    op = g.meta["op"]
    s = AVGM() if op == "avgm" else OPT()
    prev = {k[6:]: v.copy() for k, v in g.arrays.items() if k.startswith("prev0:")}
    for r in range(g.meta["rounds"]):
        avg = g.output(f"avg{r}")
        if op == "avgm":
            w = s.mean_momentum(dict(prev), avg, 0.9)
        else:
            w = s.adaptive_opt(dict(prev), avg, op)
        assert_dict_bitwise(w, g.output(f"w{r}"), f"{name} w{r}")
        assert_dict_bitwise(s.v_t, g.output(f"v{r}"), f"{name} v{r}")
        prev = {k: np.asarray(w[k]).astype(np.float32) for k in prev}


def test_empty_upload_list_exits_like_reference(cuda):
    with pytest.raises(SystemExit):
        AVG().server([], 0)


def test_shape_mismatch_is_rejected(cuda):
    a = {"w": np.ones((10, 1), np.float32)}
    b = {"w": np.ones((10,), np.float32)}
    with pytest.raises(SystemExit):
        AVG().server(upload([a, b], [1.0, 1.0]), 0)


def test_device_uploads(cuda):
    """Uploads already resident on the GPU are packed device-to-device."""
    g = Golden("avg_w1_n10")
    cl = [{k: torch.from_numpy(v).to(cuda) for k, v in c.items()} for c in g.clients()]
    s = AVG(output="device")
    got = s.server(upload(cl, g.weights()), 0)["w_glob"]
    for k, w in g.output().items():
        assert got[k].device.type == "cuda"
        assert bitwise_equal(got[k].cpu().numpy(), np.asarray(w).astype(np.float32)), k


# ---------------------------------------------------------------------------------------------
# kernel vs C oracle (seeded synthetic inputs generated on device, regenerated on the host)
# ---------------------------------------------------------------------------------------------


def _device_stack(n, stride, seed, cols=None):
    x = torch.empty((n, stride), dtype=torch.float32, device="cuda")
    agg.fill_uniform(x, seed, n_cols=cols)
    return x


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 16, 17, 100])
@pytest.mark.parametrize("ncols", [1, 3, 4, 5, 63, 1023, 2048, 2049, 4099, 70001])
def test_reduce_kernel_bit_exact(n, ncols, cuda):
    stride = -(-ncols // 64) * 64
    x = _device_stack(n, stride, seed=n * 7919 + ncols)
    w32 = (np.arange(1, n + 1, dtype=np.float64) * 0.37).astype(np.float32)
    denom = float(np.sum([float(v) for v in w32]))
    out64 = torch.empty(ncols, dtype=torch.float64, device=cuda)
    out32 = torch.empty(ncols, dtype=torch.float32, device=cuda)
    agg.reduce_stack(x, torch.from_numpy(w32).to(cuda), na.MODE_W32_DIV64, denom, n_cols=ncols,
                     out32=out32, out64=out64)
    want = oracle.c_reduce(oracle.MODE_W32_DIV64, x[:, :ncols].cpu().numpy(), w32, denom)
    assert bitwise_equal(out64.cpu().numpy(), want)
    assert bitwise_equal(out32.cpu().numpy(), want.astype(np.float32))


@pytest.mark.parametrize("n,ncols", [(3, 8388608), (5, 8388608 + 1), (2, 8388608 + 63), (9, 9000003)])
def test_reduce_kernel_big_tiles_ragged(n, ncols, cuda):
    """Buckets large enough for the one-tile-per-block 64-KiB geometry, with ragged ends."""
    stride = -(-ncols // 64) * 64
    x = _device_stack(n, stride, seed=ncols)
    w32 = np.linspace(0.5, 2.0, n).astype(np.float32)
    denom = float(np.sum([float(v) for v in w32]))
    out64 = torch.empty(ncols, dtype=torch.float64, device=cuda)
    agg.reduce_stack(x, torch.from_numpy(w32).to(cuda), na.MODE_W32_DIV64, denom, n_cols=ncols, out64=out64)
    want = oracle.c_reduce(oracle.MODE_W32_DIV64, x[:, :ncols].cpu().numpy(), w32, denom)
    assert bitwise_equal(out64.cpu().numpy(), want)


# row-pipeline geometry: each (n, ncols) lands on a different piece width V (1, 2, 4, 8, 16 KiB
# per wave) and pipeline depth D = 16/V on the 192/224-block grid, with ragged piece and window
# ends; deep stacks are the per-rank shapes of the multi-GPU runs
ROW_SHAPES = [(800, 150001), (300, 390001), (200, 700003), (64, 1500007), (40, 3300001), (17, 33), (2, 5000003),
              (10, 3300001),  # one piece per block on a widened grid (at most 13/16 of the CUs)
              (12, 3500001), (8, 4194304),  # past that: two pieces per block, row-major groups
              (20, 1600635), (30, 800318),  # a share just past a power of two: the grid that fills the piece
              (3, 14000003), (2, 9000001),  # row-major groups of 5 and 3 pieces
              (1000, 44426), (150, 44426), (300, 70001), (349, 70001), (600, 44426), (700, 3), (256, 1),
              (2000, 5)]  # narrow windows: one-wave blocks, D 16/32/40, tail rounds


@pytest.mark.parametrize("mode", [na.MODE_W32_DIV32, na.MODE_W64])
@pytest.mark.parametrize("n,ncols", [(5, 9_000_001), (1000, 44426), (400, 70001)])
def test_big_window_modes_bit_exact(mode, n, ncols, cuda):
    """Multi-piece windows (row-major geometry for fp32 sums, column-major for f64 sums) and narrow
    windows (one-wave blocks; f64 weights broadcast in two halves) in the np.float32 / np.float64
    weight modes."""
    stride = -(-ncols // 64) * 64
    x = _device_stack(n, stride, seed=ncols + mode)
    if mode == na.MODE_W64:
        w = np.linspace(0.5, 2.5, n)
        wd = torch.from_numpy(w).to(cuda)
        denom = float(np.sum(w))
    else:
        w = np.linspace(0.5, 2.5, n).astype(np.float32)
        wd = torch.from_numpy(w).to(cuda)
        denom = float(np.sum(w))  # np.float32 pairwise sum, exact as double
    out64 = torch.empty(ncols, dtype=torch.float64, device=cuda)
    out32 = torch.empty(ncols, dtype=torch.float32, device=cuda)
    agg.reduce_stack(x, wd, mode, denom, n_cols=ncols, out32=out32, out64=out64)
    want = oracle.c_reduce(mode, x[:, :ncols].cpu().numpy(), w, denom)
    got = out32.cpu().numpy() if want.dtype == np.float32 else out64.cpu().numpy()
    assert bitwise_equal(got, want)


@pytest.mark.parametrize("n,ncols", ROW_SHAPES)
def test_row_pipeline_geometries(n, ncols, cuda):
    stride = -(-ncols // 64) * 64
    x = _device_stack(n, stride, seed=n + ncols)
    w32 = np.linspace(0.25, 3.0, n).astype(np.float32)
    denom = float(np.sum([float(v) for v in w32]))
    out64 = torch.empty(ncols, dtype=torch.float64, device=cuda)
    agg.reduce_stack(x, torch.from_numpy(w32).to(cuda), na.MODE_W32_DIV64, denom, n_cols=ncols, out64=out64)
    want = oracle.c_reduce(oracle.MODE_W32_DIV64, x[:, :ncols].cpu().numpy(), w32, denom)
    assert bitwise_equal(out64.cpu().numpy(), want)


@pytest.mark.parametrize("n,ncols,op", [(300, 390001, "avgm"), (64, 1500007, "adagrad"), (800, 150001, "adam"),
                                         (50, 700003, "yogi"), (20, 3000001, "avgm"), (10, 3500001, "adagrad"),
                                         (6, 9000003, "avgm"), (1000, 44426, "avgm"), (400, 70001, "adagrad"),
                                         (120, 44426, "yogi"), (1000, 44426, "adam"),
                                         # shares of <= 8 KiB: the 4-wave kernels; past 13/16 of the CUs
                                         (100, 200080, "adagrad"), (60, 100000, "yogi"), (100, 300000, "adam"),
                                         (8, 4194304, "avgm"),
                                         # shares just past 32 / 16 KiB: filled, on 4 waves
                                         (40, 1600635, "yogi"), (50, 800318, "adagrad")])
def test_row_pipeline_fused_epilogues(n, ncols, op, cuda):
    stride = -(-ncols // 64) * 64
    x = _device_stack(n, stride, seed=ncols)
    w = np.ones(n, np.float32)
    prev = torch.empty((1, stride), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed=9)
    prev_h = prev[0, :ncols].cpu().numpy().copy()
    v = torch.full((ncols,), 0.5, dtype=torch.float64, device=cuda)
    v_h = v.cpu().numpy().copy()
    out32 = torch.empty(ncols, dtype=torch.float32, device=cuda)
    agg.reduce_stack(x, torch.from_numpy(w).to(cuda), na.MODE_W32_DIV64, float(n), n_cols=ncols, out32=out32,
                     op=na.OP_BY_NAME[op], prev=prev[0], v=v)
    g = oracle.c_reduce(oracle.MODE_W32_DIV64, x[:, :ncols].cpu().numpy(), w, float(n))
    want = oracle.c_update(op, g, prev_h, v_h)
    assert bitwise_equal(out32.cpu().numpy(), want.astype(np.float32))
    assert bitwise_equal(v.cpu().numpy(), v_h)


def test_row_pipeline_deep_window_offsets(cuda):
    """Windows of a deep stack (multi-GPU shard slices) equal the same columns of the full reduce."""
    n, stride = 400, 1 << 20
    x = _device_stack(n, stride, seed=3)
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    full = torch.empty(stride, dtype=torch.float64, device=cuda)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out64=full)
    for c0, width in [(0, 262144), (262144, 262144), (4096, 500003), (stride - 70004, 70001)]:
        part = torch.empty(width, dtype=torch.float64, device=cuda)
        agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), col_begin=c0, n_cols=width, out64=part)
        assert torch.equal(part, full[c0 : c0 + width]), c0


@pytest.mark.parametrize("dbuf", [False, True])
@pytest.mark.parametrize("p", [5_000_003, 8388608 + 5, 18_000_007])
@pytest.mark.parametrize("op", ["avgm", "adagrad", "yogi", "adam"])
def test_fused_epilogue_big_tiles(op, p, dbuf, cuda):
    """Fused f64 epilogues on row-major geometries of 2, 3 and 6 pieces per block (KG 2 / 3,
    8 waves x 8 KiB and 4 waves x 16 KiB steps: the instances whose f64 stores are regrouped into
    whole lines, DESIGN §4 finding 22), in place and double-buffered (v_out), against the C oracle."""
    n = 4
    stride = -(-p // 64) * 64
    x = _device_stack(n, stride, seed=21)
    w = np.ones(n, np.float32)
    prev = torch.empty((1, stride), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed=5)
    prev_h = prev[0, :p].cpu().numpy().copy()
    v = torch.full((p,), 0.25, dtype=torch.float64, device=cuda)
    v_h = v.cpu().numpy().copy()
    out64 = torch.empty(p, dtype=torch.float64, device=cuda)
    v_out = torch.empty_like(v) if dbuf else None
    agg.reduce_stack(x, torch.from_numpy(w).to(cuda), na.MODE_W32_DIV64, float(n), n_cols=p, out64=out64,
                     op=na.OP_BY_NAME[op], prev=prev[0], v=v, v_out=v_out)
    g = oracle.c_reduce(oracle.MODE_W32_DIV64, x[:, :p].cpu().numpy(), w, float(n))
    want = oracle.c_update(op, g, prev_h, v_h)
    assert bitwise_equal(out64.cpu().numpy(), want)
    assert bitwise_equal((v_out if dbuf else v).cpu().numpy(), v_h)


@pytest.mark.parametrize("col_begin", [0, 4, 64, 1000, 4096])
def test_column_window(col_begin, cuda):
    """A window [col_begin, +n) equals the same columns of the full reduce (sharding property)."""
    n, stride = 13, 8192
    x = _device_stack(n, stride, seed=5)
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    full = torch.empty(stride, dtype=torch.float64, device=cuda)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out64=full)
    ncols = 3001
    part = torch.empty(ncols, dtype=torch.float64, device=cuda)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), col_begin=col_begin, n_cols=ncols, out64=part)
    assert torch.equal(part, full[col_begin : col_begin + ncols])


@pytest.mark.parametrize("mode", [na.MODE_W32_DIV64, na.MODE_W32_DIV32, na.MODE_W64])
def test_modes_bit_exact(mode, cuda):
    n, p = 37, 12345
    x = _device_stack(n, 12352, seed=mode + 3)
    rng = np.random.default_rng(mode)
    wv = rng.uniform(0.1, 3.0, n)
    if mode == na.MODE_W64:
        w = wv.astype(np.float64)
        denom = float(np.sum(w))
    elif mode == na.MODE_W32_DIV32:
        w = wv.astype(np.float32)
        denom = float(np.sum(w))  # np.float32 pairwise sum, exact as double
    else:
        w = wv.astype(np.float32)
        denom = float(np.sum([float(v) for v in wv]))
    wd = torch.from_numpy(w).to(cuda)
    want = oracle.c_reduce(mode, x[:, :p].cpu().numpy(), w, denom)
    if want.dtype == np.float32:
        out = torch.empty(p, dtype=torch.float32, device=cuda)
        agg.reduce_stack(x, wd, mode, denom, n_cols=p, out32=out)
    else:
        out = torch.empty(p, dtype=torch.float64, device=cuda)
        agg.reduce_stack(x, wd, mode, denom, n_cols=p, out64=out)
    assert bitwise_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("op", ["avgm", "adagrad", "yogi", "adam"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_fused_epilogue_bit_exact(op, prec, cuda):
    n, p, stride = 11, 5001, 5056
    mode = na.MODE_W32_DIV64 if prec == "f64" else na.MODE_W32_DIV32
    x = _device_stack(n, stride, seed=17)
    w = (np.arange(n, dtype=np.float32) + 1.0).astype(np.float32)
    denom = float(np.sum([float(v) for v in w])) if prec == "f64" else float(np.sum(w))
    prev = torch.empty((1, stride), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed=99)
    prev_h = prev[0, :p].cpu().numpy().copy()
    vdt = torch.float64 if prec == "f64" else torch.float32
    v = (torch.rand(p, dtype=torch.float64, device=cuda) * 0.01).to(vdt)
    v_h = v.cpu().numpy().copy()
    out32 = torch.empty(p, dtype=torch.float32, device=cuda)
    out64 = torch.empty(p, dtype=torch.float64, device=cuda) if prec == "f64" else None
    agg.reduce_stack(x, torch.from_numpy(w).to(cuda), mode, denom, n_cols=p, out32=out32, out64=out64,
                     op=na.OP_BY_NAME[op], prev=prev[0], v=v)
    g = oracle.c_reduce(mode, x[:, :p].cpu().numpy(), w, denom)
    want = oracle.c_update(op, g, prev_h, v_h)
    assert bitwise_equal(v.cpu().numpy(), v_h)
    if prec == "f64":
        assert bitwise_equal(out64.cpu().numpy(), want)
    assert bitwise_equal(out32.cpu().numpy(), want.astype(np.float32))


def test_fused_epilogue_in_place_prev(cuda):
    """prev may double as out32 (how ServerOptimizer advances the global model)."""
    n, p = 5, 4096
    x = _device_stack(n, p, seed=1)
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    prev = torch.empty((1, p), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed=2)
    prev_h = prev[0].cpu().numpy().copy()
    v = torch.zeros(p, dtype=torch.float64, device=cuda)
    v_h = np.zeros(p)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, 5.0, out32=prev[0], op=na.OP_AVGM, prev=prev[0], v=v)
    want = oracle.c_update("avgm", oracle.c_reduce(0, x.cpu().numpy(), np.ones(n, np.float32), 5.0), prev_h, v_h)
    assert bitwise_equal(prev[0].cpu().numpy(), want.astype(np.float32))


def test_f64_and_i64_kernels(cuda):
    rng = np.random.default_rng(3)
    n, p = 9, 777
    xs = rng.standard_normal((n, p))
    w = rng.uniform(0.5, 2.0, n)
    stack = torch.zeros((n, 832), dtype=torch.float64)
    stack[:, :p] = torch.from_numpy(xs)
    out = torch.empty(832, dtype=torch.float64, device=cuda)
    agg.reduce_stack_f64(stack.to(cuda), torch.from_numpy(w).to(cuda), float(w.sum()), out)
    assert bitwise_equal(out[:p].cpu().numpy(), oracle.c_reduce("f64", xs, w, float(w.sum())))
    xi = rng.integers(-(2**40), 2**40, (n, p), dtype=np.int64)
    wi = rng.integers(1, 600, n).astype(np.int64)
    stack = torch.zeros((n, 832), dtype=torch.int64)
    stack[:, :p] = torch.from_numpy(xi)
    agg.reduce_stack_i64(stack.to(cuda), torch.from_numpy(wi).to(cuda), float(wi.sum()), out)
    assert bitwise_equal(out[:p].cpu().numpy(), oracle.c_reduce("i64", xi, wi, float(wi.sum())))


def test_misaligned_window_fails_loudly(cuda):
    x = torch.zeros((2, 128), dtype=torch.float32, device=cuda)
    w = torch.ones(2, dtype=torch.float32, device=cuda)
    out = torch.empty(10, dtype=torch.float64, device=cuda)
    with pytest.raises(na.NativeError):
        agg.reduce_stack(x, w, na.MODE_W32_DIV64, 2.0, col_begin=1, n_cols=10, out64=out)


def test_deterministic(cuda):
    x = _device_stack(50, 1 << 20, seed=8)
    w = torch.ones(50, dtype=torch.float32, device=cuda)
    a = torch.empty(1 << 20, dtype=torch.float32, device=cuda)
    b = torch.empty_like(a)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, 50.0, out32=a)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, 50.0, out32=b)
    assert torch.equal(a, b)


# BASELINE-size cases: full HIP run at the production grid, compared on EVERY element (C2, the
# north-star 100 x ResNet-50 shape, C3 fused AVGM) or on 64+ dense windows that include every
# stripe / rank boundary of the default 8-GPU plan and the row-major kernel's piece-group
# boundaries (C4, C5: 35-47 GB stacks).  Inputs are counter-based, so the host regenerates any
# column range; the C oracle reduces it in threads (ctypes releases the GIL).
# ---------------------------------------------------------------------------------------------

_HOST_WORKERS = min(16, os.cpu_count() or 1)  # the GPU box's CPU share


def _oracle_columns(n, c0, width, seed, op, prev_h):
    g = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, width, seed, row0=0, col0=c0),
                        np.ones(n, np.float32), float(n))
    if op != "mean":
        g = oracle.c_update(op, g, prev_h[c0 : c0 + width], np.zeros(width))
    return g.astype(np.float32)


def _rowmajor_piece_starts(p, cus=256):
    """Column starts of the row-major kernel's pieces and KG groups (mirror of fa_reduce.hip
    rowmajor_geometry + reduce_kernel_rowmajor's split), for placing check windows on them."""
    chunks = ((p + 3) // 4 + 63) // 64
    for d in range(0, cus - 160 + 1):
        for g in ([192 + d] if d == 0 else [192 + d, 192 - d]):
            if not 160 <= g <= cus:
                continue
            k = -(-chunks // (g * 64))
            if k < 2:
                return []
            for kg in (4, 3, 2, 5):
                if k % kg == 0 and (kg != 5 or k == 5):
                    pc = -(-chunks // (g * k))
                    starts = {pj * pc * 256 for pj in range(0, g * k, max(1, g // 4))}  # a sample of pieces
                    starts |= {(g0 * g) * pc * 256 for g0 in range(0, k, kg)}  # group starts (block 0)
                    starts |= {((g0 + kg) * g - 1) * pc * 256 for g0 in range(0, k, kg)}  # group ends
                    return sorted(s for s in starts if s < p)
    return []


def _dense_windows(p, width=4096, count=64):
    from flearn_amd.dist import ShardPlan

    starts = {(i * (p - width) // (count - 1)) & ~63 for i in range(count)}
    for r in range(8):  # stripe / rank boundaries of bench's default G=8 plan (2 stripes, 3:1)
        plan = ShardPlan.make(p, 8, r, 2, weights=(3, 1))
        for c in range(plan.stripes):
            g0 = plan.global_begin(c)
            starts |= {max(0, g0 - width // 2), min(g0 + plan.shard_of(c), p) - width // 2}
    starts |= {max(0, s - width // 2) for s in _rowmajor_piece_starts(p)}
    return sorted({(max(0, min(s, p - width)) & ~3, min(width, p)) for s in starts})


def _run_config(layout, n, op, cuda, seed=1234):
    p = layouts.padded_f32_stride(layouts.get(layout))
    x = torch.empty((n, p), dtype=torch.float32, device=cuda)
    agg.fill_uniform(x, seed=seed)
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    out32 = torch.empty(p, dtype=torch.float32, device=cuda)
    kw, prev_h = {}, None
    if op != "mean":
        prev = torch.empty((1, p), dtype=torch.float32, device=cuda)
        agg.fill_uniform(prev, seed=1)
        v = torch.zeros(p, dtype=torch.float64, device=cuda)
        kw = dict(op=na.OP_BY_NAME[op], prev=prev[0], v=v)
        prev_h = prev[0].cpu().numpy().copy()
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=out32, **kw)
    got = out32.cpu().numpy()
    del x
    torch.cuda.empty_cache()
    return p, got, prev_h


@pytest.mark.slow
@pytest.mark.timeout(600)
@pytest.mark.parametrize("layout,n,op", [("resnet18", 100, "mean"), ("resnet50", 100, "mean"),
                                         ("resnet50", 100, "avgm"), ("resnet18", 1000, "mean"),
                                         ("vit_b_16", 100, "adagrad")])
def test_baseline_config_full_parity(layout, n, op, cuda):
    """C2, the north-star shape, C3, C4 (1000 x 11.7 M: 46.8 GB of uploads) and C5 (fused Adagrad,
    100 x 86.6 M): every one of the P outputs bit-equal to the C oracle.  The host regenerates the
    counter-based inputs column chunk by column chunk (n * chunk <= 6.6 M elements per task) and
    the C oracle reduces them on the box's CPU share."""
    from concurrent.futures import ThreadPoolExecutor

    p, got, prev_h = _run_config(layout, n, op, cuda)
    chunk = max(4096, (1 << 16) * 100 // n // 64 * 64)
    bad = []

    def job(c0):
        width = min(chunk, p - c0)
        if not bitwise_equal(got[c0 : c0 + width], _oracle_columns(n, c0, width, 1234, op, prev_h)):
            bad.append(c0)

    with ThreadPoolExecutor(_HOST_WORKERS) as ex:
        list(ex.map(job, range(0, p, chunk)))
    assert not bad, (layout, op, sorted(bad)[:8])


@pytest.mark.slow
@pytest.mark.parametrize("layout,n,op", [("vit_b_16", 100, "adagrad"), ("resnet18", 1000, "mean")])
def test_baseline_config_window_parity(layout, n, op, cuda):
    """C5 and C4 at full size, fast smoke (the full compare is test_baseline_config_full_parity):
    >= 64 evenly spaced 4096-column windows plus every 8-GPU stripe / rank boundary and the
    row-major kernel's piece-group boundaries."""
    from concurrent.futures import ThreadPoolExecutor

    p, got, prev_h = _run_config(layout, n, op, cuda)
    wins = _dense_windows(p)
    assert len(wins) >= 64

    def job(win):
        c0, width = win
        return c0 if not bitwise_equal(got[c0 : c0 + width], _oracle_columns(n, c0, width, 1234, op, prev_h)) else None

    with ThreadPoolExecutor(_HOST_WORKERS) as ex:
        bad = [c for c in ex.map(job, wins) if c is not None]
    assert not bad, (layout, op, bad[:8])
    assert np.isfinite(got).all()


# ---------------------------------------------------------------------------------------------
# ---------------------------------------------------------------------------------------------
# multi-GPU code path on one GPU: a 1-rank RCCL group runs the exact all-gather call sequence
# ---------------------------------------------------------------------------------------------


@pytest.mark.parametrize("stripes,weights", [(4, None), (2, (3, 1))])
@pytest.mark.parametrize("op", ["mean", "avgm"])
def test_sharded_reducer_rccl_one_rank(op, stripes, weights, cuda, tmp_path):
    import torch.distributed as dist

    from flearn_amd.dist import ShardedReducer, ShardPlan, hip_reduce_fn

    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1,
                                device_id=cuda)
        created = True
    try:
        n, p = 9, 1_000_003
        plan = ShardPlan.make(p, 1, 0, stripes=stripes, weights=weights)
        stack = torch.empty((n, plan.local_cols), dtype=torch.float32, device=cuda)
        for c in range(plan.stripes):
            agg.fill_uniform(stack[:, plan.local_begin(c):], seed=3, col_begin=plan.global_begin(c),
                             n_cols=plan.shard_of(c))
        w = torch.ones(n, dtype=torch.float32, device=cuda)
        epi, local_out = {}, None
        if op != "mean":
            prev = torch.empty((1, plan.local_cols), dtype=torch.float32, device=cuda)
            agg.fill_uniform(prev, seed=4)
            prev_h = prev[0, :p].cpu().numpy().copy()
            epi = dict(op=na.OP_BY_NAME[op], prev=prev[0], v=torch.zeros(plan.local_cols, dtype=torch.float64, device=cuda))
            local_out = prev[0]
        red = ShardedReducer(plan, hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n), **epi), cuda,
                             local_out=local_out, gather=True)
        full = red.step().cpu().numpy()
        want = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, 3), np.ones(n, np.float32), float(n))
        if op != "mean":
            want = oracle.c_update(op, want, prev_h, np.zeros(p))
        assert bitwise_equal(full, want.astype(np.float32))
    finally:
        if created:
            dist.destroy_process_group()


@pytest.mark.parametrize("push", [True, "dma"])
def test_sharded_reducer_push_rccl_one_rank(push, cuda, tmp_path):
    """The push gather's RCCL-specific code on a 1-rank RCCL group: its barriers are 1-element
    all_reduces ordered on the pusher's stream (gloo, used by every multi-rank test on this box,
    takes the host-barrier branch instead), the bucket comes from the receive pool (exported,
    token-checked), three steps, then shutdown_push while the group exists — bit-exact."""
    import torch.distributed as dist

    from flearn_amd import dist as fd
    from flearn_amd.dist import ShardedReducer, ShardPlan, hip_reduce_fn

    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1, device_id=cuda)
        created = True
    try:
        n, p = 7, 600_001
        plan = ShardPlan.make(p, 1, 0, stripes=3)
        stack = torch.empty((n, plan.local_cols), dtype=torch.float32, device=cuda)
        for c in range(plan.stripes):
            agg.fill_uniform(stack[:, plan.local_begin(c):], seed=5, col_begin=plan.global_begin(c),
                             n_cols=plan.shard_of(c))
        w = torch.ones(n, dtype=torch.float32, device=cuda)
        red = ShardedReducer(plan, hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n)), cuda, gather=True, push=push)
        assert red.pusher is not None and red.pusher.nccl
        # both forms push from a high-priority stream (a hardware queue apart from the compute
        # stream's); the copy-engine legs' streams are normal priority.  Pushes are host-ordered,
        # so correctness does not depend on either
        from flearn_amd import streams

        assert red.pusher.stream.priority == streams.HIGH
        assert all(x.priority == 0 for x in red.pusher.peer_streams)
        want = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, 5), np.ones(n, np.float32), float(n))
        for _ in range(3):
            full = red.step()
            assert bitwise_equal(full[:p].cpu().numpy(), want.astype(np.float32))
        red.release()
        fd.shutdown_push()
        assert fd._RecvPool.bytes_held() == 0
    finally:
        if created:
            dist.destroy_process_group()


@pytest.mark.parametrize("op", ["avgm", "adagrad", "yogi", "adam"])
def test_fused_v_out_equals_in_place(op, cuda):
    """ABI 6 v_out: the double-buffered form (out32 into a fresh buffer, v_t into v_out) gives the
    in-place results bit for bit and leaves prev and v untouched."""
    n, p = 7, 300_001
    stack = torch.empty((n, p + 63), dtype=torch.float32, device=cuda)
    agg.fill_uniform(stack, seed=11)
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    prev = torch.empty((1, p + 63), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed=12)
    prev = prev[0, :p].contiguous()
    v0 = torch.full((p,), 0.125, dtype=torch.float64, device=cuda)
    kw = dict(op=na.OP_BY_NAME[op], n_cols=p)
    # in place
    prev_a, v_a = prev.clone(), v0.clone()
    agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=prev_a, prev=prev_a, v=v_a, **kw)
    # double-buffered
    prev_b, v_b = prev.clone(), v0.clone()
    out_b, vo_b = torch.empty_like(prev_b), torch.full_like(v_b, -1.0)
    agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=out_b, prev=prev_b, v=v_b, v_out=vo_b, **kw)
    assert bitwise_equal(out_b.cpu().numpy(), prev_a.cpu().numpy())
    assert bitwise_equal(vo_b.cpu().numpy(), v_a.cpu().numpy())
    assert bitwise_equal(prev_b.cpu().numpy(), prev.cpu().numpy())
    assert bitwise_equal(v_b.cpu().numpy(), v0.cpu().numpy())
    with pytest.raises(ValueError):
        agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=out_b, prev=prev_b, v=v_b, v_out=v_b, **kw)


@pytest.mark.parametrize("op,stripes", [("avgm", 1), ("adagrad", 2)])
def test_pingpong_reducer_three_steps(op, stripes, cuda):
    """bench.py's fused job: PingPong state over three steps (the buffers swap every step) equals
    three in-place oracle steps, model and v_t."""
    from flearn_amd.dist import PingPong, ShardedReducer, ShardPlan, hip_reduce_fn

    n, p = 5, 200_003
    plan = ShardPlan.make(p, 1, 0, stripes=stripes, weights=(3, 1) if stripes == 2 else None)
    stack = torch.empty((n, plan.local_cols), dtype=torch.float32, device=cuda)
    for c in range(plan.stripes):
        agg.fill_uniform(stack[:, plan.local_begin(c):], seed=21, col_begin=plan.global_begin(c),
                         n_cols=plan.shard_of(c))
    prev = torch.empty((1, plan.local_cols), dtype=torch.float32, device=cuda)
    agg.fill_uniform(prev, seed=22)
    prev_h = prev[0, :p].cpu().numpy().copy()
    state = PingPong(prev[0], torch.zeros(plan.local_cols, dtype=torch.float64, device=cuda))
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    red = ShardedReducer(plan, hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n), op=na.OP_BY_NAME[op],
                                             state=state), cuda, state=state)
    mean = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, 21), np.ones(n, np.float32), float(n))
    v_h = np.zeros(p)
    for k in range(3):
        got = red.step().cpu().numpy()
        want = oracle.c_update(op, mean, prev_h, v_h).astype(np.float32)
        assert bitwise_equal(got, want), f"step {k}"
        assert bitwise_equal(state.v[state.cur][:p].cpu().numpy(), v_h), f"v step {k}"
        prev_h = want


# ---------------------------------------------------------------------------------------------
# column shards over several devices (per-GPU parallel ingest); here 2-3 shards on one GPU
# ---------------------------------------------------------------------------------------------


@pytest.mark.parametrize("name", ["avg_w1_n10", "avg_bnmodel_pyint_n4", "avg_special_n5", "trace_lenet5_round0",
                                  "avg_np32_n10", "avg_torch_n3"])
@pytest.mark.parametrize("k", [2, 3])
def test_sharded_ingest_matches_reference(name, k, cuda):
    g = Golden(name)
    s = strategy_for(g)
    s.devices = [cuda] * k
    got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
    assert_dict_bitwise(got, g.output(), f"{name} x{k}")
    assert len(s.engine.packer.shards(s.engine.last_plan, "f32")) == k


@pytest.mark.parametrize("name", ["avgm_pyfloat_rounds3", "adagrad_np32_rounds3"])
def test_sharded_fused_optimizer_matches_reference(name, cuda):
    g = Golden(name)
    op = g.meta["op"]
    s = (AVGM(server_side=True, devices=[cuda] * 3) if op == "avgm"
         else OPT(server_side=True, method=op, devices=[cuda] * 3))
    s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
    for r in range(g.meta["rounds"]):
        clients, weights = _round_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        assert_dict_bitwise(got, g.output(f"w{r}"), f"{name} w{r}")
        assert_dict_bitwise(s.server_opt.v_t(s.engine.last_plan), g.output(f"v{r}"), f"{name} v{r}")


def test_sharded_device_output(cuda):
    g = Golden("avg_w1_n10")
    s = AVG(output="device", devices=[cuda, cuda])
    got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
    for k, w in g.output().items():
        assert bitwise_equal(got[k].cpu().numpy(), np.asarray(w).astype(np.float32)), k


# ---------------------------------------------------------------------------------------------
# FedDyn (dyn.py:10-49): fused h / theta epilogue
# ---------------------------------------------------------------------------------------------
DYN_CASES = [c for c in cases() if c.startswith("dyn_")]


def _dyn_inputs(g, r):
    from golden_io import decode_weight

    keys = g.meta["client_keys"]
    clients = [{k: g.arrays[f"r{r}x{i}:{k}"].copy() for k in keys} for i in range(g.meta["n_clients"])]
    return clients, [decode_weight(e) for e in g.meta["round_weights"][r]]


def _dyn_h0(g):
    return {k[6:]: v.copy() for k, v in g.arrays.items() if k.startswith("hinit:")}


@pytest.mark.parametrize("name", DYN_CASES)
@pytest.mark.parametrize("shards", [1, 3])
def test_dyn_strategy_matches_reference(name, shards, cuda):
    """Dyn(h).server over 3 rounds: w_glob, h (synced back into the caller's arrays) and theta
    bit-identical to the reference's; integer h entries skipped as dyn.py:24-31 does."""
    from flearn_amd import Dyn

    g = Golden(name)
    h = _dyn_h0(g)
    h_ids = {k: id(v) for k, v in h.items()}
    s = Dyn(h, devices=[cuda] * shards)
    for r in range(g.meta["rounds"]):
        clients, weights = _dyn_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        assert_dict_bitwise(got, g.output(f"w{r}"), f"{name} w{r}")
        assert s.theta is got  # dyn.py:34
        hh = s.h
        assert hh is h and all(id(hh[k]) == h_ids[k] for k in h)  # updated in place
        assert_dict_bitwise(hh, g.output(f"h{r}"), f"{name} h{r}")
        dev = s._dyn.dev_keys
        assert_dict_bitwise({k: v for k, v in s._dyn.theta_host().items() if k in dev},
                            {k: np.asarray(v) for k, v in g.output(f"theta{r}").items() if k in dev}, f"{name} theta{r}")


@pytest.mark.parametrize("name", DYN_CASES)
def test_dyn_state_restores_on_a_fresh_strategy(name, cuda):
    """A server restart between FedDyn rounds: h and theta saved after round 0 (copies of
    `strategy.h` and `strategy.theta`), a fresh Dyn(h) with `theta` assigned runs rounds 1-2 —
    w_glob, h and theta bit-identical to the reference's (dyn.py:14-36)."""
    from flearn_amd import Dyn

    g = Golden(name)
    s = Dyn(_dyn_h0(g))
    clients, weights = _dyn_inputs(g, 0)
    s.server(upload(clients, weights), 0)
    h_saved = {k: np.array(v, copy=True) for k, v in s.h.items()}
    theta_saved = {k: np.array(v, copy=True) for k, v in s.theta.items()}
    del s
    s = Dyn(h_saved)
    s.theta = theta_saved
    for r in range(1, g.meta["rounds"]):
        clients, weights = _dyn_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        assert_dict_bitwise(got, g.output(f"w{r}"), f"{name} w{r} after restore")
        assert_dict_bitwise(s.h, g.output(f"h{r}"), f"{name} h{r} after restore")


@pytest.mark.parametrize("name", DYN_CASES)
def test_dyn_float32_output(name, cuda):
    from flearn_amd import Dyn

    g = Golden(name)
    s = Dyn(_dyn_h0(g), output="float32")
    for r in range(g.meta["rounds"]):
        clients, weights = _dyn_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        for k, w in g.output(f"w{r}").items():
            w = np.asarray(w)
            if k in s._dyn.dev_keys:
                assert bitwise_equal(np.asarray(got[k]), w.astype(np.float32)), (r, k)


def test_dyn_partial_h_matches_numpy_oracle(cuda):
    """h without some fp32 keys: those keep the plain mean (mean + update on covered runs)."""
    from flearn_amd import Dyn

    g = Golden("dyn_pyfloat_rounds3")
    h0 = _dyn_h0(g)
    for drop in ("bn1.weight", "fc.bias"):
        h0.pop(drop)
    h_ora = {k: v.copy() for k, v in h0.items()}
    theta = {k: v.copy() for k, v in h0.items()}
    s = Dyn({k: v.copy() for k, v in h0.items()})
    for r in range(3):
        clients, weights = _dyn_inputs(g, r)
        got = s.server(upload(clients, weights), r)["w_glob"]
        with np.errstate(all="ignore"):
            avg = oracle.server_ensemble(weights, [{k: v.copy() for k, v in c.items()} for c in clients])
            want, theta = oracle.dyn_f(avg, h_ora, theta, len(clients))
        assert_dict_bitwise(got, want, f"partial w{r}")
        assert_dict_bitwise(s.h, h_ora, f"partial h{r}")


def test_dyn_errors_like_reference(cuda):
    from flearn_amd import Dyn

    g = Golden("dyn_pyfloat_rounds3")
    clients, weights = _dyn_inputs(g, 0)
    h = _dyn_h0(g)
    h["not.a.key"] = np.zeros(3, np.float32)
    with pytest.raises(KeyError):
        Dyn(h).server(upload(clients, weights), 0)
    with pytest.raises(AttributeError):
        Dyn(None).server(upload(clients, weights), 0)
    s = Dyn(_dyn_h0(g))
    s.server(upload(clients, weights), 0)
    with pytest.raises(SystemExit):  # theta precision would change (f64 -> fp32): refused
        s.server(upload(clients, [np.float32(w) for w in weights]), 1)


@pytest.mark.parametrize("prec", ["f64", "f32", "w64"])
@pytest.mark.parametrize("p", [1, 4093, 5001, 100001, 200081, 8388608 + 5])
def test_dyn_epilogue_vs_c_oracle(prec, p, cuda):
    """Kernel level, 2 rounds with state carried: fused reduce+FedDyn vs the C restatement,
    small (balanced grid), one-piece 4-wave (100 K, 200 K columns) and big-tile
    (buffer-descriptor path, ragged tail) buckets."""
    n = 7 if p < 10**6 else 3
    stride = -(-p // 64) * 64
    mode = {"f64": na.MODE_W32_DIV64, "f32": na.MODE_W32_DIV32, "w64": na.MODE_W64}[prec]
    tdt = torch.float32 if prec == "f32" else torch.float64
    h = torch.empty((1, stride), dtype=torch.float32, device=cuda)
    agg.fill_uniform(h, seed=41)
    h = h[0] * 0.01
    h_ora = h[:p].cpu().numpy().copy()
    theta = h.to(tdt, copy=True)
    th_ora = theta[:p].cpu().numpy().copy()
    for r in range(2):
        x = _device_stack(n, stride, seed=100 + r)
        wv = np.linspace(0.5, 2.0, n)
        w = wv.astype(np.float64 if prec == "w64" else np.float32)
        denom = float(np.sum([float(v) for v in wv])) if prec == "f64" else float(np.sum(w))
        out = torch.empty(p, dtype=tdt, device=cuda)
        kw = {"out64": out} if tdt == torch.float64 else {"out32": out}
        agg.reduce_stack(x, torch.from_numpy(w).to(cuda), mode, denom, n_cols=p, op=na.OP_DYN, h=h, v=theta, **kw)
        gm = oracle.c_reduce(mode, x[:, :p].cpu().numpy(), w, denom)
        want = oracle.c_update_dyn(gm, h_ora, th_ora, n)
        assert bitwise_equal(out.cpu().numpy(), want), r
        assert bitwise_equal(h[:p].cpu().numpy(), h_ora), r
        assert bitwise_equal(theta[:p].cpu().numpy(), th_ora), r


def test_dyn_apply_vs_c_oracle(cuda):
    p = 10007
    g = torch.rand(p, dtype=torch.float64, device=cuda)
    h = (torch.rand(p, device=cuda) * 0.1).float()
    th = torch.rand(p, dtype=torch.float64, device=cuda)
    g_h, h_h, th_h = g.cpu().numpy(), h.cpu().numpy().copy(), th.cpu().numpy().copy()
    agg.apply_dyn(g, h, th, 9, 0.05, out64=g)  # in place on the mean
    want = oracle.c_update_dyn(g_h, h_h, th_h, 9, alpha=0.05)
    assert bitwise_equal(g.cpu().numpy(), want)
    assert bitwise_equal(h.cpu().numpy(), h_h) and bitwise_equal(th.cpu().numpy(), th_h)


# ---------------------------------------------------------------------------------------------
# FedDistill (distill.py:26-46): logits mean on the device
# ---------------------------------------------------------------------------------------------
DISTILL_CASES = [c for c in cases() if c.startswith("distill_logits_")]


@pytest.mark.parametrize("name", DISTILL_CASES)
def test_distill_logits_mean_matches_reference(name, cuda):
    from flearn_amd import Distill

    g = Golden(name)
    tabs = [g.arrays[f"logits{i}"] for i in range(g.meta["n_clients"])]
    if g.meta["logits_kind"].startswith("torch"):
        tabs = [torch.from_numpy(t.copy()) for t in tabs]
    got = Distill.aggregate_logits(tabs)
    if g.meta["logits_kind"].startswith("torch"):
        assert isinstance(got, torch.Tensor) and got.device.type == "cpu"
        got = got.numpy()
    else:
        assert isinstance(got, np.ndarray)
    assert_dict_bitwise({"glob_logits": got}, g.output(), name)


def test_distill_server_matches_reference(cuda):
    from flearn_amd import Distill

    g = Golden("distill_server_n4")
    ups = upload(g.clients(), g.weights())
    for i, u in enumerate(ups):
        u["logits"] = torch.from_numpy(g.arrays[f"logits{i}"].copy())
    res = Distill().server(ups, 0)
    assert_dict_bitwise(res["w_glob"], g.output(), "distill w_glob")
    assert_dict_bitwise({"glob_logits": res["glob_logits"].numpy()}, g.output("glob"), "distill glob_logits")
    with pytest.raises(ZeroDivisionError):
        Distill.aggregate_logits([])


# ---------------------------------------------------------------------------------------------
# HTTP mode: uploads arrive as base64(pickle) strings (Encrypt.py:16-44, Server.py:126-142)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("shards", [1, 2])
@pytest.mark.parametrize("name,strategy", [("avg_lenet5_n10", "avg"), ("avg_bnmodel_pyint_n4", "avg"),
                                           ("bn_strategy_n4", "bn")])
def test_wire_uploads_through_the_engine(name, strategy, shards, fast, cuda):
    """Server.ensemble's loop: receive_processing(str) per upload, then server(); decoded fp32
    params are DMA'd straight from the codec's pinned rows when their layout is the bucket's
    (scanner route, fast=True) — small uploads by default take native base64 + unpickler."""
    from flearn_amd.wire import Encrypt

    g = Golden(name)
    enc = Encrypt(fast_min_chars=0 if fast else None)
    strs = [enc.encode({"agg_weight": w, "params": c}) for w, c in zip(g.weights(), g.clients())]
    s = (BN if strategy == "bn" else AVG)(encrypt=enc, devices=[cuda] * shards)
    ups = [s.receive_processing(x) for x in strs]
    got = s.server(ups, 0)["w_glob"]
    assert_dict_bitwise(got, g.output(), name)
    want_rows = 0 if strategy == "bn" or not fast else len(strs)  # BN drops keys: layouts differ -> plain pack
    assert s.engine.packer.last_wire_rows == want_rows
    back = enc.decode(s.upload_processing({"w_glob": got}))["w_glob"]
    assert_dict_bitwise(back, got, "round trip")


@pytest.mark.parametrize("name", ["avg_lenet5_n10", "avg_bnmodel_pyint_n4"])
def test_wire_device_staging_rounds(name, cuda):
    """stage_to_device: each decoded upload is copied to the GPU at decode time and the engine
    aggregates the staged stack — same bits as the reference, over 3 rounds (slot reuse, stack
    growth past 8 slots); a reordered upload list falls back to the pinned-row path."""
    from flearn_amd.wire import Encrypt

    g = Golden(name)
    enc = Encrypt(fast_min_chars=0, stage_to_device=True)
    strs = [enc.encode({"agg_weight": w, "params": c}) for w, c in zip(g.weights(), g.clients())]
    s = AVG(encrypt=enc)
    for r in range(3):
        ups = [s.receive_processing(x) for x in strs]
        if r == 2:
            ups = ups[::-1] + []  # order differs from the decode order: no staged stack
            want = oracle.server_ensemble(g.weights()[::-1], g.clients()[::-1])
        else:
            want = g.output()
        got = s.server(ups, r)["w_glob"]
        assert_dict_bitwise(got, want, f"{name} round {r}")
        assert s.engine.packer.last_wire_staged == (0 if r == 2 else len(strs))


def test_wire_rows_are_pinned(cuda):
    from flearn_amd import wire

    up = {"agg_weight": 1.0, "params": {"w": np.arange(1000, dtype=np.float32)}}
    d = wire.Encrypt(fast_min_chars=0).decode(wire.Encrypt().encode(up))
    row = wire.wire_row(d["params"], (("w", (1000,), 0), 1024))
    assert row is not None and row.is_pinned()


@pytest.mark.parametrize("shards", [1, 2])
def test_host_pack_mixed_upload_kinds(shards, cuda):
    """Loopback ingest above the small-bucket size (thread-pool pack) with uploads the native row
    pack takes (dict / OrderedDict of C-contiguous arrays) mixed with rows it hands back to the
    Python pack (a Fortran-order array, a read-only strided view, a numpy 0-d scalar, a Mapping
    that is not a dict): bit-exact against the oracle, twice (reused staging)."""
    import collections
    from collections.abc import Mapping

    class Upload(Mapping):
        def __init__(self, d):
            self.d = d

        def __getitem__(self, k):
            return self.d[k]

        def __iter__(self):
            return iter(self.d)

        def __len__(self):
            return len(self.d)

    rng = np.random.default_rng(11)
    shapes = {"a.weight": (512, 700), "a.bias": (700,), "b.weight": (300, 333), "s": ()}
    clients = []
    for i in range(12):
        c = {k: rng.standard_normal(sh).astype(np.float32) if sh else np.float32(rng.standard_normal())
             for k, sh in shapes.items()}
        clients.append(c)
    clients[3]["a.weight"] = np.asfortranarray(clients[3]["a.weight"])
    big = rng.standard_normal((300, 666)).astype(np.float32)
    clients[5]["b.weight"] = big[:, ::2]
    clients[5]["b.weight"].flags.writeable = False
    clients[7] = collections.OrderedDict(clients[7])
    weights = [float(w) for w in rng.integers(1, 9, size=12)]
    want = oracle.server_ensemble(weights, clients)
    s = AVG()
    s.devices = [cuda] * shards
    for _ in range(2):
        ups = upload([Upload(c) if i == 9 else c for i, c in enumerate(clients)], weights)
        got = s.server(ups, 0)["w_glob"]
        assert_dict_bitwise(got, want, f"mixed x{shards}")


@pytest.mark.parametrize("mode", ["copy-engine", "zero-copy", "zero-copy-1MiB-chunks", "dma-chunks", "dma-1MiB-chunks"])
@pytest.mark.parametrize("op", ["avgm", "adagrad", "yogi"])
def test_client_side_update_large_and_fallback_values(op, mode, cuda, monkeypatch):
    """The client update on a model above the copy-part size (parallel native packs) and with
    values the byte copy hands back to Python (a Fortran-order local array, a strided global
    view, a 0-d entry): bit-exact against the oracle over 3 rounds, state included — with two H2D
    copies and one launch, and zero-copy in one or in many chunks (the kernel reading the pinned
    staging over PCIe chunk by chunk while the next chunk is packed)."""
    from flearn_amd.strategy._update import DeviceUpdater

    monkeypatch.setattr(DeviceUpdater, "zero_copy", mode != "copy-engine")
    monkeypatch.setattr(DeviceUpdater, "transfer", "dma" if mode.startswith("dma") else "kernel")
    if mode.endswith("1MiB-chunks"):
        monkeypatch.setattr(DeviceUpdater, "chunk_bytes", 1 << 20)
    rng = np.random.default_rng(21)
    shapes = {"a": (1024, 3000), "b": (3000,), "c": (700, 900), "d": (), "e": (5, 7)}
    prev = {k: rng.standard_normal(sh).astype(np.float32) for k, sh in shapes.items()}
    prev["c"] = np.asfortranarray(prev["c"])
    s = AVGM() if op == "avgm" else OPT()
    v = None
    for r in range(3):
        glob = {k: rng.standard_normal(sh) for k, sh in shapes.items()}
        wide = rng.standard_normal((5, 14))
        glob["e"] = wide[:, ::2]
        if op == "avgm":
            want, v = oracle.mean_momentum(prev, glob, v, 0.9)
            got = s.mean_momentum(dict(prev), glob, 0.9)
        else:
            want, v = oracle.adaptive_opt(prev, glob, v, op)
            got = s.adaptive_opt(dict(prev), glob, op)
        assert_dict_bitwise(got, want, f"{op} w{r}")
        assert_dict_bitwise(s.v_t, v, f"{op} v{r}")
        prev = {k: np.asarray(got[k]).astype(np.float32) for k in shapes}
        if r == 0:
            prev["c"] = np.asfortranarray(prev["c"])


@pytest.mark.parametrize("gdt", [np.float64, np.float32])
@pytest.mark.parametrize("op", ["avgm", "adagrad", "adam"])
def test_client_side_update_native_pack(op, gdt, cuda, monkeypatch):
    """Plain C-contiguous values (what flearn's clients hold): the zero-copy chunks are packed by
    native threads (bucket.AsyncPack, 1-MiB chunks: many chunks, each launched after its own
    copies), float64 and float32 global models, bit-exact against the oracle over 3 rounds."""
    from flearn_amd.strategy._update import DeviceUpdater

    monkeypatch.setattr(DeviceUpdater, "chunk_bytes", 1 << 20)
    monkeypatch.setattr(DeviceUpdater, "first_chunk_bytes", 256 << 10)
    rng = np.random.default_rng(33)
    shapes = {"a": (1024, 3000), "b": (3000,), "c": (700, 900), "d": (), "e": (5, 7), "f": (64, 3, 7, 7)}
    prev = {k: rng.standard_normal(sh).astype(np.float32) for k, sh in shapes.items()}
    s = AVGM() if op == "avgm" else OPT()
    v = None
    for r in range(3):
        glob = {k: rng.standard_normal(sh).astype(gdt) for k, sh in shapes.items()}
        glob["d"] = np.asarray(glob["d"])  # a 0-d array (not a numpy scalar)
        if op == "avgm":
            want, v = oracle.mean_momentum(prev, glob, v, 0.9)
            got = s.mean_momentum(dict(prev), glob, 0.9)
        else:
            want, v = oracle.adaptive_opt(prev, glob, v, op)
            got = s.adaptive_opt(dict(prev), glob, op)
        up = s._get_updater() if op == "avgm" else s._get_updater(op)
        assert up.last_pack == "native"
        assert_dict_bitwise(got, want, f"{op} {gdt.__name__} w{r}")
        assert_dict_bitwise(s.v_t, v, f"{op} {gdt.__name__} v{r}")
        prev = {k: np.asarray(got[k]).astype(np.float32) for k in shapes}


@pytest.mark.parametrize("transfer", ["dma", "kernel"])
@pytest.mark.parametrize("op", ["avgm", "adagrad"])
def test_client_side_update_failure_mid_call_changes_nothing(op, transfer, cuda, monkeypatch):
    """a zero-copy chunked update that fails on a later chunk (chunks before it already
    queued) must leave v_t and w_local as they were — v_t is double-buffered and swapped only
    after every chunk ran, and the queued chunks are waited for before the error propagates — so
    retrying the round gives the reference's result."""
    from flearn_amd import aggregator
    from flearn_amd.strategy._update import DeviceUpdater

    monkeypatch.setattr(DeviceUpdater, "zero_copy", True)
    monkeypatch.setattr(DeviceUpdater, "transfer", transfer)
    monkeypatch.setattr(DeviceUpdater, "chunk_bytes", 1 << 20)
    rng = np.random.default_rng(5)
    shapes = {"a": (512, 1024), "b": (3000,), "c": (300, 700), "d": (4096,)}
    prev = {k: rng.standard_normal(sh).astype(np.float32) for k, sh in shapes.items()}
    s = AVGM() if op == "avgm" else OPT()
    v = None
    real = aggregator._epilogue
    for r in range(3):
        glob = {k: rng.standard_normal(sh) for k, sh in shapes.items()}
        if r == 1:
            calls = {"n": 0}

            def failing(*a, **k):
                calls["n"] += 1
                if calls["n"] == 3:
                    raise ValueError("refused chunk")
                return real(*a, **k)

            monkeypatch.setattr(aggregator, "_epilogue", failing)
            wl = dict(prev)
            with pytest.raises(ValueError, match="refused chunk"):
                s.mean_momentum(wl, glob, 0.9) if op == "avgm" else s.adaptive_opt(wl, glob, op)
            assert calls["n"] == 3 and all(wl[k] is prev[k] for k in prev)
            monkeypatch.setattr(aggregator, "_epilogue", real)
            if v is not None:
                assert_dict_bitwise(s.v_t, v, f"{op} v after the failed call")
        if op == "avgm":
            want, v = oracle.mean_momentum(prev, glob, v, 0.9)
            got = s.mean_momentum(dict(prev), glob, 0.9)
        else:
            want, v = oracle.adaptive_opt(prev, glob, v, op)
            got = s.adaptive_opt(dict(prev), glob, op)
        assert_dict_bitwise(got, want, f"{op} w{r}")
        assert_dict_bitwise(s.v_t, v, f"{op} v{r}")
        prev = {k: np.asarray(got[k]).astype(np.float32) for k in shapes}


class _Trainer:
    """What flearn's client_receive touches: .model and .weight (Trainer.py:228-230)."""

    def __init__(self, model):
        self.model = model

    @property
    def weight(self):
        return self.model.state_dict()


def _cuda_model(seed, cuda):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                               torch.nn.Linear(8 * 30 * 30, 65), torch.nn.LayerNorm(65),
                               torch.nn.Linear(65, 10)).to(cuda)


@pytest.mark.parametrize("op", ["avgm", "adagrad", "yogi"])
@pytest.mark.parametrize("glob_dtype", [np.float64, np.float32])
def test_client_receive_updates_a_cuda_model_in_place(op, glob_dtype, cuda, monkeypatch):
    """client_receive with a model on the GPU (flearn trains there): the update runs where the
    model lives (only w_glob crosses PCIe) and load_state_dict gets the reference's values — the
    parameters equal, bit for bit, the reference's host path (convert_to_np -> numpy update ->
    load_state_dict of the float64 arrays) over 3 rounds, v_t included; in small chunks too."""
    from flearn_amd.strategy._update import DeviceUpdater

    monkeypatch.setattr(DeviceUpdater, "chunk_bytes", 1 << 20)
    monkeypatch.setattr(DeviceUpdater, "first_chunk_bytes", 1 << 18)
    monkeypatch.setattr(DeviceUpdater, "last_chunk_bytes", 1 << 18)
    model = _cuda_model(3, cuda)
    tr = _Trainer(model)
    s = AVGM() if op == "avgm" else OPT()
    calls = {"dev": 0}
    real = DeviceUpdater.update_on_device

    def counted(self, *a, **k):
        calls["dev"] += 1
        return real(self, *a, **k)

    monkeypatch.setattr(DeviceUpdater, "update_on_device", counted)
    rng = np.random.default_rng(11)
    v = None
    for r in range(3):
        local = {k: t.detach().cpu().numpy().copy() for k, t in model.state_dict().items()}
        glob = {k: (a.astype(np.float64) + rng.standard_normal(a.shape)).astype(glob_dtype) for k, a in local.items()}
        if op == "avgm":
            want, v = oracle.mean_momentum(dict(local), glob, v, 0.9)
            s.client_receive(tr, {"w_glob": glob}, 0.9)
        else:
            want, v = oracle.adaptive_opt(dict(local), glob, v, op)
            s.client_receive(tr, {"w_glob": glob}, op)
        got = {k: t.detach().cpu().numpy() for k, t in model.state_dict().items()}
        for k in want:  # load_state_dict's cast of the reference's result
            w32 = torch.from_numpy(np.asarray(want[k])).to(torch.float32).numpy()
            assert got[k].tobytes() == w32.tobytes(), (op, r, k)
        assert_dict_bitwise(s.v_t, v, f"{op} v{r}")
    assert calls["dev"] == 3


def test_client_receive_keeps_the_host_path_for_bn_models(cuda):
    """A BN model's int64 counters make the reference's convert_to_tensor raise SystemError on the
    numpy scalars its update returns; that model keeps the host path, and its behaviour."""
    from flearn_amd.strategy._update import DeviceUpdater

    model = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.BatchNorm1d(4)).to(cuda)
    w = model.state_dict()
    glob = {k: np.asarray(t.detach().cpu().numpy(), dtype=np.float64) for k, t in w.items()}
    glob["1.num_batches_tracked"] = np.float64(0.0)
    assert not DeviceUpdater.device_model_ok(w, glob)
    with pytest.raises(SystemError):
        AVGM().client_receive(_Trainer(model), {"w_glob": glob}, 0.9)


@pytest.mark.parametrize("op", ["avgm", "adagrad", "adam"])
def test_client_side_update_bn_model(op, cuda):
    """A BatchNorm model: the server's w_glob holds np.float64 scalars for the int64
    num_batches_tracked counters and the client's state_dict int64 0-d arrays.  The fp32 keys run
    on the device, the counters through the reference's numpy ops on the host; all keys and the
    state equal the numpy restatement over 3 rounds."""
    g = Golden("avg_bnmodel_pyfloat_n4")
    prev = {k: np.asarray(v).copy() for k, v in g.clients()[0].items()}
    s = AVGM() if op == "avgm" else OPT()
    v = None
    glob = g.output()
    for r in range(3):
        if op == "avgm":
            want, v = oracle.mean_momentum(dict(prev), glob, v, 0.9)
            got = s.mean_momentum(dict(prev), glob, 0.9)
        else:
            want, v = oracle.adaptive_opt(dict(prev), glob, v, op)
            got = s.adaptive_opt(dict(prev), glob, op)
        assert set(got) == set(want)
        for k in want:
            assert type(got[k]) is type(want[k]), (k, type(got[k]), type(want[k]))
        assert_dict_bitwise(got, want, f"{op} w{r}")
        assert_dict_bitwise(s.v_t, v, f"{op} v{r}")
        prev = {k: (np.asarray(got[k]).astype(np.float32) if np.asarray(got[k]).dtype == np.float64 and
                    np.ndim(got[k]) else prev[k]) for k in prev}
        glob = {k: (val * 1.01 if np.ndim(val) else val) for k, val in glob.items()}


def test_client_side_update_refuses_a_changed_layout(cuda):
    s = AVGM()
    a = {"w": np.ones(10, np.float32)}
    s.mean_momentum(dict(a), {"w": np.zeros(10)}, 0.9)
    with pytest.raises(ValueError, match="reset"):
        s.mean_momentum({"w": np.ones(12, np.float32)}, {"w": np.zeros(12)}, 0.9)
    s._updater.reset()
    s.mean_momentum({"w": np.ones(12, np.float32)}, {"w": np.zeros(12)}, 0.9)


@pytest.mark.parametrize("name", ["avg_w1_n10", "avg_bnmodel_pyint_n4", "trace_lenet5_round0", "avg_torch_n3"])
def test_strategy_group_mode_one_rank(name, cuda, tmp_path):
    """AVG(group=True): the Strategy-level column-sharded path (pack this rank's columns, reduce,
    RCCL all_gather_into_tensor) on a 1-rank RCCL group — the multi-GPU call sequence behind
    flearn's Server.py:140, bit-exact against the reference's fixtures."""
    import torch.distributed as dist

    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1, device_id=cuda)
        created = True
    try:
        g = Golden(name)
        s = strategy_for(g)
        s.group = True
        got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
        assert_dict_bitwise(got, g.output(), name)
        a = AVGM(server_side=True, group=True)
        a.server_opt.init_global({k: np.asarray(v, np.float32) for k, v in g.output().items()
                                  if np.asarray(v).dtype == np.float64 and np.ndim(v)})
        a.server(upload(g.clients(), g.weights()), 1)
        b = AVGM(server_side=True)  # the same round without the group: same v_t
        b.server_opt.init_global({k: np.asarray(v, np.float32) for k, v in g.output().items()
                                  if np.asarray(v).dtype == np.float64 and np.ndim(v)})
        b.server(upload(g.clients(), g.weights()), 1)
        assert_dict_bitwise(a.server_opt.v_t(a.engine.last_plan), b.server_opt.v_t(b.engine.last_plan), name)
    finally:
        if created:
            dist.destroy_process_group()


@pytest.mark.parametrize("weights", [[1.0, 2.5, 0.5, 3.0], [1, 2, 3, 4]])
def test_float64_model_with_int64_counters(weights, cuda):
    """A float64 model with BatchNorm counters: with float weights the f64 tensors and the int64
    counters share the f64 bucket (numpy promotes both to float64, strategy.py:123-129); with
    int weights the counters keep int64 arithmetic.  Bit-exact vs the oracle (a plan-building
    bug once raised here: tests/test_plan_props.py found it)."""
    rng = np.random.default_rng(5)
    clients = [{"conv.weight": rng.standard_normal((8, 3, 3, 3)),
                "bn.running_mean": rng.standard_normal(8),
                "bn.num_batches_tracked": np.array(100 + i, np.int64),
                "fc.weight": rng.standard_normal((10, 72))} for i in range(len(weights))]
    want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in c.items()} for c in clients])
    got = AVG().server(upload(clients, weights), 0)["w_glob"]
    assert_dict_bitwise(got, want, f"f64 model, weights {type(weights[0]).__name__}")


@pytest.mark.parametrize("zero_copy,parts", [(False, 4), (True, 1), (True, 2), (True, 4), (True, 5)])
def test_small_round_fast_path_reuses_its_record_safely(zero_copy, parts, cuda, monkeypatch):
    """Small host rounds (every bucket < 4 MiB: flearn's config 1) take Aggregator._small_round:
    natively packed pinned staging, one H2D / launch / D2H per bucket (or, zero-copy, the kernel
    reading the pinned staging and writing the pinned result over PCIe — the fp32 bucket in
    `parts` chained launches, each after native threads packed its clients), one sync.  Round
    after round with new values (the record's staging reused) and with a value the native pack
    refuses (a non-contiguous view in an early or a late part: the general path takes over,
    nothing launched) every result is bit-equal to the oracle."""
    from flearn_amd.aggregator import Aggregator

    monkeypatch.setattr(Aggregator, "small_zero_copy", zero_copy)
    monkeypatch.setattr(Aggregator, "small_parts", parts)
    layout = layouts.get("lenet5")
    p = layouts.fp32_elems(layout)
    s = AVG()
    for r in range(6):
        flat = oracle.fill_uniform(10, p, seed=40 + r)
        clients = [layouts.synthetic_state_dict(layout, flat[i]) for i in range(10)]
        if r in (2, 4):  # a Fortran-ordered copy: same shape and dtype, not C-contiguous — in the
            # first half of the clients, and (round 4) in the second half, which the zero-copy
            # record packs only after its first launch is queued
            c = 3 if r == 2 else 7
            k = next(k for k, v in clients[c].items() if v.ndim == 2)
            clients[c][k] = np.asfortranarray(clients[c][k])
        weights = [1.0 + 0.5 * i for i in range(10)]
        got = s.server(upload(clients, weights), r)["w_glob"]
        want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in c.items()} for c in clients])
        assert_dict_bitwise(got, want, f"round {r}")
        rec = s.engine.last_plan.memo.get(("small_round", id(s.engine.packer), str(s.engine.device), "reference",
                                           zero_copy, parts))
        assert rec, "the small-round record was not built"


@pytest.mark.parametrize("wkind", ["pyfloat", "np64", "np32"])
@pytest.mark.parametrize("n,p,dev", [(3, 4099, False), (41, 4099, False), (3, 4_500_001, False),
                                     (5, 4_500_001, True)])
def test_special_values_match_reference(wkind, n, p, dev, cuda):
    """IEEE corner cases through the whole server path, against the oracle: fp32 subnormal inputs
    and products (no flush to zero), signed zeros (-0 sums stay -0), infinities, input NaNs, and
    inf - inf.  Bit-exact everywhere except the bits of NaNs the arithmetic creates (inf - inf):
    x86 SSE makes the negative default NaN, the GPU the positive canonical one — there only the
    NaN positions must agree."""
    rng = np.random.default_rng(n)
    tiny = np.float32(1.4e-45)  # the smallest fp32 subnormal
    clients = []
    for i in range(n):
        x = rng.standard_normal(p).astype(np.float32)
        if p > 260_000:  # the corner cases again at a piece boundary, mid-window and at the end
            for o in (262_144 - 100, p // 2 + 3, p - 300):
                x[o : o + 64] = tiny * (i + 1)
                x[o + 64 : o + 128] = -0.0
                x[o + 128] = np.inf if i == 0 else (-np.inf if i == n - 1 else 1.0)
        x[0:64] = tiny * (i + 1)                                  # subnormal inputs, subnormal sums
        x[64:128] = np.float32(1.1754942e-38) * rng.uniform(-1, 1, 64).astype(np.float32)  # around FLT_MIN
        x[128:192] = -0.0                                           # -0 + -0 ... = -0
        x[192:256] = 0.0 if i % 2 else -0.0                         # +0 / -0 mixed
        x[256] = np.inf                                             # +inf stays +inf
        x[257] = np.inf if i == 0 else (-np.inf if i == n - 1 else 1.0)  # inf - inf: a created NaN
        x[258] = np.float32("nan") if i == 1 else 2.0               # an input NaN propagates
        x[259] = np.float32(3.4e38)                                 # overflow to inf in the sum
        clients.append({"w": x, "b": x[:7].copy()})
    weights = {"pyfloat": [float(x) for x in rng.uniform(0.1, 3.0, n)],
               "np64": [np.float64(x) for x in rng.uniform(0.1, 3.0, n)],
               "np32": [np.float32(x) for x in rng.uniform(0.1, 3.0, n)]}[wkind]
    want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in c.items()} for c in clients])
    if dev:  # device-resident uploads: the row-pointer kernel reads them in place
        if wkind != "pyfloat":
            pytest.skip("torch uploads follow torch's promotion")
        import torch

        ups = [{"agg_weight": w, "params": {k: torch.from_numpy(v).to(cuda) for k, v in c.items()}}
               for w, c in zip(weights, clients)]
        got = {k: v.cpu().numpy() if hasattr(v, "cpu") else v for k, v in AVG().server(ups, 0)["w_glob"].items()}
    else:
        got = AVG().server(upload(clients, weights), 0)["w_glob"]
    for k in want:
        g, w = np.asarray(got[k]), np.asarray(want[k])
        assert g.dtype == w.dtype and g.shape == w.shape, k
        gn, wn = np.isnan(g), np.isnan(w)
        assert np.array_equal(gn, wn), (k, np.nonzero(gn != wn))
        assert g[~gn].tobytes() == w[~wn].tobytes(), (k, wkind, np.nonzero(g[~gn].view(np.uint8) != w[~wn].view(np.uint8)))
        if k == "w":
            assert np.all(np.signbit(g[128:192])) and np.isposinf(g[256]) and np.isnan(g[257]) and np.isnan(g[258])
            assert np.any(g[0:64] != 0)  # subnormal results were not flushed
