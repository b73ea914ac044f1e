"""Pin the CPU oracle to the reference: both restatements (numpy op-sequence and per-element C)
must reproduce every golden vector captured from flearn itself, bit for bit."""
import math

import numpy as np
import pytest

import oracle
from flearn_amd.semantics import KIND_F32, KIND_F64, KIND_I64, resolve
from golden_io import Golden, assert_dict_bitwise, bitwise_equal, cases

REDUCE_CASES = [c for c in cases() if c.startswith(("avg_", "bn_", "lg_", "trace_"))]
ROUND_CASES = [c for c in cases() if c.endswith("_rounds3") and not c.startswith("dyn_")]


def strategy_keys(g: Golden, clients):
    call = g.meta["call"]
    keys = oracle.intersect_keys(clients)
    if call.startswith("BN()"):
        return [k for k in keys if "bn" not in k]
    if call.startswith("LG("):
        return list(g.meta["shared_key_layers"])
    return None


def c_oracle_ensemble(weights, clients, keys):
    """Run the C restatement key by key with the dtypes semantics.resolve decides."""
    out = {}
    for k in keys:
        xs = [np.asarray(c[k].numpy() if hasattr(c[k], "numpy") else c[k]) for c in clients]
        nm = resolve(weights, xs[0].dtype)
        stack = np.stack([x.reshape(-1) for x in xs])
        if nm.kind == KIND_F32:
            r = oracle.c_reduce(nm.mode, stack, nm.weights, nm.denom)
        elif nm.kind == KIND_F64:
            r = oracle.c_reduce("f64", stack.astype(np.float64), nm.weights, nm.denom)
        else:
            assert nm.kind == KIND_I64
            r = oracle.c_reduce("i64", stack, nm.weights, nm.denom)
        assert r.dtype == nm.out_dtype
        r = r.reshape(xs[0].shape)
        out[k] = r.dtype.type(r[()]) if xs[0].shape == () else r
    return out


@pytest.mark.parametrize("name", REDUCE_CASES)
def test_numpy_oracle_matches_reference(name):
    g = Golden(name)
    clients, weights = g.clients(), g.weights()
    keys = strategy_keys(g, clients)
    with np.errstate(all="ignore"):
        got = oracle.server_ensemble(weights, clients, keys)
    want = g.output()
    assert_dict_bitwise(got, want, name)
    kinds = g.output_kinds()
    for k, v in got.items():
        if kinds[k].startswith("scalar:"):
            assert np.isscalar(v) and type(v).__name__ == kinds[k].split(":")[1]
        elif kinds[k].startswith("torch:"):
            assert str(v.dtype) == kinds[k][6:]


@pytest.mark.parametrize("name", REDUCE_CASES)
def test_c_oracle_matches_reference(name, oracle_lib):
    g = Golden(name)
    clients, weights = g.clients(), g.weights()
    keys = strategy_keys(g, clients) or oracle.intersect_keys(clients)
    got = c_oracle_ensemble(weights, clients, keys)
    want = {k: (v.numpy() if hasattr(v, "numpy") and not isinstance(v, np.ndarray) else v)
            for k, v in g.output().items()}
    assert_dict_bitwise(got, want, name)


def round_inputs(g: Golden, r):
    layout = [(k, tuple(s)) for k, s in g.meta["gen"]["layout"]]
    from golden_io import decode_weight, regenerate

    clients = regenerate(layout, 6, g.meta["gen"]["seeds"][r])
    weights = [decode_weight(e) for e in g.meta["round_weights"][r]]
    return clients, weights, [k for k, _ in layout]


@pytest.mark.parametrize("name", ROUND_CASES)
def test_numpy_oracle_rounds(name):
    g = Golden(name)
    op = g.meta["op"]
    prev = {k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")}
    v_t = None
    for r in range(g.meta["rounds"]):
        clients, weights, keys = round_inputs(g, r)
        avg = oracle.server_ensemble(weights, clients)
        assert_dict_bitwise(avg, g.output(f"avg{r}"), f"{name} avg{r}")
        if op == "avgm":
            w, v_t = oracle.mean_momentum(dict(prev), avg, v_t, 0.9)
        else:
            w, v_t = oracle.adaptive_opt(dict(prev), avg, v_t, op)
        assert_dict_bitwise(w, g.output(f"w{r}"), f"{name} w{r}")
        assert_dict_bitwise(v_t, g.output(f"v{r}"), f"{name} v{r}")
        prev = {k: np.asarray(w[k]).astype(np.float32) for k in keys}


@pytest.mark.parametrize("name", ROUND_CASES)
def test_c_oracle_rounds(name, oracle_lib):
    g = Golden(name)
    op = g.meta["op"]
    prev = {k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")}
    v = None
    for r in range(g.meta["rounds"]):
        clients, weights, keys = round_inputs(g, r)
        avg = c_oracle_ensemble(weights, clients, keys)
        assert_dict_bitwise(avg, g.output(f"avg{r}"), f"{name} avg{r}")
        gflat = np.concatenate([avg[k].reshape(-1) for k in keys])
        lflat = np.concatenate([prev[k].reshape(-1) for k in keys])
        if v is None:
            v = np.zeros_like(gflat)
        w = oracle.c_update(op, gflat, lflat, v)
        off = 0
        want_w, want_v = g.output(f"w{r}"), g.output(f"v{r}")
        for k in keys:
            n = math.prod(prev[k].shape)
            assert bitwise_equal(w[off : off + n].reshape(prev[k].shape), want_w[k]), f"{name} w{r} {k}"
            assert bitwise_equal(v[off : off + n].reshape(prev[k].shape), want_v[k]), f"{name} v{r} {k}"
            off += n
        prev = {k: np.asarray(want_w[k]).astype(np.float32) for k in keys}


def test_fixture_inventory():
    """The capture covers the cases SURVEY.md §8c lists."""
    names = set(cases())
    for n in (1, 2, 3, 10, 37, 100):
        assert f"avg_w1_n{n}" in names
    for must in ("avg_pyfloat_n37", "avg_pyint_n10", "avg_pyint_n100", "avg_np64_n10", "avg_np32_n10",
                 "avg_npint64_n10", "avg_special_n5", "avg_lenet5_n10", "avg_bnmodel_pyfloat_n4",
                 "avg_bnmodel_pyint_n4", "bn_strategy_n4", "lg_strategy_n4", "lg_r_strategy_n4",
                 "avg_keyintersect_n3", "avg_torch_n3", "trace_lenet5_round0", "trace_lenet5_round1"):
        assert must in names, must
    for op in ("avgm", "adagrad", "yogi", "adam"):
        assert f"{op}_pyfloat_rounds3" in names and f"{op}_np32_rounds3" in names


DYN_CASES = [c for c in cases() if c.startswith("dyn_")]


def dyn_round_inputs(g: Golden, r):
    from golden_io import decode_weight

    keys = g.meta["client_keys"]
    clients = [{k: g.arrays[f"r{r}x{i}:{k}"].copy() for k in keys} for i in range(g.meta["n_clients"])]
    return clients, [decode_weight(e) for e in g.meta["round_weights"][r]]


@pytest.mark.parametrize("name", DYN_CASES)
def test_numpy_oracle_dyn_rounds(name):
    g = Golden(name)
    h = {k[6:]: v.copy() for k, v in g.arrays.items() if k.startswith("hinit:")}
    theta = {k: v.copy() for k, v in h.items()}  # Dyn.__init__: theta = deepcopy(h)
    for r in range(g.meta["rounds"]):
        clients, weights = dyn_round_inputs(g, r)
        avg = oracle.server_ensemble(weights, clients)
        w, theta = oracle.dyn_f(avg, h, theta, len(clients))
        assert_dict_bitwise(w, g.output(f"w{r}"), f"{name} w{r}")
        assert_dict_bitwise(h, g.output(f"h{r}"), f"{name} h{r}")
        assert_dict_bitwise(theta, g.output(f"theta{r}"), f"{name} theta{r}")


@pytest.mark.parametrize("name", DYN_CASES)
def test_c_oracle_dyn_rounds(name, oracle_lib):
    g = Golden(name)
    h0 = {k[6:]: v for k, v in g.arrays.items() if k.startswith("hinit:")}
    fkeys = [k for k, v in h0.items() if v.dtype == np.float32]
    h = np.concatenate([h0[k].reshape(-1) for k in fkeys]).astype(np.float32)
    theta = None
    for r in range(g.meta["rounds"]):
        clients, weights = dyn_round_inputs(g, r)
        avg = c_oracle_ensemble(weights, clients, fkeys)
        gflat = np.concatenate([np.asarray(avg[k]).reshape(-1) for k in fkeys])
        if theta is None:
            theta = h.astype(gflat.dtype)
        w = oracle.c_update_dyn(gflat, h, theta, len(clients))
        want_w, want_h = g.output(f"w{r}"), g.output(f"h{r}")
        off = 0
        for k in fkeys:
            n = h0[k].size
            assert bitwise_equal(w[off : off + n].reshape(h0[k].shape), want_w[k]), f"{name} w{r} {k}"
            assert bitwise_equal(h[off : off + n].reshape(h0[k].shape), want_h[k]), f"{name} h{r} {k}"
            off += n


DISTILL_CASES = [c for c in cases() if c.startswith("distill_logits_")]


@pytest.mark.parametrize("name", DISTILL_CASES)
def test_numpy_oracle_logits_mean(name):
    g = Golden(name)
    tabs = [g.arrays[f"logits{i}"] for i in range(g.meta["n_clients"])]
    with np.errstate(all="ignore"):
        got = oracle.logits_mean(tabs)
    assert_dict_bitwise({"glob_logits": got}, g.output(), name)


def test_numpy_oracle_distill_server():
    g = Golden("distill_server_n4")
    clients, weights = g.clients(), g.weights()
    assert_dict_bitwise(oracle.server_ensemble(weights, clients), g.output(), "distill w_glob")
    tabs = [g.arrays[f"logits{i}"] for i in range(4)]
    assert_dict_bitwise({"glob_logits": oracle.logits_mean(tabs)}, g.output("glob"), "distill logits")
