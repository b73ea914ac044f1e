"""GPU: property test of the whole server path — random model layouts (fp32 / float64 / int64
tensors, 0-d and empty included, sizes that land on every kernel geometry from one chunk to
several pieces per block), random client counts and every weight kind numpy distinguishes —
AVG().server (plan, pack, HIP reduce, unpack) against the oracle's restatement of
strategy.py:102-130, bit for bit."""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle
from flearn_amd import AVG
from golden_io import assert_dict_bitwise

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 3, 4, 63, 64, 65, 257, 1000, 4099, 44426, 70001, 262147]


@st.composite
def case(draw):
    nkeys = draw(st.integers(1, 6))
    lay = []
    for i in range(nkeys):
        dt = draw(st.sampled_from([np.float32, np.float32, np.float32, np.float64, np.int64]))
        numel = draw(st.sampled_from(SIZES))
        shape = () if (numel == 1 and draw(st.booleans())) else (numel,)
        lay.append((f"k{i}", shape, dt))
    n = draw(st.sampled_from([1, 2, 3, 7, 17, 64, 130]))
    wkind = draw(st.sampled_from(["pyfloat", "pyint", "np32", "np64", "ones"]))
    seed = draw(st.integers(0, 2**31 - 1))
    return lay, n, wkind, seed


@settings(max_examples=int(os.environ.get("FA_PROP_EXAMPLES", "40")), deadline=None,
          suppress_health_check=list(HealthCheck))
@given(c=case())
def test_server_matches_oracle_on_random_layouts(c, cuda):
    lay, n, wkind, seed = c
    rng = np.random.default_rng(seed)
    clients = []
    for _ in range(n):
        d = {}
        for k, shape, dt in lay:
            if dt == np.int64:
                d[k] = rng.integers(-1000, 1000, size=shape).astype(np.int64)
            else:
                d[k] = rng.standard_normal(shape).astype(dt)
        clients.append(d)
    weights = {"pyfloat": [float(x) for x in rng.uniform(0.1, 3.0, n)],
               "pyint": [int(x) for x in rng.integers(1, 600, n)],
               "np32": [np.float32(x) for x in rng.uniform(0.1, 3.0, n)],
               "np64": [np.float64(x) for x in rng.uniform(0.1, 3.0, n)],
               "ones": [1.0] * n}[wkind]
    want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in cl.items()} for cl in clients])
    got = AVG().server([{"agg_weight": w, "params": cl} for w, cl in zip(weights, clients)], 0)["w_glob"]
    assert_dict_bitwise(got, want, f"{lay} n={n} {wkind}")


@settings(max_examples=int(os.environ.get("FA_PROP_EXAMPLES", "40")) // 2, deadline=None,
          suppress_health_check=list(HealthCheck))
@given(c=case())
def test_device_uploads_match_host_uploads(c, cuda):
    """The same random rounds with the uploads as CUDA tensors (flearn's run2 path: the
    row-pointer kernel and the one-launch gathers read them in place) give the values the host
    path gives (itself bit-exact against the oracle above)."""
    import torch

    lay, n, wkind, seed = c
    if wkind not in ("pyfloat", "ones"):
        return  # torch uploads follow torch's promotion; the run2 simulator sends 1.0 / len(loader)
    rng = np.random.default_rng(seed)
    clients = [{k: (rng.integers(-1000, 1000, size=shape).astype(np.int64) if dt == np.int64
                    else rng.standard_normal(shape).astype(dt)) for k, shape, dt in lay} for _ in range(n)]
    weights = [float(x) for x in rng.uniform(0.1, 3.0, n)] if wkind == "pyfloat" else [1.0] * n
    host = AVG().server([{"agg_weight": w, "params": cl} for w, cl in zip(weights, clients)], 0)["w_glob"]
    dev_clients = [{k: torch.from_numpy(np.array(v)).to(cuda) for k, v in cl.items()} for cl in clients]  # 0-d stays 0-d
    dev = AVG().server([{"agg_weight": w, "params": cl} for w, cl in zip(weights, dev_clients)], 0)["w_glob"]
    assert list(dev) == list(host)
    for k in host:
        h = np.asarray(host[k])
        d = dev[k].cpu().numpy() if isinstance(dev[k], torch.Tensor) else np.asarray(dev[k])
        assert d.shape == h.shape, k
        assert np.array_equal(d.astype(np.float64).view(np.int64), h.astype(np.float64).view(np.int64)), k


def test_fresh_servers_reusing_a_cached_plan(cuda):
    """Regression (found by the property test above): servers created one after another reuse
    the module's plan cache while their pinned stagings recycle each other's blocks; the native
    pack table must follow the pieces, not just the staging addresses.  A float64 key, an int64
    key (int weights: its own bucket) and fp32 keys, the same round on four fresh servers."""
    lay = [("k0", (65,), np.float64), ("k1", (262147,), np.float32), ("k2", (1000,), np.float32),
           ("k3", (257,), np.float32), ("k4", (65,), np.int64), ("k5", (63,), np.float32)]
    rng = np.random.default_rng(354)
    clients = [{k: (rng.integers(-1000, 1000, size=s).astype(np.int64) if dt == np.int64
                    else rng.standard_normal(s).astype(dt)) for k, s, dt in lay} for _ in range(2)]
    weights = [int(x) for x in rng.integers(1, 600, 2)]
    want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in c.items()} for c in clients])
    for rep in range(4):
        got = AVG().server([{"agg_weight": w, "params": c} for w, c in zip(weights, clients)], rep)["w_glob"]
        assert_dict_bitwise(got, want, f"fresh server {rep}")


@settings(max_examples=int(os.environ.get("FA_PROP_EXAMPLES", "40")) // 2, deadline=None,
          suppress_health_check=list(HealthCheck))
@given(c=case(), strat=st.sampled_from(["AVG", "BN", "LG"]), shards=st.integers(1, 3),
       out=st.sampled_from(["reference", "float32"]), http=st.booleans())
def test_strategies_shards_outputs_and_codec(c, strat, shards, out, http, cuda):
    """Key filters (BN: keys without "bn", bn.py:23-33; LG: the shared keys, lg.py:27-35), column
    shards over several devices (the same GPU here), output="float32" (= fl32 of the reference's
    float64 result for fp32 keys) and HTTP-mode uploads (the reference's base64(pickle) text
    through flearn_amd.Encrypt) on random layouts, against the oracle."""
    import base64
    import pickle

    from flearn_amd import BN, LG, Encrypt

    lay, n, wkind, seed = c
    lay = [(("bn." if i % 3 == 1 else "conv.") + k, s, dt) for i, (k, s, dt) in enumerate(lay)]
    rng = np.random.default_rng(seed)
    clients = [{k: (rng.integers(-1000, 1000, size=s).astype(np.int64) if dt == np.int64
                    else rng.standard_normal(s).astype(dt)) for k, s, dt in lay} for _ in range(n)]
    weights = {"pyfloat": [float(x) for x in rng.uniform(0.1, 3.0, n)],
               "pyint": [int(x) for x in rng.integers(1, 600, n)],
               "np32": [np.float32(x) for x in rng.uniform(0.1, 3.0, n)],
               "np64": [np.float64(x) for x in rng.uniform(0.1, 3.0, n)],
               "ones": [1.0] * n}[wkind]
    keys = [k for k, _, _ in lay]
    if strat == "BN":
        s, key_lst = BN(), [k for k in keys if "bn" not in k]
    elif strat == "LG":
        shared = keys[::2]
        s, key_lst = LG(shared), shared
    else:
        s, key_lst = AVG(), keys
    if not key_lst:
        return
    s.output = out
    s.devices = [cuda] * shards
    want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in cl.items()} for cl in clients], key_lst)
    ups = [{"agg_weight": w, "params": cl} for w, cl in zip(weights, clients)]
    if http:  # what a flearn HTTP server hands Strategy.server after receive_processing
        enc = Encrypt(fast_min_chars=0)
        ups = [enc.decode(base64.b64encode(pickle.dumps(u)).decode()) for u in ups]
    got = s.server(ups, 0)["w_glob"]
    assert set(got) == set(want)
    for k, w in want.items():
        g, w = np.asarray(got[k]), np.asarray(w)
        src = dict((kk, dt) for kk, _, dt in lay)[k]
        if out == "float32" and src == np.float32 and w.dtype == np.float64:
            w = w.astype(np.float32)
        assert g.shape == w.shape and g.dtype == w.dtype, (k, g.dtype, w.dtype)
        assert np.array_equal(g.reshape(-1).view(np.uint8), w.reshape(-1).view(np.uint8)), (k, strat, shards, out, http)


@settings(max_examples=int(os.environ.get("FA_PROP_EXAMPLES", "40")) // 2, deadline=None,
          suppress_health_check=list(HealthCheck))
@given(cs=st.lists(case(), min_size=2, max_size=4), order=st.lists(st.integers(0, 3), min_size=3, max_size=8))
def test_one_server_many_rounds(cs, order, cuda):
    """ONE server across rounds whose layouts, client counts and weights change and come back
    (cached plans, small-round records, pinned stagings and zero-copy buffers reused and
    switched between), with fresh values every round: every round bit-equal to the oracle."""
    s = AVG()
    for r, i in enumerate(order):
        lay, n, wkind, seed = cs[i % len(cs)]
        rng = np.random.default_rng(seed + 7919 * r)  # new values each round, same layout
        clients = [{k: (rng.integers(-1000, 1000, size=shape).astype(np.int64) if dt == np.int64
                        else rng.standard_normal(shape).astype(dt)) for k, shape, dt in lay} for _ in range(n)]
        weights = {"pyfloat": [float(x) for x in rng.uniform(0.1, 3.0, n)],
                   "pyint": [int(x) for x in rng.integers(1, 600, n)],
                   "np32": [np.float32(x) for x in rng.uniform(0.1, 3.0, n)],
                   "np64": [np.float64(x) for x in rng.uniform(0.1, 3.0, n)],
                   "ones": [1.0] * n}[wkind]
        want = oracle.server_ensemble(weights, [{k: v.copy() for k, v in cl.items()} for cl in clients])
        got = s.server([{"agg_weight": w, "params": cl} for w, cl in zip(weights, clients)], r)["w_glob"]
        assert_dict_bitwise(got, want, f"round {r}: {lay} n={n} {wkind}")


@settings(max_examples=int(os.environ.get("FA_PROP_EXAMPLES", "40")) // 2, deadline=None,
          suppress_health_check=list(HealthCheck))
@given(c=case(), op=st.sampled_from(["avgm", "adagrad", "yogi", "adam"]), init=st.booleans(),
       shards=st.integers(1, 2))
def test_server_side_optimizer_rounds_on_random_layouts(c, op, init, shards, cuda):
    """Server-fused FedAVGM / FedOPT (BASELINE configs 3 and 5) on random fp32 layouts, 3 rounds:
    round r = the reference's mean of fresh uploads, then the reference's update with w_local =
    the previous global model in fp32 (avgm.py:19-36, opt.py:23-65) — the first round adopts the
    mean when no previous model was given — composed from the oracle's restatements, bit for bit,
    with the double-buffered state in HBM (and split over column shards)."""
    from flearn_amd import AVGM, OPT

    lay, n, wkind, seed = c
    lay = [(k, shape, np.float32) for k, shape, _ in lay]  # the fused step covers the fp32 bucket
    rng = np.random.default_rng(seed)
    s = AVGM(server_side=True) if op == "avgm" else OPT(server_side=True, method=op)
    s.devices = [cuda] * shards
    prev = None
    if init:
        prev = {k: rng.standard_normal(shape).astype(np.float32) for k, shape, _ in lay}
        s.server_opt.init_global(prev)
    v = None
    for r in range(3):
        clients = [{k: rng.standard_normal(shape).astype(np.float32) for k, shape, _ in lay} for _ in range(n)]
        weights = {"pyfloat": [float(x) for x in rng.uniform(0.1, 3.0, n)],
                   "pyint": [int(x) for x in rng.integers(1, 600, n)],
                   "np32": [np.float32(x) for x in rng.uniform(0.1, 3.0, n)],
                   "np64": [np.float64(x) for x in rng.uniform(0.1, 3.0, n)],
                   "ones": [1.0] * n}[wkind]
        g = oracle.server_ensemble(weights, [{k: a.copy() for k, a in cl.items()} for cl in clients])
        if prev is None:  # first round, no previous model: the mean, state adopted
            want = g
        elif op == "avgm":
            want, v = oracle.mean_momentum(prev, g, v, 0.9)
        else:
            want, v = oracle.adaptive_opt(prev, g, v, op)
        prev = {k: np.asarray(want[k]).astype(np.float32) for k in want}
        got = s.server([{"agg_weight": w, "params": cl} for w, cl in zip(weights, clients)], r)["w_glob"]
        assert_dict_bitwise(got, want, f"round {r} {op} {lay} n={n} {wkind} init={init}")
