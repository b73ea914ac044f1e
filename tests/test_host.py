"""Host-side logic of the aggregation boundary (no GPU): numpy-semantics resolution, bucket
planning, the Strategy registry and conversions, the multi-GPU shard plan, and that the product
path refuses to run without its HIP library / GPU instead of falling back to the CPU."""
import subprocess
import sys

import numpy as np
import pytest
import torch

import flearn_amd
from flearn_amd import _native as na
from flearn_amd import layouts
from flearn_amd.bucket import ALIGN, make_plan, select_keys
from flearn_amd.dist import ShardPlan
from flearn_amd.semantics import KIND_F32, KIND_F64, KIND_I64, resolve

WEIGHT_SETS = {
    "pyfloat": [1.0, 2.5, 0.25],
    "pyint": [3, 1, 600],
    "pybool": [True, True, False],
    "np32": [np.float32(1.5), np.float32(0.5), np.float32(2)],
    "np64": [np.float64(1.5), np.float64(0.5), np.float64(2)],
    "npint64": [np.int64(3), np.int64(1), np.int64(2)],
    "np16": [np.float16(1.5), np.float16(0.5), np.float16(2)],
    "mixed_float_int": [1.0, 2, 3],
}


@pytest.mark.parametrize("wname", sorted(WEIGHT_SETS))
@pytest.mark.parametrize("xdtype", [np.float32, np.float64, np.int64])
def test_resolve_agrees_with_numpy(wname, xdtype):
    """resolve() must predict exactly the dtypes numpy gives strategy.py:123-129."""
    ws = WEIGHT_SETS[wname]
    if len({np.result_type(w, xdtype) for w in ws}) > 1:
        with pytest.raises(TypeError):  # per-client precisions differ: rejected, not guessed
            resolve(ws, xdtype)
        return
    xs = [np.array([1, 2, 3], dtype=xdtype) for _ in ws]
    acc = ws[0] * xs[0]
    for a, x in zip(ws[1:], xs[1:]):
        acc = acc + a * x
    with np.errstate(all="ignore"):
        out = np.divide(acc, np.sum(ws))
    nm = resolve(ws, xdtype)
    assert nm.acc_dtype == acc.dtype
    assert nm.out_dtype == out.dtype
    assert nm.weights.dtype == nm.acc_dtype
    assert nm.denom == float(np.sum(ws))
    expected_kind = KIND_F32 if xdtype == np.float32 else (KIND_I64 if acc.dtype == np.int64 else KIND_F64)
    assert nm.kind == expected_kind
    if nm.kind == KIND_F32:
        want_mode = {(np.float32, np.float64): na.MODE_W32_DIV64, (np.float32, np.float32): na.MODE_W32_DIV32,
                     (np.float64, np.float64): na.MODE_W64}[(acc.dtype.type, out.dtype.type)]
        assert nm.mode == want_mode


def test_resolve_rejects_mixed_promotion_and_bad_inputs():
    with pytest.raises(TypeError):
        resolve([1.0, np.float64(2.0)], np.float32)  # fp32 and f64 products in one sum
    with pytest.raises(TypeError):
        resolve([1.0, "x"], np.float32)
    with pytest.raises(TypeError):
        resolve([1.0], np.float16)
    with pytest.raises(IndexError):
        resolve([], np.float32)


def test_weight_cast_is_numpys():
    big = 2**24 + 1  # not representable in fp32: numpy rounds it to even
    nm = resolve([big, 1], np.float32)
    assert nm.weights[0] == np.float32(big) == (big * np.ones(1, np.float32))[0]


def _clients(n=3):
    out = []
    for i in range(n):
        out.append({
            "conv.weight": np.full((4, 3, 3, 3), i, np.float32),
            "bn.running_mean": np.full((4,), i, np.float32),
            "bn.num_batches_tracked": np.array(10 + i, np.int64),
            "fc.weight": np.full((10, 37), i, np.float32),
            "fc.bias": np.full((10,), i, np.float32),
        })
    return out


def test_plan_layout_and_groups():
    cl = _clients()
    plan = make_plan([1.0, 1.0, 1.0], cl)
    assert plan.keys == list(cl[0].keys())
    f32 = plan.groups[KIND_F32]
    assert [s.key for s in f32.segments] == ["conv.weight", "bn.running_mean", "fc.weight", "fc.bias"]
    for s in f32.segments:
        assert s.offset % ALIGN == 0
    assert f32.stride % ALIGN == 0 and f32.stride >= sum(s.numel for s in f32.segments)
    assert plan.key_group["bn.num_batches_tracked"] == KIND_F64  # int64 x Python float -> f64
    plan_i = make_plan([1, 2, 3], cl)
    assert plan_i.key_group["bn.num_batches_tracked"] == KIND_I64  # int64 x Python int stays int


def test_plan_key_selection_and_errors():
    cl = _clients()
    del cl[1]["fc.bias"]
    assert "fc.bias" not in select_keys(cl)  # intersection, strategy.py:119-121
    with pytest.raises(KeyError):
        make_plan([1.0] * 3, cl, key_lst=["fc.bias"])
    cl = _clients()
    cl[2]["fc.weight"] = np.zeros((37, 10), np.float32)
    with pytest.raises(ValueError):
        make_plan([1.0] * 3, cl)
    cl = _clients()
    cl[1]["fc.bias"] = cl[1]["fc.bias"].astype(np.float64)
    with pytest.raises(ValueError):
        make_plan([1.0] * 3, cl)
    with pytest.raises(IndexError):
        make_plan([], [])
    cl = _clients(2)
    cl[1] = {k: torch.from_numpy(np.asarray(v)) for k, v in cl[1].items()}
    with pytest.raises(TypeError):
        make_plan([1.0, 1.0], cl)


def test_layouts_match_survey_counts():
    assert layouts.fp32_elems(layouts.get("lenet5")) == 44_426
    assert layouts.fp32_elems(layouts.get("resnet18")) == 11_699_112
    assert layouts.fp32_tensors(layouts.get("resnet18")) == 102
    assert layouts.fp32_elems(layouts.get("resnet50")) == 25_610_152
    assert layouts.fp32_tensors(layouts.get("resnet50")) == 267
    assert layouts.fp32_elems(layouts.get("vit_b_16")) == 86_567_656
    assert layouts.fp32_tensors(layouts.get("vit_b_16")) == 152


def test_registry_mirrors_reference():
    assert type(flearn_amd.setup_strategy("avg", None)).__name__ == "AVG"
    assert type(flearn_amd.setup_strategy("AVGM", None)).__name__ == "AVGM"
    s = flearn_amd.setup_strategy("lg", None, shared_key_layers=["fc.weight"])
    assert s.shared_key_layers == ["fc.weight"]
    assert flearn_amd.setup_strategy("opt", None, server_side=True).server_side
    custom = object()
    assert flearn_amd.setup_strategy("mystrategy", custom) is custom
    with pytest.raises(SystemError):
        flearn_amd.setup_strategy("nope", None)
    assert type(flearn_amd.setup_strategy("distill", None)).__name__ == "Distill"
    for name in ("md", "pav"):
        with pytest.raises(NotImplementedError):
            flearn_amd.setup_strategy(name, None)
    h = {"w": np.zeros(3, np.float32)}
    d = flearn_amd.setup_strategy("dyn", None, h=h)
    assert type(d).__name__ == "Dyn" and d.alpha == 0.01 and d.h is h
    assert d.theta is not h and np.array_equal(d.theta["w"], h["w"])  # dyn.py:14 deepcopy


def test_conversions_mirror_reference():
    d = {"a": torch.ones(3), "b": [1, 2], "c": np.zeros(2)}
    out = flearn_amd.convert_to_np(d)
    assert out is d and all(isinstance(v, np.ndarray) for v in d.values())
    flearn_amd.convert_to_tensor(d)
    assert all(isinstance(v, torch.Tensor) for v in d.values())
    with pytest.raises(SystemError):
        flearn_amd.convert_to_tensor({"n": np.float64(3.0)})  # the 0-d buffer quirk (avg.py:41)
    with pytest.raises(SystemError):
        flearn_amd.convert_to_np({"n": 3.0})


def test_client_upload_matches_reference_contract():
    class T:
        @property
        def weight(self):
            return {"w": torch.ones(2, 2), "bn.x": torch.zeros(2)}

    up = flearn_amd.AVG().client(T())
    assert up["agg_weight"] == 1.0 and isinstance(up["params"]["w"], np.ndarray)
    up = flearn_amd.BN().client(T(), agg_weight=3)
    assert list(up["params"]) == ["w"] and up["agg_weight"] == 3


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_product_path_fails_loudly_without_gpu():
    """No CPU fallback: the server path raises NativeUnavailable (never a silent numpy result)."""
    ups = [{"agg_weight": 1.0, "params": {"w": np.ones(4, np.float32)}}]
    with pytest.raises(na.NativeUnavailable):
        flearn_amd.AVG().server(ups, 0)


@pytest.mark.parametrize("exc,exits", [
    (ValueError("shape mismatch"), True), (TypeError("dtype"), True), (KeyError("w"), True),
    (IndexError("list index out of range"), True), (NotImplementedError("sparse uploads"), True),
    (RuntimeError("[gloo/transport/tcp/pair.cc] Connection closed by peer"), False),
    (RuntimeError("Expected all tensors to be on the same device"), False),
    (torch.distributed.DistBackendError("Watchdog caught collective operation timeout"), False),
    (na.NativeError("hipErrorLaunchFailure"), False), (OSError("pinned alloc"), False),
])
def test_only_client_data_errors_take_server_exception(exc, exits):
    """avg.py:28-31 turns what numpy would raise on bad uploads into SystemExit; a failed
    collective of a group= round (a plain RuntimeError from gloo/c10d), a device-placement error
    or a HIP failure is not bad client data and must propagate unchanged."""
    class Engine:
        def ensemble(self, *a, **k):
            raise exc

    s = flearn_amd.AVG()
    s._engine = Engine()
    ups = [{"agg_weight": 1.0, "params": {"w": np.ones(4, np.float32)}}]
    if exits:
        with pytest.raises(SystemExit):
            s.server(ups, 0)
    else:
        with pytest.raises(type(exc)) as info:
            s.server(ups, 0)
        assert info.value is exc


def test_product_never_imports_the_oracle():
    code = "import sys, flearn_amd, flearn_amd.aggregator, flearn_amd.dist; print('oracle' in sys.modules)"
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         cwd=str(layouts.__file__).rsplit("/flearn_amd/", 1)[0])
    assert out.stdout.strip() == "False", out.stderr
    import pathlib

    repo = pathlib.Path(flearn_amd.__file__).parent.parent
    # the product, its tools and examples; bench.py's cpu_baseline leg is the one allowed user
    for d in ("flearn_amd", "tools", "examples"):
        for f in (repo / d).rglob("*.py"):
            assert "import oracle" not in f.read_text(), f


@pytest.mark.parametrize("n_cols,world,stripes,weights", [
    (1, 1, 1, None), (11_699_112, 8, 4, None), (44_426, 2, 3, None), (1000, 4, 4, None),
    (11_699_112, 8, 2, (3, 1)), (44_426, 2, 3, (1, 2, 1)), (63, 2, 2, (3, 1)), (25_610_152, 4, 2, (4, 1))])
def test_shard_plan_covers_columns_once(n_cols, world, stripes, weights):
    p0 = ShardPlan.make(n_cols, world, 0, stripes, weights=weights)
    seen = np.zeros(p0.padded, dtype=np.int32)
    assert p0.padded >= n_cols and p0.stripes == stripes
    for r in range(world):
        p = ShardPlan.make(n_cols, world, r, stripes, weights=weights)
        assert p.widths == p0.widths and all(w % 64 == 0 and w > 0 for w in p.widths)
        for c in range(stripes):
            g0 = p.global_begin(c)
            seen[g0 : g0 + p.shard_of(c)] += 1
            assert p.local_to_global(p.local_begin(c)) == g0
            assert p.local_to_global(p.local_begin(c) + p.shard_of(c) - 1) == g0 + p.shard_of(c) - 1
    assert (seen == 1).all()
    if weights:  # widths follow the weights (to 64-column granularity)
        tot = sum(p0.widths)
        for wd, wt in zip(p0.widths, weights):
            assert abs(wd / tot - wt / sum(weights)) <= 64 * stripes / tot + 1e-9 or tot <= 64 * stripes


def _cpu_stage(plan, kind, shards):
    from flearn_amd.bucket import Packer, _STORE

    g = plan.groups[kind]
    hosts = [torch.zeros((plan.n_clients, sh.c1 - sh.c0), dtype=torch.from_numpy(np.zeros(0, _STORE[kind])).dtype)
             for sh in shards]
    return g, Packer._pieces(g, shards), hosts


def _python_pack(plan, pieces, ups, hosts):
    out = [np.zeros(h.shape, dtype=h.numpy().dtype) for h in hosts]
    for n, w in enumerate(ups):
        for s, a, b, sh, d in pieces:
            out[sh.index][n, d: d + (b - a)] = np.asarray(w[s.key]).reshape(-1)[a:b]
    return out


@pytest.mark.parametrize("n_shards", [1, 3])
def test_native_row_pack_matches_python(n_shards):
    """fa_py_pack_rows (csrc/fa_pyhost.c) writes exactly what the Python pack writes, for whole
    keys and for keys split at shard boundaries, with wire-staged rows skipped."""
    from flearn_amd.bucket import Shard, _NativeRows, split_columns

    lay = layouts.get("lenet5")
    p = layouts.fp32_elems(lay)
    rng = np.random.default_rng(3)
    ups = [layouts.synthetic_state_dict(lay, rng.random(p, dtype=np.float32), counter=i) for i in range(5)]
    plan = make_plan([1.0] * 5, ups)
    stride = plan.groups[KIND_F32].stride
    shards = ([Shard(0, torch.device("cpu"), 0, stride)] if n_shards == 1 else
              [Shard(i, torch.device("cpu"), c0, c1) for i, (c0, c1) in
               enumerate((sh.c0, sh.c1) for sh in split_columns(stride, ["cpu"] * n_shards))])
    g, pieces, hosts = _cpu_stage(plan, KIND_F32, shards)
    assert _NativeRows.usable(pieces, hosts)
    rows = [None, None, "staged", None, None]
    nat = _NativeRows(pieces, hosts, ups, rows)
    assert nat(0, 5)
    want = _python_pack(plan, pieces, ups, hosts)
    for h, w in zip(hosts, want):
        w[2] = 0  # the staged row is not packed
        np.testing.assert_array_equal(h.numpy(), w)


def test_native_row_pack_falls_back_without_copying():
    """Values the byte copy cannot take (torch tensors, non-contiguous views, a missing key, a
    non-dict upload) make the call return False with nothing written; int64 sources stored in an
    f64 bucket are not offered to it at all."""
    from flearn_amd.bucket import Shard, _NativeRows

    base = {"a": np.arange(6, dtype=np.float32).reshape(2, 3), "b": np.ones(4, np.float32)}
    plan = make_plan([1.0, 1.0], [base, base])
    sh = [Shard(0, torch.device("cpu"), 0, plan.groups[KIND_F32].stride)]
    g, pieces, hosts = _cpu_stage(plan, KIND_F32, sh)
    bad = [
        {"a": torch.zeros(2, 3), "b": np.ones(4, np.float32)},
        {"a": np.arange(6, dtype=np.float32).reshape(3, 2).T, "b": np.ones(4, np.float32)},
        {"b": np.ones(4, np.float32)},
        {"a": np.zeros((2, 3), np.float64), "b": np.ones(4, np.float32)},
    ]
    for other in bad:
        hosts[0].zero_()
        assert not _NativeRows(pieces, hosts, [base, other], [None, None])(0, 2)
        assert not hosts[0].numpy().any()
    from collections import UserDict
    assert not _NativeRows(pieces, hosts, [base, UserDict(base)], [None, None])(0, 2)
    assert _NativeRows(pieces, hosts, [base, base], [None, None])(0, 2)
    # int64 buffers under float weights live in the f64 bucket: a cast, not a byte copy
    ints = {"n": np.array(5, dtype=np.int64)}
    plan = make_plan([1.0, 2.0], [ints, ints])
    kind = plan.key_group["n"]
    _, pieces, hosts = _cpu_stage(plan, kind, [Shard(0, torch.device("cpu"), 0, plan.groups[kind].stride)])
    assert kind == KIND_F64 and not _NativeRows.usable(pieces, hosts)


def test_plan_cache_reuses_only_identical_metadata_and_weights():
    """Repeated rounds of one model reuse the plan; any change of weights (incl. 0.0 vs -0.0,
    float vs int), shapes, dtypes, key selection or client count plans afresh; a mismatching
    client still raises after the plan was cached."""
    a = {"w": np.ones((2, 3), np.float32), "b": np.ones(3, np.float32)}
    p1 = make_plan([1.0, 2.0], [a, dict(a)])
    assert make_plan([1.0, 2.0], [dict(a), a]) is p1
    for ws in ([1.0, 2.5], [1, 2], [np.float32(1.0), np.float32(2.0)], [-0.0, 2.0]):
        assert make_plan(ws, [a, a]) is not p1
    z1, z2 = make_plan([0.0, 1.0], [a, a]), make_plan([-0.0, 1.0], [a, a])
    assert z1 is not z2 and np.signbit(z2.f32.numerics.weights[0]) and not np.signbit(z1.f32.numerics.weights[0])
    assert make_plan([1.0, 2.0], [a, a], key_lst=["w"]) is not p1
    assert make_plan([1.0, 2.0, 1.0], [a, a, a]) is not p1
    b = dict(a, w=np.ones((3, 2), np.float32))
    assert make_plan([1.0, 2.0], [b, b]) is not p1
    with pytest.raises(ValueError):
        make_plan([1.0, 2.0], [a, b])
    c = dict(a, w=torch.ones(2, 3))
    with pytest.raises(TypeError):
        make_plan([1.0, 2.0], [a, c])


def test_device_output_is_one_copy_per_shard_and_views(monkeypatch):
    """output="device" reassembly (aggregator.assemble_on_device), on CPU tensors standing in for
    per-device shard outputs: one copy per (kind, shard) into one fresh buffer per kind, and every
    key a view of that buffer at its segment offset."""
    from flearn_amd.aggregator import assemble_on_device
    from flearn_amd.bucket import split_columns

    rng = np.random.default_rng(0)
    shapes = {"conv.weight": (6, 1, 5, 5), "bn.weight": (6,), "fc.weight": (10, 84), "fc.bias": (10,),
              "bn.num_batches_tracked": ()}
    clients = []
    for _ in range(3):
        c = {k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items() if s}
        c["bn.num_batches_tracked"] = np.array(7, dtype=np.int64)
        clients.append(c)
    plan = make_plan([1.0, 2.0, 3.0], clients)
    f32 = plan.groups[KIND_F32]
    full32 = torch.arange(f32.stride, dtype=torch.float32)
    shards = split_columns(f32.stride, ["cpu", "cpu", "cpu"])
    results = {KIND_F32: [(sh, full32[sh.c0 : sh.c1].clone()) for sh in shards]}
    for kind in plan.groups:
        if kind != KIND_F32:
            st = plan.groups[kind].stride
            results[kind] = [(split_columns(st, ["cpu"])[0], torch.full((st,), 5.0, dtype=torch.float64))]
    copies = []
    orig = torch.Tensor.copy_

    def counting_copy(self, src, non_blocking=False):
        copies.append((self.numel(), src.numel()))
        return orig(self, src, non_blocking)

    monkeypatch.setattr(torch.Tensor, "copy_", counting_copy)
    glob = assemble_on_device(plan, results, "cpu")
    assert len(copies) == len(shards) + len(plan.groups) - 1  # one per shard of every kind, no per-key copies
    base = {kind: None for kind in plan.groups}
    for k in plan.keys:
        s = plan.key_segment[k]
        t = glob[k]
        assert tuple(t.shape) == tuple(s.shape)
        kind = plan.key_group[k]
        if kind == KIND_F32:
            assert torch.equal(t.reshape(-1), full32[s.offset : s.offset + s.numel])
        ptr = t.untyped_storage().data_ptr()
        assert base[kind] in (None, ptr)  # all keys of a kind view one fresh buffer
        base[kind] = ptr
    assert base[KIND_F32] != full32.untyped_storage().data_ptr()


def test_server_optimizer_restore_binds_v_t_to_the_bucket():
    """ServerOptimizer.load_state / set_v_t (host logic, CPU shards): the restored previous global
    model (cast to fp32) and v_t land at every key's columns of the f32 bucket, split over shards;
    state_dict() gives them back keyed like w_glob; set_v_t before init_global is refused."""
    from flearn_amd.aggregator import ServerOptimizer
    from flearn_amd.bucket import split_columns

    rng = np.random.default_rng(5)
    cl = [{"a": rng.random((3, 70), dtype=np.float32), "b": rng.random(5, dtype=np.float32)} for _ in range(2)]
    plan = make_plan([1.0, 2.0], cl)
    glob = {"a": rng.random((3, 70)), "b": rng.random(5)}  # f64, as w_glob comes back
    v = {"a": rng.random((3, 70)), "b": rng.random(5)}
    opt = ServerOptimizer("adagrad")
    with pytest.raises(RuntimeError):
        opt.set_v_t(v)
    with pytest.raises(RuntimeError):
        opt.state_dict(plan)  # nothing bound yet
    opt.load_state({"w_glob": glob, "v_t": v})
    shards = split_columns(plan.f32.stride, ["cpu", "cpu"])
    assert opt.prepare(plan, shards)
    got = opt.state_dict()
    for k in glob:
        assert got["w_glob"][k].dtype == np.float32 and np.array_equal(got["w_glob"][k], glob[k].astype(np.float32))
        assert got["v_t"][k].dtype == np.float64 and np.array_equal(got["v_t"][k], v[k])
    bad = ServerOptimizer("avgm")
    bad.load_state({"w_glob": glob, "v_t": {"a": v["a"]}})
    with pytest.raises(KeyError):
        bad.prepare(plan, shards)
    bad.load_state({"w_glob": glob, "v_t": {"a": v["a"], "b": np.zeros(4)}})
    with pytest.raises(ValueError):
        bad.prepare(plan, shards)


def test_slab_stack_detection():
    """Packer._slab_stack (host logic on CPU tensors): uploads carved from one allocation laid out
    as the bucket become one [N, stride] view of it — rows from a subset keep their pitch and
    offset; reversed order, a foreign tensor or another layout are refused (None)."""
    from flearn_amd import device_state_dicts
    from flearn_amd.bucket import Packer

    rng = np.random.default_rng(3)
    t = {"a": torch.from_numpy(rng.random((3, 70), dtype=np.float32)), "b": torch.from_numpy(rng.random(5, dtype=np.float32)),
         "n": torch.tensor(4)}
    sd = device_state_dicts(t, 5, device="cpu")
    for i, d in enumerate(sd):
        d["a"].add_(i)

    def stack_of(clients):
        plan = make_plan([1.0] * len(clients), clients)
        g = plan.f32
        segs = [s for s in g.segments if s.numel > 0]
        ptrs = np.array([[c[s.key].data_ptr() for c in clients] for s in segs], dtype=np.int64)
        return plan, g, Packer._slab_stack(plan, g, clients, (segs, ptrs, [], None))

    plan, g, st = stack_of(list(sd))
    assert st is not None and st.shape == (5, g.stride) and st.data_ptr() == sd.slab.data_ptr()
    assert torch.equal(st, sd.slab[:, : g.stride])
    plan, g, st = stack_of(list(sd)[2:])
    assert st is not None and st.data_ptr() == sd.slab[2].data_ptr() and st.stride(0) == sd.slab.stride(0)
    assert stack_of(list(sd)[::-1])[2] is None
    mixed = [dict(c) for c in sd]
    mixed[1]["b"] = mixed[1]["b"].clone()
    assert stack_of(mixed)[2] is None
    other = [{"a": c["a"].clone(), "b": c["b"].clone(), "n": c["n"]} for c in sd]  # separate allocations
    assert stack_of(other)[2] is None
