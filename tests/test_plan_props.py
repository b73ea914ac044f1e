"""Host (no GPU): properties of the bucket plan (flearn_amd/bucket.py make_plan) over random
model layouts — the invariants the kernels rely on (16-B aligned, disjoint segments inside the
row stride, one kind per key as numpy's promotion of strategy.py:123-129 decides, the first
client's key order), checked with hypothesis instead of hand-picked layouts."""
import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from flearn_amd.bucket import ALIGN, make_plan
from flearn_amd.semantics import KIND_F32, KIND_F64, KIND_I64

DTYPES = [np.float32, np.float32, np.float32, np.float64, np.int64]

shapes = st.lists(st.integers(0, 70), min_size=0, max_size=3).map(tuple)
layout = st.lists(st.tuples(shapes, st.sampled_from(DTYPES)), min_size=1, max_size=12)


@settings(max_examples=150, deadline=None)
@given(layout, st.integers(1, 5), st.sampled_from(["pyfloat", "pyint", "np32", "np64"]))
def test_plan_invariants(lay, n, wkind):
    keys = [f"layer{i}.{'weight' if i % 2 else 'bias'}" for i in range(len(lay))]
    clients = [{k: np.zeros(s, dt) for k, (s, dt) in zip(keys, lay)} for _ in range(n)]
    weights = {"pyfloat": [1.0] * n, "pyint": [1] * n, "np32": [np.float32(1)] * n,
               "np64": [np.float64(1)] * n}[wkind]
    try:
        plan = make_plan(weights, clients)
    except TypeError:
        # a weight / dtype pair whose per-client precisions would differ is refused, not guessed
        # (np.float32 weights on int64 buffers promote to float64 — still one precision, so only
        # dtypes outside fp32/f64/int64 reach here; none are generated)
        raise
    assert plan.keys == keys  # the first client's insertion order
    assert plan.n_clients == n
    seen = set()
    for kind, g in plan.groups.items():
        assert g.stride % ALIGN == 0
        end = 0
        for s in g.segments:
            assert s.offset % ALIGN == 0 and s.offset >= end  # aligned, disjoint, in order
            assert s.numel == int(np.prod(s.shape, dtype=np.int64))
            end = s.offset + s.numel
            assert plan.key_group[s.key] == kind and plan.key_segment[s.key] is s
            seen.add(s.key)
        assert end <= g.stride
    assert seen == set(keys)
    for k, (s, dt) in zip(keys, lay):
        prod = np.result_type(weights[0], dt)
        want = KIND_F32 if dt == np.float32 and prod == np.float32 else (KIND_I64 if prod == np.int64 else KIND_F64)
        if dt == np.float32:
            want = KIND_F32  # fp32 tensors stay in the fp32 bucket whatever the sum precision (mode)
        assert plan.key_group[k] == want, (k, dt, wkind)


weight = st.one_of(
    st.floats(0.01, 1e3, allow_nan=False), st.integers(1, 10**6), st.booleans().filter(bool),
    st.floats(0.01, 1e3).map(np.float32), st.floats(0.01, 1e3).map(np.float64),
    st.integers(1, 10**6).map(np.int64))


@settings(max_examples=300, deadline=None)
@given(st.lists(weight, min_size=1, max_size=6), st.sampled_from([np.float32, np.float64, np.int64]))
def test_resolve_matches_numpy_or_refuses(ws, xdtype):
    """semantics.resolve on arbitrary weight lists: either it refuses (the clients' products
    would have different precisions — numpy would silently mix them) or it predicts exactly the
    dtypes numpy gives strategy.py:123-129, the weights as numpy casts them, and W = np.sum."""
    from flearn_amd.semantics import resolve

    xs = [np.array([1, 2, 3], dtype=xdtype) for _ in ws]
    prods = {np.result_type(w, xdtype) for w in ws}
    if len(prods) > 1:
        try:
            resolve(ws, xdtype)
        except TypeError:
            return
        raise AssertionError("mixed per-client precisions must be refused")
    acc = ws[0] * xs[0]
    for a, x in zip(ws[1:], xs[1:]):
        acc = acc + a * x
    with np.errstate(all="ignore"):
        out = np.divide(acc, np.sum(ws))
    nm = resolve(ws, xdtype)
    assert nm.acc_dtype == acc.dtype and nm.out_dtype == out.dtype
    assert nm.denom == float(np.sum(ws))
    for w, c in zip(ws, nm.weights):
        one = (w * np.ones(1, xdtype))[0]  # numpy's cast of the weight in its product (x 1: exact)
        assert one.dtype == acc.dtype and (one == c or (np.isnan(one) and np.isnan(c)))


@settings(max_examples=120, deadline=None)
@given(layout, st.integers(1, 6), st.data())
def test_slab_stack_is_the_uploads_or_nothing(lay, n, data):
    """Packer._slab_stack over random layouts and random client selections from one
    device_state_dicts slab (CPU tensors): a selection of rows at one positive pitch (consecutive
    rows in order, or two rows with a gap) becomes a [N, stride] view whose every key segment IS
    each client's tensor (same bytes, same address); any other selection (reordered, unevenly
    gapped, a foreign tensor) is refused."""
    import torch

    from flearn_amd import device_state_dicts
    from flearn_amd.bucket import Packer

    keys = [f"layer{i}.{'weight' if i % 2 else 'bias'}" for i in range(len(lay))]
    template = {k: torch.from_numpy(np.zeros(s, dt)) for k, (s, dt) in zip(keys, lay)}
    plan0 = make_plan([1.0], [template])
    if KIND_F32 not in plan0.groups:
        return
    sd = device_state_dicts(template, n + 2, device="cpu")
    torch.manual_seed(n)
    sd.slab.copy_(torch.randn_like(sd.slab))
    start = data.draw(st.integers(0, 2))
    order = list(range(start, start + n))
    kind = data.draw(st.sampled_from(["consecutive", "reversed", "gapped", "foreign"]))
    if kind == "reversed" and n > 1:
        order = order[::-1]
    elif kind == "gapped" and n > 1 and start == 0:
        order = [0] + list(range(2, n + 1))  # row 1 skipped: one pitch only for two rows
    clients = [dict(sd[i]) for i in order]
    if kind == "foreign":  # a non-empty key (an empty tensor reads no bytes: its address is moot)
        k = next((s.key for s in plan0.groups[KIND_F32].segments if s.numel > 0), None)
        if k is None:
            return
        clients[-1][k] = clients[-1][k].clone()
    plan = make_plan([1.0] * len(clients), clients)
    g = plan.groups[KIND_F32]
    segs = [s for s in g.segments if s.numel > 0]
    if not segs:
        return
    ptrs = np.array([[c[s.key].data_ptr() for c in clients] for s in segs], dtype=np.int64)
    st_ = Packer._slab_stack(plan, g, clients, (segs, ptrs, [], None))
    # rows at one positive pitch (consecutive, or two rows with a gap) are a strided [N, stride] view
    steps = {b - a for a, b in zip(order, order[1:])}
    uniform = not steps or (len(steps) == 1 and steps.pop() > 0)
    if kind == "foreign" or not uniform:
        assert st_ is None
        return
    assert st_ is not None and st_.shape == (len(clients), g.stride)
    for r, c in enumerate(clients):
        for s in segs:
            view = st_[r, s.offset : s.offset + s.numel]
            assert view.data_ptr() == c[s.key].data_ptr() and torch.equal(view, c[s.key].reshape(-1))
