"""GPU parity of device-resident uploads read in place (fa_reduce_f32_rows / fa_gather_rows).

flearn's simulator path hands the server torch tensors (run2: flearn/server/Communicator.py:
287-292 -> Server.ensemble -> strategy.server, Server.py:140).  On the GPU each (client, key)
tensor is its own allocation; the engine reads them through a device table of pointers in one
launch instead of packing N*K tensors.  Bar: bit-exact against the reference's fixtures and
against the stack kernel (itself bit-exact vs the C oracle) on the same data."""
import numpy as np
import pytest
import torch

import oracle
from flearn_amd import AVG, AVGM, OPT, Dyn
from flearn_amd import _native as na
from flearn_amd import aggregator as agg
from flearn_amd import layouts
from golden_io import Golden, bitwise_equal

pytestmark = pytest.mark.gpu


def _to_cuda(c, cuda):
    return {k: (v.to(cuda) if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v)).to(cuda))
            for k, v in c.items()}


def _upload(clients, weights):
    return [{"agg_weight": w, "params": c} for w, c in zip(weights, clients)]


def _host(v):
    return v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


@pytest.mark.parametrize("name", ["avg_torch_n3", "avg_w1_n10", "avg_w1_n100", "avg_pyint_n100", "avg_np32_n10",
                                  "avg_np64_n10", "avg_npint64_n10", "avg_special_n5", "avg_negzero_n1",
                                  "avg_bnmodel_pyint_n4", "avg_bnmodel_pyfloat_n4", "trace_lenet5_round0",
                                  "avg_lenet5_n10"])
def test_device_uploads_read_in_place(name, cuda):
    g = Golden(name)
    clients = [_to_cuda(c, cuda) for c in g.clients()]
    s = AVG()
    got = s.server(_upload(clients, g.weights()), 0)["w_glob"]
    packer = s.engine.packer
    assert packer.last_row_tables.get("f32") == "rows", packer.last_row_tables  # no pack copy
    # int64 values of the float64 group (BN counters with float weights) take the converting
    # gather, never per-tensor copy kernels
    assert "copy" not in packer.last_row_tables.values(), packer.last_row_tables
    for k, w in g.output().items():
        assert bitwise_equal(_host(got[k]), np.asarray(w)), (name, k)


def test_gather_rows_f64_converts_like_numpy(cuda):
    """fa_gather_rows_f64: int64 -> float64 rounded to nearest as numpy's astype (values beyond
    2**53 included), float32 exact, float64 copied; segments at any column offset."""
    L = na.load()
    n, stride = 3, 256
    rng = np.random.default_rng(5)
    big = np.array([2**53 + 1, 2**53 + 3, -(2**63), 2**63 - 1, -(2**53) - 1, 0, -1, 7], dtype=np.int64)
    segs_host = []  # (col, values)
    vals = [[big, rng.integers(-2**62, 2**62, 37, dtype=np.int64), rng.standard_normal(5).astype(np.float32),
             rng.standard_normal(11)] for _ in range(n)]
    cols = [0, 9, 101, 130]
    srcs = [na.SRC_I64, na.SRC_I64, na.SRC_F32, na.SRC_F64]
    dev_vals = [[torch.from_numpy(v).to(cuda) for v in row] for row in vals]
    ptrs = np.array([[dev_vals[i][s].data_ptr() for i in range(n)] for s in range(4)], dtype=np.int64)
    ptr_d = torch.from_numpy(ptrs.reshape(-1)).to(cuda)
    segs = torch.tensor(cols + [len(v) for v in vals[0]] + srcs, dtype=torch.int64, device=cuda)
    stack = torch.full((n, stride), -5.0, dtype=torch.float64, device=cuda)
    na.check(L.fa_gather_rows_f64(stack.data_ptr(), stride, n, ptr_d.data_ptr(), segs.data_ptr(), 4,
                                  na.stream_handle(cuda)), "gather")
    got = stack.cpu().numpy()
    for i in range(n):
        want = np.full(stride, -5.0)
        for c, v in zip(cols, vals[i]):
            want[c : c + len(v)] = v.astype(np.float64)
        assert bitwise_equal(got[i], want), i


def test_gather_rows_more_clients_than_one_grid_dimension(cuda):
    """fa_gather_rows / fa_gather_rows_f64 tile the launch over blocks of 65,535
    clients (the grid's y limit) instead of refusing a bigger round: 70,001 clients."""
    L = na.load()
    n, stride = 70_001, 64
    src32 = torch.arange(2 * n, dtype=torch.float32, device=cuda) * 0.5
    src64 = torch.arange(n, dtype=torch.int64, device=cuda) * 3 - 7
    segs = torch.tensor([0, 5, 1, 2], dtype=torch.int64, device=cuda)  # cols 0, 5; lengths 1, 2
    base = src32.data_ptr()
    ptrs = torch.tensor(np.concatenate([base + 4 * np.arange(n, dtype=np.int64),  # segment 0: element i
                                        base + 4 * (n - 2 + 0 * np.arange(n, dtype=np.int64))]),  # segment 1
                        dtype=torch.int64, device=cuda)
    stack = torch.full((n, stride), -1.0, dtype=torch.float32, device=cuda)
    na.check(L.fa_gather_rows(stack.data_ptr(), stride, n, 4, ptrs.data_ptr(), segs.data_ptr(), 2,
                              na.stream_handle(cuda)), "gather")
    got = stack.cpu().numpy()
    assert bitwise_equal(got[:, 0], src32[:n].cpu().numpy())
    assert (got[:, 5:7] == src32[n - 2 : n].cpu().numpy()).all() and (got[:, 1:5] == -1).all()
    ptr64 = torch.tensor(src64.data_ptr() + 8 * np.arange(n, dtype=np.int64), dtype=torch.int64, device=cuda)
    segs64 = torch.tensor([3, 1, na.SRC_I64], dtype=torch.int64, device=cuda)
    st64 = torch.zeros((n, stride), dtype=torch.float64, device=cuda)
    na.check(L.fa_gather_rows_f64(st64.data_ptr(), stride, n, ptr64.data_ptr(), segs64.data_ptr(), 1,
                                  na.stream_handle(cuda)), "gather f64")
    assert bitwise_equal(st64[:, 3].cpu().numpy(), src64.cpu().numpy().astype(np.float64))


def test_unaligned_device_uploads_take_one_gather(cuda):
    """Views at odd element offsets cannot feed 16-B buffer loads: one fa_gather_rows launch
    packs them, and the result is still bit-exact."""
    g = Golden("avg_w1_n10")
    clients = []
    for c in g.clients():
        flat = torch.empty(sum(v.size for v in c.values()) + 1, dtype=torch.float32, device=cuda)
        d, off = {}, 1  # every view starts 4 bytes past an allocation boundary
        for k, v in c.items():
            d[k] = flat[off : off + v.size].view(v.shape)
            d[k].copy_(torch.from_numpy(v))
            off += v.size
        clients.append(d)
    s = AVG()
    got = s.server(_upload(clients, g.weights()), 0)["w_glob"]
    assert s.engine.packer.last_row_tables.get("f32") == "gather"
    for k, w in g.output().items():
        assert bitwise_equal(_host(got[k]), np.asarray(w)), k


def _separate_tensors(stack, layout):
    """Per-client dicts of separate device tensors (one allocation each), from a device stack."""
    out = []
    for i in range(stack.shape[0]):
        d, off = {}, 0
        for k, shape, t in layout:
            if t != "f32":
                continue
            n = int(np.prod(shape, dtype=np.int64))
            d[k] = stack[i, off : off + n].clone().view(shape)
            off += -(-max(n, 1) // 64) * 64
        out.append(d)
    return out


@pytest.mark.slow
@pytest.mark.parametrize("layout_name,n,op", [("resnet18", 100, "mean"), ("resnet50", 24, "avgm"),
                                              ("resnet18", 30, "adagrad")])
def test_device_upload_baseline_size(layout_name, n, op, cuda):
    """C2-size device uploads (100 x ResNet-18, 10,200 separate tensors) and fused optimizer
    steps through the row-pointer kernel: bit-equal to the stack kernel on the same data."""
    layout = layouts.get(layout_name)
    stride = layouts.padded_f32_stride(layout)
    x = torch.empty((n, stride), dtype=torch.float32, device=cuda)
    agg.fill_uniform(x, seed=99)
    clients = _separate_tensors(x, layout)
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    want = torch.empty(stride, dtype=torch.float32, device=cuda)
    kw, s = {}, AVG(output="float32")
    if op != "mean":
        prev = torch.empty((1, stride), dtype=torch.float32, device=cuda)
        agg.fill_uniform(prev, seed=5)
        kw = dict(op=na.OP_BY_NAME[op], prev=prev[0].clone(), v=torch.zeros(stride, dtype=torch.float64, device=cuda))
        s = AVGM(server_side=True, output="float32") if op == "avgm" else OPT(server_side=True, method=op,
                                                                              output="float32")
        glob0 = {}
        off = 0
        ph = prev[0].cpu().numpy()
        for k, shape, t in layout:
            if t == "f32":
                m = int(np.prod(shape, dtype=np.int64))
                glob0[k] = ph[off : off + m].reshape(shape)
                off += -(-max(m, 1) // 64) * 64
        s.server_opt.init_global(glob0)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=want, **kw)
    got = s.server(_upload(clients, [1.0] * n), 0)["w_glob"]
    assert s.engine.packer.last_row_tables.get("f32") == "rows"
    want_h = want.cpu().numpy()
    off = 0
    for k, shape, t in layout:
        if t != "f32":
            continue
        m = int(np.prod(shape, dtype=np.int64))
        assert bitwise_equal(np.asarray(got[k]).reshape(-1), want_h[off : off + m]), k
        off += -(-max(m, 1) // 64) * 64


@pytest.mark.parametrize("name", ["avgm_pyfloat_rounds3", "adagrad_np32_rounds3", "yogi_pyfloat_rounds3"])
def test_fused_optimizer_device_uploads(name, cuda):
    from golden_io import decode_weight, regenerate

    g = Golden(name)
    op = g.meta["op"]
    s = AVGM(server_side=True) if op == "avgm" else OPT(server_side=True, method=op)
    s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
    layout = [(k, tuple(sh)) for k, sh in g.meta["gen"]["layout"]]
    for r in range(g.meta["rounds"]):
        clients = [_to_cuda(c, cuda) for c in regenerate(layout, 6, g.meta["gen"]["seeds"][r])]
        weights = [decode_weight(e) for e in g.meta["round_weights"][r]]
        got = s.server(_upload(clients, weights), r)["w_glob"]
        assert s.engine.packer.last_row_tables.get("f32") == "rows"
        for k, w in g.output(f"w{r}").items():
            assert bitwise_equal(_host(got[k]), np.asarray(w)), (name, r, k)


def test_dyn_device_uploads(cuda):
    from golden_io import decode_weight

    g = Golden("dyn_pyfloat_rounds3")
    h = {k[6:]: v.copy() for k, v in g.arrays.items() if k.startswith("hinit:")}
    d = Dyn(h)
    keys = g.meta["client_keys"]
    for r in range(g.meta["rounds"]):
        clients = [_to_cuda({k: g.arrays[f"r{r}x{i}:{k}"].copy() for k in keys}, cuda) for i in range(g.meta["n_clients"])]
        weights = [decode_weight(e) for e in g.meta["round_weights"][r]]
        got = d.server(_upload(clients, weights), r)["w_glob"]
        assert d.engine.packer.last_row_tables.get("f32") == "rows"
        for k, w in g.output(f"w{r}").items():
            assert bitwise_equal(_host(got[k]), np.asarray(w)), (r, k)
        for k, w in g.output(f"h{r}").items():
            assert bitwise_equal(_host(d.h[k]), np.asarray(w)), (r, k)


def test_back_to_back_device_output_rounds_with_host_uploads(cuda):
    """rounds queued back to back with output='device' (no host sync in between)
    must not let round k+1's pack overwrite pinned staging that round k's H2D still reads."""
    n, p = 24, 1_500_000
    layout = [("w", (p,), "f32")]
    s = AVG(output="device")
    outs, wants = [], []
    for r in range(4):
        flat = oracle.fill_uniform(n, p, seed=1000 + r)
        clients = [{"w": flat[i]} for i in range(n)]
        outs.append(s.server(_upload(clients, [1.0] * n), r)["w_glob"]["w"])
        wants.append(oracle.c_reduce(oracle.MODE_W32_DIV64, flat, np.ones(n, np.float32), float(n)).astype(np.float32))
    torch.cuda.synchronize()
    for r, (o, w) in enumerate(zip(outs, wants)):
        assert bitwise_equal(o.cpu().numpy(), w), r
    assert layout


# ---------------------------------------------------------------------------------------------
# slab uploads (flearn_amd.device_state_dicts): the clients' fp32 tensors in ONE allocation laid
# out as the bucket — read in place by the stack kernel (Packer._slab_stack)
# ---------------------------------------------------------------------------------------------


def _slab_clients(clients, cuda):
    """The fixture's clients copied into device_state_dicts (values exact, dtypes kept)."""
    from flearn_amd import device_state_dicts

    cl = [_to_cuda(c, cuda) for c in clients]
    sd = device_state_dicts(cl[0], len(cl), device=cuda)
    for d, c in zip(sd, cl):
        for k, v in c.items():
            d[k].copy_(v)
    return sd


@pytest.mark.parametrize("name", ["avg_w1_n100", "avg_pyint_n100", "avg_np32_n10", "avg_special_n5",
                                  "avg_negzero_n1", "avg_bnmodel_pyfloat_n4", "trace_lenet5_round0", "avg_lenet5_n10"])
def test_slab_uploads_run_the_stack_kernel(name, cuda):
    g = Golden(name)
    sd = _slab_clients(g.clients(), cuda)
    s = AVG()
    got = s.server(_upload(list(sd), g.weights()), 0)["w_glob"]
    if "f32" in s.engine.last_plan.groups:
        assert s.engine.packer.last_row_tables.get("f32") == "slab", s.engine.packer.last_row_tables
    for k, w in g.output().items():
        assert bitwise_equal(_host(got[k]), np.asarray(w)), (name, k)


@pytest.mark.parametrize("name", ["avgm_pyfloat_rounds3", "adagrad_np32_rounds3", "adam_pyfloat_rounds3"])
def test_fused_optimizer_slab_uploads(name, cuda):
    from golden_io import decode_weight, regenerate

    g = Golden(name)
    op = g.meta["op"]
    s = AVGM(server_side=True) if op == "avgm" else OPT(server_side=True, method=op)
    s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
    layout = [(k, tuple(sh)) for k, sh in g.meta["gen"]["layout"]]
    for r in range(g.meta["rounds"]):
        sd = _slab_clients(regenerate(layout, 6, g.meta["gen"]["seeds"][r]), cuda)
        weights = [decode_weight(e) for e in g.meta["round_weights"][r]]
        got = s.server(_upload(list(sd), weights), r)["w_glob"]
        assert s.engine.packer.last_row_tables.get("f32") == "slab"
        for k, w in g.output(f"w{r}").items():
            assert bitwise_equal(_host(got[k]), np.asarray(w)), (name, r, k)


def test_slab_rows_subset_and_order(cuda):
    """Clients 1..n-1 of a slab (a row offset) still run as a stack; reversed order (negative
    pitch) or a foreign tensor among them falls back to the pointer table — same results."""
    from flearn_amd import device_state_dicts

    g = Golden("avg_w1_n10")
    sd = _slab_clients(g.clients(), cuda)
    want = None
    for sel, path in ((list(sd)[1:], "slab"), (list(sd)[::-1], "rows"), (list(sd), "slab")):
        s = AVG(output="float32")
        got = s.server(_upload(sel, [1.0] * len(sel)), 0)["w_glob"]
        assert s.engine.packer.last_row_tables.get("f32") == path, (path, s.engine.packer.last_row_tables)
        ref = AVG(output="float32").server(_upload([{k: v.cpu().numpy() for k, v in c.items()} for c in sel],
                                                   [1.0] * len(sel)), 0)["w_glob"]
        for k in ref:
            assert bitwise_equal(_host(got[k]), np.asarray(ref[k])), (path, k)
        want = got
    mixed = list(sd)
    k0 = next(iter(mixed[3]))
    mixed[3] = dict(mixed[3])
    mixed[3][k0] = mixed[3][k0].clone()  # one tensor outside the slab
    s = AVG(output="float32")
    got = s.server(_upload(mixed, [1.0] * len(mixed)), 0)["w_glob"]
    assert s.engine.packer.last_row_tables.get("f32") == "rows"
    for k in want:
        assert bitwise_equal(_host(got[k]), _host(want[k])), k
    assert isinstance(device_state_dicts(sd[0], 2, device=cuda).slab, torch.Tensor)


@pytest.mark.slow
@pytest.mark.parametrize("layout_name,n,op", [("resnet50", 100, "mean"), ("resnet50", 100, "avgm")])
def test_slab_uploads_baseline_size(layout_name, n, op, cuda):
    """NS / C3-size slab uploads (100 x ResNet-50): the engine's reduce reads the slab as its
    stack — bit-equal to the stack kernel over a packed copy of the same values."""
    from flearn_amd import device_state_dicts

    layout = layouts.get(layout_name)
    template = {k: torch.zeros(shape, dtype=torch.float32 if t == "f32" else torch.int64) for k, shape, t in layout}
    sd = device_state_dicts(template, n, device=cuda)
    agg.fill_uniform(sd.slab, seed=77)
    stride = sd.slab.shape[1]
    x = sd.slab.clone()
    w = torch.ones(n, dtype=torch.float32, device=cuda)
    want = torch.empty(stride, dtype=torch.float32, device=cuda)
    kw, s = {}, AVG(output="float32")
    if op != "mean":
        prev = torch.empty((1, stride), dtype=torch.float32, device=cuda)
        agg.fill_uniform(prev, seed=5)
        kw = dict(op=na.OP_BY_NAME[op], prev=prev[0].clone(), v=torch.zeros(stride, dtype=torch.float64, device=cuda))
        s = AVGM(server_side=True, output="float32")
        ph = prev[0].cpu().numpy()
        s.server_opt.init_global({k: ph[o : o + m].reshape(shp) for k, (o, m, shp) in sd.offsets.items()})
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=want, **kw)
    got = s.server(_upload(list(sd), [1.0] * n), 0)["w_glob"]
    assert s.engine.packer.last_row_tables.get("f32") == "slab"
    want_h = want.cpu().numpy()
    for k, (o, m, shp) in sd.offsets.items():
        assert bitwise_equal(np.asarray(got[k]).reshape(-1), want_h[o : o + m]), k
