"""Rank bodies of tests/test_gpu_multirank.py: the multi-GPU product paths (Strategy `group=`
mode — the SPMD server behind flearn's Server.py:140 — and bench's ShardedReducer) run by
several fresh processes that share cuda:0, with the real HIP kernels.

RCCL refuses two ranks on one device, so the ranks talk over gloo; flearn_amd.dist stages the
device tensors through host memory around each gloo collective (`all_gather_into`), and
everything else — column packing per rank, the sharded optimizer / FedDyn state, the
reduce launches, the post-gather divide — is the code the RCCL path runs.  Every rank checks
its own reassembled model (and state) bit for bit against the reference's fixtures or the C
oracle; any failure raises in the rank and fails the test.
"""
from __future__ import annotations

import os
import sys
import traceback
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def upload(clients, weights):
    return [{"agg_weight": w, "params": c} for w, c in zip(weights, clients)]


def _round_inputs(g, r):
    from golden_io import decode_weight, regenerate

    layout = [(k, tuple(s)) for k, s in g.meta["gen"]["layout"]]
    clients = regenerate(layout, 6, g.meta["gen"]["seeds"][r])
    return clients, [decode_weight(e) for e in g.meta["round_weights"][r]]


# ---------------------------------------------------------------------------------------------
# cases (each runs on every rank)
# ---------------------------------------------------------------------------------------------


def case_avg_fixtures(rank, world):
    """AVG / BN / LG(group=True) on the reference's fixtures: w_glob on every rank bit-equal to
    the reference (float64 outputs through the fp32-sum gather + post-gather divide), and
    output="float32" equal to fl32(reference)."""
    from flearn_amd import AVG, BN, LG, LG_R
    from golden_io import Golden, assert_dict_bitwise, bitwise_equal, cases

    def strategy_for(g, **kw):
        call = g.meta["call"]
        if call.startswith("BN()"):
            return BN(**kw)
        if call.startswith("LG_R("):
            return LG_R(g.meta["shared_key_layers"], **kw)
        if call.startswith("LG("):
            return LG(g.meta["shared_key_layers"], **kw)
        return AVG(**kw)

    names = [c for c in cases() if c.startswith(("avg_", "bn_", "lg_", "trace_"))]
    assert len(names) >= 20
    for name in names:
        g = Golden(name)
        s = strategy_for(g, group=True)
        got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
        assert_dict_bitwise(got, g.output(), f"rank {rank}/{world} {name}")
        nm = s.engine.last_plan.f32.numerics if s.engine.last_plan.f32 is not None else None
        if nm is not None and nm.out_dtype == np.float64 and nm.mode == 0:
            # the float64 result came from gathered fp32 sums (P*4 bytes on the wire)
            assert s.engine._post_denom == float(nm.denom), name
        if g.meta.get("input_kind") != "torch":
            s32 = strategy_for(g, group=True, output="float32")
            got32 = s32.server(upload(g.clients(), g.weights()), 0)["w_glob"]
            for k, w in g.output().items():
                w = np.asarray(w)
                if w.dtype == np.float64 and g.meta["in_dtypes"][k] == "float32":
                    assert bitwise_equal(np.asarray(got32[k]), w.astype(np.float32)), (name, k)


def case_setup_strategy(rank, world):
    """setup_strategy passes group= through (reference registry: common/utils.py:16-58)."""
    from flearn_amd import setup_strategy
    from golden_io import Golden, assert_dict_bitwise

    s = setup_strategy("avg", None, group=True)
    assert s.group is True
    g = Golden("avg_w1_n10")
    got = s.server(upload(g.clients(), g.weights()), 0)["w_glob"]
    assert_dict_bitwise(got, g.output(), f"rank {rank} setup_strategy avg")
    assert s.engine.packer.rank_cols == (rank, world)


def case_fused_rounds(rank, world):
    """Server-fused FedAVGM / FedOPT (adagrad, yogi, adam) with group=True over the 3-round
    fixtures: w_glob every round and the gathered v_t bit-equal to the reference's."""
    from flearn_amd import AVGM, OPT
    from golden_io import Golden, assert_dict_bitwise, cases

    names = [c for c in cases() if c.endswith("_rounds3") and not c.startswith("dyn_")]
    assert names
    for name in names:
        g = Golden(name)
        op = g.meta["op"]
        s = AVGM(server_side=True, group=True) if op == "avgm" else OPT(server_side=True, method=op, group=True)
        s.server_opt.init_global({k[6:]: v for k, v in g.arrays.items() if k.startswith("prev0:")})
        for r in range(g.meta["rounds"]):
            clients, weights = _round_inputs(g, r)
            got = s.server(upload(clients, weights), r)["w_glob"]
            assert_dict_bitwise(got, g.output(f"w{r}"), f"rank {rank} {name} w{r}")
            v = s.server_opt.v_t(s.engine.last_plan)  # collective: every rank calls it
            assert_dict_bitwise(v, g.output(f"v{r}"), f"rank {rank} {name} v{r}")


def case_first_round_adopt(rank, world):
    """FedAVGM without init_global: round 0 returns the mean and adopts it as the previous model
    (every rank, including ones whose column range is empty), round 1 is fused; both equal the
    unsharded engine's, and v_t gathers on every rank."""
    from flearn_amd import AVGM
    from golden_io import Golden, assert_dict_bitwise

    for name in ("avg_w1_n10", "trace_lenet5_round0"):
        g = Golden(name)
        a, b = AVGM(server_side=True, group=True), AVGM(server_side=True)
        for r in range(2):
            got = a.server(upload(g.clients(), g.weights()), r)["w_glob"]
            want = b.server(upload(g.clients(), g.weights()), r)["w_glob"]
            assert_dict_bitwise(got, want, f"rank {rank} {name} round {r}")
            assert_dict_bitwise(a.server_opt.v_t(a.engine.last_plan), b.server_opt.v_t(b.engine.last_plan),
                                f"rank {rank} {name} v_t round {r}")


def case_empty_ranks(rank, world):
    """A model narrower than one ALIGN unit per rank: the last ranks own no columns.  AVG, the
    adopt-then-fuse FedAVGM rounds and v_t must complete on every rank (no rank may skip a
    collective) and agree with the unsharded engine."""
    from flearn_amd import AVG, AVGM
    from golden_io import assert_dict_bitwise

    rng = np.random.default_rng(11)
    clients = [{"w": rng.standard_normal(10).astype(np.float32), "b": rng.standard_normal(3).astype(np.float32)}
               for _ in range(5)]
    weights = [1.0, 2.0, 0.5, 3.0, 1.25]
    got = AVG(group=True).server(upload(clients, weights), 0)["w_glob"]
    assert_dict_bitwise(got, AVG().server(upload(clients, weights), 0)["w_glob"], f"rank {rank} tiny AVG")
    a, b = AVGM(server_side=True, group=True), AVGM(server_side=True)
    for r in range(3):
        cl = [{k: v * (1 + r) for k, v in c.items()} for c in clients]
        got = a.server(upload(cl, weights), r)["w_glob"]
        want = b.server(upload(cl, weights), r)["w_glob"]
        assert_dict_bitwise(got, want, f"rank {rank} tiny AVGM round {r}")
        assert_dict_bitwise(a.server_opt.v_t(a.engine.last_plan), b.server_opt.v_t(b.engine.last_plan),
                            f"rank {rank} tiny v_t round {r}")


def case_dyn(rank, world):
    """Dyn(h, group=True) over the 3-round fixtures: w_glob, h (gathered and synced back into the
    caller's arrays in place) and theta bit-identical to the reference's on every rank."""
    from flearn_amd import Dyn
    from golden_io import Golden, assert_dict_bitwise, cases, decode_weight

    names = [c for c in cases() if c.startswith("dyn_")]
    assert names
    for name in names:
        g = Golden(name)
        h = {k[6:]: v.copy() for k, v in g.arrays.items() if k.startswith("hinit:")}
        h_ids = {k: id(v) for k, v in h.items()}
        s = Dyn(h, group=True)
        keys = g.meta["client_keys"]
        for r in range(g.meta["rounds"]):
            clients = [{k: g.arrays[f"r{r}x{i}:{k}"].copy() for k in keys} for i in range(g.meta["n_clients"])]
            weights = [decode_weight(e) for e in g.meta["round_weights"][r]]
            got = s.server(upload(clients, weights), r)["w_glob"]
            assert_dict_bitwise(got, g.output(f"w{r}"), f"rank {rank} {name} w{r}")
            assert s.theta is got
            hh = s.h  # collective
            assert hh is h and all(id(hh[k]) == h_ids[k] for k in h)
            assert_dict_bitwise(hh, g.output(f"h{r}"), f"rank {rank} {name} h{r}")
            dev = s._dyn.dev_keys
            assert_dict_bitwise({k: v for k, v in s._dyn.theta_host().items() if k in dev},
                                {k: np.asarray(v) for k, v in g.output(f"theta{r}").items() if k in dev},
                                f"rank {rank} {name} theta{r}")


def case_sharded_reducer(rank, world):
    """bench.py's device-resident path: ShardedReducer over this rank's block-cyclic columns with
    the HIP kernel, plans of 1, 2 (3:1) and model-chosen stripes, plain mean and fused AVGM /
    Adagrad (state sharded, prev advanced in place), two steps; every rank's reassembled model
    equals the C oracle's unsharded reduce bit for bit."""
    import oracle
    from flearn_amd import _native as na
    from flearn_amd import aggregator as agg
    from flearn_amd.dist import ShardedReducer, ShardPlan, StripeModel, hip_reduce_fn, plan_shards, plan_stripes

    cuda = torch.device("cuda", 0)
    n, p = 9, 700_001
    lc = -(-p // world)
    widths, rep = plan_shards(p, world, StripeModel(1e-6, 2e-9, 2e-6, 1e-8))  # gather-bound: a replicated tail
    assert rep > 0
    plans = [ShardPlan.make(p, world, rank, 1), ShardPlan.make(p, world, rank, 2, weights=(3, 1)),
             ShardPlan.from_widths(p, world, rank, plan_stripes(lc, StripeModel.assumed(n, world))),
             ShardPlan.from_widths(p, world, rank, widths, rep=rep)]
    w_h = np.linspace(0.5, 1.5, n).astype(np.float32)
    denom = float(np.sum([float(x) for x in w_h]))
    want_mean = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, 3), w_h, denom)
    for plan in plans:
        for op in ("mean", "avgm", "adagrad"):
            stack = torch.empty((n, plan.local_stride), dtype=torch.float32, device=cuda)
            for lo, g0, width in plan.segments():
                agg.fill_uniform(stack[:, lo:], seed=3, col_begin=g0, n_cols=width)
            w = torch.from_numpy(w_h).to(cuda)
            epi, local_out = {}, None
            if op != "mean":
                prev = torch.empty((1, plan.local_stride), dtype=torch.float32, device=cuda)
                for lo, g0, width in plan.segments():
                    agg.fill_uniform(prev[:, lo:], seed=4, col_begin=g0, n_cols=width)
                epi = dict(op=na.OP_BY_NAME[op], prev=prev[0],
                           v=torch.zeros(plan.local_stride, dtype=torch.float64, device=cuda))
                local_out = prev[0]
            red = ShardedReducer(plan, hip_reduce_fn(stack, w, na.MODE_W32_DIV64, denom, **epi), cuda,
                                 local_out=local_out, gather=True)
            want = want_mean.copy()
            prev_h = oracle.fill_uniform(1, p, 4)[0]
            v_h = np.zeros(p)
            for step in range(2):
                full = red.step().cpu().numpy()
                if op != "mean":
                    want = oracle.c_update(op, want_mean, prev_h, v_h)  # v_h updated in place
                    prev_h = want.astype(np.float32)
                assert full.tobytes() == want.astype(np.float32).tobytes(), (rank, plan.widths, op, step)


def case_sharded_reducer_push(rank, world, mode="kernel"):
    """The same ShardedReducer steps reassembled by PushGather (direct peer stores through
    IPC-mapped receive buffers: fa_push, or copy engines with mode "dma") instead of the
    all-gather: every rank's model equals the C oracle's bit for bit; plus one PushGather.gather
    of a rank-stamped slice against all_gather_into, and a push outside the receive buffer
    refused."""
    import oracle
    from flearn_amd import _native as na
    from flearn_amd import aggregator as agg
    from flearn_amd.dist import PushGather, ShardedReducer, ShardPlan, StripeModel, all_gather_into, hip_reduce_fn
    from flearn_amd.dist import plan_shards, plan_stripes

    cuda = torch.device("cuda", 0)
    n, p = 9, 700_001
    lc = -(-p // world)
    widths, rep = plan_shards(p, world, StripeModel(1e-6, 2e-9, 2e-6, 1e-8))
    plans = [ShardPlan.make(p, world, rank, 1), ShardPlan.make(p, world, rank, 2, weights=(3, 1)),
             ShardPlan.from_widths(p, world, rank, plan_stripes(lc, StripeModel.assumed(n, world))),
             ShardPlan.from_widths(p, world, rank, widths, rep=rep)]
    w_h = np.linspace(0.5, 1.5, n).astype(np.float32)
    denom = float(np.sum([float(x) for x in w_h]))
    want_mean = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, 3), w_h, denom)
    for plan in plans:
        for op in ("mean", "adagrad"):
            stack = torch.empty((n, plan.local_stride), dtype=torch.float32, device=cuda)
            for lo, g0, width in plan.segments():
                agg.fill_uniform(stack[:, lo:], seed=3, col_begin=g0, n_cols=width)
            w = torch.from_numpy(w_h).to(cuda)
            epi, local_out = {}, None
            if op != "mean":
                prev = torch.empty((1, plan.local_stride), dtype=torch.float32, device=cuda)
                for lo, g0, width in plan.segments():
                    agg.fill_uniform(prev[:, lo:], seed=4, col_begin=g0, n_cols=width)
                epi = dict(op=na.OP_BY_NAME[op], prev=prev[0],
                           v=torch.zeros(plan.local_stride, dtype=torch.float64, device=cuda))
                local_out = prev[0]
            red = ShardedReducer(plan, hip_reduce_fn(stack, w, na.MODE_W32_DIV64, denom, **epi), cuda,
                                 local_out=local_out, gather=True, push="dma" if mode == "dma" else True)
            assert red.pusher is not None
            want = want_mean.copy()
            prev_h = oracle.fill_uniform(1, p, 4)[0]
            v_h = np.zeros(p)
            for step in range(3):
                full = red.step().cpu().numpy()
                if op != "mean":
                    want = oracle.c_update(op, want_mean, prev_h, v_h)
                    prev_h = want.astype(np.float32)
                if full.tobytes() != want.astype(np.float32).tobytes():
                    bad = np.nonzero(full.view(np.uint32) != want.astype(np.float32).view(np.uint32))[0]
                    owners = sorted({next((r for r in range(world) for c in range(plan.stripes)
                                          if plan.global_begin(c, r) <= b < plan.global_begin(c, r) + plan.widths[c]),
                                          -1) for b in bad[:: max(1, len(bad) // 64)]})
                    raise AssertionError((rank, mode, plan.widths, op, step, len(bad), int(bad[0]), int(bad[-1]),
                                          "slices of ranks", owners))
            red.release()
    # kernel mode: an explicitly registered bucket, last — its unmap precedes no further export in
    # this process (the dma case runs after it: a bucket from the pool, mapped already)
    if mode == "kernel":
        full = torch.full((world * 4096,), -1.0, device=cuda)
        pg = PushGather(full, None, mode=mode)
    else:
        pg = PushGather(None, None, mode=mode, cols=world * 4096, device=cuda)
        full = pg.full
        full.fill_(-1.0)
    src = torch.arange(4096, dtype=torch.float32, device=cuda) + 10000.0 * rank
    pg.gather(src, rank * 4096)
    want = torch.empty_like(full)
    all_gather_into(want, src)
    torch.cuda.synchronize()
    assert torch.equal(full, want), rank
    try:
        pg.push(src, world * 4096 - 64)
        raise AssertionError("push past the end accepted")
    except ValueError:
        pass
    pg.close()


def case_sharded_reducer_push_dma(rank, world):
    case_sharded_reducer_push(rank, world, mode="dma")


def case_push_lifecycle(rank, world):
    """The set-up / teardown sequences behind round 4's wrong buckets, driven deterministically 12
    times each: (a) pool buckets taken, gathered into, released and parked by shutdown_push, then
    the next pool's; (b) an explicitly registered DeviceBuffer, closed (unmap + barrier) and
    parked, then the next one, sizes cycling so parked buckets are re-exported.  Every set-up
    validates every mapping by its token (`_map_peers` raises on a mismatch: a wrong import fails
    the test), every gathered bucket equals the all-gather's, the registered bucket's head bytes
    survive the token, and exported memory is re-used, never freed."""
    from flearn_amd import dist as fd

    cuda = torch.device("cuda", 0)
    pool_ptrs, own_ptrs = set(), set()
    for it in range(12):
        cols = world * (4096 + 1024 * (it % 3))
        src = torch.arange(cols // world, dtype=torch.float32, device=cuda) + 1e5 * rank + it
        want = torch.empty(cols, dtype=torch.float32, device=cuda)
        fd.all_gather_into(want, src)
        # (a) the pool: buckets parked by shutdown_push, re-exported by the next pool
        pg = fd.PushGather(None, None, mode="kernel" if it % 2 == 0 else "dma", cols=cols, device=cuda)
        assert pg.stale == [] and fd._RecvPool.bytes_held() >= cols * 4
        pool_ptrs.add(pg.full.data_ptr())
        pg.gather(src, rank * (cols // world))
        torch.cuda.synchronize()
        assert torch.equal(pg.full, want), (rank, it, "pool")
        pg.close()
        fd.shutdown_push()
        assert fd._RecvPool.bytes_held() == 0 and fd.DeviceBuffer.parked_bytes() > 0
        # (b) an explicit DeviceBuffer bucket, its head bytes preserved through registration
        buf = fd.DeviceBuffer.get(cols * 4, cuda)
        buf.tensor(torch.float32)[:cols].fill_(-7.0)
        pe = fd.PushGather(buf, None, mode="kernel")
        full = pe.full[:cols]
        assert buf.exported and full.data_ptr() == buf.ptr
        own_ptrs.add(buf.ptr)
        assert pe.stale == [] and bool((full[:4] == -7.0).all())
        pe.gather(src, rank * (cols // world))
        torch.cuda.synchronize()
        assert torch.equal(full, want), (rank, it, "explicit")
        pe.close()  # every peer unmapped (second barrier) before this rank re-uses the bucket
        del full, pe
        buf.free()  # exported: parked for the next registration, never freed
    # three sizes cycling: the parked buckets came back instead of new allocations
    assert len(pool_ptrs | own_ptrs) <= 6, (len(pool_ptrs), len(own_ptrs))


def case_push_growth_trim(rank, world):
    """Growing receive buckets (x1.25 per job, both push forms): each larger request retires the
    free bucket, and the parked bytes pass the cap (2 x the largest exported), so parked buckets
    are FREED — the operation that, with several processes on one GPU, made later imports map the
    wrong allocation.  The guarantee under test: a job either gathers exactly the all-gather's
    bucket or its set-up is refused on every rank by the token check (RCCL then); never a wrong
    bucket.  Parked bytes stay within the cap throughout."""
    from flearn_amd import dist as fd

    cuda = torch.device("cuda", 0)
    fd.shutdown_push()
    refused = 0
    cols0 = world * 65536
    for it in range(10):
        cols = (int(cols0 * 1.25 ** it) // (world * 64)) * world * 64
        src = torch.arange(cols // world, dtype=torch.float32, device=cuda) + 1e5 * rank + it
        want = torch.empty(cols, dtype=torch.float32, device=cuda)
        fd.all_gather_into(want, src)
        try:
            pg = fd.PushGather(None, None, mode="kernel" if it % 2 == 0 else "dma", cols=cols, device=cuda)
        except RuntimeError as e:  # refused together: every rank raised, nothing stays mapped
            assert "tokens" in str(e) or "could not map" in str(e), e
            refused += 1
            continue
        pg.gather(src, rank * (cols // world))
        torch.cuda.synchronize()
        assert torch.equal(pg.full, want), (rank, it)
        pg.close()
        assert fd.DeviceBuffer.parked_bytes(cuda) <= fd.DeviceBuffer.park_cap(cuda)
    fd.shutdown_push()
    assert fd.DeviceBuffer.parked_bytes(cuda) <= fd.DeviceBuffer.park_cap(cuda)
    assert fd.DeviceBuffer.trimmed()["buckets"] > 0  # the cap did free exported buckets
    print(f"[rank {rank}] growth: {fd.DeviceBuffer.trimmed()} trimmed, {refused} set-ups refused", flush=True)


CASES = {f.__name__[5:]: f for f in (case_avg_fixtures, case_setup_strategy, case_fused_rounds,
                                      case_first_round_adopt, case_empty_ranks, case_dyn, case_sharded_reducer,
                                      case_sharded_reducer_push, case_sharded_reducer_push_dma,
                                      case_push_lifecycle, case_push_growth_trim)}


def rank_main(rank, world, port, names):
    """torch.multiprocessing entry point (a fresh interpreter per rank: spawn context)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(0)  # every rank shares the one GPU of the box
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        for name in names:
            try:
                CASES[name](rank, world)
            except BaseException:
                traceback.print_exc()
                raise
            dist.barrier()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
