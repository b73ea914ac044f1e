"""flearn_amd.verify — the self-check bench.py --gpus N runs on the reassembled global model.

On CPU: the window placement, and world-size 2/4 gloo runs of ShardedReducer (the C oracle as the
per-shard reducer, as in test_dist_gloo.py) whose check passes on a correct gather and FAILS —
with the process exiting EXIT_MISMATCH, as bench.py does — when the gather lands its slices
ALIGN columns late or a rank's v_t slice is corrupted at an edge."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flearn_amd import verify
from flearn_amd.dist import ALIGN, ShardPlan

SEED = 2024


def _rendezvous():
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_verify_"), "pg")


@pytest.mark.parametrize("n_cols,world,stripes,weights,rep", [
    (25_610_152, 8, 2, (3, 1), 0), (11_699_112, 2, 3, None, 0), (86_567_656, 4, 1, None, 0),
    (44_426, 8, 2, None, 0), (1_000_003, 2, 2, None, 100_003), (5_000, 3, 1, None, 0), (63, 2, 1, None, 0)])
def test_windows_cover_every_boundary(n_cols, world, stripes, weights, rep):
    if rep:
        units = (n_cols - rep) // (world * ALIGN)
        per = units * ALIGN // stripes // ALIGN * ALIGN
        widths = [per] * (stripes - 1) + [units * ALIGN - per * (stripes - 1)]
        rep = n_cols - world * units * ALIGN
        plans = [ShardPlan.from_widths(n_cols, world, r, widths, rep=rep) for r in range(world)]
    else:
        plans = [ShardPlan.make(n_cols, world, r, stripes, weights=weights) for r in range(world)]
    wins = verify.boundary_windows(plans[0])
    w = min(4096, n_cols)
    assert all(0 <= g0 and g0 + ww <= n_cols and ww == w for g0, ww in wins)
    if n_cols >= 64 * w:
        assert len(wins) >= 64
    starts = [g0 for g0, _ in wins]

    def covered(c):  # a window holds columns on both sides of boundary c (or touches the edge)
        c = min(max(c, 0), n_cols)
        return any(g0 < c < g0 + w or (c in (0, n_cols) and (g0 == 0 or g0 + w == n_cols)) for g0 in starts)

    p = plans[0]
    for c in range(p.stripes):
        for r in range(world):
            g = p.global_begin(c, r)
            if g < n_cols:
                assert covered(g), (c, r, g)
    if p.rep:
        assert covered(p.padded) and covered(n_cols)
    # every rank's own segment edges for its state slices
    for pr in plans:
        segs = verify.segment_windows(pr)
        for lo, g0, seg in pr.segments():
            real = max(0, min(seg, n_cols - g0))
            if real:
                assert any(l == lo for l, _, _ in segs) and any(l + ww == lo + real for l, _, ww in segs)


def test_bits_equal_is_bitwise():
    a = torch.tensor([0.0, 1.0, float("nan")])
    assert verify.bits_equal(a, a.clone())
    assert not verify.bits_equal(a, torch.tensor([-0.0, 1.0, float("nan")]))
    assert not verify.bits_equal(a, a.double())


def _worker(rank, world, port, n, p, stripes, op, fault):
    import oracle
    from flearn_amd import dist as fa_dist
    from flearn_amd.dist import ShardedReducer

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    code = 0
    try:
        plan = ShardPlan.make(p, world, rank, stripes)
        local = np.zeros((n, plan.local_cols), np.float32)
        prev0 = np.zeros(plan.local_cols, np.float32)
        for lo, g0, width in plan.segments():
            width = max(0, min(width, p - g0))
            if width:
                local[:, lo : lo + width] = oracle.fill_uniform(n, width, SEED, col0=g0)
                prev0[lo : lo + width] = oracle.fill_uniform(1, width, 1, col0=g0)[0]
        w = np.ones(n, np.float32)
        denom = float(n)
        v = np.zeros(plan.local_cols)
        prev_t = torch.from_numpy(prev0.copy())

        def fn(col_begin, ncols, out_slice):
            g = oracle.c_reduce(oracle.MODE_W32_DIV64, local[:, col_begin : col_begin + ncols], w, denom)
            if op != "mean":
                vs = v[col_begin : col_begin + ncols].copy()
                g = oracle.c_update(op, g, prev_t.numpy()[col_begin : col_begin + ncols].copy(), vs)
                v[col_begin : col_begin + ncols] = vs
            out_slice.copy_(torch.from_numpy(g.astype(np.float32)))

        if fault == "gather_offset":  # what bench.py's FLEARN_BENCH_INJECT=gather_offset does
            real = fa_dist.all_gather_into

            def late(dst, src, group=None, async_op=False):
                real(dst, src, group=group)
                dst.copy_(torch.roll(dst, ALIGN))

            fa_dist.all_gather_into = late
        red = ShardedReducer(plan, fn, "cpu", local_out=prev_t if op != "mean" else None)
        full = red.step()
        if op != "mean":
            full = red.step()  # the second step from the initial state, as bench.py checks
        if fault == "state_edge" and rank == world - 1:
            lo, _, _ = plan.segments()[-1]
            v[lo] += 1.0

        def expect(g0, ww):
            x = oracle.fill_uniform(n, ww, SEED, col0=g0)
            g = oracle.c_reduce(oracle.MODE_W32_DIV64, x, w, denom)
            if op == "mean":
                return torch.from_numpy(g.astype(np.float32)), None
            pv = oracle.fill_uniform(1, ww, 1, col0=g0)[0]
            vv = np.zeros(ww)
            w1 = oracle.c_update(op, g, pv, vv).astype(np.float32)
            w2 = oracle.c_update(op, g, w1, vv).astype(np.float32)
            return torch.from_numpy(w2), torch.from_numpy(vv)

        res = verify.check_step(plan, full, expect, state=torch.from_numpy(v) if op != "mean" else None,
                                width=512, count=16)
        assert res["ranks_checked"] == world and res["windows"] >= 16
        if op != "mean":
            assert res["state_windows"] > 0
        if not res["verified"]:
            code = verify.EXIT_MISMATCH
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if code:
        raise SystemExit(code)


def _run(world, n, p, stripes, op, fault):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    ctx = mp.spawn(_worker, args=(world, _rendezvous(), n, p, stripes, op, fault), nprocs=world, join=False)
    try:
        while not ctx.join():
            pass
    except mp.ProcessExitedException as e:
        return e.exit_code
    except mp.ProcessRaisedException as e:
        if "SystemExit" in str(e):
            return verify.EXIT_MISMATCH
        raise
    return 0


@pytest.mark.parametrize("world,p,stripes,op", [(2, 50_003, 2, "mean"), (2, 30_001, 1, "avgm"),
                                                (4, 40_007, 2, "adagrad")])
def test_check_passes_on_a_correct_gather(world, p, stripes, op):
    assert _run(world, 5, p, stripes, op, None) == 0


@pytest.mark.parametrize("world,op", [(2, "mean"), (4, "adagrad")])
def test_wrong_gather_offset_fails_the_run(world, op):
    """A gather that lands every slice ALIGN columns late: the check catches it on every rank and
    the process exits non-zero."""
    assert _run(world, 5, 40_007, 2, op, "gather_offset") == verify.EXIT_MISMATCH


def test_corrupted_state_slice_edge_fails_the_run():
    """v_t is never gathered: each rank checks its own slice edges, and the verdict is shared."""
    assert _run(2, 5, 30_001, 2, "avgm", "state_edge") == verify.EXIT_MISMATCH


def test_local_model_windows_for_an_emulated_rank():
    """bench.py --emulate-world: one process holds rank 0's columns only (no gather); the model
    is checked on that rank's local segment windows, mapped to their global columns."""
    plan = ShardPlan.make(50_003, 4, 0, 2)
    glob = torch.arange(plan.full_cols + 4096, dtype=torch.float32)
    local = torch.zeros(plan.local_cols)
    for lo, g0, w in plan.segments():
        local[lo : lo + w] = glob[g0 : g0 + w]
    res = verify.check_step(plan, local, lambda g0, w: (glob[g0 : g0 + w], None), width=512, local_model=True)
    assert res["verified"] and res["windows"] == len(verify.segment_windows(plan, 512))
    local[plan.local_begin(1)] += 1
    assert not verify.check_step(plan, local, lambda g0, w: (glob[g0 : g0 + w], None), width=512,
                                 local_model=True)["verified"]
