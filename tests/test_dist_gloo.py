"""Multi-rank path on CPU: world_size-2 gloo runs of flearn_amd.dist (element-range shards,
block-cyclic stripes, all-gather reassembly, sharded optimizer state).  On the GPU each rank's
reduce_fn is the HIP kernel; here the C oracle stands in as the per-shard reducer so the test
checks the sharding + exchange logic: the reassembled model must equal the unsharded reduce
bit for bit."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SEED = 77


def _free_port():
    """A fresh file:// rendezvous (no TCP port to race for when test workers run in parallel)."""
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_gloo_"), "pg")


def _worker(rank, world, port, n, p, stripes, op, weights=None):
    import oracle
    from flearn_amd.dist import ShardedReducer, ShardPlan

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        if weights == "model":  # bench's default: widths from the two-stage pipeline model
            from flearn_amd.dist import StripeModel, plan_stripes

            model = StripeModel(1e-6, 5e-9, 2e-6, 1e-8)  # gather-bound: small stripes first
            plan = ShardPlan.from_widths(p, world, rank, plan_stripes(-(-p // world), model))
            assert plan.stripes == stripes and plan.widths[0] < plan.widths[-1], plan.widths
        elif weights == "tail":  # model-planned stripes + a replicated tail (plan_shards)
            from flearn_amd.dist import StripeModel, plan_shards

            widths, rep = plan_shards(p, world, StripeModel(1e-6, 2e-9, 2e-6, 1e-8))
            plan = ShardPlan.from_widths(p, world, rank, widths, rep=rep)
            assert plan.rep > 0 and plan.full_cols == p, (plan.widths, plan.rep)
        else:
            plan = ShardPlan.make(p, world, rank, stripes, weights=weights)
        local = np.zeros((n, plan.local_cols), np.float32)
        prev = np.zeros(plan.local_cols, np.float32)
        for lo, g0, width in plan.segments():
            width = max(0, min(width, p - g0))  # the last slices may be padding
            if width:
                local[:, lo : lo + width] = oracle.fill_uniform(n, width, SEED, col0=g0)
                prev[lo : lo + width] = oracle.fill_uniform(1, width, 1, col0=g0)[0]
        w = np.linspace(0.5, 1.5, n).astype(np.float32)
        denom = float(np.sum([float(x) for x in w]))
        v = np.zeros(plan.local_cols)
        prev_t = torch.from_numpy(prev)

        def fn(col_begin, ncols, out_slice):
            g = oracle.c_reduce(oracle.MODE_W32_DIV64, local[:, col_begin : col_begin + ncols], w, denom)
            if op != "mean":
                vs = v[col_begin : col_begin + ncols].copy()
                g = oracle.c_update(op, g, prev[col_begin : col_begin + ncols].copy(), vs)
                v[col_begin : col_begin + ncols] = vs
            out_slice.copy_(torch.from_numpy(g.astype(np.float32)))

        red = ShardedReducer(plan, fn, "cpu", local_out=prev_t if op != "mean" else None)
        full = red.step().numpy().copy()
        assert full.shape == (p,)
        # every rank holds the same, complete model
        ref = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, SEED), w, denom)
        if op != "mean":
            ref = oracle.c_update(op, ref, oracle.fill_uniform(1, p, 1)[0], np.zeros(p))
        np.testing.assert_array_equal(full.view(np.uint32), ref.astype(np.float32).view(np.uint32))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("p,stripes,op,weights", [(44_426, 4, "mean", None), (100_003, 3, "avgm", None),
                                                  (5_000, 1, "adagrad", None), (63, 2, "mean", None),
                                                  (100_003, 2, "avgm", (3, 1)), (44_426, 3, "mean", (1, 2, 1))])
def test_sharded_reduce_two_ranks(p, stripes, op, weights):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mp.spawn(_worker, args=(2, _free_port(), 7, p, stripes, op, weights), nprocs=2, join=True)


@pytest.mark.parametrize("world,op", [(2, "mean"), (2, "avgm"), (4, "adagrad"), (8, "mean")])
def test_sharded_reduce_replicated_tail(world, op):
    """Stripes + a replicated tail (plan_shards on a gather-bound model): every rank reduces the
    last columns itself — straight into the global bucket for the plain mean, through its local
    state for a fused optimizer — and the reassembled model is still the unsharded reduce."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mp.spawn(_worker, args=(world, _free_port(), 5, 90_001, None, op, "tail"), nprocs=world, join=True)


def test_sharded_reduce_four_ranks():
    """More ranks than the GPU box's CI can rehearse on one card: world 4, uneven stripes."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mp.spawn(_worker, args=(4, _free_port(), 5, 70_001, 2, "mean", (3, 1)), nprocs=4, join=True)


def test_sharded_reduce_eight_ranks():
    """The driver's scaling run at G=8, fused Adagrad, a width whose last rank's slices are
    partly padding: 3:1 stripes, and the model-planned stripes bench.py uses by default (with
    coefficients scaled so this small bucket gets several stripes, small ones first)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mp.spawn(_worker, args=(8, _free_port(), 3, 40_001, 2, "adagrad", (3, 1)), nprocs=8, join=True)
    mp.spawn(_worker, args=(8, _free_port(), 3, 40_001, 3, "adagrad", "model"), nprocs=8, join=True)


def _gather_worker(rank, world, port, stride, dtype):
    from flearn_amd.bucket import rank_width
    from flearn_amd.dist import gather_columns

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        w = rank_width(stride, world)
        assert w % 64 == 0 and w * world >= stride
        c0 = min(rank * w, stride)
        c1 = min(c0 + w, stride)
        full_ref = torch.arange(stride, dtype=dtype) * 0.5 - 7
        local = full_ref[c0:c1].clone()  # possibly short or empty on the last ranks
        got = gather_columns(local, w, stride, None)
        assert got.dtype == dtype and got.shape == (stride,)
        assert torch.equal(got, full_ref)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,stride,dtype", [(2, 44_480, torch.float64), (3, 64 * 7, torch.float32),
                                                (4, 64, torch.float32)])
def test_strategy_group_column_gather(world, stride, dtype):
    """Aggregator(group=...) (the Strategy-level RCCL path behind Server.py:140): each rank's
    equal ALIGN-aligned column range, short or empty on the last ranks, reassembled by one
    all-gather into the whole bucket on every rank."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mp.spawn(_gather_worker, args=(world, _free_port(), stride, dtype), nprocs=world, join=True)
