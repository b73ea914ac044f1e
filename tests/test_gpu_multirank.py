"""Multi-rank product paths with the real HIP kernels, on the one GPU of the box.

Each test starts `world` FRESH processes (torch.multiprocessing, spawn context: a new
interpreter per rank) that all use cuda:0 and form a gloo group — RCCL refuses two ranks on one
device.  The ranks run tests/multirank_worker.py's cases: the Strategy `group=` path (SPMD
server, the call behind flearn's Server.py:140: strategy.py:102-130, avgm.py:19-36,
opt.py:52-63, dyn.py:17-36) and bench.py's ShardedReducer, each rank checking its reassembled
model bit for bit against the reference's fixtures or the C oracle.  What this cannot cover on
one GPU: RCCL itself and xGMI (the driver's multi-GPU scaling run exercises those).
"""
import os
import socket
import time

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(world, names, deadline_s=240):
    from multirank_worker import rank_main

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    ctx = mp.start_processes(rank_main, args=(world, _free_port(), tuple(names)), nprocs=world, join=False,
                             start_method="spawn")
    t_end = time.monotonic() + deadline_s
    try:
        while not ctx.join(timeout=5):
            if time.monotonic() > t_end:
                raise TimeoutError(f"{world} ranks did not finish {names} within {deadline_s} s")
    finally:
        for p in ctx.processes:
            if p.is_alive():
                p.kill()
                p.join(10)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_strategy_group_fixtures(world, cuda):
    """AVG / BN / LG / LG_R(group=True) on every reduce fixture, output='float32', setup_strategy."""
    _run_ranks(world, ["avg_fixtures", "setup_strategy"])


@pytest.mark.timeout(300)
def test_strategy_group_fused_and_dyn(cuda):
    """AVGM / OPT(adagrad, yogi, adam)(server_side=True, group=True) 3-round fixtures incl. the
    gathered v_t, the first-round adopt path, and Dyn(h, group=True) 3 rounds (w, h, theta)."""
    _run_ranks(2, ["fused_rounds", "first_round_adopt", "dyn"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_strategy_group_empty_ranks(world, cuda):
    """A model narrower than the ranks: the last ranks own no columns and still join every
    collective (world 4 and 8: ranks with empty column ranges)."""
    _run_ranks(world, ["empty_ranks"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_reducer_hip_ranks(world, cuda):
    """bench.py's ShardedReducer with the HIP kernel on every rank: 1 stripe, 3:1 stripes and the
    model-planned stripes; mean, fused AVGM and Adagrad over two steps."""
    _run_ranks(world, ["sharded_reducer"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_reducer_push_gather(world, cuda):
    """ShardedReducer reassembled by PushGather: IPC-mapped peer buffers and one fa_push kernel
    per stripe, or one copy-engine copy per peer (here every "peer" is another process on the
    same GPU), bit-exact; world 8 = MAX_PUSH_RANKS, one MI355X node."""
    _run_ranks(world, ["sharded_reducer_push", "sharded_reducer_push_dma"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_push_setup_lifecycle(world, cuda):
    """export -> map -> unmap -> free -> re-export, 12 times for pool buckets (shutdown_push) and
    for explicitly registered DeviceBuffer buckets: every mapping holds its token, every gathered
    bucket is the all-gather's (the round-4 stale-import sequence)."""
    _run_ranks(world, ["push_lifecycle"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_push_buckets_trimmed_beyond_the_cap(world, cuda):
    """Receive buckets growing x1.25 per job: parked buckets beyond the cap are freed, and every
    later job either gathers exactly the all-gather's bucket or is refused on every rank by the
    token check — never a wrong bucket (flearn_amd.dist.DeviceBuffer)."""
    _run_ranks(world, ["push_growth_trim"])


@pytest.mark.timeout(300)
def test_push_order_under_the_products_streams(cuda, tmp_path):
    """tests/push_order_probe.py: eight processes replay the push test's sequence (mean and in-place
    Adagrad over four stripe plans, then an explicit registration) twice in both push forms, in the
    product's orders (the kernel push after a device-side wait on the reduce's stream, the
    copy-engine push in host order), every step's bucket bit-compared with the C oracle — 0 wrong
    rank-steps — with the product's streams AND with every push stream (the pusher's, each
    copy-engine leg's) forced onto high priority, so that none of them shares the compute stream's
    hardware queue.  The copy-engine push with device-side waits fails that second configuration
    (1-30% of rank-steps wrong)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    out = tmp_path / "order.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, str(Path(__file__).with_name("push_order_probe.py")), "--world", "8",
                        "--steps", "3", "--reps", "2", "--priorities", "product,high", "--out", str(out)],
                       env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    summary = json.loads(out.read_text())["summary"]
    assert set(summary) == {f"{pr}/{m}/{o}" for pr in ("product", "high")
                            for m, o in (("kernel", "-/mean"), ("kernel", "-/adagrad"), ("dma", "host/mean"),
                                         ("dma", "host/adagrad"))}
    for key, s in summary.items():
        assert s["steps"] == 8 * 4 * 2 * 3 and s["bad_steps"] == 0, (key, s["examples"])
