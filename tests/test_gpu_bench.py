"""bench.py's multi-GPU path rehearsed on the one GPU of the box: 2 ranks launched the way the
driver launches them (python -m torch.distributed.run ... bench.py --gpus 2) that share cuda:0
and talk over gloo (FLEARN_BENCH_BACKEND=gloo; RCCL refuses two ranks on one device).  It runs
the calibration, the model-planned stripes, the strong job (`value`) and the weak job beside it,
and checks the JSON line's contract fields.  Timings of this rehearsal mean nothing (the gather
is host-staged); the driver's 8-GPU run measures RCCL over xGMI."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rehearse(config, extra=(), inject=None):
    env = dict(os.environ, FLEARN_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    if inject:
        env["FLEARN_BENCH_INJECT"] = inject
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "bench.py"), "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--config", config, *extra]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=str(REPO))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_bench_two_ranks_rehearsal(config, cuda):
    p = _rehearse(config)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert d["config"]["clients"] == 100  # the fixed problem
    mg = d["multi_gpu"]
    assert mg["calibration"]["measured_gather"] is True
    # the reduce / gather contention of this node, measured concurrently, is in the fitted model
    cal = mg["calibration"]
    assert cal["c_r"] >= 0 and cal["c_g"] >= 0 and cal["concurrent_reduce_us"] > 0
    # the one-shot push gather was set up (IPC-mapped peer buffers: here two processes on one
    # GPU), checked bit for bit against the all-gather, calibrated, and timed in the trials
    pc, pd = mg["push_calibration"], mg["push_dma_calibration"]
    for c in (pc, pd):
        assert c["available"] is True and c["checked_against_rccl"] is True and c["push_kernel_us"] > 0
    assert pc["grid"] in (4, 8, 16, 32, 64, 128, 256)
    assert set(pc["gather_us_by_grid"]) == {"4", "8", "16", "32", "64", "128", "256"}
    # the grid is chosen by the push-beside-reduce pair, not by the push alone
    pair = pc["pair_us_by_grid"]
    assert set(pair) == set(pc["gather_us_by_grid"]) and pair[str(pc["grid"])] <= 1.03 * min(pair.values()) + 1e-6
    assert {t["gather"] for t in mg["plan_trials"]} == {"rccl", "push", "push_dma"}
    rb = mg["push_receive_buckets"]  # parked receive buckets stay within the cap
    assert rb["parked_bytes"] <= rb["park_cap_bytes"] and rb["pool_bytes"] > 0
    used = {"rccl": cal, "push": pc, "push_dma": pd}[mg["gather"]]
    assert mg["model"]["c_r"] == used["c_r"] and mg["model"]["c_g"] == used["c_g"]
    # the serial plan (one stripe, no tail) is among the measured trials
    assert any(len(t["stripe_widths"]) == 1 and t["replicated_cols"] == 0 for t in mg["plan_trials"])
    # stripes (padded) or stripes + a replicated tail cover the bucket
    assert sum(mg["stripe_widths"]) * 2 + mg["replicated_cols"] >= d["config"]["params"]
    if mg["replicated_cols"]:
        assert sum(mg["stripe_widths"]) * 2 + mg["replicated_cols"] == d["config"]["params"]
    assert mg["per_rank_reduce_ms"] > 0 and mg["exposed_gather_ms"] >= 0
    # the plan is the fastest measured candidate of its gather; RCCL's job ran (and was verified)
    # first, and a push plan replaced it only if its own timed job was faster and verified
    trials = [t for t in mg["plan_trials"] if t["measured_ms"] is not None]  # None: a refused set-up
    assert trials
    best = min((t for t in trials if t["gather"] == mg["gather"]), key=lambda t: t["measured_ms"])
    assert (best["stripe_widths"], best["replicated_cols"]) == (mg["stripe_widths"], mg["replicated_cols"])
    ph = mg["phases"]
    assert ph["rccl"]["verified"] is True and ph["rccl"]["ms_per_step"] > 0
    assert ph["push"]["status"] in ("adopted", "slower", "slower_in_trials", "unavailable")
    assert (mg["gather"] != "rccl") == (ph["push"]["status"] == "adopted")
    if mg["gather"] != "rccl":
        assert d["ms_per_step"] < ph["rccl"]["ms_per_step"]
    assert d["weak"]["clients"] == 200 and d["weak"]["value"] > 0
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["frac"] > 0
    # the reassembled model was checked bit for bit on >= 64 boundary windows, on both ranks
    v = d["verify"]
    assert v["verified"] is True and v["windows"] >= 64 and v["ranks_checked"] == 2 and v["comparison"] == "bitwise"
    assert v["mismatched_windows"] == 0 and (v["state_windows"] > 0) == (config == "c3")
    assert mg["verified"] is True and mg["verified_windows"] == v["windows"]
    assert mg["world_size"] == 2 and mg["backend"].startswith("gloo") and mg["allgather_probe"]["per_link_gbs"] > 0
    assert mg["calibrated_per_link_gbs"] > 0
    # the single-process multi-GPU drop-in, rehearsed as devices=[cuda:0, cuda:0]
    lb = d["loopback_multi_gpu"]
    assert lb["verified"] is True and lb["devices"] == ["cuda:0", "cuda:0"] and lb["clients"] == 100
    for o in ("reference", "device"):
        assert lb[o]["verified"] is True and lb[o]["round_ms"] > 0 and lb[o]["pack_h2d_ms"] > 0
        assert len(lb[o]["h2d_gbs_per_gpu"]) == 2 and min(lb[o]["h2d_gbs_per_gpu"]) > 0


@pytest.mark.timeout(300)
def test_bench_push_gather_is_verified(cuda):
    """--gather push --stripes 3: every stripe reassembled by direct peer stores; the line says so
    and its self-check passes on both ranks."""
    for g in ("push", "push_dma"):
        p = _rehearse("c3", ("--no-weak", "--no-loopback", "--stripes", "3", "--gather", g))
        assert p.returncode == 0, p.stderr[-4000:]
        d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
        assert d["multi_gpu"]["gather"] == g and "push all-gather" in d["config"]["parallelism"]
        assert d["verify"]["verified"] is True and d["verify"]["ranks_checked"] == 2
        # every one of 20 more steps checked end to end (each sender's slice checksums vs each
        # receiver's bucket), not only the last one
        a = d["multi_gpu"]["push_audit"]
        assert a["verified"] is True and a["audited_steps"] == 20 and a["bad_steps_by_rank"] == [0, 0]
        assert d["multi_gpu"]["phases"]["push"]["audit_verified"] is True


@pytest.mark.timeout(300)
def test_bench_keeps_rccl_when_a_push_fails_its_check(cuda):
    """FLEARN_BENCH_INJECT=push_offset with --gather push: the pushed bucket fails the self-check,
    the line records it (`push_failed_self_check`) and keeps the RCCL job timed and verified
    before the push phase, so the run still ends verified."""
    p = _rehearse("c2", ("--no-weak", "--no-loopback", "--stripes", "2", "--gather", "push"), inject="push_offset")
    assert p.returncode == 0, p.stderr[-4000:]
    assert "gather failed its step audit: keeping the RCCL line" in p.stderr  # every step is off
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    mg = d["multi_gpu"]
    assert mg["gather"] == "rccl" and mg["push_failed_self_check"]["gather"] == "push"
    assert mg["push_failed_self_check"]["mismatched_windows"] > 0  # and the last step's windows
    assert mg["push_failed_self_check"]["audit"]["bad_steps_by_rank"] == [20, 20]
    assert mg["phases"]["push"]["status"] == "failed_self_check"
    assert d["verify"]["verified"] is True and "RCCL all-gather" in d["config"]["parallelism"]


@pytest.mark.timeout(300)
def test_bench_push_audit_catches_one_bad_middle_step(cuda):
    """FLEARN_BENCH_INJECT=push_skip_mid: rank 1 skips one push in ONE audited step (neither a
    timed step nor the step verify_job bit-checks, which still passes): the step audit catches
    the stale slice on every receiver, the line keeps the RCCL job (bench.push_audit)."""
    p = _rehearse("c3", ("--no-weak", "--no-loopback", "--stripes", "2", "--gather", "push"), inject="push_skip_mid")
    assert p.returncode == 0, p.stderr[-4000:]
    assert "INJECTED: skipping one push" in p.stderr
    assert "failed its step audit: keeping the RCCL line" in p.stderr
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    mg = d["multi_gpu"]
    assert mg["gather"] == "rccl" and mg["phases"]["push"]["status"] == "failed_self_check"
    f = mg["push_failed_self_check"]
    assert f["gather"] == "push" and f["mismatched_windows"] == 0  # the last step's windows pass
    a = f["audit"]
    assert a["verified"] is False and a["bad_steps_by_rank"] == [1, 1]
    assert all(x["step"] == 7 for x in a["first_bad"]) and a["first_bad"][0]["slices"] == [{"sender": 1, "stripe": 0}]
    assert d["verify"]["verified"] is True and "RCCL all-gather" in d["config"]["parallelism"]


@pytest.mark.timeout(300)
def test_bench_line_survives_a_stalled_push_setup(cuda):
    """FLEARN_BENCH_INJECT=push_stall: rank 1 never returns from the push gather's set-up (rank 0
    then waits in its collective).  The RCCL job was timed and verified before the push phase;
    the watchdog ends both ranks at the phase budget and rank 0 prints that line, exit 0, long
    before the driver's limit."""
    import time

    t0 = time.monotonic()
    p = _rehearse("c2", ("--no-weak", "--no-loopback", "--push-budget-s", "25"), inject="push_stall")
    took = time.monotonic() - t0
    assert p.returncode == 0, p.stderr[-4000:]
    assert "INJECTED: stalling in the push set-up" in p.stderr and "WATCHDOG: push phase overran" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    mg = d["multi_gpu"]
    assert mg["gather"] == "rccl" and mg["phases"]["push"]["status"] == "timed_out"
    assert mg["phases"]["rccl"]["verified"] is True and d["verify"]["verified"] is True and d["value"] > 0
    assert took < 240, took


@pytest.mark.timeout(300)
def test_bench_line_survives_a_rank_dying_in_the_push_phase(cuda):
    """FLEARN_BENCH_INJECT=push_crash: rank 1 dies in the push gather's set-up (os._exit, standing
    in for a GPU fault's abort).  Rank 0 is then either ended by torchrun's SIGTERM (tools/lastwords.c
    writes the held line from the signal handler) or sees its next collective raise (bench's
    _end_with_held_line): either way exactly one line, the verified RCCL job, marked with the phase."""
    p = _rehearse("c2", ("--no-weak", "--no-loopback"), inject="push_crash")
    assert p.returncode != 0  # torchrun reports the dead rank
    assert "INJECTED: dying in the push set-up" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr[-3000:])
    d = json.loads(lines[0])
    mg = d["multi_gpu"]
    assert mg["gather"] == "rccl" and mg["phases"]["rccl"]["verified"] is True and d["verify"]["verified"] is True
    ended = d.get("ended_by_signal") or d.get("ended_by_error")
    assert ended is not None and ended["during"] == "push phase", d


@pytest.mark.timeout(300)
def test_bench_fails_on_a_misplaced_gather(cuda):
    """FLEARN_BENCH_INJECT=gather_offset: every gathered slice lands ALIGN columns late; the
    self-check must flag it in the line and the run must exit non-zero (EXIT_MISMATCH)."""
    from flearn_amd import verify

    p = _rehearse("c2", ("--no-weak", "--no-loopback", "--stripes", "2"), inject="gather_offset")
    assert p.returncode != 0, p.stdout[-2000:]
    assert "SELF-CHECK FAILED" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["verify"]["verified"] is False and d["verify"]["mismatched_windows"] > 0
    # a failed RCCL line is never replaced by a later (push) phase
    assert d["multi_gpu"]["gather"] == "rccl" and d["multi_gpu"]["phases"]["push"]["status"].startswith("skipped")
    assert "exitcode  : 3" in p.stderr and verify.EXIT_MISMATCH == 3  # each rank's status (torchrun exits 1)


def test_single_gpu_line_is_verified(cuda):
    """The default N=1 line checks its own output too (one launch, no gather)."""
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "3", "--warmup", "1", "--config", "c3",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=280, cwd=str(REPO))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["verify"]["verified"] is True and d["verify"]["windows"] >= 64 and d["verify"]["state_windows"] >= 2


@pytest.mark.timeout(300)
@pytest.mark.parametrize("push", [True, "dma"])
def test_push_audit_with_a_replicated_tail(push, cuda, tmp_path, monkeypatch):
    """bench.push_audit on a plan with a replicated tail (the tail is reduced, not pushed: the
    audit checks the stripes only), a 1-rank RCCL group: 20 clean steps verify; one push skipped
    in the 5th audited step is caught on that step alone."""
    import types

    import torch
    import torch.distributed as dist

    sys.path.insert(0, str(REPO))
    import bench
    from flearn_amd import _native as na
    from flearn_amd import aggregator as agg
    from flearn_amd import dist as fd
    from flearn_amd.dist import PingPong, ShardedReducer, ShardPlan, hip_reduce_fn

    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1, device_id=cuda)
        created = True
    try:
        n, p = 5, 300_032
        plan = ShardPlan.from_widths(p, 1, 0, (64_000, 128_000), rep=p - 192_000)
        stack = torch.empty((n, plan.local_stride), dtype=torch.float32, device=cuda)
        for lo, g0, width in plan.segments():
            agg.fill_uniform(stack[:, lo:], seed=9, col_begin=g0, n_cols=width)
        prev = torch.empty((1, plan.local_stride), dtype=torch.float32, device=cuda)
        agg.fill_uniform(prev, seed=4)
        state = PingPong(prev[0], torch.zeros(plan.local_stride, dtype=torch.float64, device=cuda))
        w = torch.ones(n, dtype=torch.float32, device=cuda)
        fn = hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n), op=na.OP_BY_NAME["avgm"], state=state)
        red = ShardedReducer(plan, fn, cuda, gather=True, state=state, push=push)
        job = types.SimpleNamespace(red=red, plan=plan)
        a = bench.push_audit(job, 1, cuda)
        assert a["verified"] is True and a["audited_steps"] == 20 and a["bad_steps_by_rank"] == [0]
        real_push, count = fd.PushGather.push, {"n": 0}

        def skip_one(self, src, off):
            count["n"] += 1
            if count["n"] == 2 * 4 + 2:  # the 5th step's second stripe
                return None
            return real_push(self, src, off)

        monkeypatch.setattr(fd.PushGather, "push", skip_one)
        a = bench.push_audit(job, 1, cuda)
        assert a["verified"] is False and a["bad_steps_by_rank"] == [1]
        assert a["first_bad"] == [{"step": 4, "slices": [{"sender": 0, "stripe": 1}]}]
        monkeypatch.setattr(fd.PushGather, "push", real_push)
        red.release()
        fd.shutdown_push()
    finally:
        if created:
            dist.destroy_process_group()
