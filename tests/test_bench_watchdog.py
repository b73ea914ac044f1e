"""bench.py's held line and watchdog on CPU (no GPU needed): a phase that hangs after the line was
secured still ends the process at its budget with exactly one JSON line, annotated with what
overran, and the held exit code (tests/test_gpu_bench.py rehearses the same with a stalled push
set-up on the GPU box); a process ended by a signal meanwhile (a GPU fault's abort, torchrun's
SIGTERM after another rank died) still prints the line, marked with the phase (tools/lastwords.c)."""
import json
import signal
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent

PROG = r"""
import sys, time
sys.path.insert(0, {repo!r})
import bench
held = bench.HeldLine(0)
held.set({{"metric": "m", "value": 1.5, "multi_gpu": {{}}}}, {code})
dog = bench.Watchdog(held, 0)
def note(ln):
    ln["multi_gpu"]["phases"] = {{"push": {{"status": "timed_out"}}}}
dog.arm(1.0, "push phase", note)
time.sleep(60)  # the hang
print("not reached", flush=True)
"""


def _run(code):
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", PROG.format(repo=str(REPO), code=code)], capture_output=True, text=True,
                       timeout=120)
    return p, time.monotonic() - t0


def test_watchdog_prints_the_held_line_once_and_exits():
    p, took = _run(0)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 1.5 and d["multi_gpu"]["phases"]["push"]["status"] == "timed_out"
    assert "WATCHDOG: push phase overran" in p.stderr
    assert took < 40


def test_watchdog_keeps_the_held_exit_code():
    p, _ = _run(3)
    assert p.returncode == 3
    assert len([ln for ln in p.stdout.splitlines() if ln.strip()]) == 1


def test_held_line_prints_once():
    sys.path.insert(0, str(REPO))
    import bench

    h = bench.HeldLine(1)  # not rank 0: never prints
    h.set({"v": 1}, 0)
    assert h.emit() is False
    h0 = bench.HeldLine(0)
    assert h0.emit() is False  # nothing held yet


LW_PROG = r"""
import os, signal, sys, time
sys.path.insert(0, {repo!r})
import bench
held = bench.HeldLine(0, lastwords=True)
assert held._lw is not None
held.set({{"metric": "m", "value": 2.5, "multi_gpu": {{}}}}, 0)
dog = bench.Watchdog(held, 0)
dog.arm(60.0, "push phase")
held.line["multi_gpu"]["phases"] = {{"push": {{"status": "started"}}}}
held.guard("push phase")
if {emit}:
    held.emit()
sys.stdout.flush()
{end}
time.sleep(30)
print("not reached", flush=True)
"""


def _lastwords_lib():
    lib = REPO / "tools" / "liblastwords.so"
    if not lib.exists():
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", str(REPO / "tools" / "lastwords.c"), "-o", str(lib)], check=True)


def _lw_run(end, emit=False):
    _lastwords_lib()
    return subprocess.run([sys.executable, "-c", LW_PROG.format(repo=str(REPO), end=end, emit=emit)],
                          capture_output=True, text=True, timeout=120)


def test_signal_prints_the_held_line_marked_with_its_phase():
    for end, sig in (("os.kill(os.getpid(), signal.SIGTERM)", signal.SIGTERM), ("os.abort()", signal.SIGABRT)):
        p = _lw_run(end)
        assert p.returncode == -sig, (p.returncode, p.stderr[-2000:])  # the process still ends by the signal
        lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
        assert len(lines) == 1 and "not reached" not in p.stdout, p.stdout
        d = json.loads(lines[0])
        assert d["value"] == 2.5 and d["multi_gpu"]["phases"]["push"]["status"] == "started"
        assert d["ended_by_signal"]["during"] == "push phase"


def test_signal_after_the_line_was_printed_adds_nothing():
    p = _lw_run("os.kill(os.getpid(), signal.SIGTERM)", emit=True)
    assert p.returncode == -signal.SIGTERM
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and "ended_by_signal" not in lines[0]


def _outcome_worker(rank, world, init, stuck, out):
    import torch.distributed as dist

    sys.path.insert(0, str(REPO))
    import bench

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        if stuck and rank == 1:  # a rank still inside the phase: it never posts its outcome
            time.sleep(4.0)
            return
        got = bench._agree_outcomes("adopted" if rank == 0 else "failed_self_check", rank, world, 2.0)
        Path(out).with_suffix(f".{rank}").write_text(json.dumps(got))
    finally:
        if not (stuck and rank == 1):
            time.sleep(2.5)  # let the stuck peer's sleep end before the group goes away
        dist.destroy_process_group()


def test_push_phase_outcomes_are_agreed_through_the_store(tmp_path):
    """bench._agree_outcomes: every rank's push-phase outcome through the process
    group's store, no collective — all ranks see all outcomes; a rank that never posts (stuck in
    a collective of the phase) makes the others' wait time out (None) instead of pairing with an
    unrelated collective."""
    import os

    import torch.multiprocessing as mp

    for stuck in (False, True):
        init = "file://" + os.path.join(str(tmp_path), f"pg_{stuck}")
        out = tmp_path / f"out_{stuck}"
        mp.spawn(_outcome_worker, args=(2, init, stuck, str(out)), nprocs=2, join=True)
        if stuck:
            assert json.loads(out.with_suffix(".0").read_text()) is None
        else:
            for r in (0, 1):
                assert json.loads(out.with_suffix(f".{r}").read_text()) == ["adopted", "failed_self_check"]
