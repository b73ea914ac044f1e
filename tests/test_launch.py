"""bench.py's one-process-per-GPU launcher (flearn_amd/launch.py) on CPU.

`python bench.py --gpus N` with no launcher env must start N ranks itself, fail loudly when the
node shows fewer GPUs, and never downgrade to a 1-rank measurement."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from flearn_amd import launch

REPO = Path(__file__).resolve().parent.parent
PY = sys.executable


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_two_rank_rehearsal_through_the_launcher():
    p = subprocess.run([PY, str(REPO / "tests" / "launch_rehearsal.py"), "2"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line == {"n_gpus": 2, "bit_exact": True}


def test_failing_rank_fails_the_parent():
    p = subprocess.run([PY, str(REPO / "tests" / "launch_rehearsal.py"), "2", "1"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0


def test_bench_refuses_more_gpus_than_visible():
    """This container shows 0 GPUs (a 1-GPU box shows 1): --gpus 2 must exit non-zero before any
    HIP call instead of running one rank."""
    p = subprocess.run([PY, str(REPO / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "not downgrading" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_a_mismatched_launcher_world():
    p = subprocess.run([PY, str(REPO / "bench.py"), "--gpus", "1"], env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def test_ensure_ranks_contract(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert launch.ensure_ranks(1, "x.py", [], device_count=lambda: 0) is None  # single rank: run here
    with pytest.raises(launch.LaunchError, match="not downgrading"):
        launch.ensure_ranks(8, "x.py", [], device_count=lambda: 1)
    with pytest.raises(launch.LaunchError):
        launch.ensure_ranks(0, "x.py", [])
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert launch.ensure_ranks(4, "x.py", []) is None  # already a rank of the right world
    with pytest.raises(launch.LaunchError, match="WORLD_SIZE=4"):
        launch.ensure_ranks(8, "x.py", [])
    cmd = launch.torchrun_cmd(8, "bench.py", ["--gpus", "8"], 29500)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
