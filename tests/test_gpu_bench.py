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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_bench_two_ranks_rehearsal(config, cuda):
    env = dict(os.environ, FLEARN_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "bench.py"), "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--config", config]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=str(REPO))
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert d["config"]["clients"] == 100  # the fixed problem
    mg = d["multi_gpu"]
    assert mg["calibration"]["measured_gather"] is True
    # stripes (padded) or stripes + a replicated tail cover the bucket
    assert sum(mg["stripe_widths"]) * 2 + mg["replicated_cols"] >= d["config"]["params"]
    if mg["replicated_cols"]:
        assert sum(mg["stripe_widths"]) * 2 + mg["replicated_cols"] == d["config"]["params"]
    assert mg["per_rank_reduce_ms"] > 0 and mg["exposed_gather_ms"] >= 0
    # the plan is the fastest of the measured candidates
    trials = mg["plan_trials"]
    best = min(trials, key=lambda t: t["measured_ms"])
    assert (best["stripe_widths"], best["replicated_cols"]) == (mg["stripe_widths"], mg["replicated_cols"])
    assert d["weak"]["clients"] == 200 and d["weak"]["value"] > 0
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["frac"] > 0
