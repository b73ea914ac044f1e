"""One process per GPU: the launcher behind `python bench.py --gpus N` (and any script that wants
the same contract).

    rc = ensure_ranks(n, __file__, sys.argv[1:])
    if rc is not None:          # this was the parent: the N ranks have run and exited
        sys.exit(rc)
    # ... this process is one rank (RANK / LOCAL_RANK / WORLD_SIZE set) or the only one

The parent never touches the GPU: it counts devices with torch.cuda.device_count() (on this
image that reads the driver's device list without initialising HIP), then starts N fresh children
through `python -m torch.distributed.run` on 127.0.0.1 and waits for them.  It does not exec
(replacing a process that might have initialised the GPU takes the machine down on this pool),
never downgrades to fewer ranks, and returns non-zero if any child fails (torch.distributed.run
tears the other ranks down and exits with the failure).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys


class LaunchError(SystemExit):
    """Raised (exit status 2) when the requested ranks cannot be started as asked."""

    def __init__(self, msg: str):
        super().__init__(msg)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_count() -> int:
    import torch

    return torch.cuda.device_count()


def rank_env() -> tuple[int, int, int] | None:
    """(rank, local_rank, world) when this process was started as a rank, else None."""
    if "WORLD_SIZE" not in os.environ:
        return None
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ["WORLD_SIZE"]))


def torchrun_cmd(nproc: int, script: str, argv, port: int) -> list[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(script), *argv]


def ensure_ranks(nproc: int, script: str, argv, device_count=_gpu_count, timeout: float | None = None):
    """Make `nproc` ranks run `script argv`.

    Returns None when the caller should proceed as a rank: nproc == 1 with no launcher env, or the
    launcher env already names a world of exactly nproc.  Otherwise spawns the ranks, waits and
    returns their exit status (the caller exits with it).  Raises LaunchError when fewer than
    nproc devices are visible or the launcher env disagrees with nproc.
    """
    if nproc < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {nproc})")
    env_rank = rank_env()
    if env_rank is not None:
        world = env_rank[2]
        if world != nproc:
            raise LaunchError(f"--gpus {nproc} but the launcher started WORLD_SIZE={world} ranks; "
                              f"refusing to measure a different world than asked")
        return None
    if nproc == 1:
        return None
    ndev = device_count()
    if ndev < nproc:
        raise LaunchError(f"--gpus {nproc} needs {nproc} visible GPUs, this node shows {ndev}; "
                          f"not downgrading to fewer ranks")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = torchrun_cmd(nproc, script, argv, free_port())
    print(f"[launch] {nproc} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    # own process group: a timeout ends torchrun AND its ranks, nothing else
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        rc = p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        print(f"[launch] ranks did not finish within {timeout} s", file=sys.stderr, flush=True)
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        return 124
    if rc != 0:
        print(f"[launch] a rank failed: torch.distributed.run exited {rc}", file=sys.stderr, flush=True)
    return rc
