"""Build libflearn_amd.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent
SOURCES = [HERE / "csrc" / "fa_reduce.hip"]
DEPS = [HERE / "csrc" / "fa_device.hpp"]
HEADERS = [REPO / "include" / "flearn_amd.h"]
OUT = HERE / "lib" / "libflearn_amd.so"
ARCH = os.environ.get("FLEARN_AMD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found")


def build_native(force: bool = False, verbose: bool = False) -> Path:
    newest = max(p.stat().st_mtime for p in SOURCES + DEPS + HEADERS + [Path(__file__)])
    if OUT.exists() and not force and OUT.stat().st_mtime >= newest:
        return OUT
    OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = OUT.with_suffix(".so.tmp")
    cmd = [
        hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-ffp-contract=off",  # bit-parity: no fused multiply-add anywhere in the reduce
        "-Wall",
        f"-I{REPO / 'include'}",
        "-o",
        str(tmp),
        *map(str, SOURCES),
    ]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    tmp.replace(OUT)
    return OUT


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
