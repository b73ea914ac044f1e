"""Build libflearn_amd.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent
SOURCES = [HERE / "csrc" / "fa_reduce.hip"]
HOST_SOURCES = [HERE / "csrc" / "fa_wire.cpp"]  # plain host C++ (g++), linked into the same .so
DEPS = [HERE / "csrc" / "fa_device.hpp"]
HEADERS = [REPO / "include" / "flearn_amd.h"]
OUT = HERE / "lib" / "libflearn_amd.so"
PYHOST_SOURCE = HERE / "csrc" / "fa_pyhost.c"  # Python-object pack helper (ctypes.PyDLL), not C ABI
PYHOST_OUT = HERE / "lib" / "libfa_pyhost.so"
ARCH = os.environ.get("FLEARN_AMD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found")


def build_pyhost(force: bool = False, verbose: bool = False) -> Path:
    """libfa_pyhost.so: gcc against this interpreter's and numpy's headers; Python and numpy
    symbols stay undefined / are imported at first use from the interpreter that loads it."""
    import sysconfig

    import numpy

    newest = max(PYHOST_SOURCE.stat().st_mtime, Path(__file__).stat().st_mtime)
    if PYHOST_OUT.exists() and not force and PYHOST_OUT.stat().st_mtime >= newest:
        return PYHOST_OUT
    PYHOST_OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = PYHOST_OUT.with_suffix(".so.tmp")
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-pthread", "-Wall", "-Werror",
           f"-I{sysconfig.get_paths()['include']}", f"-I{numpy.get_include()}", str(PYHOST_SOURCE), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    tmp.replace(PYHOST_OUT)
    return PYHOST_OUT


TORCHMETA_SOURCE = HERE / "csrc" / "fa_torchmeta.cpp"  # tensor-metadata walks (ctypes.PyDLL), not C ABI
TORCHMETA_OUT = HERE / "lib" / "libfa_torchmeta.so"
TORCHMETA_STAMP = HERE / "lib" / "libfa_torchmeta.stamp"  # sidecar: the stamp the .so was built with


def torch_stamp() -> str:
    """What libfa_torchmeta.so's TensorImpl reads depend on: the torch build and its C++ ABI."""
    import torch

    return f"{torch.__version__}|cxx11abi={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"


def read_torchmeta_stamp(path: Path = None):
    """The stamp compiled into a built libfa_torchmeta.so (fa_tm_stamp()), or None."""
    import ctypes

    try:
        L = ctypes.PyDLL(str(path or TORCHMETA_OUT))
        fn = L.fa_tm_stamp
    except (OSError, AttributeError):
        return None
    fn.restype = ctypes.c_char_p
    return fn().decode()


def build_torchmeta(force: bool = False, verbose: bool = False):
    """libfa_torchmeta.so: g++ against this torch's headers, linked to its libtorch_python /
    libtorch / libc10 (rpath: the same image on the GPU box).  The torch version and C++ ABI
    flag are compiled in (fa_tm_stamp); a library stamped for another torch is rebuilt here and
    refused by _native.load_torchmeta.  Best effort: the library only speeds up checks the
    Python side can also do, so a failed build removes it and the package works without it."""
    import sysconfig

    import torch
    from torch.utils.cpp_extension import include_paths

    stamp = torch_stamp()
    newest = max(TORCHMETA_SOURCE.stat().st_mtime, Path(__file__).stat().st_mtime)
    # the up-to-date check reads the sidecar stamp file, never the library itself: dlopening the
    # old .so here would leave glibc's handle cached in this process, and a later load of the
    # rebuilt file would get the stale one back (load_torchmeta then reads the old stamp)
    side = TORCHMETA_STAMP
    if (TORCHMETA_OUT.exists() and not force and TORCHMETA_OUT.stat().st_mtime >= newest
            and side.exists() and side.read_text() == stamp):
        return TORCHMETA_OUT
    TORCHMETA_OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = TORCHMETA_OUT.with_suffix(".so.tmp")
    tlib = Path(torch.__file__).resolve().parent / "lib"
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           f'-DFA_TM_STAMP="{stamp}"',
           f"-I{sysconfig.get_paths()['include']}"] + [f"-I{p}" for p in include_paths()] + [
           str(TORCHMETA_SOURCE), f"-L{tlib}", "-ltorch_python", "-ltorch", "-lc10",
           f"-Wl,-rpath,{tlib}", "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd))
    try:
        subprocess.run(cmd, check=True)
    except (subprocess.CalledProcessError, OSError) as e:
        print(f"[flearn_amd] libfa_torchmeta.so not built ({e}); device uploads use the Python metadata path")
        TORCHMETA_OUT.unlink(missing_ok=True)
        side.unlink(missing_ok=True)
        tmp.unlink(missing_ok=True)
        return None
    tmp.replace(TORCHMETA_OUT)
    side.write_text(stamp)
    return TORCHMETA_OUT


def build_native(force: bool = False, verbose: bool = False) -> Path:
    build_pyhost(force, verbose)
    build_torchmeta(force, verbose)
    newest = max(p.stat().st_mtime for p in SOURCES + HOST_SOURCES + DEPS + HEADERS + [Path(__file__)])
    if OUT.exists() and not force and OUT.stat().st_mtime >= newest:
        return OUT
    OUT.parent.mkdir(parents=True, exist_ok=True)
    tmp = OUT.with_suffix(".so.tmp")
    objs = []
    for src in HOST_SOURCES:
        obj = OUT.parent / (src.stem + ".o")
        hcmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall",
                f"-I{REPO / 'include'}", "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(hcmd))
        subprocess.run(hcmd, check=True)
        objs.append(str(obj))
    dev_objs = []
    for src in SOURCES:  # device code: compile, then link with the host objects
        obj = OUT.parent / (src.stem + ".o")
        cmd = [
            hipcc(),
            f"--offload-arch={ARCH}",
            "-O3",
            "-std=c++17",
            "-fPIC",
            "-ffp-contract=off",  # bit-parity: no fused multiply-add anywhere in the reduce
            "-Wall",
            f"-I{REPO / 'include'}",
            "-c",
            str(src),
            "-o",
            str(obj),
        ]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        dev_objs.append(str(obj))
    link = [hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", "-pthread", "-o", str(tmp), *dev_objs, *objs]
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    tmp.replace(OUT)
    return OUT


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
