"""Host: the tensor-metadata walks (csrc/fa_torchmeta.cpp) agree with the Python comparisons they
replace (bucket._raw_signature / Packer.row_table), and fall back instead of raising."""
from pathlib import Path

import numpy as np
import pytest
import torch

from flearn_amd import _native as na
from flearn_amd import bucket


@pytest.fixture(scope="module")
def L():
    lib = na.load_torchmeta()
    if lib is None:
        pytest.skip("libfa_torchmeta.so not built")
    return lib


def _clients(n=6):
    rng = np.random.default_rng(1)
    out = []
    for _ in range(n):
        out.append({"a.weight": torch.from_numpy(rng.standard_normal((4, 3)).astype(np.float32)),
                    "a.bias": torch.zeros(3), "bn.num_batches_tracked": torch.tensor(5)})
    return out


def test_same_signature_matches_python(L):
    cs = _clients()
    keys = list(cs[0])
    assert L.fa_tm_same_signature(cs, tuple(keys)) == 1
    variants = {
        "shape": lambda c: c.__setitem__("a.bias", torch.zeros(4)),
        "dtype": lambda c: c.__setitem__("a.bias", torch.zeros(3, dtype=torch.float64)),
        "type": lambda c: c.__setitem__("a.bias", torch.nn.Parameter(torch.zeros(3))),
        "0-d vs 1-d": lambda c: c.__setitem__("bn.num_batches_tracked", torch.tensor([5])),
    }
    for what, change in variants.items():
        cs2 = [dict(c) for c in cs]
        change(cs2[4])
        py = all(bucket._raw_signature(c, keys) == bucket._raw_signature(cs2[0], keys) for c in cs2)
        assert not py, what
        assert L.fa_tm_same_signature(cs2, tuple(keys)) == 0, what


def test_same_signature_cannot_tell(L):
    cs = _clients()
    keys = tuple(cs[0])
    cs2 = [dict(c) for c in cs]
    cs2[2]["a.bias"] = np.zeros(3, np.float32)  # numpy value: the Python path decides
    assert L.fa_tm_same_signature(cs2, keys) == -1
    cs3 = [dict(c) for c in cs]
    del cs3[3]["a.bias"]  # missing key: no exception left set
    assert L.fa_tm_same_signature(cs3, keys) == -1
    assert L.fa_tm_same_signature(cs, keys + ("nope",)) == -1
    assert L.fa_tm_same_signature([], keys) == -1


def test_tensor_ptrs_refuse_host_tensors_and_bad_args(L):
    cs = _clients()
    keys = ("a.weight", "a.bias")
    ptrs = np.zeros((2, len(cs)), np.int64)
    keep = [None] * (2 * len(cs))
    dts = (torch.float32, torch.float32)
    assert L.fa_tm_tensor_ptrs(cs, keys, dts, 0, ptrs.ctypes.data, keep) == 1  # CPU tensors: not device 0
    assert L.fa_tm_tensor_ptrs(cs, keys, (torch.float32,), 0, ptrs.ctypes.data, keep) == 1  # one dtype per key
    assert L.fa_tm_tensor_ptrs(cs, keys, dts, 0, ptrs.ctypes.data, [None]) == 1  # keep length
    assert L.fa_tm_tensor_ptrs(cs, keys, ("float32", "float32"), 0, ptrs.ctypes.data, keep) == 1


def test_make_plan_uses_native_signature(L):
    cs = _clients()
    assert bucket._same_signature_native(cs, list(cs[0]))
    plan = bucket.make_plan([1.0] * len(cs), cs)
    assert plan.n_clients == len(cs)


def test_sparse_and_storage_less_values_fall_back(L):
    """Sparse values answer "fallback" / a signature instead of a C++ exception crossing ctypes."""
    cs = _clients()
    keys = ("a.weight", "a.bias")
    cs2 = [dict(c) for c in cs]
    cs2[1]["a.bias"] = torch.zeros(3).to_sparse()
    py = all(bucket._raw_signature(c, list(keys)) == bucket._raw_signature(cs2[0], list(keys)) for c in cs2)
    assert L.fa_tm_same_signature(cs2, keys) == int(py)  # what the Python comparison says
    ptrs = np.zeros((2, len(cs)), np.int64)
    keep = [None] * (2 * len(cs))
    assert L.fa_tm_tensor_ptrs(cs2, keys, (torch.float32, torch.float32), 0, ptrs.ctypes.data, keep) == 1


@pytest.mark.gpu
@pytest.mark.gpu
def test_sparse_device_value_falls_back(L, cuda):
    """A sparse CUDA tensor passes the dtype and device checks: the layout check must refuse it
    before is_contiguous() (which throws for sparse tensors) is reached."""
    dev = cuda
    cs = [{k: v.to(dev) for k, v in c.items()} for c in _clients()]
    keys = ("a.weight", "a.bias")
    ptrs = np.zeros((2, len(cs)), np.int64)
    keep = [None] * (2 * len(cs))
    dts = (torch.float32, torch.float32)
    assert L.fa_tm_tensor_ptrs(cs, keys, dts, 0, ptrs.ctypes.data, keep) == 0
    cs[3]["a.bias"] = torch.zeros(3, device=dev).to_sparse()
    assert L.fa_tm_tensor_ptrs(cs, keys, dts, 0, ptrs.ctypes.data, keep) == 1


def test_up_to_date_check_never_loads_the_library():
    """build_torchmeta decides "up to date" from the sidecar stamp file: the building process
    must not dlopen the old library (glibc would hand that cached handle to the later load of the
    rebuilt file, and load_torchmeta would read the stale stamp)."""
    import subprocess
    import sys

    code = ("from flearn_amd import _build; _build.build_torchmeta(); "
            "print(any('libfa_torchmeta' in l for l in open('/proc/self/maps')))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         cwd=str(Path(__file__).resolve().parent.parent))
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "False"
