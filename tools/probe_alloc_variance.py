"""Does the NS reduce's speed depend on where its 10 GB stack lands?  One process allocates the
100 x ResNet-50 stack afresh several times — torch.empty after empty_cache, with a spacer
allocation of growing size in between that moves the next one, and (--contiguous) the same
through hipExtMallocWithFlags(hipDeviceMallocContiguous) — and times the product kernel on each
(HIP events, median of 20).  python tools/probe_alloc_variance.py [--contiguous] (GPU box)."""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "/root/repo")
from flearn_amd import _native as na  # noqa: E402
from flearn_amd import layouts  # noqa: E402

dev = torch.device("cuda", 0)
L = na.lib()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
n, p = 100, layouts.padded_f32_stride(layouts.get("resnet50"))
w = torch.ones(n, device=dev)
out = torch.empty(p, device=dev)
stream = torch.cuda.current_stream().cuda_stream


def run(ptr):
    assert L.fa_fill_uniform_f32(ptr, p, n, p, 2024, 0, 0, stream) == 0

    def red():
        assert L.fa_reduce_f32(ptr, p, n, na.MODE_W32_DIV64, w.data_ptr(), float(n), 0, p, None, out.data_ptr(),
                               None, stream) == 0
    for _ in range(3):
        red()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        red()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return round(float(np.median(ts)), 1), round(min(ts), 1)


mode = "contiguous" if "--contiguous" in sys.argv else "torch"
res, spacers = [], []
for trial in range(8):
    if mode == "torch":
        stack = torch.empty((n, p), dtype=torch.float32, device=dev)
        ptr = stack.data_ptr()
    else:
        v = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(v), n * p * 4, 0x4)  # hipDeviceMallocContiguous
        assert rc == 0, rc
        ptr = v.value
    med, mn = run(ptr)
    res.append({"trial": trial, "mode": mode, "median_us": med, "min_us": mn})
    print(res[-1], file=sys.stderr, flush=True)
    if mode == "torch":
        del stack
    else:
        torch.cuda.synchronize()
        hip.hipFree(ptr)
    spacers.append(torch.empty(int((trial + 1) * 257 * 2**20 // 4), device=dev))  # move the next allocation
    torch.cuda.empty_cache()
print(json.dumps({"rows": res}))
