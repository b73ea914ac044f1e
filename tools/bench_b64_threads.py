"""Thread scaling of the native base64 decoder (fa_b64_decode) on this host: is the HTTP-mode
decode compute- or memory-bound?  python tools/bench_b64_threads.py (host only, no GPU call)."""
import base64
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from flearn_amd import _native as na  # noqa: E402


def main():
    L = na.load()
    raw = np.random.default_rng(0).integers(0, 256, 192 * 2**20, dtype=np.uint8).tobytes()
    txt = base64.b64encode(raw)
    out = np.empty(len(raw) + 64, np.uint8)
    out[:] = 0
    fn = L.fa_b64_decode
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
    dst = np.empty_like(out)
    t0 = time.perf_counter()
    np.copyto(dst, out)
    copy_gbs = 2 * len(out) / (time.perf_counter() - t0) / 1e9
    res = {"text_MB": len(txt) / 1e6, "numpy_copy_GB_s_rw_1thread": round(copy_gbs, 1), "decode_GB_s_text": {}}
    for th in (1, 2, 4, 8, 16, 32):
        best = 1e9
        for _ in range(4):
            t = time.perf_counter()
            rc = fn(txt, len(txt), out.ctypes.data, len(out), th)
            best = min(best, time.perf_counter() - t)
            assert rc == 0
        res["decode_GB_s_text"][th] = round(len(txt) / best / 1e9, 2)
    # the same decode into pinned host memory (what HTTP-mode uploads land in) and one upload's size
    import torch

    pinned = torch.empty(len(out), dtype=torch.uint8).pin_memory()
    res["pinned_decode_GB_s_text"] = {}
    for th in (1, 16):
        best = 1e9
        for _ in range(4):
            t = time.perf_counter()
            assert fn(txt, len(txt), pinned.data_ptr(), len(out), th) == 0
            best = min(best, time.perf_counter() - t)
        res["pinned_decode_GB_s_text"][th] = round(len(txt) / best / 1e9, 2)
    small = txt[: 62 * 2**20 // 4 * 4]
    for dst_name, ptr in (("pageable", out.ctypes.data), ("pinned", pinned.data_ptr())):
        best = 1e9
        for _ in range(10):
            t = time.perf_counter()
            assert fn(small, len(small), ptr, len(out), 16) == 0
            best = min(best, time.perf_counter() - t)
        res[f"one_upload_62MB_16threads_{dst_name}_ms"] = round(best * 1e3, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
