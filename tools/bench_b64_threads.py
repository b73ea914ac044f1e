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
    print(json.dumps(res))


if __name__ == "__main__":
    main()
