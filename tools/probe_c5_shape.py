"""Why does C5 (100 x 86.6 M) stream slower per byte than NS (100 x 25.6 M)?  

    python tools/probe_c5_shape.py [--reps 5] > out.json

One process, interleaved rounds, HIP events (median): the product's plain-mean reduce
(fa_reduce_f32) on
  * ns      100 x 25,610,152   (10.2 GB, row pitch 102 MB)
  * c5      100 x 86,567,656   (34.6 GB, row pitch 346 MB)
  * c5bytes 338 x 25,610,152   (34.6 GB — C5's bytes at NS's pitch)
  * c5half  100 x 43,283,828   (17.3 GB, pitch 173 MB)
each on two allocations (placement varies per allocation: DESIGN.md section 4 finding 25), and a
plain grid-stride read (tools/libprobe_copy.so probe_read, 1024 blocks) of 10.2 and 34.6 GB.
If c5bytes streams like ns, the row pitch (shape) costs C5 its rate; if like c5, the size does.
Measurement infrastructure, not the product.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def main():
    import numpy as np
    import torch

    from flearn_amd import _native as na

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--allocs", type=int, default=2)
    a = ap.parse_args()
    L = na.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    P = ctypes.CDLL(str(REPO / "tools" / "libprobe_copy.so"))
    P.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    shapes = {"ns": (100, 25_610_152), "c5": (100, 86_567_656), "c5bytes": (338, 25_610_152),
              "c5half": (100, 43_283_828)}
    sink = torch.empty(1024 * 256 * 4, dtype=torch.int32, device=dev)
    res = {}

    def ev_time(fn, reps):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return float(np.median(ts))

    for alloc in range(a.allocs):
        for name, (n, p) in shapes.items():
            stride = -(-p // 64) * 64
            x = torch.empty((n, stride), dtype=torch.float32, device=dev)
            assert L.fa_fill_uniform_f32(x.data_ptr(), stride, n, p, 2024, 0, 0, stream) == 0
            w = torch.ones(n, dtype=torch.float32, device=dev)
            out = torch.empty(stride, dtype=torch.float32, device=dev)

            def red():
                na.check(L.fa_reduce_f32(x.data_ptr(), stride, n, na.MODE_W32_DIV64, w.data_ptr(), float(n), 0, p, None,
                                         out.data_ptr(), None, stream), "fa_reduce_f32")

            def rd():
                assert P.probe_read(x.data_ptr(), n * stride * 4 // 16, 1024, sink.data_ptr(), stream) == 0

            for _ in range(2):
                red()
                rd()
            torch.cuda.synchronize()
            tr, tl = [], []
            for _ in range(a.reps):
                tr.append(ev_time(red, 1))
                tl.append(ev_time(rd, 1))
            byts = n * p * 4 + p * 4
            r = res.setdefault(name, {"clients": n, "params": p, "bytes": byts, "reduce_us": [], "read_us": [],
                                      "reduce_tbs": [], "read_tbs": []})
            r["reduce_us"].append(round(float(np.median(tr)), 1))
            r["read_us"].append(round(float(np.median(tl)), 1))
            r["reduce_tbs"].append(round(byts / float(np.median(tr)) / 1e6, 3))
            r["read_tbs"].append(round(n * stride * 4 / float(np.median(tl)) / 1e6, 3))
            del x, out, w
            torch.cuda.empty_cache()
            print(json.dumps({name: r}), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
