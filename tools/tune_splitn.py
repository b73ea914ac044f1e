"""Geometry sweep of the split-N reduce (reduce_kernel_splitn) against the sequential kernel.

    python tools/tune_splitn.py [--shapes N:P,N:P,...] [--reps R]

For each [N, P] fp32 stack (device-generated), times the product's sequential fa_reduce_f32,
the product's fa_reduce_f32_splitn and the variants of tools/libtune_rows.so
(tune_splitn_launch: W waves = client splits per 1-KiB chunk, D rows in flight), HIP events, interleaved over R
rounds.  Each split-N result is checked against the sequential one at <= 1e-6 normwise relative
error.  Prints one JSON line per (shape, variant).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402

VARIANTS = {"w4d8": 0, "w4d16": 1, "w8d8": 2, "w8d16": 3, "w16d8": 4, "w16d4": 5, "w2d16": 6, "w16d16": 7,
            "st_w4d8": 8, "st_w8d8": 9, "st_w16d8": 10, "st_w8d16": 11, "st_w16d4": 12}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1000:44426,100:44426,1000:1000000,200:1000000,100:11699112")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    L = na.lib()
    T = ctypes.CDLL(str(REPO / "tools" / "libtune_rows.so"))
    T.tune_splitn_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    stream = na.stream_handle(dev)
    for shape in a.shapes.split(","):
        n, p = (int(v) for v in shape.split(":"))
        stride = -(-p // 64) * 64
        x = torch.empty((n, stride), dtype=torch.float32, device=dev)
        agg.fill_uniform(x, seed=11)
        w = torch.ones(n, dtype=torch.float32, device=dev)
        ref = torch.empty(stride, dtype=torch.float32, device=dev)
        out = torch.empty_like(ref)

        def seq():
            agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=out)

        def lib():
            na.check(L.fa_reduce_f32_splitn(x.data_ptr(), stride, n, na.MODE_W32_DIV64, w.data_ptr(), float(n), 0, p,
                                            None, out.data_ptr(), None, stream), "splitn")

        fns = {"sequential": seq, "lib_splitn": lib}
        for name, vid in VARIANTS.items():
            fns[name] = (lambda vid=vid: T.tune_splitn_launch(vid, x.data_ptr(), stride, n, w.data_ptr(), p, float(n),
                                                             out.data_ptr(), stream))
        agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=ref)
        torch.cuda.synchronize()
        errs = {}
        for k, f in fns.items():
            out.zero_()
            f()
            torch.cuda.synchronize()
            d = (out[:p].double() - ref[:p].double()).norm() / ref[:p].double().norm()
            errs[k] = float(d)
        times = {k: [] for k in fns}
        for _ in range(a.reps):
            for k, f in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                f()
                e0.record()
                for _ in range(a.steps):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.steps * 1e3)
        algo = n * p * 4 + p * 4
        for k, ts in times.items():
            print(json.dumps({"n": n, "p": p, "variant": k, "us_min": round(min(ts), 2),
                              "us_med": round(float(np.median(ts)), 2), "frac": round(algo / min(ts) / 8e6, 4),
                              "rel_err": errs[k]}), flush=True)
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
