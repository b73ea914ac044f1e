"""Does a column-slabbed client stack stream C5 faster?  

    python tools/probe_slabs.py [--config c5] [--op adagrad] [--slabs 1,2,4,8] [--allocs 2]

tools/probe_c5_shape.py found C5's plain mean 1-2.5% slower per byte at its 346-MB row pitch than
the same bytes at NS's 102-MB pitch (338 x 25.6 M).  Here ONE allocation of N x P floats is
reduced as S column slabs — slab s an [N][P/S] stack of its own (row pitch P/S), one launch per
slab — for each S, on the same memory (so placement is shared), interleaved rounds, HIP events,
the product kernel (fa_reduce_f32) with the config's fused epilogue and double-buffered state.
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
    from flearn_amd import aggregator as agg

    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--params", type=int, default=86_567_656)
    ap.add_argument("--op", default="adagrad")
    ap.add_argument("--slabs", default="1,2,3,4,8")
    ap.add_argument("--allocs", type=int, default=2)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--windows", action="store_true",
                    help="keep the [N][P] stack (pitch P) and split only the launches into S column windows")
    a = ap.parse_args()
    L = na.lib()
    dev = torch.device("cuda", 0)
    n, p = a.clients, a.params
    slabs = [int(x) for x in a.slabs.split(",")]
    res = {"clients": n, "params": p, "op": a.op, "mode": "windows" if a.windows else "slabs", "by_slabs": {}}
    stride_max = -(-p // 64) * 64
    for alloc in range(a.allocs):
        buf = torch.empty(n * stride_max + 64 * max(slabs) * n, dtype=torch.float32, device=dev)
        w = torch.ones(n, dtype=torch.float32, device=dev)
        prev = [torch.empty(stride_max, dtype=torch.float32, device=dev) for _ in range(2)]
        v = [torch.zeros(stride_max, dtype=torch.float64, device=dev) for _ in range(2)]
        agg.fill_uniform(prev[0][None], seed=1)
        stack = buf[: n * stride_max].view(n, stride_max)  # the plain [N][P] stack (pitch P)
        layouts = {}
        for S in slabs:
            width = -(-(-(-p // S)) // 64) * 64  # columns per slab, ALIGN-rounded
            views = []
            off = 0
            for s in range(S):
                c0 = s * width
                wc = max(0, min(width, p - c0))
                if wc == 0:
                    break
                if a.windows:  # S launches over column windows of the ONE [N][P] stack
                    views.append((stack[:, c0 : c0 + width] if c0 + width <= stride_max else stack[:, c0:], c0, wc))
                else:
                    views.append((buf[off : off + n * width].view(n, width), c0, wc))
                off += n * width
            layouts[S] = views

        def run(S, cur):
            for x, c0, wc in layouts[S]:
                kw = {}
                if a.op != "mean":
                    kw = dict(op=na.OP_BY_NAME[a.op], prev=prev[cur][c0 : c0 + wc], v=v[cur][c0 : c0 + wc],
                              v_out=v[1 - cur][c0 : c0 + wc])
                agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), n_cols=wc, out32=prev[1 - cur][c0 : c0 + wc], **kw)

        for S in slabs:  # fill each layout once (the values do not matter for timing)
            for x, c0, wc in layouts[S]:
                agg.fill_uniform(x, seed=2024, col_begin=c0, n_cols=wc)
            run(S, 0)
        torch.cuda.synchronize()
        times = {S: [] for S in slabs}
        cur = 0
        for r in range(a.reps):
            order = slabs[r % len(slabs):] + slabs[: r % len(slabs)]
            for S in order:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(S, cur)
                e1.record()
                torch.cuda.synchronize()
                times[S].append(e0.elapsed_time(e1) * 1e3)
                cur ^= 1
        alg = n * p * 4 + p * 4 + (0 if a.op == "mean" else p * 4 + 2 * p * 8)
        for S in slabs:
            t = float(np.median(times[S]))
            d = res["by_slabs"].setdefault(str(S), {"pitch_mb": round(layouts[S][0][0].stride(0) * 4 / 1e6, 1), "us": [],
                                                    "frac": []})
            d["us"].append(round(t, 1))
            d["frac"].append(round(alg / t / 8e6, 4))
        print(json.dumps(res), file=sys.stderr, flush=True)
        del buf, layouts, stack
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
