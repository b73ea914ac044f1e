"""The stack kernel at the column widths multi-GPU plans give each rank (measurement tool).

    python tools/width_sweep.py [--clients 100] [--widths 25610152,12805076,...] [--op mean|avgm]
                                [--reps 20] [--pitch contiguous|full]

One [clients, W] fp32 stack per width (pitch W rounded up to ALIGN columns, as a rank's column
shard in bench.py; --pitch full keeps the widest width's pitch and reads the first W columns, as
one stripe of a wider shard does),
reduced by the library's own geometry selection (fa_reduce_f32, FA_MODE_W32_DIV64).  Prints one
JSON line per width: the mean launch time of --reps back-to-back launches (median of 5 batches), the column windows the library
used, and the fraction of 8 TB/s of the algorithmic bytes (bench.py bytes_per_launch).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd.dist import ALIGN  # noqa: E402

NS = 25610152


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--widths", default=",".join(str(-(-NS // g)) for g in (1, 2, 4, 8, 16, 32)))
    ap.add_argument("--op", default="mean", choices=("mean", "avgm"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pitch", default="contiguous", choices=("contiguous", "full"))
    ap.add_argument("--lib", default=None, help="a tuning build of libflearn_amd.so to load instead of the product's")
    ap.add_argument("--grids", default="0", help="comma list of forced grids per width (fa_set_reduce_grid; 0 = "
                    "the library's choice); 'fit' = the grid whose share fills the piece (ceil(chunks / 2^j)); "
                    "'narrow' = a share of 2 chunks (the one-wave-per-chunk kernel)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.lib:
        na.LIB_PATH = Path(a.lib).resolve()
    L = na.lib()
    n = a.clients
    widths = [int(x) for x in a.widths.split(",")]
    full = None
    if a.pitch == "full":
        full = torch.empty((n, -(-max(widths) // ALIGN) * ALIGN), dtype=torch.float32, device=dev)
        agg.fill_uniform(full, seed=2024)
    for wdt in widths:
        if full is None:
            x = torch.empty((n, -(-wdt // ALIGN) * ALIGN), dtype=torch.float32, device=dev)
            agg.fill_uniform(x, seed=2024)
        else:
            x = full
        w = torch.ones(n, dtype=torch.float32, device=dev)
        kw = {}
        out = torch.empty(wdt, dtype=torch.float32, device=dev)
        if a.op == "avgm":
            kw = dict(op=na.OP_AVGM, prev=torch.zeros(wdt, dtype=torch.float32, device=dev),
                      v=torch.zeros(wdt, dtype=torch.float64, device=dev),
                      v_out=torch.zeros(wdt, dtype=torch.float64, device=dev))
        fn = lambda: agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), n_cols=wdt, out32=out, **kw)  # noqa: E731
        for gs in a.grids.split(","):
            chunks = -(-(-(-wdt // 4)) // 64)
            grid = fit_grid(wdt, a.op) if gs == "fit" else -(-chunks // 2) if gs == "narrow" else int(gs)
            L.fa_set_reduce_grid(grid)  # returns the previous setting
            time_one(a, L, n, wdt, fn, grid)
        L.fa_set_reduce_grid(0)
        del x


def fit_grid(wdt: int, op: str) -> int:
    """The grid near 192 whose per-block share is a whole piece of 2^j KiB (W = 4 / 8 waves)."""
    chunks = -(-(-(-wdt // 4)) // 64)
    s0 = -(-chunks // 192)
    wv = 4 if op == "mean" else 8
    cap = wv
    while cap < s0:
        cap *= 2
    return -(-chunks // (cap // 2)) if cap > wv and -(-chunks // (cap // 2)) <= 256 else 0


def time_one(a, L, n, wdt, fn, grid):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):  # back to back, as bench.py's steps: the mean launch of each batch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / a.reps)
    t = float(np.median(ts))
    algo = n * wdt * 4 + wdt * 4 + (0 if a.op == "mean" else wdt * 20)
    wins = L.fa_reduce_windows(na.OP_BY_NAME[a.op], wdt)
    print(json.dumps({"clients": n, "width": wdt, "op": a.op, "pitch": a.pitch, "grid": grid, "us": round(t, 2),
                      "us_min": round(min(ts), 2), "frac_of_8TBs": round(algo / t / 8e6, 4),
                      "windows": wins}), flush=True)


if __name__ == "__main__":
    main()
