"""Split-N (fa_reduce_f32_splitn, with its cancellation guard) vs the bit-exact sequential kernel
(fa_reduce_f32) on LeNet5-wide windows, for zero-mean uploads (the guard fires on most columns:
they cancel) and near-common uploads (clients trained from one model: a shared value + 1% noise;
the guard does not fire).  HIP events, interleaved rounds, median per launch.

    python tools/time_splitn_guard.py [--ns 16,64,100,256] [--reps 7]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="16,64,100,256")
    ap.add_argument("--p", type=int, default=44_426)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    na.lib()
    dev = torch.device("cuda", 0)
    p = a.p
    stride = -(-p // 64) * 64
    for n in (int(v) for v in a.ns.split(",")):
        for data in ("zero_mean", "near_common"):
            x = torch.empty((n, stride), dtype=torch.float32, device=dev)
            agg.fill_uniform(x, seed=5)
            if data == "near_common":
                m = torch.empty((1, stride), dtype=torch.float32, device=dev)
                agg.fill_uniform(m, seed=6)
                x.mul_(0.01).add_(m)
            w = torch.ones(n, dtype=torch.float32, device=dev)
            out = torch.empty(stride, dtype=torch.float32, device=dev)
            fns = {"sequential": lambda: agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), n_cols=p, out32=out),
                   "splitn_guarded": lambda: agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), n_cols=p, out32=out,
                                                              reorder=True)}
            times = {k: [] for k in fns}
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(a.reps):
                for k, f in fns.items():
                    f()
                    e0.record()
                    for _ in range(20):
                        f()
                    e1.record()
                    torch.cuda.synchronize()
                    times[k].append(e0.elapsed_time(e1) * 1e3 / 20)
            row = {"n": n, "p": p, "data": data}
            for k, v in times.items():
                v.sort()
                row[k + "_us"] = round(v[len(v) // 2], 2)
            row["gbs_splitn"] = round((n * p * 4 + p * 4) / 1e3 / row["splitn_guarded_us"], 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
