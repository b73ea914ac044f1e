"""Device-resident uploads (flearn's run2 path: torch tensors per client and key) on one MI355X.

    python tools/bench_rows.py [--config c2|ns|c3] [--steps K]

Times, on the same synthetic data:
  stack    : fa_reduce_f32 over a packed [N, stride] device stack (bench.py's kernel),
  rows     : fa_reduce_f32_rows reading the N*K separate tensors in place (one launch),
  server   : Strategy.server() on the full state_dict uploads, BN num_batches_tracked (int64)
             included (plan + pointer tables + H2D + the rows launch + the float64 gather),
and checks rows == stack bit for bit.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from flearn_amd import AVG, AVGM  # noqa: E402
from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import layouts  # noqa: E402
from flearn_amd.bucket import make_plan  # noqa: E402

CONFIGS = {"c2": ("resnet18", 100, "mean"), "ns": ("resnet50", 100, "mean"), "c3": ("resnet50", 100, "avgm")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--no-gc", action="store_true", help="diagnosis: time the server() calls with gc disabled")
    a = ap.parse_args()
    name, n, op = CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    layout = [x for x in layouts.get(name) if x[2] == "f32"]
    stride = layouts.padded_f32_stride(layout)
    p = layouts.fp32_elems(layout)
    x = torch.empty((n, stride), dtype=torch.float32, device=dev)
    agg.fill_uniform(x, seed=7)
    counters = [(k, shape) for k, shape, dt in layouts.get(name) if dt == "i64"]  # BN num_batches_tracked
    clients = []  # per client one model buffer (generated in place: no copy kernels), keys are views
    for i in range(n):
        buf = torch.empty((1, stride), dtype=torch.float32, device=dev)
        agg.fill_uniform(buf, seed=7, row_begin=i)
        d, off = {}, 0
        for k, shape, _ in layout:
            m = int(np.prod(shape, dtype=np.int64))
            d[k] = buf[0, off : off + m].view(shape)
            off += -(-max(m, 1) // 64) * 64
        for k, shape in counters:  # int64 with float weights: the float64 group (converting gather)
            d[k] = torch.full(shape, i + 1, dtype=torch.int64, device=dev)
        clients.append(d)
    uploads = [{"agg_weight": 1.0, "params": c} for c in clients]
    s = AVG(output="device") if op == "mean" else AVGM(server_side=True, output="device")
    w = torch.ones(n, dtype=torch.float32, device=dev)
    out_stack = torch.empty(stride, dtype=torch.float32, device=dev)
    epi = {}
    if op != "mean":
        epi = dict(op=na.OP_BY_NAME[op], prev=torch.zeros(stride, dtype=torch.float32, device=dev),
                   v=torch.zeros(stride, dtype=torch.float64, device=dev))

    def ev_time(fn, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(k):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k * 1e3  # us

    t_stack = ev_time(lambda: agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=out_stack, **epi), a.steps)
    # rows kernel alone: the table of the first server() call, relaunched
    s.server(uploads, 0)
    plan = make_plan([1.0] * n, clients)
    table = s.engine.packer.row_table(plan, plan.f32, clients, s.engine.packer.shards(plan, "f32"))
    path = dict(s.engine.packer.last_row_tables)
    out_rows = torch.empty(stride, dtype=torch.float32, device=dev)
    t_rows = ev_time(lambda: agg.reduce_stack(table, w, na.MODE_W32_DIV64, float(n), out32=out_rows, **epi), a.steps)
    if op == "mean":
        same = bool(torch.equal(out_rows.view(torch.int32)[:p], out_stack.view(torch.int32)[:p]))
    else:
        same = None  # the fused state advanced differently often; parity is in tests/test_gpu_rows.py
    torch.cuda.synchronize()
    walls = []
    if a.no_gc:
        import gc

        gc.collect()
        gc.disable()
    for r in range(a.steps):
        t0 = time.perf_counter()
        s.server(uploads, r + 1)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    algo = n * p * 4 + p * 4 + (0 if op == "mean" else p * 20)
    print(json.dumps({
        "config": a.config, "clients": n, "params": p, "tensors_per_client": len(layout) + len(counters), "op": op,
        "stack_kernel_us": round(t_stack, 1), "rows_kernel_us": round(t_rows, 1),
        "stack_frac_of_8TBs": round(algo / t_stack / 8e6, 4), "rows_frac_of_8TBs": round(algo / t_rows / 8e6, 4),
        "rows_bit_equal_stack": same,
        "server_call_ms_median": round(float(np.median(walls)) * 1e3, 3),
        "server_call_ms_min": round(min(walls) * 1e3, 3),
        "server_call_ms_all": [round(x * 1e3, 2) for x in walls],
        "path": path,
    }), flush=True)


if __name__ == "__main__":
    main()
