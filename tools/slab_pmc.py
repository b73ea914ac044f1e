"""Slab uploads (flearn_amd.device_state_dicts) against the packed stack, for rocprofv3 passes.

    python tools/slab_pmc.py [--config ns|c3] [--which engine|stack|both] [--reps 10]

engine: 100 clients' ResNet-50 state_dicts carved from one allocation, aggregated through the
        product's Strategy.server (output="device": no D2H) — the Packer recognises the slab and
        launches the stack kernel (reduce_kernel_rowmajor) on the clients' own memory;
stack:  the same values in a separate [N, stride] stack, fa_reduce_f32 launched directly
        (bench.py's kernel).
Prints one JSON line: HIP-event kernel times of each (median of --reps), the server() call's wall
time, and whether the two results are bit-equal.  Run one --which per process under
`rocprofv3 --pmc` (both launch the same kernel name).  Measurement infrastructure.
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

from flearn_amd import AVG, AVGM, device_state_dicts  # noqa: E402
from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import layouts  # noqa: E402

CONFIGS = {"ns": ("resnet50", 100, "mean"), "c3": ("resnet50", 100, "avgm"), "c2": ("resnet18", 100, "mean")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--which", default="both", choices=("engine", "stack", "both"))
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    name, n, op = CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    na.lib()
    layout = layouts.get(name)
    template = {k: torch.zeros(shape, dtype=torch.float32 if t == "f32" else torch.int64) for k, shape, t in layout}
    sd = device_state_dicts(template, n, device=dev)
    agg.fill_uniform(sd.slab, seed=2024)  # generated in place: no copy kernels in the passes
    stride = sd.slab.shape[1]
    p = sum(m for _, m, _ in sd.offsets.values())
    uploads = [{"agg_weight": 1.0, "params": c} for c in sd]
    res = {"config": a.config, "clients": n, "params": p, "tensors_per_client": len(layout), "op": op,
           "slab_bytes": sd.slab.numel() * 4}

    def ev_time(fn, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(k):
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return float(np.median(ts))

    algo = n * p * 4 + p * 4 + (0 if op == "mean" else p * 20)
    out_engine = out_stack = None
    if a.which in ("engine", "both"):
        s = AVG(output="device") if op == "mean" else AVGM(server_side=True, output="device")
        if op != "mean":
            s.server_opt.init_global({k: np.zeros(shp, np.float32) for k, (_, _, shp) in sd.offsets.items()})
        s.server(uploads, 0)
        torch.cuda.synchronize()
        assert s.engine.packer.last_row_tables.get("f32") == "slab", s.engine.packer.last_row_tables
        walls = []
        for r in range(a.reps):
            t0 = time.perf_counter()
            g = s.server(uploads, r + 1)["w_glob"]
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
        t = ev_time(lambda: s.server(uploads, 99), a.reps)
        out_engine = torch.cat([g[k].reshape(-1) for k in sd.offsets]) if op == "mean" else None
        res.update(engine_server_call_us=round(t, 1), engine_server_wall_ms_median=round(float(np.median(walls)) * 1e3, 3),
                   engine_path=dict(s.engine.packer.last_row_tables))
    if a.which in ("stack", "both"):
        x = sd.slab.clone()
        w = torch.ones(n, dtype=torch.float32, device=dev)
        out = torch.empty(stride, dtype=torch.float32, device=dev)
        kw = {}
        if op != "mean":
            pv = [torch.zeros(stride, dtype=torch.float32, device=dev) for _ in range(2)]
            vv = [torch.zeros(stride, dtype=torch.float64, device=dev) for _ in range(2)]
            kw = dict(op=na.OP_BY_NAME[op], prev=pv[0], v=vv[0], v_out=vv[1])
            out = pv[1]
        t = ev_time(lambda: agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=out, **kw), a.reps)
        out_stack = torch.cat([out[o : o + m] for o, m, _ in sd.offsets.values()]) if op == "mean" else None
        res.update(stack_kernel_us=round(t, 1), stack_frac_of_8TBs=round(algo / t / 8e6, 4))
    if out_engine is not None and out_stack is not None:
        res["engine_bit_equal_stack"] = bool(torch.equal(out_engine.view(torch.int32), out_stack.view(torch.int32)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
