"""Row-pointer kernel vs stack kernel on the same client data, for rocprofv3 --pmc passes
(why does reduce_kernel_segrows_rm run 7-10% behind reduce_kernel_rowmajor?).

flearn's run2 simulator hands the server each client's CUDA state_dict (Communicator.py:287-292):
every tensor its own allocation.  The product reads them in place through a per-(key, client)
pointer table (fa_reduce_f32_rows, via AVG(output="device").server); the stack kernel
(fa_reduce_f32 over one [N, stride] array) reads the same values packed.  This launches both,
alternating, --reps times each, and prints their HIP-event times; run it under
`rocprofv3 --pmc ...` to get per-kernel counters.

    python tools/rows_pmc.py [--config ns|c3] [--alloc clones|views|stack] [--reps 10]

--alloc: clones = one allocation per (client, tensor) as deepcopy makes them; views = one flat
allocation per client, tensors are views into it; stack = tensors are views into ONE [N, stride]
stack (the row kernel then reads exactly the stack kernel's addresses).
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

import flearn_amd  # noqa: E402
from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import layouts  # noqa: E402

CONFIGS = {"ns": ("resnet50", 100, "mean"), "c3": ("resnet50", 100, "avgm"), "c2": ("resnet18", 100, "mean")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--alloc", default="clones", choices=("clones", "views", "stack"))
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    name, n, op = CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    na.lib()
    lay = [(k, s, t) for k, s, t in layouts.get(name) if t == "f32"]
    stride = layouts.padded_f32_stride(lay)
    p = layouts.fp32_elems(lay)
    stack = torch.empty((n, stride), dtype=torch.float32, device=dev)
    agg.fill_uniform(stack, seed=2024)
    offs, o = [], 0
    for k, s, _ in lay:
        m = int(np.prod(s)) if s else 1
        offs.append((k, s, o, m))
        o += -(-m // 64) * 64
    clients = []
    for i in range(n):
        d = {}
        if a.alloc == "views":
            flat = stack[i].clone()
        for k, s, off, m in offs:
            if a.alloc == "clones":
                d[k] = stack[i, off : off + m].clone().view(s)
            elif a.alloc == "views":
                d[k] = flat[off : off + m].view(s)
            else:
                d[k] = stack[i, off : off + m].view(s)
        clients.append(d)
    ups = [{"agg_weight": 1.0, "params": c} for c in clients]
    w = torch.ones(n, dtype=torch.float32, device=dev)
    out = torch.empty(stride, dtype=torch.float32, device=dev)
    if op == "mean":
        s = flearn_amd.AVG(output="device")
        kw = {}
    else:
        s = flearn_amd.AVGM(server_side=True, output="device")
        prev = torch.empty((1, stride), dtype=torch.float32, device=dev)
        agg.fill_uniform(prev, seed=1)
        s.server_opt.init_global({k: prev[0, off : off + m].view(sh).cpu().numpy() for k, sh, off, m in offs})
        v = [torch.zeros(stride, dtype=torch.float64, device=dev) for _ in range(2)]
        pv = [prev[0], torch.empty(stride, dtype=torch.float32, device=dev)]
        kw = dict(op=na.OP_BY_NAME[op])
    for _ in range(2):
        s.server(ups, 0)
    assert s.engine.packer.last_row_tables.get("f32") == "rows" or "rows" in s.engine.packer.last_row_tables.values(), \
        s.engine.packer.last_row_tables
    t_rows, t_stack = [], []
    cur = 0
    for r in range(a.reps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        s.server(ups, r)
        e1.record()
        if op == "mean":
            agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=out)
        else:
            agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=pv[1 - cur], prev=pv[cur], v=v[cur],
                             v_out=v[1 - cur], **kw)
            cur ^= 1
        e2.record()
        torch.cuda.synchronize()
        t_rows.append(e0.elapsed_time(e1) * 1e3)
        t_stack.append(e1.elapsed_time(e2) * 1e3)
    alg = n * p * 4 + p * 4 + (0 if op == "mean" else p * 4 + 2 * p * 8)
    print(json.dumps({"config": a.config, "alloc": a.alloc, "clients": n, "params": p,
                      "server_call_us_median": round(float(np.median(t_rows)), 1),
                      "stack_kernel_us_median": round(float(np.median(t_stack)), 1),
                      "stack_frac": round(alg / float(np.median(t_stack)) / 8e6, 4),
                      "note": "server_call = the whole AVG.server call on the stream (row kernel + its small launches); "
                              "take the row kernel's own time from rocprof"}))


if __name__ == "__main__":
    main()
