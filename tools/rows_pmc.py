"""Row-pointer kernel vs stack kernel on the same client data, for rocprofv3 --pmc passes
(why does reduce_kernel_segrows_rm run 7-10% behind reduce_kernel_rowmajor?).

flearn's run2 simulator hands the server each client's CUDA state_dict (Communicator.py:287-292):
every tensor its own allocation.  The product reads them in place through a per-(key, client)
pointer table (fa_reduce_f32_rows, the engine's Packer building the table); the stack kernel
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

from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import layouts  # noqa: E402
from flearn_amd.aggregator import Aggregator  # noqa: E402
from flearn_amd.bucket import RowTable, make_plan  # noqa: E402
from flearn_amd.semantics import KIND_F32  # noqa: E402

CONFIGS = {"ns": ("resnet50", 100, "mean"), "c3": ("resnet50", 100, "avgm"), "c2": ("resnet18", 100, "mean")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--alloc", default="clones", choices=("clones", "views", "stack"))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kernel", default="product", choices=("product", "lt"),
                    help="lt: the row kernel with the group's row pointers staged in LDS (tools/libtune_rows.so "
                         "variant 16, the product's V8 W8 KG2 geometry and piece table; mean only)")
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
    # the uploads hold the stack's values without a torch copy kernel (the PMC passes crashed the
    # profiler inside torch's device-to-device copy): every tensor is generated in place with the
    # stack's (seed, client, column) coordinates
    clients = []
    for i in range(n):
        d = {}
        flat = None
        if a.alloc == "views":
            flat = torch.empty(stride, dtype=torch.float32, device=dev)
            agg.fill_uniform(flat, seed=2024, row_begin=i)
        for k, sh, off, m in offs:
            if a.alloc == "clones":
                t = torch.empty(m, dtype=torch.float32, device=dev)
                agg.fill_uniform(t, seed=2024, row_begin=i, col_begin=off)
                d[k] = t.view(sh)
            elif a.alloc == "views":
                d[k] = flat[off : off + m].view(sh)
            else:
                d[k] = stack[i, off : off + m].view(sh)
        clients.append(d)
    w = torch.ones(n, dtype=torch.float32, device=dev)
    out = torch.empty(stride, dtype=torch.float32, device=dev)
    out_rows = torch.empty(stride, dtype=torch.float32, device=dev)
    eng = Aggregator(output="device")
    eng.packer.use_slabs = False  # --alloc stack IS a slab: measure the pointer-table kernel on it
    plan = make_plan([1.0] * n, clients)
    if op != "mean":  # double-buffered (prev, v_t) per kernel, same initial state
        pv, pr = ([torch.empty(stride, dtype=torch.float32, device=dev) for _ in range(2)] for _ in range(2))
        agg.fill_uniform(pv[0], seed=1)
        agg.fill_uniform(pr[0], seed=1)
        v = [torch.zeros(stride, dtype=torch.float64, device=dev) for _ in range(2)]
        vr = [torch.zeros(stride, dtype=torch.float64, device=dev) for _ in range(2)]

    T = None
    if a.kernel == "lt":
        import ctypes

        if op != "mean":
            raise SystemExit("--kernel lt: mean only")
        T = ctypes.CDLL(str(REPO / "tools" / "libtune_rows.so"))
        P = ctypes.c_void_p
        T.tune_rows_rm_launch.argtypes = [ctypes.c_int, P, ctypes.c_int, P, P, ctypes.c_int64, ctypes.c_int, P,
                                          ctypes.c_double, P, P]

    def rows_launch(cur):
        (sh, table), = eng.packer.pack(plan, clients)[KIND_F32]
        assert isinstance(table, RowTable), type(table)
        if T is not None:
            pieces, npieces, grid = table.piece_table(0)
            rc = T.tune_rows_rm_launch(16, table.ptrs.data_ptr(), n, w.data_ptr(), pieces.data_ptr(), npieces, grid,
                                       table.work.data_ptr(), float(n), out_rows.data_ptr(), na.stream_handle(dev))
            assert rc == 0, rc
            table.release()
        elif op == "mean":
            agg.reduce_stack(table, w, na.MODE_W32_DIV64, float(n), out32=out_rows)
        else:
            agg.reduce_stack(table, w, na.MODE_W32_DIV64, float(n), out32=pr[1 - cur], prev=pr[cur], v=vr[cur],
                             v_out=vr[1 - cur], op=na.OP_BY_NAME[op])

    def stack_launch(cur):
        if op == "mean":
            agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=out)
        else:
            agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=pv[1 - cur], prev=pv[cur], v=v[cur],
                             v_out=v[1 - cur], op=na.OP_BY_NAME[op])

    cur = 0
    for _ in range(2):
        rows_launch(cur)
        stack_launch(cur)
        cur ^= 1
    torch.cuda.synchronize()
    # compare the tensors' columns only (the stack's alignment gaps hold fill values the row
    # kernel never reads or writes)
    a_, b_ = (out_rows if op == "mean" else pr[cur]), (out if op == "mean" else pv[cur])
    same = all(bool(torch.equal(a_[off : off + m].view(torch.int32), b_[off : off + m].view(torch.int32)))
               for _, _, off, m in offs)
    t_rows, t_stack = [], []
    for r in range(a.reps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        rows_launch(cur)
        e1.record()
        stack_launch(cur)
        e2.record()
        cur ^= 1
        torch.cuda.synchronize()
        t_rows.append(e0.elapsed_time(e1) * 1e3)
        t_stack.append(e1.elapsed_time(e2) * 1e3)
    alg = n * p * 4 + p * 4 + (0 if op == "mean" else p * 4 + 2 * p * 8)
    print(json.dumps({"config": a.config, "alloc": a.alloc, "kernel": a.kernel, "clients": n, "params": p, "bit_equal": same,
                      "rows_us_median": round(float(np.median(t_rows)), 1),
                      "stack_kernel_us_median": round(float(np.median(t_stack)), 1),
                      "stack_frac": round(alg / float(np.median(t_stack)) / 8e6, 4),
                      "note": "rows = the pointer-table H2D + the row kernel on the stream; the kernel's own "
                              "time from rocprof"}))


if __name__ == "__main__":
    main()
