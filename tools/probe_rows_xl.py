"""Row-pointer kernel, fused FedAVGM (C3's shape: 100 x ResNet-50 uploads, one allocation per
(client, tensor) as flearn's run2 deepcopy makes them): half-line vs whole-line f64 state stores.

    python tools/probe_rows_xl.py [--reps 9]

The product's piece table and grid (RowTable.piece_table), the kernel through tools/libtune_rows.so
(tune_rows_rm_avgm, xl 0 / 1), double-buffered state, interleaved rounds, HIP events around the
launch only; both outputs bit-compared with the stack kernel's.  Measurement infrastructure.
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
from flearn_amd import layouts  # noqa: E402
from flearn_amd.aggregator import Aggregator  # noqa: E402
from flearn_amd.bucket import RowTable, make_plan  # noqa: E402
from flearn_amd.semantics import KIND_F32  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--layout", default="resnet50")
    ap.add_argument("--clients", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    na.lib()
    n = a.clients
    lay = [(k, s, t) for k, s, t in layouts.get(a.layout) if t == "f32"]
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
        for k, sh, off, m in offs:
            t = torch.empty(m, dtype=torch.float32, device=dev)
            agg.fill_uniform(t, seed=2024, row_begin=i, col_begin=off)
            d[k] = t.view(sh)
        clients.append(d)
    w = torch.ones(n, dtype=torch.float32, device=dev)
    eng = Aggregator(output="device")
    plan = make_plan([1.0] * n, clients)
    (sh, table), = eng.packer.pack(plan, clients)[KIND_F32]
    assert isinstance(table, RowTable)
    pieces, npieces, grid = table.piece_table(na.OP_AVGM)
    T = ctypes.CDLL(str(REPO / "tools" / "libtune_rows.so"))
    P = ctypes.c_void_p
    T.tune_rows_rm_avgm.argtypes = [ctypes.c_int, P, ctypes.c_int, P, P, ctypes.c_int64, ctypes.c_int, P,
                                    ctypes.c_double, P, P, P, P, P]
    prev0 = torch.empty(stride, dtype=torch.float32, device=dev)
    agg.fill_uniform(prev0[None], seed=1)
    outs = {}
    stream = na.stream_handle(dev)

    def launch(xl, prev, v, v_out, out):
        rc = T.tune_rows_rm_avgm(xl, table.ptrs.data_ptr(), n, w.data_ptr(), pieces.data_ptr(), npieces, grid,
                                 table.work.data_ptr(), float(n), prev.data_ptr(), v.data_ptr(), v_out.data_ptr(),
                                 out.data_ptr(), stream)
        assert rc == 0, rc

    bufs = {xl: (torch.zeros(stride, dtype=torch.float64, device=dev), torch.empty(stride, dtype=torch.float64, device=dev),
                 torch.empty(stride, dtype=torch.float32, device=dev)) for xl in (0, 1)}
    for xl in (0, 1):  # one step from (prev0, v = 0): the outputs to compare
        v, v_out, out = bufs[xl]
        launch(xl, prev0, v, v_out, out)
    want_v = torch.empty(stride, dtype=torch.float64, device=dev)
    want = torch.empty(stride, dtype=torch.float32, device=dev)
    agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=want, prev=prev0,
                     v=torch.zeros(stride, dtype=torch.float64, device=dev), v_out=want_v, op=na.OP_AVGM)
    torch.cuda.synchronize()
    same = {}
    for xl in (0, 1):
        v, v_out, out = bufs[xl]
        same[xl] = all(bool(torch.equal(out[o0:o0 + m].view(torch.int32), want[o0:o0 + m].view(torch.int32))) and
                       bool(torch.equal(v_out[o0:o0 + m].view(torch.int64), want_v[o0:o0 + m].view(torch.int64)))
                       for _, _, o0, m in offs)
    times = {0: [], 1: []}
    for r in range(a.reps):
        for xl in ((0, 1) if r % 2 == 0 else (1, 0)):
            v, v_out, out = bufs[xl]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(xl, prev0, v, v_out, out)
            e1.record()
            torch.cuda.synchronize()
            times[xl].append(e0.elapsed_time(e1) * 1e3)
    alg = n * p * 4 + p * 4 + p * 4 + 2 * p * 8
    res = {"layout": a.layout, "clients": n, "params": p, "grid": grid, "pieces": npieces,
           "bit_equal_to_stack_kernel": {"half_line": same[0], "whole_line": same[1]}}
    for xl, name in ((0, "half_line"), (1, "whole_line")):
        t = float(np.median(times[xl]))
        res[name] = {"us_median": round(t, 1), "frac": round(alg / t / 8e6, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
