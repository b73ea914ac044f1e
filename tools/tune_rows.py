"""Work-plan sweep for fa_reduce_f32_rows (device uploads read in place), one MI355X.

    python tools/tune_rows.py [--config c2|ns] [--alloc views|clones|stack] [--reps R]

Times the product kernel (lib: fa_reduce_f32_rows with fa_rows_plan's table) against variants
of its geometry (V quads per lane, D rows in flight, W waves; pieces of C KiB of a row, largest
first, claimed dynamically) built through tools/libtune_rows.so, and the stack kernel on the
same data; HIP events, interleaved over R rounds; every variant is bit-compared with the stack
kernel.  Prints one JSON line per variant.
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

TUNE_LIB = REPO / "tools" / "libtune_rows.so"
PIECE = np.dtype([("col", "<i8"), ("seg_off", "<i8"), ("seg", "<i4"), ("n_cols", "<i4"), ("aux", "<i8")])
CONFIGS = {"c2": ("resnet18", 100), "ns": ("resnet50", 100), "c4s": ("resnet18", 800),
           "c2flat": ("flat:11699136", 100), "c2wide": ("flat:2359296x5", 100)}  # synthetic: big tensors only


def cut(segs, max_chunks):
    out = []
    for s, (col, n) in enumerate(segs):
        off = 0
        while off < n:
            w = min(max_chunks * 256, n - off)
            out.append((col + off, off, s, w))
            off += w
    return out


def product_plan(segs, pc, kg=2, wide_cols=64 * 8 * 4):
    """fa_rows_plan's table for a given piece width pc (chunks): pieces cut as its cut_segment,
    largest first (stable), pieces[0].aux = the wide ones."""
    out = []
    for s, (col, n) in enumerate(segs):
        chunks = -(-n // 256)
        if chunks == 0:
            continue
        npc = -(-chunks // pc)
        per = -(-chunks // npc) * 256
        off = 0
        while off < n:
            w = min(per, n - off)
            out.append((col + off, off, s, w))
            off += per
    out.sort(key=lambda q: -q[3])
    arr = np.zeros(len(out), PIECE)
    for i, q in enumerate(out):
        arr[i] = (q[0], q[1], q[2], q[3], 0)
    if len(out):
        arr[0]["aux"] = sum(1 for q in out if q[3] > wide_cols)
    return arr


def filled_plan(segs, kg, pmax=64, wv=8, target=192):
    """The product planner's search (fa_rows_plan) for group size kg and pieces of at most pmax
    chunks: the widest pieces and a grid in [target - target/8, target] whose groups fill whole
    rounds.  Returns (table, grid)."""
    best = None
    for pc in range(pmax, pmax * 5 // 8 - 1, -1):
        arr = product_plan(segs, pc, kg, wide_cols=64 * wv * 4)
        groups = -(-int(arr[0]["aux"]) // kg) if len(arr) else 0
        for g in range(target, target - target // 8 - 1, -1):
            rounds = -(-groups // g)
            fill = groups / (rounds * g) if groups else 1.0
            if best is None or fill > best[0] + 1e-9:
                best = (fill, arr, g)
            if fill >= 1.0:
                break
        if best[0] >= 1.0:
            break
    return best[1], best[2]


def block_major(per_block, kg=1):
    k = max(len(b) for b in per_block)
    k = -(-k // kg) * kg
    arr = np.zeros(len(per_block) * k, PIECE)
    for b, lst in enumerate(per_block):
        for j, p in enumerate(lst):
            arr[b * k + j] = (p[0], p[1], p[2], p[3], 0)
    return arr, len(per_block)


def rr(pieces, g, kg=1):
    per = [[] for _ in range(min(g, len(pieces)))]
    for i, p in enumerate(pieces):
        per[i % len(per)].append(p)
    return block_major(per, kg)


def by_alloc(arr, ptrs):
    """arr (a fa_rows_plan table) with its wide pieces, then its narrow pieces, each sorted by the
    address of client 0's bytes of the piece; pieces[0].aux = the wide count, as the kernel reads."""
    nw = int(arr[0]["aux"]) if len(arr) else 0
    addr = ptrs[arr["seg"], 0] + arr["seg_off"] * 4
    out = arr.copy()
    for lo, hi in ((0, nw), (nw, len(arr))):
        out[lo:hi] = arr[lo + np.argsort(addr[lo:hi], kind="stable")]
    out["aux"] = 0
    if len(out):
        out[0]["aux"] = nw
    return out


def lib_plan(segs, g):
    L = na.load()
    cols = np.array([c for c, _ in segs], np.int64)
    lens = np.array([n for _, n in segs], np.int64)
    cnt, gg = ctypes.c_int64(), ctypes.c_int32()
    na.check(L.fa_rows_plan(len(segs), cols.ctypes.data, lens.ctypes.data, 0, g, None, 0, ctypes.byref(cnt),
                            ctypes.byref(gg)), "plan")
    arr = np.zeros(cnt.value, PIECE)
    na.check(L.fa_rows_plan(len(segs), cols.ctypes.data, lens.ctypes.data, 0, g, arr.ctypes.data, cnt.value,
                            ctypes.byref(cnt), ctypes.byref(gg)), "plan")
    return arr, gg.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--alloc", default="views", choices=("views", "clones", "stack"))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--only", default="", help="comma list of kernel-name substrings ('lib' adds the library plan)")
    ap.add_argument("--trace", action="store_true", help="per-block claim timeline of the product plan, then exit")
    ap.add_argument("--plans", default="", help="comma list of PC:GRID piece-width/grid plans run through the "
                    "product kernel (fa_reduce_f32_rows) beside its own plan")
    a = ap.parse_args()
    L = na.lib()
    name, n = CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    if name.startswith("flat:"):  # one (or k) equal fp32 tensors per client: every piece full width
        m, _, k = name[5:].partition("x")
        layout = [(f"t{i}", (int(m),), "f32") for i in range(int(k or 1))]
    else:
        layout = [x for x in layouts.get(name) if x[2] == "f32"]
    stride = layouts.padded_f32_stride(layout)
    p = layouts.fp32_elems(layout)
    x = torch.empty((n, stride), dtype=torch.float32, device=dev)
    agg.fill_uniform(x, seed=7)
    segs, off = [], 0
    for k, shape, _ in layout:
        m = int(np.prod(shape, dtype=np.int64))
        segs.append((off, m))
        off += -(-max(m, 1) // 64) * 64
    ptrs = np.empty((len(segs), n), np.int64)
    keep = []
    for i in range(n):
        if a.alloc == "stack":  # the row pointers point into the client stack itself
            for j, (c0, m) in enumerate(segs):
                ptrs[j, i] = x[i, c0:].data_ptr()
        elif a.alloc == "views":
            buf = torch.empty((1, stride), dtype=torch.float32, device=dev)
            agg.fill_uniform(buf, seed=7, row_begin=i)
            for j, (c0, m) in enumerate(segs):
                ptrs[j, i] = buf[0, c0:].data_ptr()
            keep.append(buf)
        else:
            for j, (c0, m) in enumerate(segs):
                t = x[i, c0 : c0 + m].clone()
                ptrs[j, i] = t.data_ptr()
                keep.append(t)
    ptr_d = torch.from_numpy(ptrs.reshape(-1)).to(dev)
    w = torch.ones(n, dtype=torch.float32, device=dev)
    want = torch.empty(stride, dtype=torch.float32, device=dev)
    agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=want)
    T = ctypes.CDLL(str(TUNE_LIB))
    T.tune_rows_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p,
                                   ctypes.c_void_p]
    work = torch.zeros(1, dtype=torch.int32, device=dev)
    # name -> (kernel variant (V, D, W), piece chunks)
    kernels = {"v8d2w4_c32": (0, 32), "v16d1w4_c64": (1, 64), "v8d1w8_c64": (2, 64), "v8d2w8_c64": (3, 64),
               "v8d4w4_c32": (4, 32), "v4d4w4_c16": (5, 16), "v4d2w8_c32": (6, 32), "v16d2w4_c64": (7, 64),
               "v8d2w4_c16": (0, 16), "v16d1w4_c32": (1, 32)}
    T.tune_rows_rm_launch.argtypes = T.tune_rows_launch.argtypes
    variants = {"stack": None, "lib": (None,) + lib_plan(segs, 0)}
    # the product plan with its pieces in ALLOCATION order (address of client
    # 0's bytes of the piece; wide pieces stay first, so groups are claimed the same way) instead
    # of largest first: do blocks streaming neighbouring addresses read the scattered uploads better?
    base, gb = lib_plan(segs, 0)
    variants["lib_alloc_order"] = (None, by_alloc(base, ptrs), gb)
    for spec in filter(None, a.plans.split(",")):
        pc, g = (int(x) for x in spec.split(":"))
        variants[f"plan_pc{pc}_g{g}"] = (None, product_plan(segs, pc), g)
    # row-major grouped kernel: pieces of 64 KiB, largest first, pieces[0].aux = the wide ones
    # name -> (kernel variant, waves, piece chunks = V * W KiB per row)
    rm_kernels = {"rm_v8w8kg2": (0, 8, 64), "rm_v8w8kg3": (1, 8, 64), "rm_v8w8kg4": (2, 8, 64),
                  "rm_v16w4kg2": (3, 4, 64), "rm_v8w8kg2ds2": (4, 8, 64), "rm_v8w8kg4ds2": (5, 8, 64),
                  "rm_v16w4kg2ds2": (6, 4, 64), "rm_v4w8kg4ds2": (7, 8, 32), "rm_v4w8kg4ds4": (8, 8, 32),
                  "rm_v8w8kg2sg": (9, 8, 64), "rm_v16w4kg2sg": (10, 4, 64), "rm_v8w8kg3sg": (11, 8, 64),
                  "rm_v8w8kg2pf2": (12, 8, 64), "rm_v8w8kg2pf4": (13, 8, 64), "rm_v8w8kg2pf8": (14, 8, 64),
                  "rm_v16w4kg2pf4": (15, 4, 64), "rm_v8w8kg2lt": (16, 8, 64), "rm_v16w4kg2lt": (17, 4, 64),
                  "rm_v8w8kg2ds2lt": (18, 8, 64), "rm_v8w8kg3lt": (19, 8, 64)}
    for kname, (kid, wv, pchunks) in rm_kernels.items():
        if a.only and not any(o in kname for o in a.only.split(",")):
            continue
        kg = int(kname.split("kg")[1][0])
        arr, g = filled_plan(segs, kg, pchunks, wv)
        variants[f"{kname}_filled_g{g}"] = (100 + kid, arr, min(g, len(arr)))
    for kname, (kid, c) in kernels.items():
        if a.only and not any(o in kname for o in a.only.split(",")):
            continue
        pcs = sorted(cut(segs, c), key=lambda q: -q[3])
        for g in (192, 256, 384):
            arr = np.zeros(len(pcs), PIECE)
            for i, q in enumerate(pcs):
                arr[i] = (q[0], q[1], q[2], q[3], 0)
            variants[f"{kname}_g{g}"] = (kid, arr, min(g, len(pcs)))
    dev_tabs = {k: (v[0], torch.from_numpy(v[1].view(np.uint8)).to(dev), len(v[1]), v[2])
                for k, v in variants.items() if v}
    if a.trace:
        out = torch.empty(stride, dtype=torch.float32, device=dev)
        _trace(T, dev_tabs["lib"], ptr_d, n, w, work, out, dev, na.stream_handle(dev), segs, variants["lib"][1])
        return
    out = torch.empty(stride, dtype=torch.float32, device=dev)
    stream = na.stream_handle(dev)

    def launch(k):
        if k == "stack":
            agg.reduce_stack(x, w, na.MODE_W32_DIV64, float(n), out32=out)
            return
        kid, t, cnt, g = dev_tabs[k]
        if kid is None:
            na.check(L.fa_reduce_f32_rows(ptr_d.data_ptr(), n, na.MODE_W32_DIV64, w.data_ptr(), float(n), t.data_ptr(),
                                          cnt, g, work.data_ptr(), None, out.data_ptr(), None, stream), k)
            return
        fn = T.tune_rows_rm_launch if kid >= 100 else T.tune_rows_launch
        rc = fn(kid % 100, ptr_d.data_ptr(), n, w.data_ptr(), t.data_ptr(), cnt, g, work.data_ptr(), float(n),
                out.data_ptr(), stream)
        assert rc == 0, (k, rc)

    times = {k: [] for k in variants}
    for k in variants:  # check
        out.zero_()
        launch(k)
        torch.cuda.synchronize()
        assert torch.equal(out[:p].view(torch.int32), want[:p].view(torch.int32)) or k == "stack" or \
            _segments_equal(out, want, segs), k
    for _ in range(a.reps):
        for k in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            launch(k)
            e0.record()
            for _ in range(a.steps):
                launch(k)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.steps * 1e3)
    algo = n * p * 4 + p * 4
    for k, ts in times.items():
        print(json.dumps({"config": a.config, "alloc": a.alloc, "variant": k, "us_min": round(min(ts), 1),
                          "us_med": round(float(np.median(ts)), 1), "frac": round(algo / min(ts) / 8e6, 4)}), flush=True)


def _trace(T, tab, ptr_d, n, w, work, out, dev, stream, segs, plan):
    """Claim timeline of the product kernel on the product plan: when each block starts each of
    its claims, how many it made, when it exits (us from the first block's first claim)."""
    T.tune_rows_rm_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]
    _, t, cnt, g = tab
    nwide = int(plan[0]["aux"]) if len(plan) else 0
    print(json.dumps({"pieces": int(cnt), "wide": nwide, "groups": (nwide + 1) // 2, "narrow": int(cnt) - nwide,
                      "grid": g, "wide_cols": [int(x) for x in np.unique(plan["n_cols"][:nwide])][:8]}), flush=True)
    for rep in range(3):
        tr = torch.zeros(g * 32, dtype=torch.int64, device=dev)
        rc = T.tune_rows_rm_trace(ptr_d.data_ptr(), n, w.data_ptr(), t.data_ptr(), cnt, g, work.data_ptr(), float(n),
                                  out.data_ptr(), tr.data_ptr(), stream)
        assert rc == 0
        torch.cuda.synchronize()
        h = tr.view(g, 32).cpu().numpy().astype(np.float64)
        t0 = h[:, 1][h[:, 1] > 0].min()
        nclaim = h[:, 31].astype(int)
        end = (h[:, 0] - t0) / 100.0
        starts = [(h[b, 1 : 1 + min(nclaim[b], 30)] - t0) / 100.0 for b in range(g)]
        first_narrow = []
        q = lambda x: [round(float(np.percentile(x, p)), 1) for p in (0, 10, 50, 90, 100)]
        print(json.dumps({"rep": rep, "claims_per_block": np.bincount(nclaim).tolist(),
                          "end_us_p0_10_50_90_100": q(end),
                          "claim2_start_us": q([s[1] for s in starts if len(s) > 1]),
                          "claim3_start_us": q([s[2] for s in starts if len(s) > 2]),
                          "last_claim_start_us": q([s[-1] for s in starts if len(s)])}), flush=True)


def _segments_equal(out, want, segs):
    o, w = out.cpu().numpy().view(np.uint32), want.cpu().numpy().view(np.uint32)
    return all(np.array_equal(o[c : c + m], w[c : c + m]) for c, m in segs)


if __name__ == "__main__":
    main()
