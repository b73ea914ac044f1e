"""Can the aggregation reduce and a collective overlap on one MI355X?  

The multi-GPU pipeline (flearn_amd.dist) overlaps stripe c's RCCL all-gather with stripe c+1's
reduce; its model (StripeModel) assumed the two do not slow each other down.  On the one-GPU box
this measures it: the product's fp32 reduce of a device-resident client stack runs on one stream
while a stand-in for the gather's traffic runs on another —

  * `copy B`: a 16-B grid-stride copy kernel on B blocks (tools/probe_copy.hip): RCCL's kernels
    occupy CUs and move data through HBM; a local copy reads AND writes local HBM, so at equal
    rate it is the pessimistic side of a gather (which only writes the received bytes here);
  * `dma`: hipMemcpyAsync device-to-device (torch copy_): no reduce-visible CU use if the
    runtime picks a DMA engine.

for reduce grids from the library's default (192 blocks on 256 CUs) up to one block per CU and
down (fa_set_reduce_grid): each pair alone, then concurrently (both start on one event), median
of --reps.  Prints one JSON object: per (grid, copy) the reduce time alone / concurrent, the copy
rate alone / concurrent and the reduce's slowdown factor — the contention term StripeModel uses.

    python tools/overlap_probe.py [--config ns] [--grids 0,256,224,192,160] [--copy 16,32,64,dma]
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

LAYOUTS = {"ns": ("resnet50", 100), "c2": ("resnet18", 100), "c5": ("vit_b_16", 100)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns", choices=sorted(LAYOUTS))
    ap.add_argument("--grids", default="0,256,224,192,160")
    ap.add_argument("--copy", default="16,32,64,dma")
    ap.add_argument("--copy-mb", type=int, default=256, help="bytes of one copy launch")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--push-cus", type=int, default=0,
                    help="run the copy stream on this many CUs only (a CU-masked stream), spread evenly")
    ap.add_argument("--mask-reduce", action="store_true",
                    help="with --push-cus: the reduce's stream gets the other CUs (disjoint masks)")
    ap.add_argument("--push-cu-layout", default="spread", choices=["spread", "low"],
                    help="which CUs the copy stream gets: every (CUs/K)-th, or the lowest K")
    ap.add_argument("--keep-streams", action="store_true",
                    help="leave the CU-masked streams alive at exit (round 5's behaviour: a SIGSEGV in "
                         "__cxa_finalize under rocprofv3, DESIGN.md section 7)")
    a = ap.parse_args()
    L = ctypes.CDLL(str(REPO / "tools" / "libprobe_copy.so"))
    L.probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
    L.probe_copy.restype = ctypes.c_int
    L.probe_copy_rep.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                 ctypes.c_void_p]
    L.probe_copy_rep.restype = ctypes.c_int
    L.probe_spin.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    L.probe_spin.restype = ctypes.c_int
    L.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    L.probe_read.restype = ctypes.c_int
    L.probe_write.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
    L.probe_write.restype = ctypes.c_int
    L.probe_blit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.probe_blit.restype = ctypes.c_int
    na.lib()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    name, n = LAYOUTS[a.config]
    p = layouts.padded_f32_stride(layouts.get(name))
    stack = torch.empty((n, p), dtype=torch.float32, device=dev)
    agg.fill_uniform(stack, seed=2024)
    w = torch.ones(n, dtype=torch.float32, device=dev)
    out = torch.empty(p, dtype=torch.float32, device=dev)
    nbytes = a.copy_mb << 20
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    masks = None
    created = []  # CU-masked streams this probe made: destroyed before exit
    if a.push_cus:
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        words = (ncu + 31) // 32
        step = ncu // a.push_cus
        cus = ([i * step for i in range(a.push_cus)] if a.push_cu_layout == "spread" else list(range(a.push_cus)))
        mb, ma = [0] * words, [0] * words
        for c in range(ncu):
            (mb if c in cus else ma)[c // 32] |= 1 << (c % 32)
        L.probe_stream_cumask.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
        L.probe_stream_cumask_get.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32)]

        def masked(m):
            h = ctypes.c_void_p()
            assert L.probe_stream_cumask((ctypes.c_uint32 * words)(*m), words, ctypes.byref(h)) == 0
            got = (ctypes.c_uint32 * words)()
            assert L.probe_stream_cumask_get(h, words, got) == 0
            created.append(h.value)
            return torch.cuda.ExternalStream(h.value, device=dev), [int(x) for x in got]

        sb, got_b = masked(mb)
        masks = {"copy_cus": cus, "copy_mask_read_back": [hex(x) for x in got_b]}
        if a.mask_reduce:
            sa, got_a = masked(ma)
            masks["reduce_mask_read_back"] = [hex(x) for x in got_a]
    alg_bytes = n * p * 4 + p * 4

    def reduce():
        with torch.cuda.stream(sa):
            agg.reduce_stack(stack, w, na.MODE_W32_DIV64, float(n), out32=out)

    small = torch.empty(1 << 19, dtype=torch.float32, device=dev).fill_(1.0)  # 2 MiB: stays in L2
    small_dst = torch.empty_like(small)
    spin_out = torch.empty(256 * 256, dtype=torch.float32, device=dev)

    sink = torch.empty(4096 * 256 * 4, dtype=torch.int32, device=dev)
    host_dst = None

    def copy_fn(kind):
        nonlocal host_dst
        if kind.startswith("rd"):  # HBM reads only
            blocks = int(kind[2:])

            def f():
                assert L.probe_read(src.data_ptr(), nbytes // 16, blocks, sink.data_ptr(), sb.cuda_stream) == 0
            return f
        if kind.startswith("wr"):  # HBM writes only
            blocks = int(kind[2:])

            def f():
                assert L.probe_write(dst.data_ptr(), nbytes // 16, blocks, sb.cuda_stream) == 0
            return f
        if kind.startswith("spin"):  # ALU only, no memory traffic: do CUs / dispatch interfere?
            blocks = int(kind[4:])

            def f():
                assert L.probe_spin(spin_out.data_ptr(), blocks, 200000, sb.cuda_stream) == 0
            return f
        if kind.startswith("l2copy"):  # cache-resident copy: CU + L2 traffic, no HBM
            blocks = int(kind[6:])

            def f():
                assert L.probe_copy_rep(small_dst.data_ptr(), small.data_ptr(), small.numel() // 4, blocks, 64,
                                        sb.cuda_stream) == 0
            return f
        if kind.startswith("pushhost"):  # fa_push into pinned host memory: a LINK-bound push kernel (PCIe
            # standing in for an xGMI link), which reads its source once from local HBM and
            # writes nothing to it — the sender's side of the one-shot push gather
            if host_dst is None:
                host_dst = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
            Lf = na.lib()
            dsts = (ctypes.c_void_p * 1)(host_dst.data_ptr())
            pgrid = int(kind[8:] or 0)  # pushhost<B>: B blocks (none: the library's default)

            def f():
                assert Lf.fa_push(src.data_ptr(), nbytes, dsts, 1, pgrid, sb.cuda_stream) == 0
            return f
        if kind.startswith("cphost") or kind == "blithost":  # a plain 16-B copy kernel (probe_copy16,
            # cphost<B>: B blocks of 256) or the runtime's blit kernel (hipMemcpyDeviceToDevice) into
            # pinned host memory: which store pattern lets a link-bound copy leave the reduce alone?
            if host_dst is None:
                host_dst = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
            blocks = int(kind[6:]) if kind.startswith("cphost") else 0

            def f():
                if blocks:
                    assert L.probe_copy(host_dst.data_ptr(), src.data_ptr(), nbytes // 16, blocks, sb.cuda_stream) == 0
                else:
                    assert L.probe_blit(host_dst.data_ptr(), src.data_ptr(), nbytes, sb.cuda_stream) == 0
            return f
        if kind.startswith("paced"):  # paced<U>x<B>: the paced push stand-in into pinned host memory,
            # U quads per lane per round, B blocks, each wave's stores drained before its next loads
            if host_dst is None:
                host_dst = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
            u, b = (int(x) for x in kind[5:].split("x"))
            L.probe_push_paced.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_void_p]

            def f():
                assert L.probe_push_paced(host_dst.data_ptr(), src.data_ptr(), nbytes // 16, b, u, sb.cuda_stream) == 0
            return f
        if kind == "dmahost":  # a copy engine moving device memory to pinned host memory over PCIe:
            # the sender's side of the copy-engine push (an SDMA leg over a link)
            if host_dst is None:
                host_dst = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
            Ld = na.lib()

            def f():
                assert Ld.fa_copy_dma(host_dst.data_ptr(), src.data_ptr(), nbytes, sb.cuda_stream) == 0
            return f
        if kind == "dmadev":  # a copy engine (fa_copy_dma, NoCU) between two device buffers: the
            # sender's side of the copy-engine push with an HBM destination standing in for a peer's
            def f():
                assert na.lib().fa_copy_dma(dst.data_ptr(), src.data_ptr(), nbytes, sb.cuda_stream) == 0
            return f
        if kind == "dma":
            def f():
                with torch.cuda.stream(sb):
                    dst.copy_(src, non_blocking=True)
            return f
        blocks = int(kind)

        def f():
            rc = L.probe_copy(dst.data_ptr(), src.data_ptr(), nbytes // 16, blocks, sb.cuda_stream)
            assert rc == 0, rc
        return f

    def timed(fn, stream, reps=1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e3  # us

    def together(k, cfn):
        """reduce on sa, k copies on sb, both released by one event; (reduce us, copies us)."""
        go = torch.cuda.Event()
        torch.cuda.current_stream(dev).synchronize()
        ea0, ea1, eb0, eb1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        go.record(torch.cuda.current_stream(dev))
        sa.wait_event(go)
        sb.wait_event(go)
        ea0.record(sa)
        eb0.record(sb)
        reduce()
        for _ in range(k):
            cfn()
        ea1.record(sa)
        eb1.record(sb)
        torch.cuda.synchronize(dev)
        return ea0.elapsed_time(ea1) * 1e3, eb0.elapsed_time(eb1) * 1e3

    res = {"config": a.config, "clients": n, "cols": p, "copy_bytes": nbytes, "device": torch.cuda.get_device_name(0),
           "cu_masks": masks,
           "cus": torch.cuda.get_device_properties(0).multi_processor_count, "rows": []}
    kinds = [k.strip() for k in a.copy.split(",") if k.strip()]
    for g in [int(x) for x in a.grids.split(",")]:
        agg.set_reduce_grid(g)
        for _ in range(2):
            timed(reduce, sa)
        alone = float(np.median([timed(reduce, sa) for _ in range(a.reps)]))
        row = {"grid": g or "default", "reduce_us": round(alone, 1),
               "reduce_gbs": round(alg_bytes / alone / 1e3, 1), "with": {}}
        for kind in kinds:
            cfn = copy_fn(kind)
            for _ in range(2):
                timed(cfn, sb)
            c_alone = float(np.median([timed(cfn, sb) for _ in range(a.reps)]))
            k = max(1, int(round(alone / c_alone)))  # copies spanning about the reduce's time
            pairs = [together(k, cfn) for _ in range(a.reps)]
            r_c = float(np.median([x for x, _ in pairs]))
            c_c = float(np.median([y for _, y in pairs]))
            row["with"][kind] = {
                "copy_alone_us": round(c_alone, 1), "copy_alone_gbs": round(nbytes / c_alone / 1e3, 1),
                "copies": k, "reduce_concurrent_us": round(r_c, 1), "copies_concurrent_us": round(c_c, 1),
                "copy_concurrent_gbs": round(k * nbytes / c_c / 1e3, 1),
                "reduce_slowdown": round(r_c / alone, 4), "copy_slowdown": round(c_c / (k * c_alone), 4),
            }
            print(f"grid {g or 'default'} copy {kind}: reduce {alone:.1f} -> {r_c:.1f} us, "
                  f"copy {k} x {c_alone:.1f} -> {c_c:.1f} us", file=sys.stderr, flush=True)
        res["rows"].append(row)
    agg.set_reduce_grid(0)
    res["note"] = ("copy GB/s counts bytes copied (each read once and written once locally); a gather's local "
                   "HBM traffic at the same GB/s is about half of the copy's")
    print(json.dumps(res), flush=True)
    if created and not a.keep_streams:
        # a hipStream the runtime did not make for torch must be destroyed by its maker, before
        # the HIP runtime's own static teardown (ExternalStream never destroys what it wraps)
        torch.cuda.synchronize(dev)
        sa = sb = None
        L.probe_stream_destroy.argtypes = [ctypes.c_void_p]
        for h in created:
            assert L.probe_stream_destroy(h) == 0
        print(f"destroyed {len(created)} CU-masked stream(s)", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
