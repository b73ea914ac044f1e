"""Do the copy-engine push's legs run at once?

    rocprofv3 --memory-copy-trace --kernel-trace --stats -d gpurun_out/dma -o legs -- \
        python3 tools/probe_dma_legs.py --legs 7 --mib 64 --out gpurun_out/dma/legs.json

PushGather(mode="dma") issues one hipMemcpyAsync per peer, each on its own stream, behind one
event of the stripe's reduce (C ABI fa_push_dma).  On one GPU there are no peers; the legs go to
`legs` pinned host buffers instead (every leg then crosses the same PCIe link, so what the trace
answers is whether the copies' INTERVALS overlap — the engines run at once, sharing the link — or
follow each other — one engine / one queue at a time), and, second, to `legs` device buffers
(same-device copies).  Timed with HIP events on the pusher's stream: one leg alone, then all
legs through fa_push_dma + fa_stream_join.  Measurement infrastructure, not the product.

Time it WITHOUT a profiler: under rocprofv3 the runtime routes these copies differently (kernel
trace: copy kernels; memory-copy trace: ~60 GB/s per engine), so a traced run says which path
ran, not how fast ("The copy paths, traced and untraced").
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
    import torch

    from flearn_amd import _native as na

    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", type=int, default=7)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/dma/legs.json")
    args = ap.parse_args()
    L = na.lib()
    dev = torch.device("cuda", 0)
    n = args.mib << 20
    src = torch.empty(n // 4, dtype=torch.float32, device=dev).uniform_()
    main_s = torch.cuda.Stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(args.legs)]
    handles = (ctypes.c_void_p * args.legs)(*[s.cuda_stream for s in streams])
    out = {"legs": args.legs, "bytes_per_leg": n, "device": torch.cuda.get_device_name(0)}

    def timed(fn, reps):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            fn()
            e1.record(main_s)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / 1e3)
        ts.sort()
        return ts[len(ts) // 2]

    for kind in ("pinned_host", "device"):
        if kind == "pinned_host":
            dsts = [torch.empty(n // 4, dtype=torch.float32, pin_memory=True) for _ in range(args.legs)]
        else:
            dsts = [torch.empty(n // 4, dtype=torch.float32, device=dev) for _ in range(args.legs)]
        ptrs = (ctypes.c_void_p * args.legs)(*[d.data_ptr() for d in dsts])
        for path in ("engine", "blit"):
            # engine: the product's legs (fa_copy_dma / fa_push_dma: hipMemcpyDeviceToDeviceNoCU);
            # blit: the same copies through torch (hipMemcpyDeviceToDevice-style: a copy kernel)
            def one(path=path):
                if path == "engine":
                    na.check(L.fa_copy_dma(dsts[0].data_ptr(), src.data_ptr(), n, main_s.cuda_stream), "fa_copy_dma")
                else:
                    with torch.cuda.stream(main_s):
                        dsts[0].copy_(src, non_blocking=True)

            def all_legs(k=args.legs, path=path):
                if path == "engine":
                    na.check(L.fa_push_dma(src.data_ptr(), n, ptrs, k, handles, main_s.cuda_stream), "fa_push_dma")
                    na.check(L.fa_stream_join(main_s.cuda_stream, handles, k), "fa_stream_join")
                else:
                    for i in range(k):
                        streams[i].wait_stream(main_s)
                        with torch.cuda.stream(streams[i]):
                            dsts[i].copy_(src, non_blocking=True)
                    for i in range(k):
                        main_s.wait_stream(streams[i])

            one()
            all_legs()
            t1 = timed(one, args.reps)
            res = {"one_leg_ms": round(t1 * 1e3, 4), "one_leg_gbs": round(n / t1 / 1e9, 2)}
            for k in sorted({2, 4, args.legs}):
                if k > args.legs:
                    continue
                tk = timed(lambda k=k: all_legs(k), args.reps)
                res[f"legs{k}_ms"] = round(tk * 1e3, 4)
                res[f"legs{k}_gbs_total"] = round(k * n / tk / 1e9, 2)
                # 1.0: the legs took as long as one leg (concurrent, no shared bottleneck); k: k
                # times one leg (serial, or concurrent but sharing one link)
                res[f"legs{k}_over_one"] = round(tk / t1, 3)
            torch.cuda.synchronize(dev)
            ok = all(torch.equal(d.to(dev) if kind == "pinned_host" else d, src) for d in dsts)
            for d in dsts:
                d.zero_()
            res["copies_correct"] = bool(ok)
            out[f"{kind}_{path}"] = res
        del dsts
        torch.cuda.empty_cache()
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
