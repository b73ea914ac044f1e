"""Does the stripe pipeline overlap the way the model assumes?  (round 5)

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe -o pipe -- \
        python3 tools/trace_pipeline.py --gather push --stripes 4
    python3 tools/trace_pipeline.py --analyze gpurun_out/pipe/.../pipe_kernel_trace.csv

One process, a 1-rank RCCL group on cuda:0, the NS stack (100 x ResNet-50 columns), and
flearn_amd.dist.ShardedReducer over S stripes with the gather named (`rccl`: RCCL's all-gather on
its own stream; `push` / `push_dma`: the one-shot push, which at world 1 is this rank's own copy
into its receive bucket).  Several steps, then --analyze reads the kernel trace: per step, the
reduce launches on the compute stream, the gather's kernels on the other streams, and how much of
each gather ran while a reduce was running — the stripe c gather beside the stripe c+1 reduce the
StripeModel prices.  At world 1 no link is crossed: this shows the streams' structure, not xGMI.
Measurement infrastructure, not the product.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def run(a):
    import tempfile

    import torch
    import torch.distributed as dist

    from flearn_amd import _native as na
    from flearn_amd import aggregator as agg
    from flearn_amd import dist as fd
    from flearn_amd import layouts

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_pipe_"), "pg")
    kw = {}
    if a.nccl_high:  # RCCL's internal stream from the high-priority pool
        kw["pg_options"] = dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)
    dist.init_process_group("nccl", init_method=init, rank=0, world_size=1, device_id=dev, **kw)
    try:
        p = a.cols or layouts.padded_f32_stride(layouts.get("resnet50"))
        n = a.clients
        plan = fd.ShardPlan.make(p, 1, 0, stripes=a.stripes)
        stack = torch.empty((n, plan.local_cols), dtype=torch.float32, device=dev)
        agg.fill_uniform(stack, seed=2024)
        w = torch.ones(n, dtype=torch.float32, device=dev)
        push = {"rccl": False, "push": True, "push_dma": "dma"}[a.gather]
        fd._PUSH_ORDER = a.order  # auto (the product), host, or producer (a device-side event wait)
        red = fd.ShardedReducer(plan, fd.hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n)), dev, gather=True,
                                push=push)
        if red.pusher is not None and a.pusher_stream != "default":
            red.pusher.stream = new_stream(a.pusher_stream, dev)
            if red.pusher.peer_streams:
                import ctypes

                red.pusher.peer_streams = [new_stream(a.pusher_stream, dev) for _ in red.pusher.peer_streams]
                red.pusher._peer_handles = (ctypes.c_void_p * len(red.pusher.peer_streams))(
                    *[x.cuda_stream for x in red.pusher.peer_streams])
        for _ in range(2):
            red.step()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            red.step()
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / a.steps
        red.release()
        fd.shutdown_push()
        print(json.dumps({"gather": a.gather, "stripes": a.stripes, "clients": n, "cols": p, "steps": a.steps,
                          "pusher_stream": a.pusher_stream, "nccl_high": a.nccl_high, "order": a.order,
                          "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "ms_per_step": round(ms, 4)}))
    finally:
        dist.destroy_process_group()


def new_stream(kind: str, dev):
    """A stream for the gather: `normal` — a normal-priority torch stream (the product's stream
    before round 5's fix: it may share the compute stream's hardware queue); `high` — the
    product's side stream (flearn_amd.streams.side_stream).  (A stream created with a CU mask of
    every CU also got a queue of its own, but its process crashed at exit under the profiler.)"""
    import torch

    return torch.cuda.Stream(dev, priority=-1 if kind == "high" else 0)


def analyze(path: str):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Stream_Id"])) for r in rows]
    queue = {(int(r["Start_Timestamp"]), r["Kernel_Name"]): int(r["Queue_Id"]) for r in rows}
    red = sorted(k for k in ks if "reduce_kernel" in k[2])
    if red:  # the pipeline's window: from the first reduce on (set-up copies before it are not gathers)
        ks = [k for k in ks if k[0] >= red[0][0] - 1000]
    gat = sorted(k for k in ks if ("push_kernel" in k[2] or "copy_kernel" in k[2] or "nccl" in k[2].lower()
                                   or "rccl" in k[2].lower() or "copyBuffer" in k[2]))
    if not red:
        return {"error": "no reduce kernels in the trace"}

    def overlap(a0, a1):
        return sum(max(0, min(a1, r1) - max(a0, r0)) for r0, r1, _, _ in red)

    g_total = sum(g1 - g0 for g0, g1, _, _ in gat)
    g_beside = sum(overlap(g0, g1) for g0, g1, _, _ in gat)
    names = sorted({k[2][:60] for k in gat})
    return {"reduce_queues": sorted({queue[(k[0], k[2])] for k in red}),
            "gather_queues": sorted({queue[(k[0], k[2])] for k in gat}),
            "reduce_launches": len(red), "reduce_streams": sorted({k[3] for k in red}),
            "gather_launches": len(gat), "gather_streams": sorted({k[3] for k in gat}), "gather_kernels": names,
            "gather_us_total": round(g_total / 1e3, 1), "gather_us_beside_a_reduce": round(g_beside / 1e3, 1),
            "gather_frac_beside_a_reduce": round(g_beside / g_total, 3) if g_total else None,
            "reduce_us_total": round(sum(r1 - r0 for r0, r1, _, _ in red) / 1e3, 1),
            "first_step": [{"kernel": k[2][:40], "stream": k[3], "start_us": round((k[0] - red[0][0]) / 1e3, 1),
                            "dur_us": round((k[1] - k[0]) / 1e3, 1)}
                           for k in sorted(red + gat)[: 2 * 8]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gather", default="push", choices=["rccl", "push", "push_dma"])
    ap.add_argument("--stripes", type=int, default=4)
    ap.add_argument("--order", default="auto", choices=["auto", "host", "producer"],
                    help="how each stripe's push follows its reduce (flearn_amd.dist._PUSH_ORDER; auto: the "
                         "product's — producer for the kernel push, host for the copy-engine push)")
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--cols", type=int, default=0, help="columns of the stack (0: NS, 100 x ResNet-50; "
                    "a multi-GPU rank's share, e.g. 3201280 for NS at G = 8)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--analyze", default=None, help="a rocprofv3 kernel_trace.csv of a run")
    ap.add_argument("--pusher-stream", default="default", choices=["default", "normal", "high"],
                    help="default: as the product creates it (high priority since round 5)")
    ap.add_argument("--nccl-high", action="store_true", help="RCCL's stream from the high-priority pool")
    a = ap.parse_args()
    if a.analyze:
        print(json.dumps(analyze(a.analyze), indent=1))
    else:
        run(a)


if __name__ == "__main__":
    main()
