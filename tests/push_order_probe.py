"""Are the push gather's copies ordered after the stripe's reduce when the pusher's streams have
their own hardware queue?  (rounds 5-6)

    python tests/push_order_probe.py --world 8 --steps 3 --reps 6 --priorities normal,high,product \
        --dma-orders host,producer,chain [--forensic]

(round 5: with the copy-engine push's pusher stream at high priority, 32 of 576 in-place Adagrad
rank-steps were wrong.  Round 6: with every push stream at high priority the copy-engine legs AND
the pusher's own-copy kernel copied stripes before their reduce had finished, whatever the
device-side order — `--dma-orders chain` (round 5: an event of the pusher's stream), `producer` (an
event of the reduce's own stream), with L2 fences (or, in round 6's first build, one-wave gate kernels
around each leg) — while `host`, the product's
order now, issues each stripe's legs only after the host has seen its reduce complete.  "high" puts
the pusher's stream AND every leg's stream at high priority: none of them shares the compute
stream's hardware queue; "hipusher" / "hipeers" only one side)

`world` processes share cuda:0 over gloo (like tests/test_gpu_multirank.py); each runs
ShardedReducer steps with the fused Adagrad epilogue in place (the reduce reads `prev` and writes
the new model over it; the pushes read that model) under four stripe plans, with the pusher's
streams at normal priority (may share the compute stream's hardware queue) or high priority (a
queue of their own: flearn_amd.streams.side_stream), and compares every step's bucket with the C
oracle.  For a mismatch it records which ranks' slices were wrong and whether the wrong values are
the PREVIOUS step's model (a copy that read its source before the reduce had written it) or
something else.  Prints one JSON object.  Test infrastructure (it checks against the C oracle, so it
lives under tests/), run by tools/gpu_run.sh push_order and by tests/test_gpu_multirank.py.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def _worker(rank, world, port, modes, priorities, steps, reps, out_path, dma_orders=("host",), fences=("none",),
            forensic=False, compute="default", kernel_orders=("-",)):
    import numpy as np
    import torch
    import torch.distributed as dist

    import oracle
    from flearn_amd import _native as na
    from flearn_amd import aggregator as agg
    from flearn_amd import dist as fd
    from flearn_amd.dist import ShardedReducer, ShardPlan, StripeModel, hip_reduce_fn, plan_shards, plan_stripes

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cuda = torch.device("cuda", 0)
    n, p = 9, 700_001
    lc = -(-p // world)
    widths, rep = plan_shards(p, world, StripeModel(1e-6, 2e-9, 2e-6, 1e-8))
    plans = [ShardPlan.make(p, world, rank, 1), ShardPlan.make(p, world, rank, 2, weights=(3, 1)),
             ShardPlan.from_widths(p, world, rank, plan_stripes(lc, StripeModel.assumed(n, world))),
             ShardPlan.from_widths(p, world, rank, widths, rep=rep)]
    w_h = np.linspace(0.5, 1.5, n).astype(np.float32)
    denom = float(np.sum([float(x) for x in w_h]))
    want_mean = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(n, p, 3), w_h, denom)
    results = []

    L = na.lib()

    def fence(kind):
        na.check(L.fa_cache_fence(kind, torch.cuda.current_stream(cuda).cuda_stream), "fa_cache_fence")

    def run_plans(mode, prio, rep, order, fen):
        for pi, plan in enumerate(plans):
            for op in ("mean", "adagrad"):  # the test's order (tests/multirank_worker.py)
                stack = torch.empty((n, plan.local_stride), dtype=torch.float32, device=cuda)
                for lo, g0, width in plan.segments():
                    agg.fill_uniform(stack[:, lo:], seed=3, col_begin=g0, n_cols=width)
                w = torch.from_numpy(w_h).to(cuda)
                epi, local_out = {}, None
                if op != "mean":
                    prev = torch.empty((1, plan.local_stride), dtype=torch.float32, device=cuda)
                    for lo, g0, width in plan.segments():
                        agg.fill_uniform(prev[:, lo:], seed=4, col_begin=g0, n_cols=width)
                    epi = dict(op=na.OP_BY_NAME["adagrad"], prev=prev[0],
                               v=torch.zeros(plan.local_stride, dtype=torch.float64, device=cuda))
                    local_out = prev[0]
                fn = hip_reduce_fn(stack, w, na.MODE_W32_DIV64, denom, **epi)
                if fen.split("+")[0] in ("release", "both"):  # L2 written back after every stripe's reduce
                    def fn(lo, sc, out, _f=fn):
                        _f(lo, sc, out)
                        fence(na.FENCE_RELEASE)
                red = ShardedReducer(plan, fn, cuda, local_out=local_out, gather=True,
                                     push="dma" if mode == "dma" else True)
                prev_h = oracle.fill_uniform(1, p, 4)[0]
                v_h = np.zeros(p)
                last = prev_h.astype(np.float32) if op != "mean" else want_mean.astype(np.float32)
                bad_steps = []
                if forensic:  # global column -> (owner rank, owner's local column) of the stripes
                    own_r = np.full(p, -1, dtype=np.int64)
                    own_l = np.zeros(p, dtype=np.int64)
                    for c in range(plan.stripes):
                        for r in range(world):
                            g0 = plan.global_begin(c, r)
                            w_ = max(0, min(plan.widths[c], p - g0))
                            own_r[g0 : g0 + w_] = r
                            own_l[g0 : g0 + w_] = plan.local_begin(c) + np.arange(w_)
                for step in range(steps):
                    if forensic:  # what each sender's source and this rank's bucket held before
                        src_snap = red.local_out.clone()
                        bkt_snap = red.full[:p].clone()
                    full = red.step()
                    if fen.split("+")[0] in ("acquire", "both"):  # L2 invalidated before the bucket is read
                        fence(na.FENCE_ACQUIRE)
                    full = full.cpu().numpy()
                    if forensic:
                        srcs = [None] * world
                        dist.all_gather_object(srcs, src_snap.cpu().numpy())
                        bkt_before = bkt_snap.cpu().numpy()
                    if op == "mean":
                        want = want_mean.astype(np.float32)
                    else:
                        want = oracle.c_update("adagrad", want_mean, prev_h, v_h).astype(np.float32)
                        prev_h = want
                    if full.tobytes() != want.tobytes():
                        bad = np.nonzero(full.view(np.uint32) != want.view(np.uint32))[0]
                        stale = int(np.sum(full[bad].view(np.uint32) == last[bad].view(np.uint32)))
                        owners = sorted({next((r for r in range(world) for c in range(plan.stripes)
                                               if plan.global_begin(c, r) <= b < plan.global_begin(c, r)
                                               + plan.widths[c]), -1) for b in bad[:: max(1, len(bad) // 64)]})
                        rec = {"step": step, "bad": int(len(bad)), "stale_prev_step": stale,
                               "owners": owners, "first": int(bad[0]), "last": int(bad[-1])}
                        if forensic:
                            u = lambda a: a.view(np.uint32)  # noqa: E731
                            ob = bad[own_r[bad] >= 0]
                            pre_src = np.array([srcs[own_r[b]][own_l[b]] for b in ob], dtype=np.float32)
                            rec["pushed_cols"] = int(len(ob))
                            # = the sender's source BEFORE this step's reduce: the leg read it early
                            rec["eq_sender_src_before"] = int(np.sum(u(full[ob]) == u(pre_src)))
                            # = this rank's bucket before the step: the leg had not landed
                            rec["eq_bucket_before"] = int(np.sum(u(full[bad]) == u(bkt_before[bad])))
                            time.sleep(0.05)
                            torch.cuda.synchronize()
                            again = red.full[:p].cpu().numpy()
                            # right when read again 50 ms later: the leg landed after the read
                            rec["right_when_reread"] = int(np.sum(u(again[bad]) == u(want[bad])))
                        bad_steps.append(rec)
                    last = want
                red.release()
                results.append({"priority": prio, "mode": mode, "order": order, "fence": fen, "rep": rep, "plan": pi,
                                "op": op,
                                "widths": list(plan.widths), "steps": steps, "bad_steps": bad_steps})
                del stack, red

    def explicit_registration(mode):
        """The test's last part: kernel mode registers a torch tensor (its caching-allocator
        segment is exported, then dropped), dma mode a pool bucket."""
        if mode == "kernel":
            full = torch.full((world * 4096,), -1.0, device=cuda)
            pg = fd.PushGather(full, None, mode=mode)
        else:
            pg = fd.PushGather(None, None, mode=mode, cols=world * 4096, device=cuda)
            full = pg.full
            full.fill_(-1.0)
        src = torch.arange(4096, dtype=torch.float32, device=cuda) + 10000.0 * rank
        pg.gather(src, rank * 4096)
        want = torch.empty_like(full)
        fd.all_gather_into(want, src)
        torch.cuda.synchronize()
        ok = bool(torch.equal(full, want))
        pg.close()
        return ok

    try:
        product = (fd.side_stream, fd.peer_stream)
        for prio in priorities:
            if prio == "product":  # the streams as flearn_amd.dist creates them
                fd.side_stream, fd.peer_stream = product
            else:  # "high": pusher and legs; "hipusher" / "hipeers": only that one at high priority
                hi, lo = (lambda dev: torch.cuda.Stream(dev, priority=-1)), (lambda dev: torch.cuda.Stream(dev, priority=0))
                fd.side_stream = hi if prio in ("high", "hipusher") else lo
                fd.peer_stream = hi if prio in ("high", "hipeers") else lo
            for rep in range(reps):
                for mode in modes:
                    for order in (dma_orders if mode == "dma" else kernel_orders):
                        fd._PUSH_ORDER = order if order != "-" else "auto"
                        for fen in fences:
                            if compute == "created":  # the whole job on a created compute stream
                                with torch.cuda.stream(torch.cuda.Stream(cuda)):
                                    run_plans(mode, prio, rep, order, fen + "+created")
                                    torch.cuda.synchronize()
                            else:
                                run_plans(mode, prio, rep, order, fen)
                            if rank == 0:
                                print(f"{prio} rep {rep} {mode} {order} {fen}: done", file=sys.stderr, flush=True)
                        if not explicit_registration(mode):
                            results.append({"priority": prio, "mode": mode, "order": order, "rep": rep,
                                            "plan": "explicit", "op": "-", "widths": [], "steps": 1,
                                            "bad_steps": [{"step": 0, "bad": -1}]})
                dist.barrier()
            fd.shutdown_push()
        fd.side_stream, fd.peer_stream = product
        fd._PUSH_ORDER = "auto"
        gathered = [None] * world
        dist.all_gather_object(gathered, results)
        if rank == 0:
            summary = {}
            for r, res in enumerate(gathered):
                for x in res:
                    fen = x.get("fence", "none")
                    key = f"{x['priority']}/{x['mode']}/{x.get('order', '-')}/" + (f"{fen}/" if fen != "none" else "") + x["op"]
                    s = summary.setdefault(key, {"runs": 0, "steps": 0, "bad_steps": 0, "bad_by_step": {},
                                                 "bad_by_plan": {}, "bad_elems": 0, "stale_prev_step": 0,
                                                 "examples": []})
                    if x["bad_steps"]:
                        s["bad_by_plan"][str(x["plan"])] = s["bad_by_plan"].get(str(x["plan"]), 0) + len(x["bad_steps"])
                    for b in x["bad_steps"]:
                        for f in ("pushed_cols", "eq_sender_src_before", "eq_bucket_before", "right_when_reread"):
                            if f in b:
                                s[f] = s.get(f, 0) + b[f]
                    s["runs"] += 1
                    s["steps"] += x["steps"]
                    s["bad_steps"] += len(x["bad_steps"])
                    for b in x["bad_steps"]:
                        s["bad_by_step"][str(b["step"])] = s["bad_by_step"].get(str(b["step"]), 0) + 1
                        s["bad_elems"] += max(b["bad"], 0)
                        s["stale_prev_step"] += b.get("stale_prev_step", 0)
                    if x["bad_steps"] and len(s["examples"]) < 6:
                        s["examples"].append({"rank": r, "plan": x["plan"], "widths": x["widths"], **x["bad_steps"][0]})
            Path(out_path).write_text(json.dumps({"world": world, "summary": summary}, indent=1))
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--modes", default="kernel,dma")
    ap.add_argument("--reps", type=int, default=3, help="times the test's whole sequence runs per priority")
    ap.add_argument("--priorities", default="normal,high")
    ap.add_argument("--kernel-orders", default="-",
                    help="comma list for the kernel push: host / producer ('-': the product's order, labelled '-')")
    ap.add_argument("--dma-orders", default="host",
                    help="how the copy-engine legs follow their reduce: host (the product), producer (an event of "
                         "the reduce's stream) and/or chain (round 5: an event of the pusher's stream)")
    ap.add_argument("--fences", default="none",
                    help="none / release (L2 written back after each stripe's reduce) / acquire (L2 invalidated "
                         "before the bucket is read) / both: which cache fence removes wrong buckets")
    ap.add_argument("--forensic", action="store_true",
                    help="classify wrong values: the sender's source before the step (a leg read early), this "
                         "rank's bucket before the step (a leg not landed), right when re-read 50 ms later")
    ap.add_argument("--compute", default="default", choices=("default", "created"),
                    help="the reduces' stream: torch's default (null) stream, or a created one")
    ap.add_argument("--out", default="gpurun_out/push_order.json")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    mp.spawn(_worker, args=(a.world, port, a.modes.split(","), a.priorities.split(","), a.steps, a.reps, a.out,
                            tuple(a.dma_orders.split(",")), tuple(a.fences.split(",")), a.forensic, a.compute,
                            tuple(a.kernel_orders.split(","))),
             nprocs=a.world, join=True)
    print(Path(a.out).read_text())


if __name__ == "__main__":
    main()
