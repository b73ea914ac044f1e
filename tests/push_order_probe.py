"""Are the push gather's copies ordered after the stripe's reduce when the pusher's streams have
their own hardware queue?  (round 5)

    python tests/push_order_probe.py --world 8 --steps 3 --reps 6 --priorities normal,high,product

(round 5: with the copy-engine push's streams at high priority, 32 of 576 in-place Adagrad
rank-steps were wrong; flearn_amd.dist now gives only the kernel push a high-priority stream)

`world` processes share cuda:0 over gloo (like tests/test_gpu_multirank.py); each runs
ShardedReducer steps with the fused Adagrad epilogue in place (the reduce reads `prev` and writes
the new model over it; the pushes read that model) under four stripe plans, with the pusher's
streams at normal priority (may share the compute stream's hardware queue) or high priority (a
queue of their own: flearn_amd.streams.side_stream), and compares every step's bucket with the C
oracle.  For a mismatch it records which ranks' slices were wrong and whether the wrong values are
the PREVIOUS step's model (a copy that read its source before the reduce had written it) or
something else.  Prints one JSON object.  Test infrastructure (it checks against the C oracle, so it
lives under tests/), run by hand or by tools/gpu_r05a*.sh, not by pytest.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def _worker(rank, world, port, modes, priorities, steps, reps, out_path):
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

    def run_plans(mode, prio, rep):
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
                red = ShardedReducer(plan, hip_reduce_fn(stack, w, na.MODE_W32_DIV64, denom, **epi), cuda,
                                     local_out=local_out, gather=True, push="dma" if mode == "dma" else True)
                prev_h = oracle.fill_uniform(1, p, 4)[0]
                v_h = np.zeros(p)
                last = prev_h.astype(np.float32) if op != "mean" else want_mean.astype(np.float32)
                bad_steps = []
                for step in range(steps):
                    full = red.step().cpu().numpy()
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
                        bad_steps.append({"step": step, "bad": int(len(bad)), "stale_prev_step": stale,
                                          "owners": owners, "first": int(bad[0]), "last": int(bad[-1])})
                    last = want
                red.release()
                results.append({"priority": prio, "mode": mode, "rep": rep, "plan": pi, "op": op,
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
        for prio in priorities:
            if prio != "product":  # "product": the streams as flearn_amd.dist creates them
                fd.side_stream = (lambda dev: torch.cuda.Stream(dev, priority=-1)) if prio == "high" else (
                    lambda dev: torch.cuda.Stream(dev, priority=0))
            for rep in range(reps):
                for mode in modes:
                    run_plans(mode, prio, rep)
                    if not explicit_registration(mode):
                        results.append({"priority": prio, "mode": mode, "rep": rep, "plan": "explicit", "op": "-",
                                        "widths": [], "steps": 1, "bad_steps": [{"step": 0, "bad": -1}]})
                dist.barrier()
            fd.shutdown_push()
        gathered = [None] * world
        dist.all_gather_object(gathered, results)
        if rank == 0:
            summary = {}
            for r, res in enumerate(gathered):
                for x in res:
                    key = f"{x['priority']}/{x['mode']}/{x['op']}"
                    s = summary.setdefault(key, {"runs": 0, "steps": 0, "bad_steps": 0, "examples": []})
                    s["runs"] += 1
                    s["steps"] += x["steps"]
                    s["bad_steps"] += len(x["bad_steps"])
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
    ap.add_argument("--out", default="gpurun_out/push_order.json")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    mp.spawn(_worker, args=(a.world, port, a.modes.split(","), a.priorities.split(","), a.steps, a.reps, a.out),
             nprocs=a.world, join=True)
    print(Path(a.out).read_text())


if __name__ == "__main__":
    main()
