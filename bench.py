"""Device-resident FedAVG-family aggregation throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ns|c2|c3|c4|c5|c1k]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N` with no launcher env starts the N ranks itself (flearn_amd/launch.py: fresh children
through torch.distributed.run, before any HIP call in the parent); it fails loudly when fewer
than N GPUs are visible and never measures a smaller world than asked.

One "step" = one server aggregation over device-resident client uploads: the fused HIP reduce of
N clients x P fp32 parameters (+ the fused AVGM/Adagrad update for c3/c5) into the fp32 global
model, and for N>1 GPUs the RCCL all-gather that reassembles it on every GPU.  Inputs are
synthetic (splitmix64 U(-1,1), generated on device), weights are Python 1.0 — flearn's default
(Client.py:157) — so the arithmetic is FA_MODE_W32_DIV64, bit-identical to the reference.

Configs (BASELINE.json):  ns  FedAVG    100 x ResNet-50 (25,610,152 fp32)      [default: the
                              north star's "100 clients x 25 M fp32 at 1 GPU" headline shape]
                          c2  FedAVG    100 x ResNet-18 (11,699,112 fp32)
                          c3  FedAVGM   100 x ResNet-50 (25,610,152 fp32)
                          c4  FedAVG   1000 x ResNet-18
                          c5  FedOPT-Adagrad 100 x ViT-B/16 (86,567,656 fp32)
Multi-GPU (element-range column shards + RCCL all-gather, flearn_amd/dist.py):
  --scaling strong (default) `value` is the config's fixed problem (its clients) on G GPUs, so the
                   N-GPU values divide directly by the 1-GPU line (the north star's speedup);
                   the weak job (clients x G uploads, every GPU streaming the 1-GPU bytes) runs
                   after it and is reported in the "weak" field (--no-weak skips it)
  --scaling weak   the other way round
  stripes          by default the reduce/gather pipeline is planned per job from a two-stage
                   model whose coefficients are fitted on the running job (reduce of the whole
                   and 1/8 of the local width, RCCL all-gather of both; max over ranks): the
                   "multi_gpu" field reports the widths, the model, its prediction, the measured
                   per-rank reduce time and the exposed gather time; --stripes K fixes K stripes.
                   The plan may end in a replicated tail (flearn_amd.dist.plan_shards): the last
                   columns are reduced by EVERY rank instead of gathered — redundant HBM reads
                   traded for xGMI bytes where the gather sets the step (G = 2, 4: one link per
                   peer); `value` counts every column once ("replicated_cols" in "multi_gpu")
  --emulate-world G  one GPU runs rank 0's share of a G-GPU job (no collective): the per-rank
                   reduce of the multi-GPU runs, measurable on a single-GPU box
Prints ONE JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import threading
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import dist as fa_dist  # noqa: E402
from flearn_amd import launch, layouts, verify  # noqa: E402
from flearn_amd.dist import (ALIGN, PingPong, ShardedReducer, ShardPlan, StripeModel,  # noqa: E402
                             all_gather_into, hip_reduce_fn, shard_candidates)

METRIC = "device-resident GiB/s, FedAVG N-client weighted tensor reduce; %HBM peak"
UPLOAD_SEED, PREV_SEED = 2024, 1  # synthetic client uploads / previous global model
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = 1024.0**3

CONFIGS = {
    "ns": dict(layout="resnet50", clients=100, op="mean",
               workload="NS: FedAVG reduce, 100 clients x ResNet-50 state_dict (25,610,152 fp32 / 267 tensors) "
                        "- the north star's 100 x 25 M headline shape"),
    "c2": dict(layout="resnet18", clients=100, op="mean",
               workload="C2: FedAVG reduce, 100 clients x ResNet-18 state_dict (11,699,112 fp32 / 102 tensors)"),
    "c3": dict(layout="resnet50", clients=100, op="avgm",
               workload="C3: FedAVGM (server momentum fused into reduce), 100 clients x ResNet-50 (25,610,152 fp32)"),
    "c4": dict(layout="resnet18", clients=1000, op="mean",
               workload="C4: FedAVG reduce, 1000 clients x ResNet-18 (11,699,112 fp32)"),
    "c1k": dict(layout="lenet5", clients=1000, op="mean",
                workload="C1k: FedAVG reduce, 1000 clients x LeNet5 (44,426 fp32) - small-P / deep-N shape"),
    "c5": dict(layout="vit_b_16", clients=100, op="adagrad",
               workload="C5: FedOPT-Adagrad fused with reduce, 100 clients x ViT-B/16 (86,567,656 fp32)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(n_clients: int, cols: int, op: str) -> int:
    """FedAVG N*P*4 + P*4 (fp32 out); fused AVGM/OPT adds P*4 prev + 2*P*8 v_t."""
    b = n_clients * cols * 4 + cols * 4
    if op != "mean":
        b += cols * 4 + 2 * cols * 8
    return b


def host_cpu_name() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.machine()


def cpu_baseline(stack: torch.Tensor, layout, n_sample: int, reps: int = 3):
    """flearn's CPU path: the oracle's numpy restatement of Strategy.server_ensemble
    (strategy.py:102-130, bit-exact to the reference by tests/test_oracle_golden.py), timed on
    this host over a sample of the same workload (n_sample clients, full layout)."""
    import oracle

    fp32 = [(k, s, t) for k, s, t in layout if t == "f32"]
    p = layouts.fp32_elems(fp32)
    host = stack[:n_sample, :p].cpu().numpy()
    clients = [layouts.synthetic_state_dict(fp32, host[i]) for i in range(n_sample)]
    weights = [1.0] * n_sample
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        oracle.server_ensemble(weights, clients)
        best = min(best, time.perf_counter() - t0)
    gib = algorithmic_bytes(n_sample, p, "mean") / GIB / best
    return {
        "value": round(gib, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n_sample} clients x full {len(fp32)}-tensor layout ({p} fp32), numpy op-sequence "
                  f"restatement of server_ensemble, best of {reps} ({best:.3f} s); numpy ufuncs are "
                  f"single-threaded (1 core used); host {host_cpu_name()}, nproc={os.cpu_count()}",
    }


def load_traffic(config: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py)."""
    f = REPO / "profiles" / "traffic.json"
    if not f.exists():
        return None, None
    d = json.loads(f.read_text()).get(config)
    if not d:
        return None, None
    return d.get("hbm_bytes_per_launch"), d.get("source")


class Job:
    """One aggregation job on this rank: n clients x the config's layout, this rank's block-cyclic
    columns (plan) resident in HBM, the fused HIP reduce per stripe and (world > 1) the RCCL
    all-gather of every stripe."""

    def __init__(self, cfg, layout, n, plan, dev, world, reorder, push=False, push_grid=0, reducer=True):
        """reducer=False: allocate and fill only (local); make_reducer() then builds the sharded
        reducer — collective when pushing (the peers map each other's buckets)."""
        self.cfg, self.n, self.plan, self.dev = cfg, n, plan, dev
        self.world, self.push, self.push_grid = world, push, push_grid
        self.red = None
        cols, stride = plan.local_cols, plan.local_stride
        log(f"[rank {plan.rank}] alloc {n} x {cols} fp32 = {n * cols * 4 / 1e9:.2f} GB, stripes {plan.widths}"
            + (f" + replicated tail {plan.rep}" if plan.rep else ""))
        self.stack = torch.empty((n, stride), dtype=torch.float32, device=dev)
        for lo, g0, width in plan.segments():
            agg.fill_uniform(self.stack[:, lo:], seed=UPLOAD_SEED, row_begin=0, col_begin=g0, n_cols=width)
        self.weights = torch.ones(n, dtype=torch.float32, device=dev)  # Python 1.0 -> fl32(1.0)
        self.denom = float(np.sum([1.0] * n))  # np.sum(agg_weight_lst), strategy.py:127
        self.reorder = reorder
        epi, state = {}, None
        if cfg["op"] != "mean":
            prev = torch.empty((1, stride), dtype=torch.float32, device=dev)
            # the fused step reads (prev, v_t) and writes the new global model and v_t into a
            # second pair, swapped every step — as the product's ServerOptimizer does
            state = PingPong(prev[0], torch.zeros(stride, dtype=torch.float64, device=dev))
            self.reset_state(state)
            epi = dict(op=na.OP_BY_NAME[cfg["op"]], state=state)
        self.fn = hip_reduce_fn(self.stack, self.weights, na.MODE_W32_DIV64, self.denom, reorder=reorder, **epi)
        self._state = state
        if reducer:
            self.make_reducer()

    def make_reducer(self):
        self.red = ShardedReducer(self.plan, self.fn, self.dev, gather=self.world > 1, state=self._state, push=self.push,
                                  push_grid=self.push_grid)

    def reset_state(self, state=None):
        """The fused optimizers' initial state: prev = the seed-1 synthetic model on this rank's
        columns, v_t = 0 (np.zeros_like on first use, avgm.py:27 / opt.py:35)."""
        st = state if state is not None else self.red.state
        st.cur = 0
        for lo, g0, width in self.plan.segments():
            agg.fill_uniform(st.prev[0][lo:], seed=PREV_SEED, col_begin=g0, n_cols=width)
        st.v[0].zero_()

    def release(self):
        """Collective for a push-gathered job (peers unmap this rank's buffer first)."""
        if self.red is not None:
            self.red.release()
        self.stack = self.red = self.fn = None
        torch.cuda.empty_cache()

    def reduce_only(self):
        """The reduce launches of one step (every stripe and the replicated tail), no collective."""
        for lo, _, width in self.plan.segments():
            self.fn(lo, width, self.red.local_out[lo : lo + width])


def _event_time(fn, reps: int) -> float:
    """Seconds per call of fn, HIP events on torch's current stream (what the launches use)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def _max_over_ranks(vals, world, dev):
    if world == 1:
        return list(vals)
    on = dev if dist.get_backend() == "nccl" else "cpu"  # gloo: host tensors
    t = torch.tensor(list(vals), dtype=torch.float64, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def calibrate(job: Job, world: int, dev, reps: int = 5):
    """Fit the stripe model on the running job: the reduce of the whole local width and of 1/8 of
    it, and an all-gather of each width (real RCCL over xGMI), max over ranks.  Returns
    (StripeModel, the raw measurements).  On one GPU (--emulate-world) the gather terms are the
    model's a priori ones (StripeModel.assumed)."""
    p = job.plan
    big = p.local_cols
    small = max(ALIGN, (big // 8) // ALIGN * ALIGN)
    out = job.red.local_out
    r_big = _event_time(lambda: job.fn(0, big, out[:big]), reps)
    r_small = _event_time(lambda: job.fn(0, small, out[:small]), reps)
    r_conc = g_conc = None
    if world > 1:
        full = torch.empty(world * big, dtype=torch.float32, device=dev)
        for _ in range(2):  # RCCL's first calls set up channels / buffers
            all_gather_into(full, out[:big])
            all_gather_into(full[: world * small], out[:small])
        torch.cuda.synchronize()
        dist.barrier()
        g_big = _event_time(lambda: all_gather_into(full, out[:big]), reps)
        g_small = _event_time(lambda: all_gather_into(full[: world * small], out[:small]), reps)
        r_conc, g_conc = _contention(job, full, out, big, dev, reps)
        del full
    else:
        m = StripeModel.assumed(job.n, p.world)
        g_big, g_small = m.a_g + m.b_g * big, m.a_g + m.b_g * small
    vals = (r_big, r_small, g_big, g_small) + ((r_conc, g_conc) if r_conc is not None else ())
    vals = _max_over_ranks(vals, world, dev)
    r_big, r_small, g_big, g_small = vals[:4]
    c_r = c_g = 0.0
    cal = dict(width_cols=[big, small], reduce_us=[round(r_big * 1e6, 2), round(r_small * 1e6, 2)],
               gather_us=[round(g_big * 1e6, 2), round(g_small * 1e6, 2)], measured_gather=world > 1)
    if r_conc is not None:
        r_conc, g_conc = vals[4:]
        # the slowdown each stream saw while the other ran (equal widths: the shorter one was
        # concurrent for all of its time, the longer one for part of it — an effective value)
        c_r, c_g = max(r_conc / r_big - 1.0, 0.0), max(g_conc / g_big - 1.0, 0.0)
        cal.update(concurrent_reduce_us=round(r_conc * 1e6, 2), concurrent_gather_us=round(g_conc * 1e6, 2),
                   c_r=round(c_r, 4), c_g=round(c_g, 4))
    return StripeModel.fit(big, small, r_big, r_small, g_big, g_small, c_r=c_r, c_g=c_g), cal


PUSH_GRIDS = (4, 8, 16, 32, 64, 128, 256)  # the paced push kernel: few blocks can fill a link
PUSH_MODE = {"push": "kernel", "push_dma": "dma"}  # --gather name -> PushGather mode


def calibrate_push(job: Job, world: int, dev, r_big: float, reps: int = 5, mode: str = "kernel"):
    """The one-shot push all-gather (fa_dist.PushGather) on the running job: availability (every
    rank maps its peers' buffers), a bit-compare against RCCL's all-gather of the same slices, the
    gather of the whole local width and of 1/8 of it, and its contention with the reduce.
    Returns (StripeModel or None, calibration dict)."""
    p = job.plan
    big = p.local_cols
    small = max(ALIGN, (big // 8) // ALIGN * ALIGN)
    out = job.red.local_out
    try:  # a bucket from the receive pool: the jobs and trials after this one map no new buffer
        pg = fa_dist.PushGather(None, mode=mode, cols=world * big, device=dev)
    except RuntimeError as e:
        return None, {"available": False, "reason": str(e)}
    full = pg.full
    try:
        pg.gather(out[:big], p.rank * big)
        want = torch.empty_like(full)
        all_gather_into(want, out[:big])
        torch.cuda.synchronize(dev)
        same = _max_over_ranks((0.0 if torch.equal(full, want) else 1.0,), world, dev)[0] == 0.0
        del want
        if not same:
            return None, {"available": False, "reason": "pushed buckets differ from RCCL's all-gather"}
        for _ in range(2):
            pg.gather(out[:big], p.rank * big)
            pg.gather(out[:small], p.rank * small)
        torch.cuda.synchronize(dev)
        dist.barrier()
        # the push kernel's grid: the smallest whose push BESIDE a reduce of the same width ends
        # both within 3% of the best such pair.  More blocks keep more stores in flight for the
        # links, but stores backed up behind a link slow the reduce through the data fabric — on
        # one GPU's PCIe stand-in 3x at the grid that fills the link — so
        # the gather alone picks the wrong grid.
        by_grid, pair_by_grid = {}, {}
        for g in (PUSH_GRIDS if mode == "kernel" else ()):
            pg.grid = g
            by_grid[g] = _event_time(lambda: pg.gather(out[:big], p.rank * big), 3)
            pair_by_grid[g] = _pair_time(job, pg, out, big, dev, 3)
        if by_grid:
            times = _max_over_ranks(list(by_grid.values()) + list(pair_by_grid.values()), world, dev)
            by_grid = dict(zip(PUSH_GRIDS, times[:len(PUSH_GRIDS)]))
            pair_by_grid = dict(zip(PUSH_GRIDS, times[len(PUSH_GRIDS):]))
            best = min(pair_by_grid.values())
            pg.grid = min(g for g, t in pair_by_grid.items() if t <= 1.03 * best)
        g_big = _event_time(lambda: pg.gather(out[:big], p.rank * big), reps)
        g_small = _event_time(lambda: pg.gather(out[:small], p.rank * small), reps)
        r_conc, g_conc, g_alone = _contention_push(job, pg, out, big, dev, reps)
        grid = pg.grid
    finally:
        pg.close()
    r_small = _event_time(lambda: job.fn(0, small, out[:small]), reps)
    g_big, g_small, r_conc, g_conc, g_alone, r_small = _max_over_ranks(
        (g_big, g_small, r_conc, g_conc, g_alone, r_small), world, dev)
    c_r, c_g = max(r_conc / r_big - 1.0, 0.0), max(g_conc / max(g_alone, 1e-9) - 1.0, 0.0)
    cal = dict(available=True, mode=mode, checked_against_rccl=True, width_cols=[big, small], grid=grid,
               gather_us_by_grid={str(g): round(t * 1e6, 2) for g, t in by_grid.items()},
               pair_us_by_grid={str(g): round(t * 1e6, 2) for g, t in pair_by_grid.items()},
               gather_us=[round(g_big * 1e6, 2), round(g_small * 1e6, 2)],
               push_kernel_us=round(g_alone * 1e6, 2), concurrent_reduce_us=round(r_conc * 1e6, 2),
               concurrent_push_us=round(g_conc * 1e6, 2), c_r=round(c_r, 4), c_g=round(c_g, 4),
               per_link_gbs=round(big * 4 / max(g_alone, 1e-9) / 1e9, 2))
    return StripeModel.fit(big, small, r_big, r_small, g_big, g_small, c_r=c_r, c_g=c_g), cal


def _pair_time(job, pg, out, cols, dev, reps: int) -> float:
    """A push of `cols` columns and a reduce of as many, started together: the time until both
    are done (median of reps) — what a stripe's push beside the next stripe's reduce costs."""
    out2 = torch.empty_like(out)
    cur = torch.cuda.current_stream(dev)
    src, off = out[:cols], job.plan.rank * cols
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        pg.begin()
        pg.push(src, off)
        job.fn(0, cols, out2[:cols])
        pg.end()
        e1.record(cur)
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1) / 1e3)
    return float(np.median(ts))


def _contention_push(job, pg, out, cols, dev, reps: int):
    """(reduce time beside a push, push-kernel time beside a reduce, push-kernel time alone)."""
    side = torch.cuda.Stream(dev)
    out2 = torch.empty_like(out)
    cur = torch.cuda.current_stream(dev)
    r_t, g_t, a_t = [], [], []
    src, off = out[:cols], job.plan.rank * cols
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        pg.begin()
        pg.push(src, off)
        job.fn(0, cols, out2[:cols])
        e1.record(cur)
        pg.end()
        torch.cuda.synchronize(dev)
        r_t.append(e0.elapsed_time(e1) / 1e3)
        for beside in (True, False):
            dist.barrier()
            e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            pg.begin()
            side.wait_stream(pg.stream)  # the reduce starts with the push, after the barrier
            if beside:
                with torch.cuda.stream(side):
                    job.fn(0, cols, out2[:cols])
            e2.record(pg.stream)
            pg.push(src, off)
            pg.join()
            e3.record(pg.stream)
            pg.end()
            cur.wait_stream(side)
            torch.cuda.synchronize(dev)
            (g_t if beside else a_t).append(e2.elapsed_time(e3) / 1e3)
    return float(np.median(r_t)), float(np.median(g_t)), float(np.median(a_t))


def _contention(job, full, out, cols, dev, reps: int):
    """The reduce and the all-gather of the whole local width run concurrently (real RCCL over
    xGMI at N > 1): (reduce time beside the gather, gather time beside the reduce), each taken on
    the stream of the one being measured.  Host-staged gloo gathers are synchronous: no overlap."""
    side = torch.cuda.Stream(dev)
    out2 = torch.empty_like(out)
    cur = torch.cuda.current_stream(dev)
    r_t, g_t = [], []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        dist.barrier()
        # (a) the reduce on this stream, the gather issued first on RCCL's
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        w = all_gather_into(full, out[:cols], async_op=True)
        job.fn(0, cols, out2[:cols])
        e1.record(cur)
        if w is not None:
            w.wait()
        torch.cuda.synchronize(dev)
        r_t.append(e0.elapsed_time(e1) / 1e3)
        dist.barrier()
        # (b) the gather enqueued on this stream's order, the reduce on a side stream
        e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        side.wait_stream(cur)
        e2.record(cur)
        with torch.cuda.stream(side):
            job.fn(0, cols, out2[:cols])
        all_gather_into(full, out[:cols])
        e3.record(cur)
        cur.wait_stream(side)
        torch.cuda.synchronize(dev)
        g_t.append(e2.elapsed_time(e3) / 1e3)
    return float(np.median(r_t)), float(np.median(g_t))


def _probe_job(cfg, layout, n, args, world, rank, dev, g_eff):
    """A one-stripe job of this rank's columns, warmed up: what the calibrations run on."""
    p_real = layouts.fp32_elems(layout)
    probe = Job(cfg, layout, n, ShardPlan.make(p_real, g_eff, rank, 1), dev, world, args.reorder)
    for _ in range(2):
        probe.reduce_only()
    return probe


def _trial(cfg, layout, n, args, world, rank, dev, g_eff, gather, widths, rep, model, push_grid=0) -> dict:
    """One candidate plan timed for 5 steps on a fresh job (max over ranks: every rank sees the
    same numbers and picks the same plan)."""
    p_real = layouts.fp32_elems(layout)
    rec = {"gather": gather, "stripe_widths": list(widths), "replicated_cols": rep,
           "predicted_ms": round(model.makespan(widths, rep)[0] * 1e3, 4)}
    # the allocation is local, so it may fail on some ranks only (out of memory): agree on it
    # before anything collective, so that every rank skips the candidate together
    tj, err = None, None
    try:
        tj = Job(cfg, layout, n, ShardPlan.from_widths(p_real, g_eff, rank, widths, rep=rep), dev, world, args.reorder,
                 push=PUSH_MODE.get(gather, False), push_grid=push_grid, reducer=False)
    except (torch.OutOfMemoryError, RuntimeError) as e:
        err = f"{type(e).__name__}: {e}"[:200]
    if _max_over_ranks((0.0 if tj is not None else 1.0,), world, dev)[0] > 0.0:
        tj = None
        torch.cuda.empty_cache()
        rec.update(measured_ms=None, error=err or "another rank could not allocate this candidate")
        return rec
    try:
        tj.make_reducer()
    except RuntimeError as e:  # a push that every rank refused to set up (PushGather, collective)
        tj = None
        torch.cuda.empty_cache()
        rec.update(measured_ms=None, error=str(e))
        return rec
    for _ in range(2):
        tj.red.step()
    t = _max_over_ranks((_event_time(tj.red.step, 5),), world, dev)[0]
    tj.release()
    rec["measured_ms"] = round(t * 1e3, 4)
    return rec


def _model_info(model, cal, plan):
    pred, _red, exposed = model.makespan(plan.widths, plan.rep)
    return dict(model={"a_r_us": round(model.a_r * 1e6, 3), "b_r_ns_per_col": round(model.b_r * 1e9, 5),
                       "a_g_us": round(model.a_g * 1e6, 3), "b_g_ns_per_col": round(model.b_g * 1e9, 5),
                       "c_r": round(model.c_r, 4), "c_g": round(model.c_g, 4)},
                calibration=cal, predicted_ms=round(pred * 1e3, 4), predicted_exposed_gather_ms=round(exposed * 1e3, 4))


def plan_rccl(cfg, layout, n, args, world, rank, dev, g_eff):
    """The reduce/gather plan with RCCL's all-gather: stripes fixed by --stripes, or the fitted
    model's candidates (flearn_amd.dist.shard_candidates) each timed on the job, the fastest
    kept.  Returns (plan, info, fastest measured trial in s or None)."""
    p_real = layouts.fp32_elems(layout)
    if g_eff == 1:
        return ShardPlan.make(p_real, 1, 0, args.stripes or 1), {}, None
    if args.stripes:
        sw = (None if args.stripe_weights in (None, "equal") or args.stripes == 1 else
              tuple(float(x) for x in args.stripe_weights.split(",")))
        return ShardPlan.make(p_real, g_eff, rank, args.stripes, weights=sw), {"stripe_choice": "fixed by --stripes"}, None
    probe = _probe_job(cfg, layout, n, args, world, rank, dev, g_eff)
    model, cal = calibrate(probe, world, dev)
    probe.release()
    cands = shard_candidates(p_real, g_eff, model)
    widths, rep = min(cands, key=lambda c: model.makespan(c[0], c[1])[0])
    trials, best_s = [], None
    if world > 1 and len(cands) > 1:
        trials = [_trial(cfg, layout, n, args, world, rank, dev, g_eff, "rccl", w_c, r_c, model) for w_c, r_c in cands]
        ok = [k for k in range(len(cands)) if trials[k]["measured_ms"] is not None]
        if ok:  # (a candidate some rank could not allocate is skipped on every rank)
            i = min(ok, key=lambda k: trials[k]["measured_ms"])
            widths, rep = cands[i]
            best_s = trials[i]["measured_ms"] * 1e-3
    plan = ShardPlan.from_widths(p_real, g_eff, rank, widths, rep=rep)
    info = dict(stripe_choice=("model (flearn_amd.dist.plan_shards: stripes + replicated tail), coefficients fitted "
                               "on this job" + ("; the fastest of the model's plan and its neighbours over 5 measured "
                                                "steps each" if trials else "")),
                **_model_info(model, cal, plan))
    if trials:
        info["plan_trials"] = trials
    return plan, info, best_s


def plan_push(cfg, layout, n, args, world, rank, dev, g_eff, r_big_s):
    """The one-shot push gathers (kernel stores, copy engines): each form set up on a probe job,
    bit-checked against RCCL's all-gather, calibrated; its model's candidates timed on the job.
    Returns (plan, gather, info, fastest measured trial in s or None); plan None: no push form
    available here (the info says why)."""
    p_real = layouts.fp32_elems(layout)
    forms = [(g, m, k) for g, m, k in (("push", "kernel", "push_calibration"), ("push_dma", "dma", "push_dma_calibration"))
             if args.gather in ("auto", g)]
    info = {}
    if args.stripes:  # a forced push form on the fixed stripes: no calibration, no trials
        g = forms[0][0]
        plan, _i, _b = plan_rccl(cfg, layout, n, args, world, rank, dev, g_eff)
        return plan, g, {"stripe_choice": "fixed by --stripes", "push_grid": None}, None
    probe = _probe_job(cfg, layout, n, args, world, rank, dev, g_eff)
    models, grids = {}, {}
    if r_big_s <= 0:  # the reduce of the whole local width (the contention terms' reference)
        big = probe.plan.local_cols
        r_big_s = _max_over_ranks((_event_time(lambda: probe.fn(0, big, probe.red.local_out[:big]), 5),), world, dev)[0]
    try:
        for g, mode, key in forms:
            m, c = calibrate_push(probe, world, dev, r_big_s, mode=mode)
            info[key] = c
            if m is not None:
                models[g] = m
                grids[g] = c.get("grid", 0) if mode == "kernel" else 0
    finally:
        probe.release()
    if not models:
        return None, None, info, None
    cands = [(g, w_c, r_c) for g, m in models.items() for w_c, r_c in shard_candidates(p_real, g_eff, m)]
    trials = [_trial(cfg, layout, n, args, world, rank, dev, g_eff, g, w_c, r_c, models[g], grids[g])
              for g, w_c, r_c in cands]
    ok = [k for k in range(len(cands)) if trials[k]["measured_ms"] is not None]
    if not ok:
        info["plan_trials"] = trials
        return None, None, info, None
    i = min(ok, key=lambda k: trials[k]["measured_ms"])
    g, widths, rep = cands[i]
    plan = ShardPlan.from_widths(p_real, g_eff, rank, widths, rep=rep)
    mi = _model_info(models[g], None, plan)
    mi.pop("calibration")  # "calibration" stays RCCL's; the push forms' are push(_dma)_calibration
    info.update(mi)
    info.update(plan_trials=trials, push_grid=grids[g] if g == "push" else None,
                stripe_choice="push gathers' models, the fastest candidate over 5 measured steps each")
    return plan, g, info, trials[i]["measured_ms"] * 1e-3


def timed_job(cfg, layout, n, plan, gather, push_grid, args, world, dev, g_eff):
    """Build the job on `plan` with `gather`, warm up, time args.steps steps (barrier + sync on
    both sides, HIP events on the launch stream, max over ranks).  Returns (job, step_s, wall_s,
    info)."""
    info = {}
    job = Job(cfg, layout, n, plan, dev, world, args.reorder, push=PUSH_MODE.get(gather, False), push_grid=push_grid or 0)
    for _ in range(args.warmup):
        job.red.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        job.red.step()
    ev1.record()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = max(ev0.elapsed_time(ev1) / 1e3, 0.0)  # s, on the stream the kernels run on
    elapsed, wall = _max_over_ranks((elapsed, wall), world, dev)
    step_s = elapsed / args.steps
    if g_eff > 1:  # this rank's reduce launches of one step alone (no collective), max over ranks
        red_s = _max_over_ranks((_event_time(job.reduce_only, max(3, min(args.steps, 20))),), world, dev)[0]
        info["per_rank_reduce_ms"] = round(red_s * 1e3, 4)
        info["exposed_gather_ms"] = round(max(step_s - red_s, 0.0) * 1e3, 4)
    info["stripe_widths"] = list(plan.widths)
    # columns every rank reduces itself (no gather): redundant work, counted once in `value`
    info["replicated_cols"] = plan.rep
    info["gather"] = gather if world > 1 else None
    info["push_grid"] = push_grid if gather == "push" else None
    return job, step_s, wall, info


def run_job(cfg, layout, n, args, world, rank, dev, g_eff, gather: str = "rccl"):
    """Plan with `gather` ("rccl", or a push form: planned by plan_push) and time it.
    Returns (job, step_s, wall_s, info)."""
    if gather == "rccl" or world == 1:
        plan, info, _best = plan_rccl(cfg, layout, n, args, world, rank, dev, g_eff)
        push_grid = 0
    else:
        plan, gather, info, _best = plan_push(cfg, layout, n, args, world, rank, dev, g_eff, 0.0)
        push_grid = info.get("push_grid") or 0
        if plan is None:  # no push form available for this job: RCCL's all-gather
            plan, rinfo, _best = plan_rccl(cfg, layout, n, args, world, rank, dev, g_eff)
            info = {**info, **rinfo, "push_unavailable": True}
            gather, push_grid = "rccl", 0
    job, step_s, wall, tinfo = timed_job(cfg, layout, n, plan, gather, push_grid, args, world, dev, g_eff)
    info.update(tinfo)
    return job, step_s, wall, info


def verify_job(job, cfg, world, dev, emulated: bool = False) -> dict:
    """After the timed region: prove the reassembled global model right (flearn_amd.verify).
    Windows on every slice start / rank boundary / replicated-tail edge (>= 64) are regenerated
    for all N clients and reduced UNSHARDED with the same kernel; the bucket the sharded step
    returned (RCCL all-gather at N > 1) must match bit for bit, on every rank.  Fused configs
    restart from the initial state and check the second step's model and every rank's own v_t
    slices.  No oracle: the product kernel against itself."""
    op = cfg["op"]
    n, plan = job.n, job.plan
    fused = op != "mean"
    if fused:
        job.reset_state()
        job.red.step()
    full = job.red.step()
    torch.cuda.synchronize(dev)
    state = job.red.state.v[job.red.state.cur] if fused else None
    width = 4096
    x = torch.empty((n, width), dtype=torch.float32, device=dev)
    prev = torch.empty(width, dtype=torch.float32, device=dev)
    v0 = torch.zeros(width, dtype=torch.float64, device=dev)
    w1, v1, w2, v2 = (torch.empty(width, dtype=dt, device=dev) for dt in
                      (torch.float32, torch.float64, torch.float32, torch.float64))
    kw = dict(op=na.OP_BY_NAME[op]) if fused else {}

    def expect(g0, w):
        agg.fill_uniform(x, seed=UPLOAD_SEED, col_begin=g0, n_cols=w)
        if not fused:
            agg.reduce_stack(x, job.weights, na.MODE_W32_DIV64, job.denom, n_cols=w, out32=w2)
            return w2, None
        agg.fill_uniform(prev, seed=PREV_SEED, col_begin=g0, n_cols=w)
        agg.reduce_stack(x, job.weights, na.MODE_W32_DIV64, job.denom, n_cols=w, out32=w1, prev=prev, v=v0,
                         v_out=v1, **kw)
        agg.reduce_stack(x, job.weights, na.MODE_W32_DIV64, job.denom, n_cols=w, out32=w2, prev=w1, v=v1,
                         v_out=v2, **kw)
        return w2, v2

    compare = None
    if job.reorder:  # the split-N order is not the list order: its documented bound instead
        def compare(a, b):
            a64, b64 = a.double(), b.double()
            return bool(torch.linalg.vector_norm(a64 - b64) <= 1e-6 * torch.linalg.vector_norm(b64))
    res = verify.check_step(plan, full, expect, state=state, width=width, compare=compare, local_model=emulated)
    res["comparison"] = "<= 1e-6 normwise (--reorder)" if job.reorder else "bitwise"
    res["what"] = ("the returned global bucket vs the unsharded same-kernel reduce of regenerated inputs, on "
                   "windows at every stripe/rank slice boundary and replicated-tail edge"
                   + (" (2nd step from the initial state; v_t on every rank's own slice edges)" if fused else ""))
    return res


#: tests/test_gpu_bench.py's fault injection into one audited step (set by _install_injections)
_AUDIT_FAULT = None
AUDIT_STEPS = 20


def _checksums(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """Two exact integer checksums of an fp32 range's bit patterns: their sum, and their sum
    weighted by position (a range shifted or permuted changes the second)."""
    b = t.view(torch.int32).to(torch.int64)
    return torch.stack([b.sum(), (b * idx[: b.numel()]).sum()])


def push_audit(job, world, dev, steps: int = AUDIT_STEPS) -> dict:
    """After a push job's timed region: `steps` more steps, every one checked end to end.  Each
    rank checksums its own slice of every stripe on the compute stream right after the stripe's
    reduce (what it then pushes), and after the step every slice of the reassembled bucket; the
    senders' checksums are all-gathered and every receiver compares them with what landed — so a
    gather that corrupted one step in the middle, and not the last, is caught (the windowed
    bit-check of verify_job covers the last step only).  Collective: every rank runs the same
    steps and reaches the same verdict."""
    red, p = job.red, job.plan
    if red.pusher is None or red.full is None:
        return {"audited_steps": 0, "verified": True, "note": "no push gather"}
    idx = (torch.arange(max(p.widths), dtype=torch.int64, device=dev) % 65521) + 1
    real = red.reduce_fn
    sent = {}
    starts = {p.local_begin(c) for c in range(p.stripes)}  # the replicated tail is not pushed

    def hooked(lo, sc, out):
        real(lo, sc, out)
        if lo in starts:
            sent[lo] = _checksums(out, idx)

    red.reduce_fn = hooked
    bad = []
    try:
        for s in range(steps):
            if _AUDIT_FAULT is not None:
                _AUDIT_FAULT(s, red)
            sent.clear()
            red.step()
            mine = torch.stack([sent[p.local_begin(c)] for c in range(p.stripes)])  # [stripes, 2]
            every = torch.empty((world, p.stripes, 2), dtype=torch.int64, device=dev)
            fa_dist.all_gather_into(every.view(-1), mine.reshape(-1), group=None)
            got = torch.stack([torch.stack([_checksums(red.full[p.global_begin(c, r): p.global_begin(c, r) + p.widths[c]], idx)
                                            for c in range(p.stripes)]) for r in range(world)])
            wrong = (got != every).any(dim=2).nonzero().tolist()
            if wrong:
                bad.append({"step": s, "slices": [{"sender": r, "stripe": c} for r, c in wrong][:8]})
    finally:
        red.reduce_fn = real
    # every rank's verdict (a slice may be wrong on one receiver only)
    flags = torch.tensor([len(bad)], dtype=torch.int64, device=dev)
    all_flags = torch.empty(world, dtype=torch.int64, device=dev)
    fa_dist.all_gather_into(all_flags, flags)
    n_bad = [int(x) for x in all_flags.tolist()]
    return {"audited_steps": steps, "verified": sum(n_bad) == 0, "bad_steps_by_rank": n_bad,
            "first_bad": bad[:3], "checksums": "sum and position-weighted sum of the fp32 bit patterns, per "
                                                "(sender, stripe) slice: sender's after its reduce vs every receiver's bucket"}


def gather_probe(job, world, dev, reps: int = 5) -> dict:
    """All-gather rate of this job's local width (RCCL over xGMI at N > 1), outside the timed
    region: every GPU receives (world-1) slices, one over each peer link (one xGMI link per peer
    on an MI355X node)."""
    cols = job.plan.local_cols
    src = job.red.local_out[:cols]
    full = torch.empty(world * cols, dtype=torch.float32, device=dev)
    for _ in range(2):
        all_gather_into(full, src)
    torch.cuda.synchronize(dev)
    dist.barrier()
    t = _max_over_ranks((_event_time(lambda: all_gather_into(full, src), reps),), world, dev)[0]
    per_link = cols * 4 / t / 1e9
    return {"cols_per_rank": cols, "us": round(t * 1e6, 2), "ingress_gbs_per_gpu": round(per_link * (world - 1), 2),
            "per_link_gbs": round(per_link, 2)}


def rccl_version() -> str | None:
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - a build without RCCL: nothing to report
        return None


def loopback_multi_gpu(devices, rounds: int = 5, config: str = "c2") -> dict:
    """flearn's in-process server on an N-GPU node: Communicator.run collects every upload in ONE
    process (Communicator.py:127-141) and Server.ensemble calls strategy.server once
    (Server.py:126-142), so the drop-in there is AVG(devices=[cuda:0..N-1]) — each GPU packs and
    reduces its column share of the host uploads through its own PCIe link.  Times C2 loopback
    (100 x ResNet-18 host numpy uploads with BN counters) for output="reference" (host float64
    dict, the reference's types) and output="device" (tensors on cuda:0, peer copies over xGMI),
    checks each result bit for bit against the one-device call on the same uploads, and reports
    the per-GPU H2D rate of the pack phase."""
    import flearn_amd

    cfg = CONFIGS[config]
    layout = layouts.get(cfg["layout"])
    n, p = cfg["clients"], layouts.fp32_elems(layout)
    d0 = devices[0]
    x = torch.empty((n, p), dtype=torch.float32, device=d0)
    agg.fill_uniform(x, seed=UPLOAD_SEED)
    host = x.cpu().numpy()
    del x
    torch.cuda.empty_cache()
    uploads = [{"agg_weight": 1.0, "params": layouts.synthetic_state_dict(layout, host[i], counter=100 + i)}
               for i in range(n)]

    def sync():
        for d in set(devices):
            torch.cuda.synchronize(d)

    def host_of(v):
        if isinstance(v, torch.Tensor):
            return v.detach().cpu().numpy()
        return np.asarray(v)

    out = {"config": config, "clients": n, "params": p, "devices": [str(d) for d in devices],
           "upload_bytes": int(host.nbytes)}
    for output in ("reference", "device"):
        one = flearn_amd.AVG(output=output, devices=[d0])
        want = {k: host_of(v) for k, v in one.server(uploads, 0)["w_glob"].items()}
        one = None
        s = flearn_amd.AVG(output=output, devices=list(devices))
        eng = s.engine
        orig = eng.packer.pack
        pack_t, ingest = [], {}

        def pack(plan, w, orig=orig, pack_t=pack_t, ingest=ingest):
            t0 = time.perf_counter()
            stacks = orig(plan, w)
            sync()
            pack_t.append(time.perf_counter() - t0)
            for parts in stacks.values():
                for sh, st in parts:
                    if isinstance(st, torch.Tensor):
                        ingest[sh.index] = ingest.get(sh.index, 0) + n * sh.width * st.element_size()
            return stacks

        eng.packer.pack = pack
        times, got = [], None
        for r in range(rounds + 2):
            t0 = time.perf_counter()
            res = s.server(uploads, r)["w_glob"]
            sync()
            dt = time.perf_counter() - t0
            if r >= 2:
                times.append(dt)
            if r == 0:
                got = res
        ok = set(got) == set(want) and all(
            host_of(got[k]).dtype == want[k].dtype and host_of(got[k]).shape == want[k].shape
            and host_of(got[k]).tobytes() == want[k].tobytes() for k in want)
        calls = rounds + 2
        per_dev = {i: b / calls for i, b in ingest.items()}
        pk = float(np.median(pack_t[2:])) if len(pack_t) > 2 else float(np.median(pack_t))
        out[output] = {
            "round_ms": round(float(np.median(times)) * 1e3, 3),
            "pack_h2d_ms": round(pk * 1e3, 3),
            "h2d_gbs_per_gpu": [round(b / pk / 1e9, 2) for _, b in sorted(per_dev.items())],
            "h2d_gbs_total": round(sum(per_dev.values()) / pk / 1e9, 2),
            "verified": bool(ok),
        }
        eng.packer.pack = orig
        s = eng = None
        torch.cuda.empty_cache()
    out["verified"] = all(out[o]["verified"] for o in ("reference", "device"))
    out["what"] = ("AVG(devices=[...]).server(host uploads) per round (pack+H2D per GPU, reduce, D2H or device "
                   "assembly), median of the rounds after 2 warm-up calls; bit-compared with the 1-device call")
    return out


def _load_lastwords():
    """tools/liblastwords.so (built by __graft_entry__.build()): the held line written to stdout if a
    signal ends the process (a GPU fault's abort, torchrun's SIGTERM after another rank died)."""
    import ctypes

    path = Path(__file__).resolve().parent / "tools" / "liblastwords.so"
    if not path.exists():
        log(f"[rank 0] {path.name} not built: a crash in the later phases would lose the held line")
        return None
    lib = ctypes.CDLL(str(path))
    lib.lw_set.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    lib.lw_set.restype = ctypes.c_int
    lib.lw_clear.argtypes = []
    lib.lw_clear.restype = ctypes.c_int
    return lib


class HeldLine:
    """Rank 0's JSON line, built as soon as the RCCL job is timed and verified and refined by
    the later phases; printed exactly once — at the end, or by the Watchdog when a later phase
    overruns its budget, or (tools/lastwords.c) by a signal handler if the process is killed or
    aborts meanwhile: then the line carries `ended_by_signal.during` = the phase that was running."""

    def __init__(self, rank: int, lastwords=False):
        self.rank, self.line, self.exit_code = rank, None, 0
        self._lock = threading.Lock()
        self._printed = False
        self._phase = "between phases"
        self._lw = _load_lastwords() if lastwords and rank == 0 else None

    def set(self, line, exit_code: int):
        with self._lock:
            self.line, self.exit_code = line, exit_code
        self.guard(self._phase)

    def guard(self, phase: str):
        """Hand the current line, marked with `phase`, to the signal handler."""
        self._phase = phase
        if self._lw is None or self.line is None:
            return
        with self._lock:
            if self._printed:
                return
            data = json.dumps({**self.line, "ended_by_signal": {
                "during": phase, "note": "the process was ended by a signal (GPU fault, abort, or torchrun's "
                                         "SIGTERM after another rank died); this is the line held at that point"}})
            rc = self._lw.lw_set(data.encode(), len(data.encode()))
            if rc:
                log(f"[rank 0] lastwords: lw_set returned {rc}")

    def emit(self) -> bool:
        with self._lock:
            if self._printed or self.line is None or self.rank != 0:
                return False
            print(json.dumps(self.line), flush=True)
            self._printed = True
            if self._lw is not None:
                self._lw.lw_clear()
            return True


class Watchdog:
    """Bounds the phases after the secured RCCL line (the push gathers' set-up, calibration,
    trials and job; the weak job; the loopback): armed with a budget, it fires if the phase has
    not been disarmed in time — a hang in a collective or in a GPU wait, on any rank — annotates
    the held line with what overran, prints it (rank 0) and ends the process with os._exit (every
    rank has its own watchdog, so every rank ends).  No exec, no restart."""

    def __init__(self, held: HeldLine, rank: int):
        self.held, self.rank = held, rank
        self._lock = threading.Lock()
        self._deadline = None
        self._what = None
        self._annotate = None
        threading.Thread(target=self._run, daemon=True, name="bench-watchdog").start()

    def arm(self, seconds: float, what: str, annotate=None):
        with self._lock:
            self._deadline, self._what, self._annotate = time.monotonic() + seconds, what, annotate
        self.held.guard(what)

    def disarm(self):
        with self._lock:
            self._deadline = self._what = self._annotate = None
        self.held.guard("between phases")

    def _run(self):
        while True:
            time.sleep(0.25)
            with self._lock:
                fire = self._deadline is not None and time.monotonic() > self._deadline
                what, annotate = self._what, self._annotate
            if not fire:
                continue
            try:
                log(f"[rank {self.rank}] WATCHDOG: {what} overran its budget; ending with the held line")
                with self.held._lock:  # a copy: the main thread may still be refining the line
                    line = None if self.held.line is None else json.loads(json.dumps(self.held.line))
                if line is not None and annotate is not None:
                    try:
                        annotate(line)
                    except Exception:  # noqa: BLE001 - the line goes out whatever the annotation does
                        pass
                    with self.held._lock:
                        self.held.line = line
                self.held.emit()
                sys.stdout.flush()
                sys.stderr.flush()
            finally:  # whatever the emit did, the hang it bounds ends here
                os._exit(self.held.exit_code)


def job_extras(job, step_s, info, args, cfg, world, dev, g_eff, main_n, backend):
    """The collective measurements around a timed job: the dominant kernel's launch time (the
    reduce of this rank's whole local width), and at N > 1 the all-gather probe."""
    plan, cols = job.plan, job.plan.local_cols
    if g_eff == 1 and plan.stripes == 1:
        launch_s = step_s  # the step IS one kernel launch
    else:  # the reduce of this rank's whole local width as one launch (no gather)
        launch_s = _max_over_ranks((_event_time(lambda: job.fn(0, cols, job.red.local_out), args.steps),), world, dev)[0]
    if world > 1:
        info["world_size"] = dist.get_world_size()
        info["backend"] = dist.get_backend()
        info["rccl_version"] = rccl_version() if backend == "nccl" else None
        info["allgather_probe"] = gather_probe(job, world, dev)
        cal = info.get("calibration")
        if cal and cal.get("measured_gather"):
            c_cols, g_us = cal["width_cols"][0], cal["gather_us"][0]
            info["calibrated_per_link_gbs"] = round(c_cols * 4 / (g_us * 1e-6) / 1e9, 2) if g_us > 0 else None
    return launch_s


def build_line(args, cfg, world, g_eff, emu, main_n, job, step_s, wall, info, check, launch_s, cpu, backend):
    """Rank 0's JSON line (the driver's contract) for one timed job."""
    layout_p = job.plan.n_cols
    plan, cols = job.plan, job.plan.local_cols
    job_bytes = algorithmic_bytes(main_n, layout_p, cfg["op"]) if not emu else algorithmic_bytes(main_n, cols, cfg["op"])
    value = job_bytes / GIB / step_s
    # fa_reduce_f32 may run a wide window as several launches of consecutive column windows
    # (fa_reduce_windows): the per-launch bytes and time are the step's divided by that count
    launches = max(1, na.lib().fa_reduce_windows(na.OP_BY_NAME[cfg["op"]], cols))
    launch_bytes = algorithmic_bytes(main_n, cols, cfg["op"]) // launches
    launch_s = launch_s / launches
    achieved = launch_bytes / 1e9 / launch_s
    traffic, traffic_src = load_traffic(args.config) if g_eff == 1 else (None, None)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "bytes_per_launch": launch_bytes,
                "launch_us": round(launch_s * 1e6, 2), "launches_per_step": launches}
    if traffic_src:
        roofline["traffic_source"] = traffic_src
    weak_main = args.scaling == "weak" and g_eff > 1
    gather = info.get("gather")
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if weak_main else "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: device-generated splitmix64 U(-1,1) client uploads, agg_weight 1.0 (flearn default)",
        "config": {
            "workload": (f"{cfg['workload']}, weak-scaled: {main_n} clients on {g_eff} GPUs" if weak_main
                         else cfg["workload"] + (f" on {g_eff} GPUs (fixed problem)" if g_eff > 1 else "")),
            "config": args.config,
            "clients": main_n,
            "params": layout_p,
            "layout": cfg["layout"],
            "epilogue": cfg["op"],
            "order": ("split-N allowed (fixed-order tree of client splits, <= 1e-6 normwise)" if args.reorder
                      else "reference client order (bit-exact)"),
            "parallelism": ("single GPU" if g_eff == 1 else
                            f"element-range shards x{g_eff} + "
                            + {"push": "one-shot push all-gather over xGMI (peer stores)",
                               "push_dma": "one-shot push all-gather over xGMI (copy engines, one per peer)"}.get(
                                   gather, "RCCL all-gather") + f" ({plan.stripes} stripes"
                            + (f", widths {'/'.join(str(x) for x in plan.widths)}" if plan.stripes > 1 else "")
                            + (f"; the last {plan.rep} columns reduced by every rank, not gathered" if plan.rep else "")
                            + ")"
                            + (f"; EMULATED: rank 0's reduce of a {emu}-GPU job on one GPU, no gather" if emu else "")),
            # `value` against the HBM peak of the GPUs that produced it (N x 8 TB/s; at N > 1
            # the step includes the all-gather, so this is the job's, not a kernel's, fraction)
            "hbm_peak_frac_of_value": round(value * GIB / 1e9 / (HBM_PEAK_GBS * (world if not emu else 1)), 4),
            "hbm_peak_gbs_all_gpus": HBM_PEAK_GBS * (world if not emu else 1),
            "wall_s_timed_region": round(wall, 4),
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "verify": check,
    }
    if g_eff > 1:
        line["multi_gpu"] = dict(info)
        if world > 1 and backend != "nccl":
            line["multi_gpu"]["backend"] = f"{backend} (rehearsal: host-staged gather, not xGMI)"
        if check is not None:
            line["multi_gpu"]["verified"] = check["verified"]
            line["multi_gpu"]["verified_windows"] = check["windows"]
    return line


def _end_with_held_line(held, rank, e):
    """A later phase raised (multi-GPU): print the held line, marked with the phase and the error,
    and end this rank now — os._exit, since the process group's teardown may wait on dead peers."""
    log(f"[rank {rank}] a later phase failed: {type(e).__name__}: {e}; ending with the held line")
    if held.line is not None:
        held.line["ended_by_error"] = {"during": held._phase, "error": f"{type(e).__name__}: {e}"[:400]}
    held.emit()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(held.exit_code)


_OUTCOME_ROUND = [0]


def _agree_outcomes(status: str, rank: int, world: int, timeout_s: float):
    """Every rank's push-phase outcome via the process group's store (no collective); None when
    some rank has not posted within timeout_s."""
    from datetime import timedelta

    store = dist.distributed_c10d._get_default_store()
    _OUTCOME_ROUND[0] += 1
    keys = [f"flearn_bench/push_outcome/{_OUTCOME_ROUND[0]}/{r}" for r in range(world)]
    store.set(keys[rank], status)
    try:
        store.wait(keys, timedelta(seconds=timeout_s))
    except Exception:  # noqa: BLE001 - a timeout: a peer is stuck or gone
        return None
    return [store.get(k).decode() for k in keys]


def _exit_code(check) -> int:
    return verify.EXIT_MISMATCH if (check is not None and not check["verified"]) else 0


def _install_injections(rank):
    inject = os.environ.get("FLEARN_BENCH_INJECT", "")
    if inject == "gather_offset":
        # rehearsal of a mis-gathering collective (tests/test_gpu_bench.py): every stripe's
        # gathered range lands ALIGN columns late — the self-check must catch it and fail the run
        real_gather = fa_dist.all_gather_into

        def late_gather(dst, src, group=None, async_op=False):
            real_gather(dst, src, group=group, async_op=False)
            dst.copy_(torch.roll(dst, ALIGN))

        fa_dist.all_gather_into = late_gather
    if inject == "push_offset":
        # rehearsal of a mis-placed push (tests/test_gpu_bench.py): every pushed slice lands ALIGN
        # columns off — the self-check must catch it and the line keep RCCL's all-gather
        real_push = fa_dist.PushGather.push

        def off_push(self, src, elem_offset):
            shifted = elem_offset + ALIGN
            if shifted + src.numel() > self.full.numel():
                shifted = elem_offset - ALIGN
            return real_push(self, src, shifted)

        fa_dist.PushGather.push = off_push
    if inject == "push_skip_mid" and rank == 1:
        # rehearsal of a gather that goes wrong in ONE step that is neither the last timed step nor
        # the one verify_job bit-checks (tests/test_gpu_bench.py): rank 1 skips its push of the
        # first stripe in the 8th audited step — the step audit must catch it, the line keep RCCL
        real_push = fa_dist.PushGather.push
        skip = {"armed": False}

        def skipping_push(self, src, elem_offset):
            if skip["armed"]:
                skip["armed"] = False
                log("[rank 1] INJECTED: skipping one push in an audited step")
                return None
            return real_push(self, src, elem_offset)

        def fault(step, red):
            if step == 7:
                skip["armed"] = True

        fa_dist.PushGather.push = skipping_push
        global _AUDIT_FAULT
        _AUDIT_FAULT = fault
    if inject == "push_stall" and rank == 1:
        # rehearsal of a rank that never comes back from the push set-up (tests/test_gpu_bench.py):
        # the watchdog must still print the verified RCCL line within the budget
        real_init = fa_dist.PushGather.__init__

        def stalled_init(self, *a, **k):
            log("[rank 1] INJECTED: stalling in the push set-up")
            while True:
                time.sleep(1.0)

        fa_dist.PushGather.__init__ = stalled_init
        del real_init
    if inject == "push_crash" and rank == 1:
        # rehearsal of a rank that dies in the push set-up (a GPU fault's abort, say): torchrun
        # then ends the others with SIGTERM, or their next collective raises — rank 0 must still
        # print the verified RCCL line (tools/lastwords.c, _end_with_held_line)
        def crashing_init(self, *a, **k):
            log("[rank 1] INJECTED: dying in the push set-up")
            sys.stderr.flush()
            os._exit(7)

        fa_dist.PushGather.__init__ = crashing_init
    return inject


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=None,
                    help="fix the reduce/gather pipeline depth (N>1); default: the calibrated model's plan")
    ap.add_argument("--stripe-weights", default=None,
                    help="relative stripe widths with --stripes, e.g. 3,1; 'equal' (default) for equal")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="N>1: which job is `value` (the other one is reported beside it)")
    ap.add_argument("--no-weak", action="store_true", help="N>1: skip the weak-scaling job")
    ap.add_argument("--emulate-world", type=int, default=None,
                    help="single process: time rank 0's reduce of a G-GPU job (no gather)")
    ap.add_argument("--cpu-sample", type=int, default=None, help="clients in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reorder", action="store_true",
                    help="allow the split-N kernel (deterministic, <= 1e-6 normwise, not bit-exact)")
    ap.add_argument("--no-verify", action="store_true", help="skip the post-run check of the reassembled model")
    ap.add_argument("--gather", choices=("auto", "rccl", "push", "push_dma"), default="auto",
                    help="N>1: how stripes are reassembled — RCCL's all-gather, the one-shot push over "
                         "xGMI by kernel stores or by copy engines (flearn_amd.dist.PushGather), or "
                         "whichever measures fastest.  The RCCL job is always timed and verified first")
    ap.add_argument("--push-budget-s", type=float, default=float(os.environ.get("FLEARN_BENCH_PUSH_BUDGET_S", 120)),
                    help="N>1: wall-clock budget of the push phase (set-up, calibration, trials, job)")
    ap.add_argument("--phase-budget-s", type=float, default=float(os.environ.get("FLEARN_BENCH_PHASE_BUDGET_S", 120)),
                    help="N>1: budget of the weak job and of the loopback, each")
    ap.add_argument("--deadline-s", type=float, default=float(os.environ.get("FLEARN_BENCH_DEADLINE_S", 480)),
                    help="N>1: an optional phase (push, weak job, loopback) starts only if it can end within "
                         "this many seconds of the start, budget included (the driver's limit is ~600 s)")
    ap.add_argument("--no-loopback", action="store_true",
                    help="N>1: skip the single-process AVG(devices=[...]) loopback measurement")
    args = ap.parse_args()
    t_start = time.monotonic()

    def time_for(budget: float) -> bool:  # may an optional phase of this budget still start?
        return time.monotonic() - t_start + budget <= args.deadline_s

    # one process per GPU: with no launcher env, --gpus N > 1 starts the N ranks here, BEFORE any
    # HIP call in this process (na.lib(), torch.cuda.set_device, ...), and exits with their status
    if args.emulate_world is not None and args.gpus != 1:
        raise SystemExit("--emulate-world is a single-process mode (use --gpus 1)")
    rc = launch.ensure_ranks(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # FLEARN_BENCH_BACKEND=gloo (tests/test_gpu_bench.py): rehearse the N>1 path with several
    # ranks sharing the GPUs there are (RCCL refuses two ranks on one device); the gather is then
    # host-staged and its times say nothing about xGMI.  The real runs use RCCL.
    backend = os.environ.get("FLEARN_BENCH_BACKEND", "nccl")
    na.lib()
    if backend != "nccl":
        local_rank %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    _install_injections(rank)

    cfg = CONFIGS[args.config]
    layout = layouts.get(cfg["layout"])
    emu = args.emulate_world
    g_eff = emu or world  # GPUs of the (possibly emulated) job
    strong_n, weak_n = cfg["clients"], cfg["clients"] * g_eff
    main_n = strong_n if args.scaling == "strong" else weak_n
    held = HeldLine(rank, lastwords=world > 1)  # multi-GPU: a crash in a later phase still prints the line
    dog = Watchdog(held, rank) if world > 1 else None

    def self_check(job):
        if args.no_verify:
            return None
        log(f"[rank {rank}] verifying the reassembled model ...")
        c = verify_job(job, cfg, world, dev, emulated=bool(emu))
        if rank == 0:
            log(f"[rank 0] verified={c['verified']} windows={c['windows']} mismatched={c['mismatched_windows']}")
        return c

    # ---- phase 1: RCCL's all-gather (one GPU: the kernel alone) — timed, verified, held -------
    job, step_s, wall, info = run_job(cfg, layout, main_n, args, world, rank, dev, g_eff, gather="rccl")
    check = self_check(job)
    launch_s = job_extras(job, step_s, info, args, cfg, world, dev, g_eff, main_n, backend)
    cpu = None
    if rank == 0 and g_eff == 1 and not args.no_cpu_baseline:
        sample = args.cpu_sample or min(main_n, 100)
        log(f"[rank 0] CPU baseline over {sample} clients ...")
        cpu = cpu_baseline(job.stack, layout, sample)
    line = build_line(args, cfg, world, g_eff, emu, main_n, job, step_s, wall, info, check, launch_s, cpu, backend)
    held.set(line, _exit_code(check))
    rccl = {"gather": "rccl", "ms_per_step": round(step_s * 1e3, 4), "value": line["value"],
            "verified": None if check is None else check["verified"]}
    if g_eff > 1:
        line["multi_gpu"]["phases"] = {"rccl": rccl}
    gather_main = "rccl"
    if world > 1:
        dist.barrier()

    # the phases after the secured line: an exception in any of them (a peer that died mid-collective
    # raises on gloo) ends every rank with the held line, not a traceback without one
    try:
        # ---- phase 2: the one-shot push gathers, bounded; adopted only if faster AND verified ------
        # (not when the RCCL job failed its self-check: that line stands, and the run exits non-zero)
        rccl_failed = check is not None and not check["verified"]
        if rccl_failed and g_eff > 1:
            line["multi_gpu"]["phases"]["push"] = {"status": "skipped: the RCCL job failed its self-check"}
        # every rank decides alike: rank 0's clock, broadcast
        def agreed(flag: bool) -> bool:
            if world == 1:
                return flag
            box = [flag]
            dist.broadcast_object_list(box, src=0)
            return bool(box[0])

        push_time = agreed(time_for(args.push_budget_s)) if world > 1 and args.gather != "rccl" and not rccl_failed else True
        if not push_time:
            line["multi_gpu"]["phases"]["push"] = {"status": "skipped: out of time", "deadline_s": args.deadline_s}
        if world > 1 and args.gather != "rccl" and not rccl_failed and push_time:
            t_phase = time.perf_counter()
            ph = {"status": "started", "budget_s": args.push_budget_s}
            line["multi_gpu"]["phases"]["push"] = ph

            def overran(ln, t_phase=t_phase):
                p = ln["multi_gpu"]["phases"]["push"]
                p.update(status="timed_out", elapsed_s=round(time.perf_counter() - t_phase, 1),
                         note="a rank did not finish the push phase within its budget: the RCCL line stands")

            dog.arm(args.push_budget_s, "push phase", overran)
            status, pjob, pinfo = "error", None, {}
            try:
                r_big = (info.get("calibration") or {}).get("reduce_us", [0.0])[0] * 1e-6
                pplan, pg_name, pinfo, pbest = plan_push(cfg, layout, main_n, args, world, rank, dev, g_eff, r_big)
                best_rccl = min((t["measured_ms"] for t in info.get("plan_trials", []) if t["measured_ms"]), default=None)
                if pplan is None:
                    status = "unavailable"
                elif args.gather == "auto" and best_rccl is not None and pbest is not None and pbest * 1e3 >= best_rccl:
                    status = "slower_in_trials"
                else:
                    pjob, pstep, pwall, ptinfo = timed_job(cfg, layout, main_n, pplan, pg_name, pinfo.get("push_grid"),
                                                           args, world, dev, g_eff)
                    pinfo.update(ptinfo)
                    log(f"[rank {rank}] auditing {AUDIT_STEPS} more steps of the {pg_name} gather ...")
                    paudit = push_audit(pjob, world, dev)
                    pinfo["push_audit"] = paudit
                    pcheck = self_check(pjob)
                    if not paudit["verified"]:
                        status = "failed_self_check"
                        pinfo["push_failed_self_check"] = {"gather": pg_name, "audit": paudit,
                                                           "mismatched_windows": None if pcheck is None else
                                                           pcheck["mismatched_windows"]}
                        log(f"[rank {rank}] the {pg_name} gather failed its step audit: keeping the RCCL line")
                    elif pcheck is not None and not pcheck["verified"]:
                        status = "failed_self_check"
                        pinfo["push_failed_self_check"] = {"gather": pg_name, "mismatched_windows": pcheck["mismatched_windows"],
                                                           "first_mismatches": pcheck.get("first_mismatches")}
                        log(f"[rank {rank}] the {pg_name} gather failed the self-check: keeping the RCCL line")
                    elif args.gather == "auto" and pstep >= step_s:
                        status = "slower"
                    else:
                        status = "adopted"
                    ph.update(ms_per_step=round(pstep * 1e3, 4), gather=pg_name,
                              verified=None if pcheck is None else pcheck["verified"],
                              audited_steps=paudit["audited_steps"], audit_verified=paudit["verified"])
            except Exception as e:  # noqa: BLE001 - any failure here leaves the RCCL line standing
                log(f"[rank {rank}] push phase failed: {type(e).__name__}: {e}")
                ph["error"] = f"{type(e).__name__}: {e}"
            # every rank's outcome, through the store rather than a collective: a rank that raised
            # may have left its peers inside one of the phase's collectives, and a collective here
            # could pair with theirs.  Peers that never post theirs are stuck: this rank then ends
            # with the held line (and their watchdogs end them)
            outcomes = _agree_outcomes(status, rank, world, max(args.push_budget_s - (time.perf_counter() - t_phase), 5.0))
            if outcomes is None:
                ph["status"] = "error"
                _end_with_held_line(held, rank, RuntimeError("a peer never posted its push-phase outcome"))
            adopt = all(o == "adopted" for o in outcomes)
            ph["status"] = "adopted" if adopt else next((o for o in outcomes if o != "adopted"), status)
            ph["rank_outcomes"] = outcomes
            for k in ("push_calibration", "push_dma_calibration"):
                if k in pinfo:
                    line["multi_gpu"][k] = pinfo[k]
            if "plan_trials" in pinfo:
                line["multi_gpu"]["plan_trials"] = line["multi_gpu"].get("plan_trials", []) + pinfo["plan_trials"]
            if "push_failed_self_check" in pinfo:
                line["multi_gpu"]["push_failed_self_check"] = pinfo["push_failed_self_check"]
            if adopt:
                job.release()
                job, step_s, wall, info, check = pjob, pstep, pwall, {**info, **pinfo}, pcheck
                gather_main = pg_name
                launch_s = job_extras(job, step_s, info, args, cfg, world, dev, g_eff, main_n, backend)
                phases = line["multi_gpu"]["phases"]
                trials = line["multi_gpu"].get("plan_trials")
                line = build_line(args, cfg, world, g_eff, emu, main_n, job, step_s, wall, info, check, launch_s, cpu, backend)
                line["multi_gpu"]["phases"] = phases
                if trials is not None:
                    line["multi_gpu"]["plan_trials"] = trials
                held.set(line, _exit_code(check))
            elif pjob is not None:
                pjob.release()
            ph["elapsed_s"] = round(time.perf_counter() - t_phase, 1)
            # the push gathers' receive buckets on this rank: mapped by the pool, and released ones
            # parked for reuse (bounded: fa_dist.PARK_CAP x the largest exported)
            line["multi_gpu"]["push_receive_buckets"] = {
                "pool_bytes": fa_dist._RecvPool.bytes_held(), "parked_bytes": fa_dist.DeviceBuffer.parked_bytes(dev),
                "park_cap_bytes": fa_dist.DeviceBuffer.park_cap(dev), "trimmed": fa_dist.DeviceBuffer.trimmed()}
            dist.barrier()
            dog.disarm()

        # ---- phase 3: the weak job beside it, the loopback drop-in — each bounded -------------------
        weak_time = agreed(time_for(args.phase_budget_s)) if g_eff > 1 and emu is None else True
        if g_eff > 1 and not args.no_weak and emu is None and not rccl_failed and not weak_time:
            line["weak"] = {"status": "skipped: out of time", "deadline_s": args.deadline_s}
        if g_eff > 1 and not args.no_weak and emu is None and not rccl_failed and weak_time:
            def weak_overran(ln):
                ln["weak"] = {"status": "timed_out", "budget_s": args.phase_budget_s}

            dog.arm(args.phase_budget_s, "weak job", weak_overran)
            job.release()
            other_n = weak_n if args.scaling == "strong" else strong_n
            ojob, ostep, _, oinfo = run_job(cfg, layout, other_n, args, world, rank, dev, g_eff, gather=gather_main)
            line[("weak" if args.scaling == "strong" else "strong")] = {
                "scaling": "weak" if args.scaling == "strong" else "strong",
                "clients": other_n,
                "value": round(algorithmic_bytes(other_n, layouts.fp32_elems(layout), cfg["op"]) / GIB / ostep, 2),
                "unit": "GiB/s",
                "ms_per_step": round(ostep * 1e3, 4),
                **oinfo,
            }
            ojob.release()
            dist.barrier()
            dog.disarm()

        if world > 1:
            if job is not None and job.red is not None:
                job.red.release()  # collective: the bucket back to the pool while the group exists
            fa_dist.shutdown_push()  # every peer unmaps, then the receive buckets are parked
            dist.barrier()
            dist.destroy_process_group()
        loop = None
        if world > 1 and rank == 0 and not args.no_loopback and not rccl_failed and not time_for(args.phase_budget_s):
            line["loopback_multi_gpu"] = {"status": "skipped: out of time", "deadline_s": args.deadline_s}
        elif world > 1 and rank == 0 and not args.no_loopback and not rccl_failed:
            # the single-process multi-GPU drop-in (flearn's Communicator collects every upload in one
            # process): rank 0 alone, after the process group is gone, drives every GPU of the node
            ndev = max(torch.cuda.device_count(), 1)
            devices = [torch.device("cuda", i % ndev) for i in range(world)]
            job.release()
            job = None

            def loop_overran(ln):
                ln["loopback_multi_gpu"] = {"status": "timed_out", "budget_s": args.phase_budget_s}

            dog.arm(args.phase_budget_s, "loopback", loop_overran)
            log(f"[rank 0] loopback AVG(devices={[str(d) for d in devices]}) ...")
            loop = loopback_multi_gpu(devices)
            dog.disarm()
            line["loopback_multi_gpu"] = loop
            if not loop["verified"]:
                held.set(line, verify.EXIT_MISMATCH)

    except Exception as e:  # noqa: BLE001
        if world == 1:
            raise
        _end_with_held_line(held, rank, e)

    held.emit()
    if held.exit_code:
        log(f"[rank {rank}] SELF-CHECK FAILED: the reassembled global model differs from the unsharded reduce")
        sys.exit(held.exit_code)


if __name__ == "__main__":
    main()
