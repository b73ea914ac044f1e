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
  --scaling weak   (default) the job aggregates clients x G uploads on G GPUs, so every GPU
                   streams the same bytes as the 1-GPU run (G=8 from c2: 800 clients x
                   ResNet-18, the shape of BASELINE config 4)
  --scaling strong the config's clients on G GPUs (each GPU reduces P/G columns)
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
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from flearn_amd import _native as na  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import launch, layouts  # noqa: E402
from flearn_amd.dist import ShardedReducer, ShardPlan, hip_reduce_fn  # noqa: E402

METRIC = "device-resident GiB/s, FedAVG N-client weighted tensor reduce; %HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = 1024.0**3
DEFAULT_STRIPES = 2  # N>1: stripe 0's all-gather overlaps stripe 1's reduce ...
DEFAULT_STRIPE_WEIGHTS = (3, 1)  # ... and the small last stripe leaves little of the gather exposed

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=None, help="reduce/gather pipeline depth (N>1)")
    ap.add_argument("--stripe-weights", default=None,
                    help="relative stripe widths, e.g. 3,1 (default for 2 stripes); 'equal' for equal")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--emulate-world", type=int, default=None,
                    help="single process: time rank 0's reduce of a G-GPU job (no gather)")
    ap.add_argument("--cpu-sample", type=int, default=None, help="clients in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reorder", action="store_true",
                    help="allow the split-N kernel (deterministic, <= 1e-6 normwise, not bit-exact)")
    args = ap.parse_args()

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
    na.lib()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = CONFIGS[args.config]
    layout = layouts.get(cfg["layout"])
    emu = args.emulate_world
    if emu is not None and world != 1:
        raise SystemExit("--emulate-world is a single-process mode")
    g_eff = emu or world  # GPUs of the (possibly emulated) job
    n = cfg["clients"] * (g_eff if args.scaling == "weak" else 1)
    p_real = layouts.fp32_elems(layout)
    stripes = args.stripes or (1 if g_eff == 1 else DEFAULT_STRIPES)
    if args.stripe_weights == "equal" or stripes == 1:
        sw = None
    elif args.stripe_weights:
        sw = tuple(float(x) for x in args.stripe_weights.split(","))
    else:
        sw = DEFAULT_STRIPE_WEIGHTS if stripes == len(DEFAULT_STRIPE_WEIGHTS) else None
    plan = ShardPlan.make(p_real, g_eff, rank, stripes, weights=sw)
    cols = plan.local_cols

    # ---- device-resident synthetic uploads: this rank's columns of all N clients ----
    log(f"[rank {rank}] alloc {n} x {cols} fp32 = {n * cols * 4 / 1e9:.2f} GB")
    stack = torch.empty((n, cols), dtype=torch.float32, device=dev)
    for c in range(stripes):
        lo = plan.local_begin(c)
        agg.fill_uniform(stack[:, lo:], seed=2024, row_begin=0, col_begin=plan.global_begin(c),
                         n_cols=plan.shard_of(c))
    weights = torch.ones(n, dtype=torch.float32, device=dev)  # Python 1.0 -> fl32(1.0)
    denom = float(np.sum([1.0] * n))  # np.sum(agg_weight_lst), strategy.py:127
    epi = {}
    local_out = None
    if cfg["op"] != "mean":
        prev = torch.empty((1, cols), dtype=torch.float32, device=dev)
        for c in range(stripes):
            lo = plan.local_begin(c)
            agg.fill_uniform(prev[:, lo:], seed=1, col_begin=plan.global_begin(c), n_cols=plan.shard_of(c))
        prev = prev[0]
        v = torch.zeros(cols, dtype=torch.float64, device=dev)
        epi = dict(op=na.OP_BY_NAME[cfg["op"]], prev=prev, v=v)
        local_out = prev  # the fused step advances the global model in place
    fn = hip_reduce_fn(stack, weights, na.MODE_W32_DIV64, denom, reorder=args.reorder, **epi)
    red = ShardedReducer(plan, fn, dev, local_out=local_out, gather=world > 1)

    # ---- warmup + timed steps ----
    for _ in range(args.warmup):
        red.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        red.step()
    ev1.record()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = ev0.elapsed_time(ev1) / 1e3  # s, on the stream the kernels run on
    elapsed = max(elapsed, 0.0)
    if world > 1:
        t = torch.tensor([elapsed, wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, wall = t.tolist()
    step_s = elapsed / args.steps
    job_bytes = algorithmic_bytes(n, p_real, cfg["op"])
    if emu:  # rank 0's columns only
        job_bytes = algorithmic_bytes(n, plan.local_cols, cfg["op"])
    value = job_bytes / GIB / step_s

    # ---- roofline of the dominant kernel: per-launch algorithmic bytes / launch time ----
    if g_eff == 1 and stripes == 1:
        launch_s = step_s  # the step IS one kernel launch
        launch_cols = p_real
    else:  # time the reduce launches alone (no gather) on this rank
        k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k0.record()
        for _ in range(args.steps):
            fn(0, cols, red.local_out)
        k1.record()
        torch.cuda.synchronize(dev)
        launch_s = k0.elapsed_time(k1) / 1e3 / args.steps
        launch_cols = cols
    launch_bytes = algorithmic_bytes(n, launch_cols, cfg["op"])
    achieved = launch_bytes / 1e9 / launch_s
    traffic, traffic_src = load_traffic(args.config) if g_eff == 1 else (None, None)
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "bytes_per_launch": launch_bytes,
        "launch_us": round(launch_s * 1e6, 2),
    }
    if traffic_src:
        roofline["traffic_source"] = traffic_src

    cpu = None
    if rank == 0 and g_eff == 1 and not args.no_cpu_baseline:
        sample = args.cpu_sample or min(n, 100)
        log(f"[rank 0] CPU baseline over {sample} clients ...")
        cpu = cpu_baseline(stack, layout, sample)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic: device-generated splitmix64 U(-1,1) client uploads, agg_weight 1.0 (flearn default)",
            "config": {
                "workload": (cfg["workload"] if g_eff == 1 or args.scaling == "strong" else
                             f"{cfg['workload']}, weak-scaled: {n} clients on {g_eff} GPUs"),
                "config": args.config,
                "clients": n,
                "params": p_real,
                "layout": cfg["layout"],
                "epilogue": cfg["op"],
                "order": ("split-N allowed (fixed-order tree of client splits, <= 1e-6 normwise)" if args.reorder
                          else "reference client order (bit-exact)"),
                "parallelism": ("single GPU" if g_eff == 1 else
                                f"element-range shards x{g_eff} + RCCL all-gather ({stripes} stripes"
                                + (f", widths {'/'.join(str(x) for x in plan.widths)}" if stripes > 1 else "") + ")"
                                + (f"; EMULATED: rank 0's reduce of a {emu}-GPU job on one GPU, no gather"
                                   if emu else "")),
                "hbm_peak_frac_of_value": round(value * GIB / 1e9 / HBM_PEAK_GBS, 4),
                "wall_s_timed_region": round(wall, 4),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
