"""Strong-scaling projection of bench.py --gpus G from the stripe model
(flearn_amd.dist.StripeModel / plan_stripes) with a per-link xGMI assumption.

On an 8-GPU MI355X node every GPU has one xGMI link to each peer, so an all-gather among G GPUs
brings (G-1)/G of the bucket into each GPU over G-1 links: ingress(G) = (G-1) * link rate.  The
reduce coefficients are the measured 1-GPU kernel rates (profiles/r03/final), the launch and
collective constants the model's a priori ones.  A PROJECTION: nothing here has run on more than
one GPU.

    python tools/project_scaling.py [--link-gbs 50,64] [--json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from flearn_amd.dist import ALIGN, StripeModel, plan_shards, plan_stripes  # noqa: E402

# config -> (clients, fp32 params, 1-GPU step of the final profile pass in s, algorithmic bytes/col)
CONFIGS = {
    "ns": (100, 25_610_152),
    "c4": (1000, 11_699_112),
    "c5": (100, 86_567_656),
}


def one_gpu_step(cfg: str) -> float:
    """The newest profile pass's 1-GPU step (profiles/r05/final, else r03)."""
    for rnd in ("r05", "r03"):
        f = REPO / "profiles" / rnd / "final" / cfg / f"bench_{cfg}.json"
        if f.exists():
            return json.loads(f.read_text())["ms_per_step"] / 1e3
    raise FileNotFoundError(cfg)


OVERLAP = (REPO / "profiles" / "r04" / "overlap" / "overlap.json",
           REPO / "profiles" / "r04" / "overlap" / "overlap_rw.json")


def contention(ingress_bs: float, paths=OVERLAP, local_traffic: float = 2.0):
    """(c_r, c_g, the stand-in used) for a gather bringing `ingress_bs` into each GPU: from the
    one-GPU overlap probes (tools/overlap_probe.py) at the library's default reduce grid, the
    smallest copy stand-in whose local HBM traffic (2 x its copy rate: read + write) is at least
    the gather's (2 x ingress: the received bytes written, the rank's own slice read once per
    peer) — the next measured point above, or the largest.  Copy points of every probe file
    (2-64 blocks: 19-552 GB/s)."""
    pts = []
    for path in paths:
        if not Path(path).exists():
            continue
        d = json.loads(Path(path).read_text())
        row = next(r for r in d["rows"] if r["grid"] == "default")
        pts += [(v["copy_alone_gbs"] * 1e9, v["reduce_slowdown"] - 1.0, v["copy_slowdown"] - 1.0, k)
                for k, v in row["with"].items() if k.isdigit()]
    pts.sort()
    for rate, c_r, c_g, k in pts:
        if 2.0 * rate >= local_traffic * ingress_bs:
            return c_r, c_g, f"copy on {k} blocks ({rate / 1e9:.0f} GB/s)"
    rate, c_r, c_g, k = pts[-1]
    return c_r, c_g, f"copy on {k} blocks ({rate / 1e9:.0f} GB/s)"


PUSH_PROBE = REPO / "profiles" / "r04" / "overlap" / "overlap_push.json"
PUSH_DMA_PROBE = REPO / "profiles" / "r04" / "overlap" / "overlap_push_dma.json"


def push_dma_contention(ingress_bs: float, path=PUSH_DMA_PROBE, push_path=PUSH_PROBE):
    """(c_r, c_g, stand-in) of the copy-engine push: the sender's legs are copy-engine transfers
    over a link (dmahost: device -> pinned memory over PCIe), the receiver's HBM takes the peers'
    stores like a write-only stream at the ingress rate (wr<B> from the push probe)."""
    d = json.loads(Path(path).read_text())
    v = next(r for r in d["rows"] if r["grid"] == "default")["with"]["dmahost"]
    w = next(r for r in json.loads(Path(push_path).read_text())["rows"] if r["grid"] == "default")["with"]
    wr = sorted((x["copy_alone_gbs"] * 1e9, x) for k, x in w.items() if k.startswith("wr"))
    rate, wv = next(((r, x) for r, x in wr if r >= ingress_bs), wr[-1])
    c_r = (v["reduce_slowdown"] - 1.0) + (wv["reduce_slowdown"] - 1.0)
    return c_r, max(v["copy_slowdown"] - 1.0, 0.0), f"copy engine + writes at {rate / 1e9:.0f} GB/s"


def push_contention(ingress_bs: float, path=PUSH_PROBE, blocks=None):
    """(c_r, c_g, stand-in) of the one-shot push from the one-GPU probe: the sender's push kernel
    (pushhost<B>: a link-bound fa_push into pinned memory over PCIe, at the smallest grid that
    reaches 95% of its best rate) slows the reduce and is slowed by it; the peers' stores landing
    in this GPU's HBM act like a write-only stream at the ingress rate (wr<B>: the first one at
    or above it).  The two reduce terms add."""
    d = json.loads(Path(path).read_text())
    w = next(r for r in d["rows"] if r["grid"] == "default")["with"]
    ph = sorted((int(k[8:]), v) for k, v in w.items() if k.startswith("pushhost") and k[8:])
    top = max(v["copy_alone_gbs"] for _, v in ph)
    b, v = (next((b, v) for b, v in ph if b == blocks) if blocks else
            next((b, v) for b, v in ph if v["copy_alone_gbs"] >= 0.95 * top))
    wr = sorted((v["copy_alone_gbs"] * 1e9, v) for k, v in w.items() if k.startswith("wr"))
    rate, wv = next(((r, v) for r, v in wr if r >= ingress_bs), wr[-1])
    c_r = (v["reduce_slowdown"] - 1.0) + (wv["reduce_slowdown"] - 1.0)
    return c_r, v["copy_slowdown"] - 1.0, f"push on {b} blocks + writes at {rate / 1e9:.0f} GB/s"


def project(cfg: str, g: int, link_bs: float, launch_s=10e-6, collective_s=30e-6, tail=True, contended=False,
            push=False, barrier_s=15e-6, dma=False, dma_egress_bs=None, push_probe=PUSH_PROBE, serial=False,
            push_blocks=None):
    """push: the one-shot push gather (flearn_amd.dist.PushGather) — a launch per stripe instead
    of a collective, two barriers per step, and local HBM traffic of ingress * (1 + 1/(G-1))
    (received bytes written, the own slice read once) instead of a ring's ~2 x ingress.
    dma_egress_bs (with dma): what the copy engines that run at once move out of one GPU in all
    (round 5, tools/probe_dma_legs.py untraced: ~955 GB/s for 7 device-to-device legs; the ~140
    GB/s first read from a profiled run was the profiler's); every leg then gets
    min(link, egress / (G-1))."""
    n, p = CONFIGS[cfg]
    if push and dma and dma_egress_bs and g > 1:
        link_bs = min(link_bs, dma_egress_bs / (g - 1))
    t1 = one_gpu_step(cfg)
    local = -(-p // g)
    local = -(-local // ALIGN) * ALIGN
    b_r = t1 / p  # the 1-GPU per-column cost (fused state traffic included)
    b_g = (g - 1) * 4.0 / ((g - 1) * link_bs) if g > 1 else 0.0
    a_g = (launch_s if push else collective_s) if g > 1 else 0.0
    m = StripeModel(launch_s, b_r, a_g, b_g)
    stand_in = None
    if contended and g > 1:
        ingress = (g - 1) * link_bs
        c_r, c_g, stand_in = (push_dma_contention(ingress, PUSH_DMA_PROBE if str(push_probe) == str(PUSH_PROBE)
                                                  else push_probe, push_probe) if push and dma else
                              push_contention(ingress, push_probe, push_blocks) if push else contention(ingress))
        m = m.with_contention(c_r, c_g)
    if g == 1 or serial:
        widths, rep = (local,), 0
    elif tail:
        widths, rep = plan_shards(p, g, m)
    else:
        widths, rep = plan_stripes(local, m), 0
    step, red, exposed = m.makespan(widths, rep)
    if push and g > 1:
        step += 2 * barrier_s
    return {"config": cfg, "gather": "push" if push else "rccl", "gpus": g, "link_GBs": link_bs / 1e9, "ingress_GBs": (g - 1) * link_bs / 1e9,
            "stripes": len(widths), "replicated_frac": round(rep / p, 3), "step_ms": round(step * 1e3, 3),
            "reduce_ms": round(red * 1e3, 3), "exposed_gather_ms": round(exposed * 1e3, 3),
            "speedup": round(t1 / step, 2), "c_r": round(m.c_r, 3), "c_g": round(m.c_g, 3), "stand_in": stand_in}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--link-gbs", default="50,64")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--no-tail", action="store_true", help="stripes only (no replicated tail)")
    ap.add_argument("--push", action="store_true", help="the one-shot push gather instead of RCCL's all-gather")
    ap.add_argument("--dma", action="store_true", help="with --push: its copy-engine form (one leg per peer)")
    ap.add_argument("--dma-egress-gbs", type=float, default=None,
                    help="with --push --dma: the copy engines' total egress per GPU (measured untraced: ~955)")
    ap.add_argument("--push-probe", default=str(PUSH_PROBE),
                    help="the push contention probe (round 5's untraced rerun: profiles/r05/copy_paths/overlap_push_r05.json)")
    ap.add_argument("--push-blocks", type=int, default=None,
                    help="with --push: the stand-in's block count (default: the fewest within 95%% of its best rate)")
    ap.add_argument("--serial", action="store_true",
                    help="one stripe, no overlap: what a gather whose stream shares the compute stream's hardware "
                         "queue gets (DESIGN.md section 6, the pipeline's streams)")
    ap.add_argument("--contended", action="store_true",
                    help="reduce / gather slowed by the measured one-GPU contention (profiles/r04/overlap)")
    a = ap.parse_args()
    egress = a.dma_egress_gbs * 1e9 if a.dma_egress_gbs else None
    rows = [project(c, g, float(l) * 1e9, tail=not a.no_tail, contended=a.contended, push=a.push, dma=a.dma,
                    dma_egress_bs=egress, push_probe=a.push_probe, serial=a.serial, push_blocks=a.push_blocks)
            for l in a.link_gbs.split(",") for c in CONFIGS for g in (2, 4, 8)]
    if a.json:
        print(json.dumps(rows, indent=1))
        return
    for r in rows:
        print(f"{r['link_GBs']:>5.0f} GB/s/link  {r['config']:>3}  G={r['gpus']}  ingress {r['ingress_GBs']:>4.0f} GB/s  "
              f"{r['stripes']} stripes  tail {r['replicated_frac']:.3f}  step {r['step_ms']:.3f} ms  (reduce {r['reduce_ms']:.3f}, exposed gather "
              f"{r['exposed_gather_ms']:.3f})  {r['speedup']:.2f}x  c_r {r['c_r']} c_g {r['c_g']}")


if __name__ == "__main__":
    main()
