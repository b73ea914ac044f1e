"""Per-launch counter table of the row-pointer kernel vs the stack kernel from a
`tools/gpu_run.sh rows_pmc` / `slab_pmc` pass directory (rocprofv3 csv).

    python tools/rows_pmc_table.py gpurun_out/<OUT> [--json] [--pair=tagA,tagB ...]
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

KERNELS = {"rows": "reduce_kernel_segrows_rm", "stack": "reduce_kernel_rowmajor"}


def counters(path: Path):
    """{kernel: {counter: mean per dispatch}} (dispatch values summed over dimensions first)."""
    per = defaultdict(lambda: defaultdict(float))
    for f in path.glob("**/*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                for kind, kn in KERNELS.items():
                    if kn in row["Kernel_Name"]:
                        per[(kind, row["Counter_Name"])][row["Dispatch_Id"]] += float(row["Counter_Value"])
    out = defaultdict(dict)
    for (kind, ctr), d in per.items():
        out[kind][ctr] = sum(d.values()) / len(d)
    return out


def stats(path: Path):
    out = {}
    for f in path.glob("**/*kernel_stats.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                for kind, kn in KERNELS.items():
                    if kn in row["Name"]:
                        out[kind] = {"calls": int(row["Calls"]), "avg_us": float(row["AverageNs"]) / 1e3}
    return out


def main():
    root = Path(sys.argv[1])
    tags = sorted({p.name.split("_", 1)[1] for p in root.iterdir() if p.is_dir() and p.name.startswith("trace_")})
    res = {}
    for tag in tags:
        rec = {"time": stats(root / f"trace_{tag}"), "counters": defaultdict(dict)}
        for d in root.iterdir():
            if d.is_dir() and d.name.endswith("_" + tag) and not d.name.startswith("trace_"):
                for kind, ctrs in counters(d).items():
                    rec["counters"][kind].update(ctrs)
        res[tag] = rec
    if "--json" in sys.argv:
        print(json.dumps(res, indent=1))
        return
    pairs = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--pair=")]
    if pairs:  # two tags that ran the SAME kernel in separate processes (slab_pmc: engine vs stack)
        for pr in pairs:
            ta, tb = pr.split(",")
            ra, rb = res[ta], res[tb]
            print(f"\n### {ta} vs {tb} (reduce_kernel_rowmajor in both)\n")
            print(f"| counter (per launch) | {ta} | {tb} | ratio |")
            print("|---|---|---|---|")
            sa, sb = ra["time"].get("stack"), rb["time"].get("stack")
            if sa and sb:
                print(f"| kernel time (us, rocprof; calls {sa['calls']} / {sb['calls']}) | {sa['avg_us']:.1f} | "
                      f"{sb['avg_us']:.1f} | {sa['avg_us'] / sb['avg_us']:.3f} |")
            ca, cb = ra["counters"].get("stack", {}), rb["counters"].get("stack", {})
            for ctr in sorted(set(ca) | set(cb)):
                a, b = ca.get(ctr), cb.get(ctr)
                ratio = f"{a / b:.3f}" if a is not None and b else "-"
                print(f"| {ctr} | {'-' if a is None else f'{a:.4g}'} | {'-' if b is None else f'{b:.4g}'} | {ratio} |")
        return
    for tag, rec in res.items():
        print(f"\n### {tag}\n")
        t = rec["time"]
        print("| counter (per launch) | row-pointer kernel | stack kernel | rows / stack |")
        print("|---|---|---|---|")
        if "rows" in t and "stack" in t:
            print(f"| kernel time (us, rocprof) | {t['rows']['avg_us']:.1f} | {t['stack']['avg_us']:.1f} | "
                  f"{t['rows']['avg_us'] / t['stack']['avg_us']:.3f} |")
        c = rec["counters"]
        for ctr in sorted(set(c.get("rows", {})) | set(c.get("stack", {}))):
            a, b = c.get("rows", {}).get(ctr), c.get("stack", {}).get(ctr)
            ratio = f"{a / b:.3f}" if a is not None and b else "-"
            fa = f"{a:.4g}" if a is not None else "-"
            fb = f"{b:.4g}" if b is not None else "-"
            print(f"| {ctr} | {fa} | {fb} | {ratio} |")


if __name__ == "__main__":
    main()
