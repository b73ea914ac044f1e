"""Summarise rocprofv3 runs of bench.py into per-launch numbers for the dominant kernel.

    python tools/pmc_traffic.py --config c2 --stats DIR/x_kernel_stats.csv \
        --fetch DIR/x_counter_collection.csv --write DIR/y_counter_collection.csv \
        --bytes-per-launch B --out profiles/traffic.json

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are collected in separate --pmc passes (TCC slots), both are in KiB, and on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
from __future__ import annotations

import argparse
import csv
import json
from pathlib import Path

KERNEL = "fa::reduce_kernel"  # the engine's reduce kernels (not torch's at::native::reduce_kernel)


def dominant_kernel(stats_csv: Path, kernel: str = KERNEL):
    """The engine reduce kernel with the largest total time in a rocprofv3 kernel_stats file: the
    bench's own launches (bench.py's self-check adds narrow-window launches of other kernels)."""
    best = None
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                tot = float(row.get("TotalDurationNs") or 0.0) or float(row["AverageNs"]) * int(row["Calls"])
                if best is None or tot > best[0]:
                    best = (tot, row)
    return None if best is None else best[1]


def per_dispatch(counter_csv: Path, counter: str, kernel: str = KERNEL, exact: str | None = None):
    """Per-dispatch values of `counter` for the kernel named `exact` (else: every kernel whose
    name contains `kernel`, keeping the name with the most bytes per dispatch)."""
    vals, names, grids = {}, {}, {}
    with open(counter_csv) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if (name == exact if exact else kernel in name) and row["Counter_Name"] == counter:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = name
                grids[row["Dispatch_Id"]] = int(row["Grid_Size"])
    if vals:  # the bench's launches: the largest grid of each kernel (the self-check's windows are narrower)
        top = {}
        for d, g in grids.items():
            top[names[d]] = max(top.get(names[d], 0), g)
        vals = {d: v for d, v in vals.items() if grids[d] == top[names[d]]}
    if exact or not vals:
        return list(vals.values())
    by = {}
    for d, v in vals.items():
        by.setdefault(names[d], []).append(v)
    return max(by.values(), key=lambda xs: sum(xs) / len(xs))


def kernel_stats(stats_csv: Path, kernel: str = KERNEL):
    """The dominant kernel's launch statistics: from the kernel trace next to the stats file
    (its largest-grid dispatches only: bench.py's own launches, not the self-check's narrow
    windows), else from the stats file."""
    row = dominant_kernel(stats_csv, kernel)
    if row is None:
        return None
    trace = Path(str(stats_csv).replace("_kernel_stats.csv", "_kernel_trace.csv"))
    if trace.exists():
        durs = []
        with open(trace) as f:
            rows = [r for r in csv.DictReader(f) if r["Kernel_Name"] == row["Name"]]
        if rows:
            top = max(int(r["Grid_Size_X"]) for r in rows)
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if int(r["Grid_Size_X"]) == top]
        if durs:
            return {"name": row["Name"], "calls": len(durs), "avg_ns": sum(durs) / len(durs), "min_ns": float(min(durs)),
                    "max_ns": float(max(durs)), "from": "kernel trace, the bench's largest-grid dispatches"}
    return {"name": row["Name"], "calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
            "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--bytes-per-launch", type=float, required=True, help="algorithmic bytes per launch")
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--source", default=None)
    a = ap.parse_args()
    exact = None
    if a.stats:
        dk = dominant_kernel(Path(a.stats))
        exact = dk["Name"] if dk is not None else None
    fetch = per_dispatch(Path(a.fetch), "FETCH_SIZE", exact=exact)
    write = per_dispatch(Path(a.write), "WRITE_SIZE", exact=exact)
    if not fetch or not write:
        raise SystemExit("no reduce_kernel dispatches with FETCH_SIZE / WRITE_SIZE found")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    rec = {
        "hbm_bytes_per_launch": round(hbm),
        "fetch_size_kib_raw": round(f_kib, 1),
        "write_size_kib": round(w_kib, 1),
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "algorithmic_bytes_per_launch": a.bytes_per_launch,
        "traffic_over_algorithmic": round(hbm / a.bytes_per_launch, 4),
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)",
        "source": a.source or f"{a.fetch} + {a.write}",
    }
    if a.stats:
        ks = kernel_stats(Path(a.stats))
        if ks:
            rec["rocprof_kernel_stats"] = ks
    out = Path(a.out)
    data = json.loads(out.read_text()) if out.exists() else {}
    data[a.config] = rec
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(data, indent=2) + "\n")
    print(json.dumps({a.config: rec}, indent=2))


if __name__ == "__main__":
    main()
