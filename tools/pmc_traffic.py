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

KERNEL = "reduce_kernel"


def per_dispatch(counter_csv: Path, counter: str, kernel: str = KERNEL):
    vals = {}
    with open(counter_csv) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def kernel_stats(stats_csv: Path, kernel: str = KERNEL):
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                return {"name": row["Name"], "calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                        "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
    return None


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
    fetch = per_dispatch(Path(a.fetch), "FETCH_SIZE")
    write = per_dispatch(Path(a.write), "WRITE_SIZE")
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
