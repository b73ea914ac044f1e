"""Summarise a rocprofv3 --memory-copy-trace of tools/probe_dma_legs.py: do the copy-engine legs
of one fa_push_dma call run at the same time?

    python tools/dma_trace_summary.py gpurun_out/r05b/dma/trace > profiles/r05/push_dma_trace/summary.json

Groups the copies into bursts (copies whose intervals chain within 50 us of each other) and, per
burst, reports the copies' count, total span, the sum of their durations, and the peak number of
copies in flight at once: concurrency = sum(durations) / span (1.0 = one after the other, k = k
at once).  Measurement infrastructure."""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path


def load(root: Path):
    files = sorted(root.rglob("*memory_copy_trace.csv"))
    if not files:
        raise SystemExit(f"no *memory_copy_trace.csv under {root}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append(r)
    return rows


def field(r, *names):
    for n in names:
        for k in r:
            if k.lower() == n.lower():
                return r[k]
    return None


def main():
    root = Path(sys.argv[1])
    rows = load(root)
    copies = []
    for r in rows:
        t0, t1 = int(field(r, "Start_Timestamp")), int(field(r, "End_Timestamp"))
        copies.append({"start": t0, "end": t1, "dir": field(r, "Direction", "Kind"), "bytes": field(r, "Size", "Bytes"),
                       "src": field(r, "Source_Agent_Id", "Src_Agent_Id"), "dst": field(r, "Destination_Agent_Id",
                                                                                     "Dst_Agent_Id")})
    copies.sort(key=lambda c: c["start"])
    bursts, cur = [], []
    for c in copies:
        if cur and c["start"] > max(x["end"] for x in cur) + 50_000:
            bursts.append(cur)
            cur = []
        cur.append(c)
    if cur:
        bursts.append(cur)
    out = []
    for b in bursts:
        span = max(c["end"] for c in b) - min(c["start"] for c in b)
        busy = sum(c["end"] - c["start"] for c in b)
        ev = sorted([(c["start"], 1) for c in b] + [(c["end"], -1) for c in b])
        live = peak = 0
        for _, d in ev:
            live += d
            peak = max(peak, live)
        out.append({"copies": len(b), "span_us": round(span / 1e3, 2), "sum_of_durations_us": round(busy / 1e3, 2),
                    "concurrency": round(busy / max(span, 1), 2), "peak_in_flight": peak,
                    "durations_us": [round((c["end"] - c["start"]) / 1e3, 1) for c in b],
                    "starts_us_rel": [round((c["start"] - b[0]["start"]) / 1e3, 1) for c in b],
                    "dirs": sorted({str(c["dir"]) for c in b})})
    print(json.dumps({"columns": list(rows[0].keys()) if rows else [], "bursts": out}, indent=1))


if __name__ == "__main__":
    main()
