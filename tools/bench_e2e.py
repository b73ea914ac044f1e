"""End-to-end server aggregation through the Strategy API, uploads in host memory.

    python tools/bench_e2e.py [--config c2] [--rounds 5] [--output reference|float32]

flearn's loopback Server hands `Strategy.server` a list of client uploads whose params are host
numpy arrays (Communicator.py:127-141 -> Server.py:126-140); the result goes back to the clients
as host arrays.  This times AVG().server(uploads, r) on that input — plan, pack into pinned
staging, H2D, the fused HIP reduce, D2H, unpack — and splits the time by phase.  It is the
PCIe-inclusive rate recorded in DESIGN.md, never bench.py's `value`.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import flearn_amd  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import layouts  # noqa: E402
from _refavg import reference_avg  # noqa: E402

CONFIGS = {"c2": ("resnet18", 100), "c3": ("resnet50", 100), "c1": ("lenet5", 10)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--output", default="reference")
    ap.add_argument("--devices", type=int, default=1, help="split columns over the first K GPUs")
    ap.add_argument("--native-pack", type=int, default=None, help="Packer.native_async (0: the Python pool)")
    ap.add_argument("--zero-copy-out", type=int, default=None, help="Packer.zero_copy_out (0: copy engine + host copy)")
    ap.add_argument("--lookahead", type=int, default=None, help="Packer.async_lookahead (chunks packed ahead; 0: all)")
    ap.add_argument("--pack-threads", type=int, default=None, help="Packer.async_threads")
    ap.add_argument("--ab", default=None,
                    help="alternate round by round between Packer settings, e.g. "
                         "'native_async=0;native_async=1,async_lookahead=2': per-setting medians")
    a = ap.parse_args()
    name, n = CONFIGS[a.config]
    layout = layouts.get(name)
    p = layouts.fp32_elems(layout)
    dev = torch.device("cuda", 0)
    x = torch.empty((n, p), dtype=torch.float32, device=dev)
    agg.fill_uniform(x, seed=2024)
    host = x.cpu().numpy()  # the clients' uploads live in host memory
    del x
    uploads = [{"agg_weight": 1.0, "params": layouts.synthetic_state_dict(layout, host[i], counter=100 + i)}
               for i in range(n)]
    if a.devices > torch.cuda.device_count():
        raise SystemExit(f"--devices {a.devices} but only {torch.cuda.device_count()} GPU(s) visible")
    s = flearn_amd.AVG(output=a.output, devices=[torch.device("cuda", i) for i in range(a.devices)])
    eng = s.engine
    if a.native_pack is not None:
        eng.packer.native_async = bool(a.native_pack)
    if a.zero_copy_out is not None:
        eng.packer.zero_copy_out = bool(a.zero_copy_out)
    if a.lookahead is not None:
        eng.packer.async_lookahead = a.lookahead
    if a.pack_threads is not None:
        eng.packer.async_threads = a.pack_threads
    # phase timers around the engine's own steps
    t = {"plan_pack_h2d": [], "reduce": [], "d2h_unpack": [], "total": []}
    orig_pack, orig_finish = eng.packer.pack, eng._finish

    def sync_all():
        for d in eng.devices:
            torch.cuda.synchronize(d)

    def pack(plan, w):
        t0 = time.perf_counter()
        out = orig_pack(plan, w)
        sync_all()
        t["plan_pack_h2d"].append(time.perf_counter() - t0)
        t["_red0"] = time.perf_counter()
        return out

    def finish(plan, results):
        sync_all()
        t["reduce"].append(time.perf_counter() - t["_red0"])
        t0 = time.perf_counter()
        out = orig_finish(plan, results)
        t["d2h_unpack"].append(time.perf_counter() - t0)
        return out

    eng.packer.pack, eng._finish = pack, finish
    if a.ab:
        return ab(a, s, uploads, t, layout)
    for r in range(a.rounds + 1):
        t0 = time.perf_counter()
        w_glob = s.server(uploads, r)["w_glob"]
        t["total"].append(time.perf_counter() - t0)
    assert len(w_glob) == len(layout)
    med = {k: float(np.median(v[1:])) for k, v in t.items() if not k.startswith("_")}
    # the reference's loopback server step on the same uploads (numpy, 1 core), best of a few
    ref_s = []
    ws, ps = [u["agg_weight"] for u in uploads], [u["params"] for u in uploads]
    for _ in range(3 if n * p > 1 << 24 else 30):
        t0 = time.perf_counter()
        reference_avg(ws, ps)
        ref_s.append(time.perf_counter() - t0)
    in_bytes = n * p * 4
    out_bytes = p * (8 if a.output == "reference" else 4)
    res = {
        "config": a.config, "layout": name, "clients": n, "params": p, "output": a.output, "devices": a.devices,
        "median_s": {k: round(v, 5) for k, v in med.items()},
        "e2e_GiB_s_algorithmic": round((in_bytes + out_bytes) / 2**30 / med["total"], 2),
        "h2d_input_GB": round(in_bytes / 1e9, 3),
        "pack_h2d_GB_s": round(in_bytes / 1e9 / med["plan_pack_h2d"], 2),
        "reference_server_s": round(min(ref_s), 5),
        "speedup_vs_reference": round(min(ref_s) / med["total"], 2),
        "pack_path": eng.packer.last_pack_paths.get("f32"), "native_pack": eng.packer.native_async,
        "zero_copy_out": eng.packer.zero_copy_out, "lookahead": eng.packer.async_lookahead,
        "pack_threads": eng.packer.async_threads,
        "note": "uploads are host numpy views (flearn loopback); first round (pinned-buffer allocation) excluded",
    }
    print(json.dumps(res))


def ab(a, s, uploads, t, layout):
    """Interleaved A/B of Packer settings in one process: round r uses setting r % k; medians
    per setting over the rounds after each setting's first."""
    settings = []
    for spec in a.ab.split(";"):
        kv = {}
        for item in filter(None, spec.split(",")):
            k, v = item.split("=")
            kv[k.strip()] = int(v)
        settings.append(kv)
    eng = s.engine
    per = [{"plan_pack_h2d": [], "d2h_unpack": [], "total": [], "path": None} for _ in settings]
    for r in range((a.rounds + 1) * len(settings)):
        i = r % len(settings)
        for k, v in settings[i].items():
            setattr(eng.packer, k, type(getattr(eng.packer, k))(v))
        n0 = len(t["plan_pack_h2d"])
        t0 = time.perf_counter()
        w_glob = s.server(uploads, r)["w_glob"]
        per[i]["total"].append(time.perf_counter() - t0)
        per[i]["plan_pack_h2d"].append(t["plan_pack_h2d"][n0])
        per[i]["d2h_unpack"].append(t["d2h_unpack"][n0])
        per[i]["path"] = eng.packer.last_pack_paths.get("f32")
        assert len(w_glob) == len(layout)
    res = {"config": a.config, "rounds_per_setting": a.rounds, "settings": []}
    for kv, d in zip(settings, per):
        res["settings"].append({"set": kv, "path": d["path"],
                                **{k + "_ms": round(float(np.median(v[1:])) * 1e3, 2) for k, v in d.items() if k != "path"},
                                "total_ms_all": [round(x * 1e3, 1) for x in d["total"]]})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
