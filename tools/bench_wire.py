"""HTTP-mode server round: N base64(pickle) uploads -> global model string.

    python tools/bench_wire.py [--config c2] [--rounds 3] [--ref-sample 8]

flearn's HTTP server decodes every upload with Encrypt.decode (base64 + pickle.loads,
Encrypt.py:32-44) inside Server.ensemble (Server.py:126-131), aggregates (strategy.server) and
encodes the result (Server.py:142).  This times that round through flearn_amd (wire.Encrypt +
the HIP engine), phase by phase, and the reference's codec on a bounded sample of the same
uploads (numpy AVG on the host for the aggregation leg, scaled linearly to N and labelled so).
"""
from __future__ import annotations

import argparse
import base64
import json
import pickle
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import flearn_amd  # noqa: E402
from flearn_amd import aggregator as agg  # noqa: E402
from flearn_amd import layouts, wire  # noqa: E402
from _refavg import reference_avg as _reference_avg  # noqa: E402

CONFIGS = {"c1": ("lenet5", 10), "c2": ("resnet18", 100), "c3": ("resnet50", 100)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ref-sample", type=int, default=8, help="uploads the reference codec is timed on")
    ap.add_argument("--stage", action="store_true", help="Encrypt(stage_to_device=True): H2D during decode")
    a = ap.parse_args()
    name, n = CONFIGS[a.config]
    lay = layouts.get(name)
    p = layouts.fp32_elems(lay)
    dev = torch.device("cuda", 0)
    x = torch.empty((n, p), dtype=torch.float32, device=dev)
    agg.fill_uniform(x, seed=2025)
    host = x.cpu().numpy()
    del x
    t0 = time.perf_counter()
    strs = [wire.b64encode(pickle.dumps({"agg_weight": 1.0,
                                         "params": layouts.synthetic_state_dict(lay, host[i], counter=100 + i)}))
            for i in range(n)]
    gen_s = time.perf_counter() - t0
    del host
    b64_bytes = sum(len(s) for s in strs)

    # ---- flearn_amd: Server.ensemble's loop with the wire codec and the engine -------------
    s = flearn_amd.AVG(encrypt=wire.Encrypt(stage_to_device=a.stage))
    ph = {"decode": [], "server": [], "encode": [], "total": []}
    out_len = 0
    for _ in range(a.rounds + 1):
        t0 = time.perf_counter()
        ups = [s.receive_processing(x) for x in strs]
        t1 = time.perf_counter()
        glob = s.server(ups, 0)
        t2 = time.perf_counter()
        payload = s.upload_processing(glob)
        t3 = time.perf_counter()
        out_len = len(payload)
        for k, v in (("decode", t1 - t0), ("server", t2 - t1), ("encode", t3 - t2), ("total", t3 - t0)):
            ph[k].append(v)
        rows = s.engine.packer.last_wire_rows
        staged = s.engine.packer.last_wire_staged
        del ups, glob, payload
    med = {k: float(np.median(v[1:])) for k, v in ph.items()}

    # ---- reference codec + numpy AVG on a bounded sample -----------------------------------
    k = min(a.ref_sample, n)
    t0 = time.perf_counter()
    dec = [pickle.loads(base64.b64decode(x.encode())) for x in strs[:k]]  # Encrypt.decode
    t1 = time.perf_counter()
    w = _reference_avg([d["agg_weight"] for d in dec], [d["params"] for d in dec])
    t2 = time.perf_counter()
    enc = base64.b64encode(pickle.dumps({"w_glob": w})).decode()  # Encrypt.encode
    t3 = time.perf_counter()
    ref = {"decode": (t1 - t0) * n / k, "server": (t2 - t1) * n / k, "encode": t3 - t2}
    ref["total"] = sum(ref.values())

    res = {
        "config": a.config, "layout": name, "clients": n, "params": p,
        "b64_MB_in": round(b64_bytes / 1e6, 1), "b64_MB_out": round(out_len / 1e6, 1),
        "wire_rows_dma": rows,
        "wire_rows_staged_at_decode": staged,
        "flearn_amd_s": {k2: round(v, 4) for k2, v in med.items()},
        "flearn_amd_decode_GB_s_b64": round(b64_bytes / 1e9 / med["decode"], 2),
        "reference_s_scaled": {k2: round(v, 3) for k2, v in ref.items()},
        "reference_sample": f"{k} of {n} uploads decoded + averaged on 1 core (numpy), scaled x{n / k:g}; encode of 1 model",
        "speedup_total": round(ref["total"] / med["total"], 1),
        "generate_s": round(gen_s, 2),
        "note": "rounds after the first (pinned-row allocation) are the median",
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
