"""Client-side FedAVGM / FedOPT update (flearn's client_receive math) on the GPU vs the
reference's numpy, per call, for one model: host fp32 w_local + host float64 w_glob in, new
w_local out — AVGM.mean_momentum (avgm.py:19-36) / OPT.adaptive_opt (opt.py:23-65).

    python tools/bench_client_update.py [--layout resnet50] [--rounds 4]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import flearn_amd  # noqa: E402
from flearn_amd import layouts  # noqa: E402
from _refavg import ReferenceClientUpdate  # noqa: E402


def model(lay, seed, dtype, counters=True):
    """One state_dict of the layout: float keys in `dtype`; with `counters` the BN
    num_batches_tracked keys too — int64 arrays in a client's w_local, numpy float64 scalars in
    the server's w_glob (what the reference's server mean makes of a 0-d int64 value)."""
    p = layouts.fp32_elems(lay)
    flat = np.random.default_rng(seed).standard_normal(p).astype(dtype)
    sd = layouts.synthetic_state_dict(lay, flat.astype(np.float32), counter=1)
    out = {}
    for k, v in sd.items():
        if v.dtype == np.float32:
            out[k] = v.astype(dtype)
        elif counters:
            out[k] = v.copy() if dtype == np.float32 else np.float64(seed)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="resnet50")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--ref-rounds", type=int, default=2)
    ap.add_argument("--no-counters", action="store_true", help="drop the BN num_batches_tracked keys")
    ap.add_argument("--ab", action="store_true",
                    help="DeviceUpdater copy-engine vs zero-copy chunked, alternating, outputs compared")
    ap.add_argument("--zero-copy", type=int, default=None, help="DeviceUpdater.zero_copy (default: the class default)")
    ap.add_argument("--chunk-mb", type=float, default=None, help="DeviceUpdater.chunk_bytes in MiB")
    ap.add_argument("--first-mb", type=float, default=None, help="DeviceUpdater.first_chunk_bytes in MiB")
    ap.add_argument("--last-mb", type=float, default=None, help="DeviceUpdater.last_chunk_bytes in MiB")
    ap.add_argument("--native-pack", type=int, default=None, help="DeviceUpdater.native_pack (0: Python pool)")
    ap.add_argument("--phases", action="store_true", help="record the zero-copy pipeline's per-chunk times")
    ap.add_argument("--device-model", action="store_true",
                    help="client_receive with the model on the GPU: device path vs the reference's host path")
    ap.add_argument("--transfer", default=None, choices=("dma", "dma_in", "kernel"), help="DeviceUpdater.transfer")
    a = ap.parse_args()
    from flearn_amd.strategy._update import DeviceUpdater

    if a.first_mb is not None:
        DeviceUpdater.first_chunk_bytes = int(a.first_mb * (1 << 20))
    if a.last_mb is not None:
        DeviceUpdater.last_chunk_bytes = int(a.last_mb * (1 << 20))
    if a.phases:
        DeviceUpdater.trace = []
    if a.transfer is not None:
        DeviceUpdater.transfer = a.transfer
    if a.native_pack is not None:
        DeviceUpdater.native_pack = bool(a.native_pack)

    if a.zero_copy is not None:
        DeviceUpdater.zero_copy = bool(a.zero_copy)
    if a.chunk_mb is not None:
        DeviceUpdater.chunk_bytes = int(a.chunk_mb * (1 << 20))
    if a.ab:
        return ab(a)
    if a.device_model:
        return device_model(a)
    lay = layouts.get(a.layout)
    w_local0 = model(lay, 1, np.float32, not a.no_counters)
    globs = [model(lay, 10 + r, np.float64, not a.no_counters) for r in range(a.rounds)]
    p = sum(v.size for v in w_local0.values() if v.dtype == np.float32)
    res = {"layout": a.layout, "params": p, "keys": len(w_local0),
           "int64_counters": sum(1 for v in w_local0.values() if v.dtype == np.int64)}
    for method in ("avgm", "adagrad"):
        s = flearn_amd.AVGM() if method == "avgm" else flearn_amd.OPT()
        fn = ((lambda wl, wg: s.mean_momentum(wl, wg, 0.9)) if method == "avgm"
              else (lambda wl, wg: s.adaptive_opt(wl, wg, "adagrad")))
        ts = []
        for r in range(a.rounds):
            wl = dict(w_local0)
            t0 = time.perf_counter()
            fn(wl, globs[r])
            ts.append(time.perf_counter() - t0)
        ref = ReferenceClientUpdate(method)
        rs = []
        for r in range(a.ref_rounds):
            wl = dict(w_local0)
            t0 = time.perf_counter()
            ref(wl, globs[r])
            rs.append(time.perf_counter() - t0)
        med = float(np.median(ts[1:]))
        if a.phases and DeviceUpdater.trace:
            last = DeviceUpdater.trace[-1]
            calls = DeviceUpdater.trace[1:] or DeviceUpdater.trace

            def med_ms(f):
                return round(float(np.median([f(t) for t in calls])) * 1e3, 3)

            res[f"{method}_phases"] = {
                "launched_ms": round(last["launched_s"] * 1e3, 3), "done_ms": round(last["done_s"] * 1e3, 3),
                "chunks": [[n, round(t0 * 1e3, 3), round(t1 * 1e3, 3)] for n, t0, t1 in last["chunks"]],
                "median": {"first_launch_ms": med_ms(lambda t: t["chunks"][0][2]),
                           "launched_ms": med_ms(lambda t: t["launched_s"]), "done_ms": med_ms(lambda t: t["done_s"]),
                           "call_ms": med_ms(lambda t: t.get("call_s", float("nan")))},
                "note": "per chunk (last call): [elements, pack start ms, launch queued ms]; median over calls after the first"}
            DeviceUpdater.trace.clear()
        res[method] = {"flearn_amd_s": round(med, 4), "first_call_s": round(ts[0], 4),
                       "reference_s": round(float(np.median(rs[1:] if len(rs) > 1 else rs)), 4),
                       "speedup": round(float(np.median(rs[1:] if len(rs) > 1 else rs)) / med, 1)}
    from flearn_amd.strategy._update import DeviceUpdater

    res["zero_copy"] = DeviceUpdater.zero_copy
    res["transfer"] = DeviceUpdater.transfer
    res["chunk_bytes"] = DeviceUpdater.chunk_bytes
    res["first_chunk_bytes"] = DeviceUpdater.first_chunk_bytes
    res["last_chunk_bytes"] = DeviceUpdater.last_chunk_bytes
    res["native_pack"] = DeviceUpdater.native_pack
    res["note"] = "host arrays in and out (PCIe-inclusive); reference = its numpy ops on 1 core; median after round 0"
    print(json.dumps(res))


class _Model:
    """load_state_dict / state_dict over a dict of CUDA tensors (param.copy_(value), as
    torch.nn.Module.load_state_dict does)."""

    def __init__(self, tensors):
        self.t = tensors

    def state_dict(self):
        return dict(self.t)

    def load_state_dict(self, d):
        import torch

        with torch.no_grad():
            for k, t in self.t.items():
                v = d[k]
                t.copy_(v if isinstance(v, torch.Tensor) else torch.as_tensor(v))


class _Trainer:
    def __init__(self, model):
        self.model = model

    @property
    def weight(self):
        return self.model.state_dict()


def device_model(a):
    """client_receive (avgm.py:38-45 / opt.py:67-76) with the model's tensors on the GPU, fp32
    keys only (BN counters make the reference path raise): the device path (only w_glob crosses
    PCIe) against the reference's path on the same object (convert_to_np -> update -> load)."""
    import torch

    from flearn_amd.strategy._update import DeviceUpdater

    lay = [x for x in layouts.get(a.layout) if x[2] == "f32"]
    p = layouts.fp32_elems(lay)
    w0 = model(lay, 1, np.float32, False)
    globs = [model(lay, 10 + r, np.float64, False) for r in range(a.rounds)]
    res = {"layout": a.layout, "params": p, "keys": len(w0)}
    real_ok = DeviceUpdater.device_model_ok
    for method in ("avgm", "adagrad"):
        out = {}
        for mode in ("device", "host"):
            DeviceUpdater.device_model_ok = staticmethod(real_ok if mode == "device" else (lambda w, g: False))
            s = flearn_amd.AVGM() if method == "avgm" else flearn_amd.OPT()
            tensors = {k: torch.from_numpy(v).to("cuda") for k, v in w0.items()}
            tr = _Trainer(_Model(tensors))
            ts = []
            for r in range(a.rounds):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if method == "avgm":
                    s.client_receive(tr, {"w_glob": globs[r]}, 0.9)
                else:
                    s.client_receive(tr, {"w_glob": globs[r]}, "adagrad")
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            out[mode] = (float(np.median(ts[1:])), {k: t.cpu().numpy().copy() for k, t in tensors.items()})
        DeviceUpdater.device_model_ok = staticmethod(real_ok)
        same = all(out["device"][1][k].tobytes() == out["host"][1][k].tobytes() for k in w0)
        res[method] = {"device_path_s": round(out["device"][0], 4), "host_path_s": round(out["host"][0], 4),
                       "bit_equal": same}
    res["note"] = ("client_receive per round incl. load_state_dict, model tensors on the GPU; host path = the "
                   "reference's convert_to_np -> update -> load_state_dict on this engine; median after round 0")
    print(json.dumps(res))


def ab(a):
    from flearn_amd.strategy._update import DeviceUpdater

    lay = layouts.get(a.layout)
    w_local0 = model(lay, 1, np.float32, not a.no_counters)
    globs = [model(lay, 10 + r, np.float64, not a.no_counters) for r in range(a.rounds)]
    res = {"layout": a.layout}
    for method in ("avgm", "adagrad"):
        # one strategy object per mode (its pinned staging persists), called alternately
        objs = {zc: (flearn_amd.AVGM() if method == "avgm" else flearn_amd.OPT()) for zc in (False, True)}
        times, outs = {False: [], True: []}, {False: [], True: []}
        for rep in range(3):
            for r in range(a.rounds):
                for zc in (False, True):
                    DeviceUpdater.zero_copy = zc
                    s = objs[zc]
                    wl = dict(w_local0)
                    # drop the previous call's result before the clock starts: freeing the copy-engine
                    # path's fresh 205-MB array (munmap) inside the next call's timing charged ~8 ms
                    # to whichever mode ran next (round 4 traces)
                    out = None
                    t0 = time.perf_counter()
                    out = s.mean_momentum(wl, globs[r], 0.9) if method == "avgm" else s.adaptive_opt(wl, globs[r], "adagrad")
                    dt = time.perf_counter() - t0
                    if rep or r:
                        times[zc].append(dt)
                    if rep == 0:
                        outs[zc].append({k: np.array(v, copy=True) for k, v in out.items()})
        same = all(np.array_equal(np.asarray(x[k]), np.asarray(y[k])) and np.asarray(x[k]).dtype == np.asarray(y[k]).dtype
                   for x, y in zip(outs[False], outs[True]) for k in x)
        res[method] = {"copy_engine_s": round(float(np.median(times[False])), 4),
                       "zero_copy_s": round(float(np.median(times[True])), 4), "bit_equal": same,
                       "zero_copy_all_s": [round(t, 4) for t in times[True]],
                       "copy_engine_all_s": [round(t, 4) for t in times[False]]}
        if DeviceUpdater.trace:
            res[method]["zero_copy_alloc_launched_done_call_ms"] = [
                [round(t["alloc_s"] * 1e3, 2), round(t["launched_s"] * 1e3, 2), round(t["done_s"] * 1e3, 2),
                 round(t.get("call_s", 0) * 1e3, 2)] for t in DeviceUpdater.trace]
            DeviceUpdater.trace.clear()
    DeviceUpdater.zero_copy = True
    print(json.dumps(res))


if __name__ == "__main__":
    main()
