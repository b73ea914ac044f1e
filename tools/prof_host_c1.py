"""cProfile of the loopback C1 server step (10 LeNet5 uploads as host numpy dicts): median round
time, then the hottest host functions.  python tools/prof_host_c1.py (on a GPU box)."""
import cProfile
import pstats
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import flearn_amd  # noqa: E402
from flearn_amd import layouts  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent))
from _refavg import reference_avg  # noqa: E402


def main(rounds=300):
    lay = layouts.get("lenet5")
    p = layouts.fp32_elems(lay)
    rng = np.random.default_rng(0)
    ups = [{"agg_weight": 1.0,
            "params": layouts.synthetic_state_dict(lay, rng.random(p, dtype=np.float32), counter=100 + i)}
           for i in range(10)]
    s = flearn_amd.AVG()
    for r in range(20):
        s.server(ups, r)
    ts = []
    for r in range(rounds):
        t = time.perf_counter()
        s.server(ups, r)
        ts.append(time.perf_counter() - t)
    print("median us", np.median(ts) * 1e6, "min", min(ts) * 1e6)
    if "--ab" in sys.argv:  # copy-engine vs zero-copy small rounds, alternating in one process
        from flearn_amd.aggregator import Aggregator

        # two upload sets, alternated call by call: a stale cached line of the reused pinned
        # staging (or result) would show as a mismatch
        ups2 = [{"agg_weight": 1.0, "params": layouts.synthetic_state_dict(lay, rng.random(p, dtype=np.float32),
                                                                            counter=200 + i)} for i in range(10)]
        sets = (ups, ups2)
        refs = [{k: np.array(v, copy=True) for k, v in s.server(u, 0)["w_glob"].items()} for u in sets]
        res = {False: [], True: [], "numpy": []}
        for rep in range(6):
            for r in range(rounds // 3):  # the reference's numpy server step on the same uploads
                u = sets[r % 2]
                t = time.perf_counter()
                reference_avg([c["agg_weight"] for c in u], [c["params"] for c in u])
                res["numpy"].append(time.perf_counter() - t)
            for zc in (False, True):
                Aggregator.small_zero_copy = zc
                for r in range(20):
                    s.server(sets[r % 2], r)
                for r in range(rounds // 3):
                    t = time.perf_counter()
                    out = s.server(sets[r % 2], r)["w_glob"]
                    res[zc].append(time.perf_counter() - t)
                    ref = refs[r % 2]
                    assert all(np.array_equal(out[k], ref[k]) for k in ref), f"zero-copy={zc}: result differs"
        for zc in (False, True, "numpy"):
            name = {False: "copy-engine", True: "zero-copy", "numpy": "reference numpy"}[zc]
            print(f"{name} median us {np.median(res[zc]) * 1e6:.1f} min {min(res[zc]) * 1e6:.1f}")
        Aggregator.small_zero_copy = True
    if "--parts" in sys.argv:  # zero-copy small rounds in 1 / 2 / 3 / 4 chained launches, alternating
        from flearn_amd.aggregator import Aggregator

        ups2 = [{"agg_weight": 1.0, "params": layouts.synthetic_state_dict(lay, rng.random(p, dtype=np.float32),
                                                                            counter=300 + i)} for i in range(10)]
        sets = (ups, ups2)
        refs = [{k: np.array(v, copy=True) for k, v in s.server(u, 0)["w_glob"].items()} for u in sets]
        kinds = (1, 2, 3, 4)
        res = {k: [] for k in kinds}
        res["numpy"] = []
        for rep in range(6):
            for r in range(rounds // 3):
                u = sets[r % 2]
                t = time.perf_counter()
                reference_avg([c["agg_weight"] for c in u], [c["params"] for c in u])
                res["numpy"].append(time.perf_counter() - t)
            for k in kinds:
                Aggregator.small_parts = k
                for r in range(20):
                    s.server(sets[r % 2], r)
                for r in range(rounds // 3):
                    t = time.perf_counter()
                    out = s.server(sets[r % 2], r)["w_glob"]
                    res[k].append(time.perf_counter() - t)
                    ref = refs[r % 2]
                    assert all(np.array_equal(out[kk], ref[kk]) for kk in ref), f"parts={k}: result differs"
        for k in (*kinds, "numpy"):
            name = f"{k} launches" if k != "numpy" else "reference numpy"
            print(f"{name} median us {np.median(res[k]) * 1e6:.1f} min {min(res[k]) * 1e6:.1f}")
        Aggregator.small_parts = 1
    pr = cProfile.Profile()
    pr.enable()
    for r in range(rounds):
        s.server(ups, r)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
