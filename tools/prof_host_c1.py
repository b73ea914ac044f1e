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
    pr = cProfile.Profile()
    pr.enable()
    for r in range(rounds):
        s.server(ups, r)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
