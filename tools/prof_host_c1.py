"""cProfile of the loopback C1 server step (10 LeNet5 uploads as host numpy dicts): median round
time, then the hottest host functions.  python tools/prof_host_c1.py (on a GPU box)."""
import sys, time, cProfile, pstats
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np, torch
import flearn_amd
from flearn_amd import layouts
lay = layouts.get("lenet5"); p = layouts.fp32_elems(lay)
rng = np.random.default_rng(0)
ups = [{"agg_weight": 1.0, "params": layouts.synthetic_state_dict(lay, rng.random(p, dtype=np.float32), counter=100+i)} for i in range(10)]
s = flearn_amd.AVG()
for r in range(20): s.server(ups, r)
ts=[]
for r in range(300):
    t=time.perf_counter(); s.server(ups, r); ts.append(time.perf_counter()-t)
print("median us", np.median(ts)*1e6, "min", min(ts)*1e6)
pr = cProfile.Profile(); pr.enable()
for r in range(300): s.server(ups, r)
pr.disable(); pstats.Stats(pr).sort_stats("tottime").print_stats(30)
