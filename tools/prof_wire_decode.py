"""Split of one ResNet-18 upload decode (HTTP mode): total, native scan, planning, full base64
decode, and a cProfile of the Python side.  python tools/prof_wire_decode.py"""
import sys, time, pickle, cProfile, pstats
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np
from flearn_amd import layouts, wire
lay = layouts.get("resnet18"); p = layouts.fp32_elems(lay)
rng = np.random.default_rng(0)
s = wire.b64encode(pickle.dumps({"agg_weight": 1.0, "params": layouts.synthetic_state_dict(lay, rng.random(p, dtype=np.float32), counter=1)}))
E = wire.Encrypt()
for _ in range(3): E.decode(s)
t=time.perf_counter()
for _ in range(10): E.decode(s)
print("decode ms", (time.perf_counter()-t)/10*1e3, "chars", len(s))
pr=cProfile.Profile(); pr.enable()
for _ in range(10): E.decode(s)
pr.disable(); pstats.Stats(pr).sort_stats("tottime").print_stats(15)
import ctypes, json
L = wire.na.load()
ptr, n = wire._ascii_ptr(s)
buf = ctypes.create_string_buffer(1<<20); need = ctypes.c_int64(0)
t=time.perf_counter()
for _ in range(10): L.fa_pickle_scan_b64(ptr, n, buf, 1<<20, ctypes.byref(need))
print("scan ms", (time.perf_counter()-t)/10*1e3, need.value)
tree = json.loads(buf.raw[:need.value].decode())
t=time.perf_counter()
for _ in range(10):
    dec = wire._Decoder(L, ptr, n); planned = dec.plan_row(tree); dec.assign(tree)
print("plan+assign ms", (time.perf_counter()-t)/10*1e3)
out = np.empty(p+100000, np.float32)
raw = wire.b64decode(s)
t=time.perf_counter()
for _ in range(10): wire.b64decode(s)
print("full b64decode ms", (time.perf_counter()-t)/10*1e3, "threads", wire._THREADS)
