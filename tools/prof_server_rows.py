import cProfile, pstats, sys, time, io
sys.path.insert(0, '/root/repo')
import numpy as np, torch
from flearn_amd import AVG, layouts
from flearn_amd import aggregator as agg
name = sys.argv[1] if len(sys.argv) > 1 else 'resnet50'
n = 100
dev = torch.device('cuda', 0)
layout = [x for x in layouts.get(name)]
clients = []
for i in range(n):
    d = {}
    for k, shape, dt in layout:
        d[k] = torch.empty(shape, dtype=torch.float32 if dt == 'f32' else (torch.int64 if dt == 'i64' else torch.float64), device=dev)
        if dt == 'f32':
            d[k].uniform_()
        else:
            d[k].zero_()
    clients.append(d)
ups = [{"agg_weight": 1.0, "params": c} for c in clients]
s = AVG(output="device")
for r in range(3):
    s.server(ups, r)
torch.cuda.synchronize()
walls = []
for r in range(10):
    t = time.perf_counter(); s.server(ups, r); torch.cuda.synchronize(); walls.append(time.perf_counter() - t)
print('server ms median', np.median(walls) * 1e3, 'min', min(walls) * 1e3, 'path', s.engine.packer.last_row_tables)
pr = cProfile.Profile(); pr.enable()
for r in range(5):
    s.server(ups, r)
torch.cuda.synchronize()
pr.disable()
st = io.StringIO(); pstats.Stats(pr, stream=st).sort_stats('cumtime').print_stats(25); print(st.getvalue())
