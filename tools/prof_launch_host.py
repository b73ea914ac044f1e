"""Host time per reduce launch through the Python path (dist.hip_reduce_fn -> aggregator.reduce_stack
-> fa_reduce_f32), plain mean and fused Adagrad on a narrow window (GPU time negligible): what a
multi-stripe step pays per stripe on the host.  python tools/prof_launch_host.py (GPU box)."""
import time, torch, numpy as np, sys
sys.path.insert(0, "/root/repo")
from flearn_amd import _native as na, aggregator as agg
from flearn_amd.dist import hip_reduce_fn, PingPong
dev = torch.device("cuda", 0)
n, cols = 100, 64 * 1024
stack = torch.empty((n, cols), device=dev); agg.fill_uniform(stack, seed=1)
w = torch.ones(n, device=dev)
out = torch.empty(cols, device=dev)
fn = hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n))
prev = torch.zeros(cols, device=dev)
st = PingPong(prev, torch.zeros(cols, dtype=torch.float64, device=dev))
fn2 = hip_reduce_fn(stack, w, na.MODE_W32_DIV64, float(n), op=na.OP_BY_NAME["adagrad"], state=st)
for f, name in ((fn, "mean"), (fn2, "adagrad")):
    for _ in range(50): f(0, 4096, out[:4096])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2000): f(0, 4096, out[:4096])
    dt = (time.perf_counter() - t) / 2000
    torch.cuda.synchronize()
    print(name, "host us per launch", round(dt * 1e6, 2))
