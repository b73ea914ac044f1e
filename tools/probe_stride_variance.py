"""Is the NS reduce's placement sensitivity a matter of the row stride?  One process allocates a
stack for 100 x ResNet-50 rows afresh several times (spacer allocations of growing size in
between move it) and, on each allocation, times the product kernel with the row stride padded by
0 / 64 / 320 / 1088 / 4160 floats (or: probe_stride_variance.py PADS [TRIALS [LAYOUT [N]]]) (the rows lie that much further apart; the columns reduced are
the same 25.6 M).  HIP events, median of 15.  python tools/probe_stride_variance.py (GPU box)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "/root/repo")
from flearn_amd import _native as na  # noqa: E402
from flearn_amd import layouts  # noqa: E402

dev = torch.device("cuda", 0)
L = na.lib()
LAYOUT = sys.argv[3] if len(sys.argv) > 3 else "resnet50"
n = int(sys.argv[4]) if len(sys.argv) > 4 else 100
p = layouts.padded_f32_stride(layouts.get(LAYOUT))
PADS = tuple(int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,64,320,1088,4160".split(",")))
w = torch.ones(n, device=dev)
out = torch.empty(p, device=dev)
stream = torch.cuda.current_stream().cuda_stream
res, spacers = [], []
for trial in range(int(sys.argv[2]) if len(sys.argv) > 2 else 6):
    stack = torch.empty(n * (p + max(PADS)), dtype=torch.float32, device=dev)
    row = {"trial": trial}
    times = {pad: [] for pad in PADS}
    order = list(PADS)
    for rnd in range(3):  # interleaved rounds, the pad order rotated: no drift favours a pad
        for pad in order[rnd % len(order):] + order[: rnd % len(order)]:
            stride = p + pad
            assert L.fa_fill_uniform_f32(stack.data_ptr(), stride, n, p, 2024, 0, 0, stream) == 0

            def red():
                assert L.fa_reduce_f32(stack.data_ptr(), stride, n, na.MODE_W32_DIV64, w.data_ptr(), float(n), 0, p,
                                       None, out.data_ptr(), None, stream) == 0
            for _ in range(2):
                red()
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                red()
                e1.record()
                torch.cuda.synchronize()
                times[pad].append(e0.elapsed_time(e1) * 1e3)
    for pad in PADS:
        row[str(pad)] = round(float(np.median(times[pad])), 1)
    res.append(row)
    print(row, file=sys.stderr, flush=True)
    del stack
    spacers.append(torch.empty(int((trial + 1) * 257 * 2**20 // 4), device=dev))
    torch.cuda.empty_cache()
print(json.dumps({"layout": LAYOUT, "clients": n, "pads_floats": PADS, "rows": res}))
