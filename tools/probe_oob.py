"""Probe the gfx950 raw-buffer range check for a 16-byte load that is partly out of range.
Prints, for num_records in 0..20 bytes and offsets 0/16, what the four lanes of the quad return."""
import ctypes
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from flearn_amd import _native as na  # noqa: E402

T = ctypes.CDLL(str(REPO / "tools" / "libtune_rows.so"))
T.tune_oob_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda", 0)
src = torch.arange(1, 9, dtype=torch.float32, device=dev)
out = torch.empty(4, dtype=torch.float32, device=dev)
res = {}
for off in (0, 16):
    for b in range(0, 33, 4):
        out.fill_(-1)
        assert T.tune_oob_probe(src.data_ptr(), b, off, out.data_ptr(), na.stream_handle(dev)) == 0
        torch.cuda.synchronize()
        res[f"off{off}_bytes{b}"] = out.tolist()
print(json.dumps(res))
