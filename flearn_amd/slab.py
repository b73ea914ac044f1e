"""Device-resident client uploads carved from ONE allocation (the row-pointer path's fast form).

flearn's run2 simulator hands the server each client's CUDA state_dict
(/root/reference/flearn/server/Communicator.py:287-292): every tensor its own allocation.  The
engine reads such uploads in place through a per-(key, client) pointer table
(fa_reduce_f32_rows), at 7-8% below the stack kernel — the cost is address translation of
thousands of separate allocations (UTCL2 busy 2x, profiles/r05/rows_pmc/), not the kernel.
`device_state_dicts(template, n)` gives a caller that owns its clients' device models the
other layout: N state_dicts whose fp32 tensors are views of one [n, stride] allocation, laid out
exactly as the engine's fp32 bucket (same key order, same 64-column-aligned offsets).  The
Packer recognises it (Packer._slab_stack) and hands the stack kernel the allocation itself — no
pointer table, no copy, the stack kernel's speed.  Anything else (a subset of the dicts'
rows, other keys, extra tensors) still works through the pointer table.
"""
from __future__ import annotations

import numpy as np
import torch

from .bucket import make_plan
from .semantics import KIND_F32


class SlabStateDicts(list):
    """N state_dicts (a list) whose fp32 tensors are views of `slab` ([n, stride] fp32, one
    allocation); `keys_f32` / `offsets`: the fp32 keys and their column offsets in a row."""

    slab: torch.Tensor
    offsets: dict


def _host(v):
    if isinstance(v, torch.Tensor):
        return v.detach()
    return torch.from_numpy(np.ascontiguousarray(v))


def device_state_dicts(template, n: int, device=None) -> SlabStateDicts:
    """N state_dicts shaped like `template` (a state_dict of tensors / arrays, or an nn.Module),
    each initialised with the template's values, on `device` (default: the current CUDA device).
    The fp32 tensors of all N dicts live in one [n, stride] fp32 allocation, each client's row
    laid out as the aggregation bucket; other dtypes (BN num_batches_tracked, ...) get tensors of
    their own.  Uploading these dicts (AVG / AVGM / OPT / Dyn .server with torch uploads) runs
    the stack kernel on the allocation in place (Packer._slab_stack)."""
    if hasattr(template, "state_dict") and callable(template.state_dict):
        template = template.state_dict()
    if n < 1:
        raise ValueError("n must be >= 1")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    plan = make_plan([1.0], [dict(template)])
    g = plan.groups.get(KIND_F32)
    stride = g.stride if g is not None else 0
    slab = torch.zeros((n, max(stride, 1)), dtype=torch.float32, device=dev)
    offsets = {}
    if g is not None:
        for s in g.segments:
            offsets[s.key] = (s.offset, s.numel, tuple(s.shape))
            src = _host(template[s.key]).to(dev, torch.float32).reshape(1, -1)
            slab[:, s.offset : s.offset + s.numel].copy_(src.expand(n, -1))
    out = SlabStateDicts()
    for i in range(n):
        d = {}
        for k, v in template.items():
            if k in offsets:
                o, m, shape = offsets[k]
                d[k] = slab[i, o : o + m].view(shape)
            else:
                d[k] = _host(v).to(dev, copy=True)
        out.append(d)
    out.slab, out.offsets = slab, offsets
    return out
