"""Device-side AVGM / FedOPT update of a received global model (the client_receive form).

The reference runs `mean_momentum` (avgm.py:19-36) and `adaptive_opt` (opt.py:23-65) per client
in numpy float64.  `DeviceUpdater` flattens w_local (fp32) and w_glob (the server's float64 —
or float32 — arrays) into aligned device buffers, keeps v_t resident in HBM across rounds and
runs one fa_opt_apply launch, with the reference's operation order and precision.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native as na
from ..bucket import ALIGN
from .utils import _ERR


class DeviceUpdater:
    def __init__(self, op: str, device=None, beta=0.9, eta=1e-1, tau=1e-9, beta2=0.99):
        self.op = na.OP_BY_NAME[op]
        self.device = device
        self.params = dict(beta=beta, eta=eta, tau=tau, beta2=beta2)
        self.layout = None  # [(key, shape, offset, numel)]
        self.v = None

    def _layout(self, w_glob):
        lay, off = [], 0
        for k, g in w_glob.items():
            shape = tuple(np.shape(g))
            n = int(np.prod(shape)) if shape else 1
            lay.append((k, shape, off, n))
            off += -(-max(n, 1) // ALIGN) * ALIGN
        return lay, off

    def reset(self):
        self.layout, self.v = None, None

    def state(self):
        """v_t as the reference exposes it: {key: ndarray}."""
        if self.v is None:
            return {}
        host = self.v.cpu().numpy()
        return {k: host[o : o + n].reshape(s).copy() for k, s, o, n in self.layout}

    def __call__(self, w_local, w_glob, **override):
        na.lib()
        glob = {}
        for k, g in w_glob.items():
            if isinstance(g, torch.Tensor):
                g = g.detach().cpu().numpy()
            if not isinstance(g, np.ndarray):
                raise SystemError(_ERR, type(g))
            glob[k] = g
        dts = {g.dtype for g in glob.values()}
        if len(dts) != 1 or dts.pop() not in (np.float64, np.float32):
            raise TypeError("w_glob values must all be float64 (or all float32) arrays")
        gdt = next(iter(glob.values())).dtype
        local = {}
        for k in glob:
            lv = w_local[k]
            if isinstance(lv, torch.Tensor):
                lv = lv.detach().cpu().numpy()
            if not isinstance(lv, np.ndarray) or lv.dtype != np.float32 or lv.shape != glob[k].shape:
                raise TypeError(f"w_local[{k!r}] must be an fp32 array shaped like w_glob[{k!r}]")
            local[k] = lv
        lay, total = self._layout(glob)
        dev = torch.device(self.device) if self.device is not None else torch.device("cuda", torch.cuda.current_device())
        tdt = torch.float64 if gdt == np.float64 else torch.float32
        if self.layout != lay or self.v is None or self.v.dtype != tdt:
            self.layout = lay
            self.v = torch.zeros(total, dtype=tdt, device=dev)  # np.zeros_like(delta) on first use
        lh = torch.zeros(total, dtype=torch.float32, pin_memory=True)
        gh = torch.zeros(total, dtype=tdt, pin_memory=True)
        for k, s, o, n in lay:
            lh.numpy()[o : o + n] = local[k].reshape(-1)
            gh.numpy()[o : o + n] = glob[k].reshape(-1)
        with torch.cuda.device(dev):
            ld = lh.to(dev, non_blocking=True)
            gd = gh.to(dev, non_blocking=True)
            out = torch.empty(total, dtype=tdt, device=dev)
            from ..aggregator import apply_update

            params = dict(self.params, **override)
            kw = {"out64": out} if tdt == torch.float64 else {"out32": out}
            apply_update(self.op, ld, gd, self.v, **kw, **params)
            host = out.cpu().numpy()
        for k, s, o, n in lay:  # in place, like the reference (avgm.py:34-35, opt.py:62-63)
            w_local[k] = host[o : o + n].reshape(s).copy()
        return w_local
