"""Device-side AVGM / FedOPT update of a received global model (the client_receive form).

The reference runs `mean_momentum` (avgm.py:19-36) and `adaptive_opt` (opt.py:23-65) per client
in numpy float64.  `DeviceUpdater` flattens w_local (fp32) and w_glob (the server's float64 —
or float32 — arrays) into aligned device buffers, keeps v_t resident in HBM across rounds and
runs one fa_opt_apply launch, with the reference's operation order and precision.
"""
from __future__ import annotations

import concurrent.futures
import ctypes
import math
import os
import time

import numpy as np
import torch

from .. import _native as na
from ..bucket import ALIGN, AsyncPack

_FMT = {np.dtype(np.float32): ord("f"), np.dtype(np.float64): ord("d")}
_F32 = np.dtype(np.float32)
_DEV_GLOB = (np.dtype(np.float64), _F32)  # w_glob dtypes the device path takes
_PART_BYTES = 16 << 20  # host copies are split into parts of about this size, one per pool task
_POOL = None


def _pool() -> concurrent.futures.ThreadPoolExecutor:
    global _POOL
    if _POOL is None:
        # the pack is host-memory copies (the GIL released): as many threads as the process may
        # use, up to 16 (the GPU box's CPU share per GPU)
        try:
            cpus = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            cpus = os.cpu_count() or 8
        _POOL = concurrent.futures.ThreadPoolExecutor(max(4, min(16, cpus)), thread_name_prefix="fa-update")
    return _POOL


def _run(tasks):
    """Run zero-argument callables (copies that release the GIL) on the pool; their results."""
    if len(tasks) == 1:
        return [tasks[0]()]
    return [f.result() for f in [_pool().submit(t) for t in tasks]]


class _DictPack:
    """Copies one dict's arrays into a flat staging buffer at the layout's offsets with
    fa_py_pack_rows (csrc/fa_pyhost.c), in byte-balanced parts run on the pool; False when a
    value is not a C-contiguous array of the expected dtype (the caller then copies in Python)."""

    def __init__(self, lay, dtype, dst_ptr, part_bytes=_PART_BYTES):
        self.fn = na.load_pyhost().fa_py_pack_rows
        item, fmt = np.dtype(dtype).itemsize, _FMT[np.dtype(dtype)]
        parts, cur, size = [], [], 0
        for k, _s, o, n in lay:
            cur.append((k, n, o))
            size += n * item
            if size >= part_bytes:
                parts.append(cur)
                cur, size = [], 0
        if cur:
            parts.append(cur)
        self.parts = []
        for part in parts:  # desc table: total, src_lo, nbytes, fmt, dst_base, dst_row, dst_off; skip
            m = len(part)
            desc = np.zeros(7 * m + 1, dtype=np.int64)
            nb = np.array([n for _, n, _ in part], dtype=np.int64) * item
            desc[0:m] = nb
            desc[2 * m:3 * m] = nb
            desc[3 * m:4 * m] = fmt
            desc[4 * m:5 * m] = dst_ptr
            desc[6 * m:7 * m] = np.array([o for _, _, o in part], dtype=np.int64) * item
            self.parts.append((tuple(k for k, _, _ in part), desc))

    def tasks(self, d: dict):
        """The pack as pool tasks (one per part); each returns 0 on success."""
        if type(d) is not dict:
            d = dict(d)
        clients = [d]
        return [(lambda keys=keys, desc=desc: self.fn(clients, keys, len(keys), desc.ctypes.data, 0, 1))
                for keys, desc in self.parts]

    def __call__(self, d: dict) -> bool:
        return all(rc == 0 for rc in _run(self.tasks(d)))


class _AsyncPack(AsyncPack):
    """The zero-copy chunk plan's copies into the pinned staging as one native job list: per
    key, w_local's float32 value (when `lh_ptr` is given) and w_glob's value, in chunk order."""

    def __init__(self, chunks, lh_ptr, gh_ptr, gdtype):
        item = torch.empty((), dtype=gdtype).element_size()
        gfmt = ord("d") if item == 8 else ord("f")
        keys, rows = [], []
        for j, (_f, _e, _pl, _pg, g) in enumerate(chunks):
            for k, _s, o, n in g:
                if lh_ptr is not None:
                    keys.append(k)
                    rows.append((0, n * 4, ord("f"), lh_ptr + o * 4, j, 0, n * 4))
                keys.append(k)
                rows.append((1, n * item, gfmt, gh_ptr + o * item, j, 0, n * item))
        super().__init__(tuple(keys), np.array(rows, dtype=np.int64).reshape(-1, 7), len(chunks))

    def start(self, local, glob):
        return super().start((local if local is not None else {}, glob))


class DeviceUpdater:
    #: zero-copy, chunked: the update kernel reads w_local / w_glob from the pinned staging and
    #: writes the result straight into a fresh pinned buffer over PCIe, one chunk of keys at a
    #: time, while the pool packs the next chunk; the new w_local values are views of that buffer
    #: (no copy-out).  False: pack everything, two H2D copies, one launch, one D2H, a host copy
    #: out; tools/bench_client_update.py --ab times both
    zero_copy = True
    #: with zero_copy: how the chunks cross PCIe.  "dma": each packed chunk is copied to the GPU
    #: by a copy engine on its own stream, updated there, and its result copied back into the
    #: pinned result by another copy engine — H2D and D2H run concurrently at DMA rate;
    #: "kernel": the update kernel itself reads the pinned staging and writes the pinned result
    #: over PCIe (zero-copy loads run below the DMA rate: 38 vs ~55 GB/s, round 4)
    transfer = "kernel"
    chunk_bytes = 64 << 20  # w_glob bytes per zero-copy chunk (the middle ones; 32 MiB: +0.3-0.8 ms, round 4)
    first_chunk_bytes = 4 << 20  # the first chunks grow from this (x2 each) so the GPU starts early
    last_chunk_bytes = 8 << 20  # ... and the last ones shrink towards this: a short exposed tail
    #: the zero-copy chunks are packed by native threads (fa_py_pack_start: 512 KiB jobs, no
    #: interpreter work per job, the waiting thread copies too); False: Python pool tasks of
    #: 4 MiB parts (the fallback for values the native pack refuses)
    native_pack = True
    #: a list to receive per-call phase times (tools/bench_client_update.py --phases), or None
    trace = None

    def __init__(self, op: str, device=None, beta=0.9, eta=1e-1, tau=1e-9, beta2=0.99):
        self.op = na.OP_BY_NAME[op]
        self.device = device
        self.params = dict(beta=beta, eta=eta, tau=tau, beta2=beta2)
        self.layout = None  # [(key, shape, offset, numel)]
        self.v = None
        self._v_next = None  # the zero-copy path's second v_t buffer (double-buffered: all or nothing)
        self.v_host = {}  # v_t of the keys computed on the host (integer buffers, scalars)
        self._stage = None  # pinned staging of the current layout (local, global, result)

    def _layout(self, w_glob):
        """[(key, shape, offset, numel)], total — cached on the (key, shape) signature: the same
        model comes back every round."""
        sig = tuple((k, g.shape) for k, g in w_glob.items())
        hit = getattr(self, "_lay_cache", None)
        if hit is not None and hit[0] == sig:
            return hit[1], hit[2]
        lay, off = [], 0
        for k, shape in sig:
            n = math.prod(shape) if shape else 1
            lay.append((k, shape, off, n))
            off += -(-max(n, 1) // ALIGN) * ALIGN
        self._lay_cache = (sig, lay, off)
        return lay, off

    def reset(self):
        """Forget v_t (device and host keys): the next call starts from zeros, as a fresh
        strategy object would."""
        self.layout, self.v, self._v_next, self._stage, self.v_host = None, None, None, None, {}

    def state(self):
        """v_t as the reference exposes it: {key: ndarray}."""
        out = {}
        if self.v is not None:
            host = self.v.cpu().numpy()
            out = {k: host[o : o + n].reshape(s).copy() for k, s, o, n in self.layout}
        out.update(self.v_host)
        return out

    def __call__(self, w_local, w_glob, **override):
        t_call = time.perf_counter()
        n_trace = len(self.trace) if self.trace is not None else 0
        self._call(w_local, w_glob, **override)
        if self.trace is not None and len(self.trace) > n_trace:
            self.trace[-1]["call_s"] = time.perf_counter() - t_call
        return w_local

    def _call(self, w_local, w_glob, **override):
        na.lib()
        glob, local, host_keys = {}, {}, []
        gdt = None
        nd, tt = np.ndarray, torch.Tensor
        for k, g in w_glob.items():
            lv = w_local[k]
            # exact-type tests first: this loop runs over every key of every call (~0.2 ms for
            # ResNet-50's 320 keys with isinstance chains, part of what the call costs)
            if type(g) is not nd:
                if isinstance(g, tt):
                    g = g.detach().cpu().numpy()
                elif not isinstance(g, nd):
                    host_keys.append(k)
                    continue
            if type(lv) is not nd:
                if isinstance(lv, tt):
                    lv = lv.detach().cpu().numpy()
                elif not isinstance(lv, nd):
                    host_keys.append(k)
                    continue
            # the device handles fp32 parameters against a float64 / float32 global model, one
            # precision per call (the first key's); anything else (BN num_batches_tracked: int64
            # local, numpy-scalar global) takes the reference's numpy ops on the host, key by key,
            # as avgm.py / opt.py compute them
            dt = g.dtype
            if (g.ndim >= 1 and lv.dtype == _F32 and lv.shape == g.shape and dt in _DEV_GLOB
                    and (gdt is None or dt == gdt)):
                gdt = dt
                glob[k], local[k] = g, lv
            else:
                host_keys.append(k)
        if glob:
            self._device_step(w_local, glob, local, gdt, **override)
        if host_keys:
            self._host_step(w_local, w_glob, host_keys, **override)
        return w_local

    def _host_step(self, w_local, w_glob, keys, **override):
        """The reference's per-key numpy arithmetic (avgm.py:19-36 / opt.py:23-65) for the keys the
        device path does not take; their v_t lives on the host (np.zeros_like(delta) first).
        The common case — BN num_batches_tracked: a 0-d int64 local value against a float64
        scalar in w_glob — runs as ONE vectorised numpy evaluation of the same expressions over
        all such keys (elementwise, so every value is what the per-key scalar ops give; results
        are handed back as the np.float64 scalars numpy returns for 0-d operands)."""
        p = dict(self.params, **override)
        vh = self.v_host
        batch = [k for k in keys if type(w_local[k]) is np.ndarray and w_local[k].ndim == 0
                 and w_local[k].dtype == np.int64 and type(w_glob[k]) in (np.float64, float)
                 and (k not in vh or type(vh[k]) is np.float64)]
        if len(batch) > 1:
            lv = np.array([w_local[k] for k in batch], dtype=np.int64)
            g = np.array([w_glob[k] for k in batch], dtype=np.float64)
            delta = g - lv
            v = np.array([vh[k] if k in vh else 0.0 for k in batch], dtype=np.float64)
            if self.op == na.OP_AVGM:
                v = delta + p["beta"] * v
                out = lv + v
            else:
                sq = np.multiply(delta, delta)
                if self.op == na.OP_ADAGRAD:
                    v = v + sq
                elif self.op == na.OP_YOGI:
                    v = v - (1 - p["beta2"]) * sq * np.sign(v - sq)
                else:
                    v = p["beta2"] * v + (1 - p["beta2"]) * sq
                out = lv + p["eta"] * delta / (np.sqrt(v) + p["tau"])
            for i, k in enumerate(batch):
                w_local[k] = out[i]
                vh[k] = v[i]
            done = set(batch)
            keys = [k for k in keys if k not in done]
        for k in keys:
            lv = w_local[k]
            if isinstance(lv, torch.Tensor):
                lv = lv.detach().cpu().numpy()
            g = w_glob[k]
            if isinstance(g, torch.Tensor):
                g = g.detach().cpu().numpy()
            delta = g - lv
            v = vh.get(k)
            if v is None:
                v = np.zeros_like(delta)
            if self.op == na.OP_AVGM:
                v = delta + p["beta"] * v
                w_local[k] = lv + v
            else:
                sq = np.multiply(delta, delta)
                if self.op == na.OP_ADAGRAD:
                    v = v + sq
                elif self.op == na.OP_YOGI:
                    v = v - (1 - p["beta2"]) * sq * np.sign(v - sq)
                else:
                    v = p["beta2"] * v + (1 - p["beta2"]) * sq
                w_local[k] = lv + p["eta"] * delta / (np.sqrt(v) + p["tau"])
            vh[k] = v

    def _device_step(self, w_local, glob, local, gdt, **override):
        lay, total = self._layout(glob)
        dev = torch.device(self.device) if self.device is not None else torch.device("cuda", torch.cuda.current_device())
        tdt = torch.float64 if gdt == np.float64 else torch.float32
        if self.v is not None and (self.layout != lay or self.v.dtype != tdt):
            raise ValueError("the model layout or w_glob's dtype changed between rounds: v_t no longer matches; "
                             "call reset() to start the optimizer state afresh")
        if self.v is None:
            self.layout = lay
            self.v = torch.zeros(total, dtype=tdt, device=dev)  # np.zeros_like(delta) on first use
            self._v_next = None
            self._stage = None
        st = self._staging(lay, total, tdt, dev)
        ev = getattr(self, "_h2d_done", None)
        if ev is not None:  # update_on_device's DMAs out of the shared pinned staging are done
            ev.synchronize()
            self._h2d_done = None
        if self.zero_copy:
            return self._device_step_zc(w_local, glob, local, lay, total, tdt, dev, **override)
        lh, gh, oh, pack_l, pack_g = st
        if oh is None:  # staging made for the zero-copy path: the copy-engine path needs a result buffer
            oh = torch.empty(total, dtype=tdt, pin_memory=True)
            self._stage = (lh, gh, oh, pack_l, pack_g)
        with torch.cuda.device(dev):
            # local -> pinned -> device, then the global model while the local one is in flight
            if not pack_l(local):
                for k, s, o, n in lay:
                    lh.numpy()[o : o + n] = local[k].reshape(-1)
            ld = lh.to(dev, non_blocking=True)
            if not pack_g(glob):
                for k, s, o, n in lay:
                    gh.numpy()[o : o + n] = glob[k].reshape(-1)
            gd = gh.to(dev, non_blocking=True)
            out = torch.empty(total, dtype=tdt, device=dev)
            from ..aggregator import apply_update

            params = dict(self.params, **override)
            kw = {"out64": out} if tdt == torch.float64 else {"out32": out}
            apply_update(self.op, ld, gd, self.v, **kw, **params)
            oh.copy_(out, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()  # staging is reused by the next call
        # one fresh array for the new w_local, filled from the pinned result by the pool
        src = oh.numpy()
        fresh = np.empty(total, dtype=src.dtype)
        step = 1 << 22
        _run([(lambda a=a: np.copyto(fresh[a : a + step], src[a : a + step])) for a in range(0, total, step)])
        for k, s, o, n in lay:  # replaced per key, like the reference (avgm.py:34-35, opt.py:62-63)
            w_local[k] = fresh[o : o + n].reshape(s)

    def _chunks(self, lay, total, tdt):
        """[(first, end, pack_local, pack_glob)]: runs of whole keys of about chunk_bytes of w_glob,
        in layout order, with their own pack tables into the shared staging (cached per layout)."""
        if getattr(self, "_chunk_plan", None) is not None and self._chunk_plan[0] is self._stage:
            return self._chunk_plan[1]
        lh, gh = self._stage[0], self._stage[1]
        gdt = np.float64 if tdt == torch.float64 else np.float32
        item = np.dtype(gdt).itemsize
        # target sizes: first_chunk_bytes doubling up to chunk_bytes, then chunk_bytes, and the
        # last ones halving down to last_chunk_bytes (the exposed ends of the pipeline: the first
        # chunk's pack before the GPU starts, the last chunk's kernel after the pack is done)
        total_b = sum(e[3] for e in lay) * item
        head, b = [], max(1, int(self.first_chunk_bytes))
        while b < self.chunk_bytes and sum(head) + b < total_b:
            head.append(b)
            b *= 2
        tail, b = [], max(1, int(self.last_chunk_bytes))
        while b < self.chunk_bytes and sum(head) + sum(tail) + b < total_b:
            tail.append(b)
            b *= 2
        tail.reverse()
        mid = max(0, total_b - sum(head) - sum(tail))
        targets = head + [self.chunk_bytes] * max(1, -(-mid // max(1, self.chunk_bytes))) + tail
        groups, cur, size = [], [], 0
        for e in lay:
            cur.append(e)
            size += e[3] * item
            if size >= targets[min(len(groups), len(targets) - 1)]:
                groups.append(cur)
                cur, size = [], 0
        if cur:
            groups.append(cur)
        out = []
        for j, g in enumerate(groups):
            first = g[0][2] if j else 0
            end = groups[j + 1][0][2] if j + 1 < len(groups) else total
            out.append((first, end, _DictPack(g, np.float32, lh.data_ptr(), 4 << 20),
                        _DictPack(g, gdt, gh.data_ptr(), 4 << 20), g))
        self._chunk_plan = (self._stage, out)
        self._apacks = {}
        return out

    def _apack(self, chunks, with_local: bool):
        """The chunk plan's native async pack (w_glob only, or w_local and w_glob), cached with it."""
        ap = self._apacks.get(with_local)
        if ap is None:
            ap = self._apacks[with_local] = _AsyncPack(chunks, self._stage[0].data_ptr() if with_local else None,
                                                       self._stage[1].data_ptr(), self._stage[1].dtype)
        return ap

    def _device_step_zc(self, w_local, glob, local, lay, total, tdt, dev, **override):
        """All or nothing: v_t advances into the second buffer, which becomes v_t only after
        every chunk ran; on any error the queued chunks are waited for (they read the staging
        the next call repacks) and v_t, the staging and w_local are as before the call."""
        from ..aggregator import _epilogue

        lh, gh = self._stage[0], self._stage[1]
        L = na.lib()
        prec = na.PREC_F64 if tdt == torch.float64 else na.PREC_F32
        p = dict(self.params, **override)
        if self._v_next is None or self._v_next.shape != self.v.shape or self._v_next.dtype != self.v.dtype:
            self._v_next = torch.empty_like(self.v)
        v_in, v_out = self.v, self._v_next
        # the new w_local lives in a fresh pinned buffer the kernel writes over PCIe; the values
        # handed out are views of it (torch's host caching allocator recycles it once they die)
        t_alloc = time.perf_counter()
        res = torch.empty(total, dtype=tdt, pin_memory=True)
        dma = self.transfer in ("dma", "dma_in")
        dma_out = self.transfer == "dma"
        if dma:
            dbuf = getattr(self, "_dbuf", None)
            if dbuf is None or dbuf[0] is not self._stage:
                # device copies of the staging and the result, and the copy-in / copy-out streams
                dbuf = self._dbuf = (self._stage, torch.empty(total, dtype=torch.float32, device=dev),
                                     torch.empty(total, dtype=tdt, device=dev), torch.empty(total, dtype=tdt, device=dev),
                                     torch.cuda.Stream(dev), torch.cuda.Stream(dev))
            _, dl, dg, dout, s_in, s_out = dbuf
        tr = [] if self.trace is not None else None
        t0 = time.perf_counter()
        chunks = self._chunks(lay, total, tdt)
        # every chunk's copies are queued at once, in chunk order: native threads (or, for values
        # the native pack refuses, the Python pool) stay busy whatever the chunk sizes, and each
        # chunk's kernel is launched as soon as its own copies are in
        ap = self._apack(chunks, True) if self.native_pack else None
        h = ap.start(local, glob) if ap is not None else None
        self.last_pack = "native" if h is not None else "pool"
        futs = None
        if h is None:
            pool = _pool()
            futs = [([pool.submit(t) for t in pack_l.tasks(local)], [pool.submit(t) for t in pack_g.tasks(glob)])
                    for _first, _end, pack_l, pack_g, _g in chunks]
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev)
            sh = stream.cuda_stream
            try:
                for j, (first, end, pack_l, pack_g, g) in enumerate(chunks):
                    tp = time.perf_counter()
                    if h is not None:
                        ap.wait(h, j)
                    else:
                        fl, fg = futs[j]
                        if any(f.result() for f in fl):  # a value the native pack refuses: copy in Python
                            for k, s, o, n in g:
                                lh.numpy()[o : o + n] = local[k].reshape(-1)
                        if any(f.result() for f in fg):
                            for k, s, o, n in g:
                                gh.numpy()[o : o + n] = glob[k].reshape(-1)
                    n = end - first
                    if dma:  # copy engine in (own stream), the update on the device, copy engine out
                        with torch.cuda.stream(s_in):
                            dl[first:end].copy_(lh[first:end], non_blocking=True)
                            dg[first:end].copy_(gh[first:end], non_blocking=True)
                        stream.wait_stream(s_in)
                        src_l, src_g = dl[first:end], dg[first:end]
                        out = (dout if dma_out else res)[first:end].data_ptr()
                    else:  # the kernel reads the pinned staging and writes the pinned result over PCIe
                        src_l, src_g, out = lh[first:end], gh[first:end], res[first:end].data_ptr()
                    epi = _epilogue(self.op, src_l, v_in[first:end], p["beta"], p["eta"], p["tau"], p["beta2"],
                                    v_out=v_out[first:end])
                    na.check(L.fa_opt_apply(prec, ctypes.byref(epi), src_l.data_ptr(), src_g.data_ptr(),
                                            n, None if prec == na.PREC_F64 else out,
                                            out if prec == na.PREC_F64 else None, sh), "fa_opt_apply")
                    if dma_out:
                        s_out.wait_stream(stream)
                        with torch.cuda.stream(s_out):
                            res[first:end].copy_(dout[first:end], non_blocking=True)
                    if tr is not None:
                        tr.append((end - first, tp - t0, time.perf_counter() - t0))
            except BaseException:
                if h is not None:  # no pack may still write the staging ...
                    ap.end(h)
                else:
                    for fl, fg in futs:
                        for f in fl + fg:
                            f.cancel()
                    concurrent.futures.wait([f for fl, fg in futs for f in fl + fg])
                stream.synchronize()  # ... nor a queued chunk read it or write `res`
                if dma:
                    s_in.synchronize()
                    s_out.synchronize()
                raise
            ts = time.perf_counter()
            if h is not None:
                ap.end(h)  # every copy is done: releases the values
            # the new values' views are made while the GPU finishes (they read nothing yet)
            fresh = res.numpy()
            views = [(k, fresh[o : o + n].reshape(s)) for k, s, o, n in lay]
            stream.synchronize()
            if dma:
                s_out.synchronize()
        self.v, self._v_next = v_out, v_in
        if tr is not None:
            self.trace.append({"chunks": tr, "launched_s": ts - t0, "done_s": time.perf_counter() - t0,
                               "alloc_s": t0 - t_alloc})
        w_local.update(views)  # replaced per key, like the reference (avgm.py:34-35, opt.py:62-63)

    # ---- the model already on the GPU (client_receive with a CUDA model) ---------------------
    @staticmethod
    def device_model_ok(weights, w_glob) -> bool:
        """True when client_receive can update the model where it lives: every state_dict value
        a contiguous float32 CUDA tensor on one device, and every w_glob value an ndarray of the
        same shape, all float64 or all float32 (what the server returns for fp32 models).
        Anything else — BN counters (whose numpy scalars make the reference's convert_to_tensor
        raise), CPU models, other dtypes — takes the reference's host path unchanged."""
        if not weights or not w_glob:
            return False
        devs = set()
        for v in weights.values():
            if not (isinstance(v, torch.Tensor) and v.is_cuda and v.dtype == torch.float32 and v.is_contiguous()):
                return False
            devs.add(v.device)
        if len(devs) != 1:
            return False
        gdt = None
        for k, g in w_glob.items():
            lv = weights.get(k)
            if lv is None or type(g) is not np.ndarray or g.dtype not in (np.float64, np.float32):
                return False
            if tuple(g.shape) != tuple(lv.shape):
                return False
            if gdt is None:
                gdt = g.dtype
            elif g.dtype != gdt:
                return False
        return True

    def update_on_device(self, local: dict, w_glob: dict, **override) -> dict:
        """The update of a model that lives on the GPU: w_local's values are the model's float32
        CUDA tensors (gathered in one launch, fa_gather_rows), w_glob's host arrays go to the GPU
        in chunks (packed by the pool into pinned staging, one DMA each) and each chunk's update
        runs as soon as it lands.  Returns {key: the new value as a CUDA tensor in w_glob's dtype}
        for w_glob's keys — what load_state_dict then casts into the float32 parameters, exactly
        as it casts the reference's float64 host arrays.  Only the server's model crosses PCIe
        (the reference moves the local model down and the result back up as well).  v_t is the
        same double-buffered state the host path keeps, so the two paths may alternate."""
        na.lib()
        glob = {k: np.ascontiguousarray(g) for k, g in w_glob.items()}
        gdt = next(iter(glob.values())).dtype
        tdt = torch.float64 if gdt == np.float64 else torch.float32
        dev = next(iter(local.values())).device
        lay, total = self._layout(glob)
        if self.v is not None and (self.layout != lay or self.v.dtype != tdt):
            raise ValueError("the model layout or w_glob's dtype changed between rounds: v_t no longer matches; "
                             "call reset() to start the optimizer state afresh")
        if self.v is None:
            self.layout = lay
            self.v = torch.zeros(total, dtype=tdt, device=dev)
            self._v_next = None
            self._stage = None
        self._staging(lay, total, tdt, dev)
        gh = self._stage[1]
        ev = getattr(self, "_h2d_done", None)
        if ev is not None:  # the previous call's DMAs out of the pinned staging are complete
            ev.synchronize()
        key = ("devmodel", self._stage[1].data_ptr(), str(dev))
        db = getattr(self, "_devbuf", None)
        if db is None or db[0] != key:
            segs = torch.tensor([o for _, _, o, _ in lay] + [n for _, _, _, n in lay], dtype=torch.int64).to(dev)
            db = self._devbuf = (key, torch.zeros(total, dtype=torch.float32, device=dev),
                                 torch.empty(total, dtype=tdt, device=dev), torch.empty(total, dtype=tdt, device=dev),
                                 segs, torch.empty(len(lay), dtype=torch.int64, pin_memory=True),
                                 torch.empty(len(lay), dtype=torch.int64, device=dev))
        _, dl, dg, dout, segs, ptr_h, ptr_d = db
        if self._v_next is None or self._v_next.shape != self.v.shape or self._v_next.dtype != self.v.dtype:
            self._v_next = torch.empty_like(self.v)
        v_in, v_out = self.v, self._v_next
        from ..aggregator import _epilogue

        L = na.lib()
        prec = na.PREC_F64 if tdt == torch.float64 else na.PREC_F32
        p = dict(self.params, **override)
        chunks = self._chunks(lay, total, tdt)
        ap = self._apack(chunks, False) if self.native_pack else None
        h = ap.start(None, glob) if ap is not None else None
        futs = None
        if h is None:
            pool = _pool()
            futs = [[pool.submit(t) for t in pack_g.tasks(glob)] for _f, _e, _pl, pack_g, _g in chunks]
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev)
            sh = stream.cuda_stream
            try:
                # the local model: one gather launch of every tensor into its layout slot
                ptr_h.numpy()[:] = [local[k].data_ptr() for k, _, _, _ in lay]
                ptr_d.copy_(ptr_h, non_blocking=True)
                na.check(L.fa_gather_rows(dl.data_ptr(), total, 1, 4, ptr_d.data_ptr(), segs.data_ptr(), len(lay), sh),
                         "fa_gather_rows")
                for j, (first, end, _pl, _pg, g) in enumerate(chunks):
                    if h is not None:
                        ap.wait(h, j)
                    elif any(f.result() for f in futs[j]):  # a value the native pack refuses: copy in Python
                        for k, _s, o, n in g:
                            gh.numpy()[o : o + n] = glob[k].reshape(-1)
                    dg[first:end].copy_(gh[first:end], non_blocking=True)
                    epi = _epilogue(self.op, dl[first:end], v_in[first:end], p["beta"], p["eta"], p["tau"], p["beta2"],
                                    v_out=v_out[first:end])
                    out = dout[first:end].data_ptr()
                    na.check(L.fa_opt_apply(prec, ctypes.byref(epi), dl[first:end].data_ptr(), dg[first:end].data_ptr(),
                                            end - first, None if prec == na.PREC_F64 else out,
                                            out if prec == na.PREC_F64 else None, sh), "fa_opt_apply")
            except BaseException:
                if h is not None:
                    ap.end(h)
                else:
                    for fg in futs:
                        for f in fg:
                            f.cancel()
                    concurrent.futures.wait([f for fg in futs for f in fg])
                stream.synchronize()
                raise
            if h is not None:
                ap.end(h)
            done = torch.cuda.Event()
            done.record(stream)
        self._h2d_done = done
        self.v, self._v_next = v_out, v_in
        # fresh result buffer per call: the returned tensors must not be overwritten by the next
        res = dout
        self._devbuf = db[:3] + (torch.empty(total, dtype=tdt, device=dev),) + db[4:]
        return {k: res[o : o + n].view(s) for k, s, o, n in lay}

    def _staging(self, lay, total, tdt, dev):
        """Pinned staging for this layout, reused across calls (zeroed once: only the segments
        are ever written, so the alignment gaps stay zero)."""
        if getattr(self, "_stage", None) is None:
            lh = torch.zeros(total, dtype=torch.float32, pin_memory=True)
            gh = torch.zeros(total, dtype=tdt, pin_memory=True)
            oh = None if self.zero_copy else torch.empty(total, dtype=tdt, pin_memory=True)
            gdt = np.float64 if tdt == torch.float64 else np.float32
            self._stage = (lh, gh, oh, _DictPack(lay, np.float32, lh.data_ptr()), _DictPack(lay, gdt, gh.data_ptr()))
        return self._stage
