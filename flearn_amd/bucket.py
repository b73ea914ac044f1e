"""Bucket planning and host<->device packing of client state_dicts.

The reference reduces key by key, N x K numpy calls over many small tensors
(flearn/common/strategy/strategy.py:123-126; ResNet-18 has 102 fp32 tensors, median 256
elements).  Here every selected key of every client is flattened into ONE row of a device
matrix per arithmetic kind ("bucket"), so a whole aggregation is one kernel launch:

    f32 bucket  [N, stride]  fp32 tensors (weights, biases, BN running stats)
    f64 bucket  [N, stride]  float64 tensors, and int64 buffers numpy promotes to float64
    i64 bucket  [N, stride]  int64 buffers under integer weights (stay int64 in numpy)

Each key occupies a segment [offset, offset+numel) of its bucket row; segments start on
ALIGN-element (256-byte) boundaries and the row stride is a multiple of ALIGN, so every row of
every segment is 16-byte aligned for the dwordx4 loads, and rows never share a cache line.
Padding elements are zero and never read back.
"""
from __future__ import annotations

import concurrent.futures
import math
from dataclasses import dataclass, field
from functools import reduce

import numpy as np
import torch

from .semantics import KIND_F32, KIND_F64, KIND_I64, Numerics, resolve

ALIGN = 64  # elements: 256 B for fp32, 512 B for 8-byte kinds

_STORE = {KIND_F32: np.float32, KIND_F64: np.float64, KIND_I64: np.int64}
_TORCH = {np.float32: torch.float32, np.float64: torch.float64, np.int64: torch.int64}


@dataclass
class Segment:
    key: str
    shape: tuple
    numel: int
    offset: int
    src_dtype: np.dtype


@dataclass
class Group:
    kind: str
    numerics: Numerics
    segments: list = field(default_factory=list)
    stride: int = 0

    @property
    def store_dtype(self):
        return _STORE[self.kind]


@dataclass
class BucketPlan:
    keys: list  # output key order
    groups: dict  # kind -> Group
    key_group: dict  # key -> kind
    key_segment: dict  # key -> Segment
    n_clients: int
    input_kind: str  # "numpy" | "torch"

    @property
    def f32(self):
        return self.groups.get(KIND_F32)


def _as_array_meta(v, where):
    """(dtype, shape, kind) of one uploaded value without copying it."""
    if isinstance(v, torch.Tensor):
        return np.dtype(str(v.dtype).replace("torch.", "")), tuple(v.shape), "torch"
    if isinstance(v, (np.ndarray, np.generic)):
        return v.dtype, tuple(np.shape(v)), "numpy"
    raise TypeError(f"{where}: unsupported value type {type(v).__name__} (expected ndarray or Tensor)")


def select_keys(w_local_lst, key_lst=None):
    """strategy.py:119-121: the keys common to every client when key_lst is None, else key_lst.
    Ordered by the first client's insertion order (the reference's order is set-hash order,
    so any fixed order is equally faithful; this one is deterministic)."""
    if key_lst is not None:
        keys = list(key_lst)
        for n, w in enumerate(w_local_lst):
            for k in keys:
                if k not in w:
                    raise KeyError(k)
        return keys
    common = reduce(lambda a, b: a & b, [set(w.keys()) for w in w_local_lst])
    return [k for k in w_local_lst[0].keys() if k in common]


def make_plan(agg_weight_lst, w_local_lst, key_lst=None) -> BucketPlan:
    if len(w_local_lst) == 0 or len(agg_weight_lst) == 0:
        raise IndexError("list index out of range")  # reference: agg_weight_lst[0] (strategy.py:123)
    if len(agg_weight_lst) != len(w_local_lst):
        raise ValueError("agg_weight_lst and w_local_lst differ in length")
    keys = select_keys(w_local_lst, key_lst)
    numerics_by_dtype = {}
    groups: dict = {}
    key_group = {}
    key_segment = {}
    input_kinds = set()
    for k in keys:
        dt, shape, ik = _as_array_meta(w_local_lst[0][k], f"client 0 key {k!r}")
        input_kinds.add(ik)
        for n in range(1, len(w_local_lst)):
            dtn, shn, ikn = _as_array_meta(w_local_lst[n][k], f"client {n} key {k!r}")
            input_kinds.add(ikn)
            if dtn != dt or shn != shape:
                raise ValueError(
                    f"client {n} key {k!r}: {dtn}{list(shn)} does not match client 0's {dt}{list(shape)}"
                )
        if dt not in numerics_by_dtype:
            numerics_by_dtype[dt] = resolve(agg_weight_lst, dt)
        nm = numerics_by_dtype[dt]
        g = groups.get(nm.kind)
        if g is None:
            g = groups[nm.kind] = Group(nm.kind, nm)
        elif g.numerics != nm and not _same_numerics(g.numerics, nm):
            raise TypeError(f"key {k!r} needs different arithmetic than the rest of its bucket")
        numel = int(math.prod(shape))
        seg = Segment(k, shape, numel, g.stride, dt)
        g.segments.append(seg)
        key_segment[k] = seg
        g.stride += -(-max(numel, 1) // ALIGN) * ALIGN
        key_group[k] = nm.kind
    if len(input_kinds) > 1:
        raise TypeError("mixing numpy arrays and torch tensors in one aggregation is not supported")
    return BucketPlan(keys, groups, key_group, key_segment, len(w_local_lst), input_kinds.pop() if input_kinds else "numpy")


def _same_numerics(a: Numerics, b: Numerics) -> bool:
    return (a.kind, a.mode, a.denom, a.out_dtype) == (b.kind, b.mode, b.denom, b.out_dtype) and np.array_equal(
        a.weights, b.weights
    )


class Packer:
    """Owns reusable pinned staging and device buckets; packs uploads, unpacks results."""

    def __init__(self, device, workers: int = 8):
        self.device = torch.device(device)
        self.workers = workers
        self._pinned = {}
        self._dev = {}

    def _buf(self, cache, key, shape, dtype, **kw):
        t = cache.get(key)
        if t is None or t.numel() < math.prod(shape) or t.dtype != dtype:
            cache.pop(key, None)
            t = torch.zeros(math.prod(shape), dtype=dtype, **kw)
            cache[key] = t
        return t[: math.prod(shape)].view(shape)

    def device_bucket(self, tag, shape, dtype):
        """A reusable device buffer (contents undefined)."""
        return self._buf(self._dev, tag, shape, dtype, device=self.device)

    def pack(self, plan: BucketPlan, w_local_lst) -> dict:
        """Copy every client's selected tensors into the device buckets: kind -> [N, stride]."""
        out = {}
        for kind, g in plan.groups.items():
            tdt = _TORCH[g.store_dtype]
            dev = self.device_bucket(("in", kind), (plan.n_clients, g.stride), tdt)
            if plan.input_kind == "torch" and all(
                w_local_lst[0][s.key].device.type == "cuda" for s in g.segments
            ):
                for n, w in enumerate(w_local_lst):
                    for s in g.segments:
                        dev[n, s.offset : s.offset + s.numel].copy_(w[s.key].reshape(-1))
                out[kind] = dev
                continue
            host = self._buf(self._pinned, kind, (plan.n_clients, g.stride), tdt, pin_memory=True)
            self._pack_pipelined(plan, g, w_local_lst, host, dev)
            out[kind] = dev
        return out

    def _pack_pipelined(self, plan: BucketPlan, g: Group, w_local_lst, host, dev):
        """Host ingest: client rows are packed into pinned staging by a thread pool, chunk by
        chunk, and each finished chunk's H2D copy is queued at once, so the DMA of chunk k runs
        while the CPU packs chunk k+1 (flearn's uploads are pageable host arrays: they must be
        copied once into pinned memory before the DMA engine can read them)."""
        host_np = host.numpy()

        def fill(n):
            row = host_np[n]
            w = w_local_lst[n]
            for s in g.segments:
                v = w[s.key]
                if isinstance(v, torch.Tensor):
                    v = v.detach().cpu().numpy()
                row[s.offset : s.offset + s.numel] = np.asarray(v).reshape(-1)

        n = plan.n_clients
        workers = max(1, min(self.workers, n))
        chunk = max(workers, -(-n // 8))  # ~8 chunks, at least one row per worker
        if workers == 1:
            for r in range(n):
                fill(r)
            dev.copy_(host, non_blocking=True)
            return
        with concurrent.futures.ThreadPoolExecutor(workers) as ex:
            for lo in range(0, n, chunk):
                hi = min(n, lo + chunk)
                list(ex.map(fill, range(lo, hi)))
                dev[lo:hi].copy_(host[lo:hi], non_blocking=True)

    def unpack(self, plan: BucketPlan, results: dict, as_torch: bool, out_dtype_override=None) -> dict:
        """results: kind -> device tensor [stride].  Returns {key: fresh value} in plan order,
        with the reference's types: ndarray (numpy scalar for 0-d keys) or torch CPU tensor.
        D2H goes to reusable pinned staging (full PCIe rate); the result is then copied, by a
        thread pool in slices, into ONE freshly allocated buffer per call whose views are handed
        out — nothing returned is shared with staging or with later calls."""
        host = {}
        for kind, t in results.items():
            h = self._buf(self._pinned, ("out", kind, t.dtype), tuple(t.shape), t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            host[kind] = h
        torch.cuda.current_stream(self.device).synchronize()
        fresh = {}
        for kind, h in host.items():
            src = h.numpy()
            dst = np.empty_like(src)
            step = 1 << 22  # 4M elements per slice
            if src.size > step and self.workers > 1:
                with concurrent.futures.ThreadPoolExecutor(self.workers) as ex:
                    list(ex.map(lambda lo: np.copyto(dst[lo : lo + step], src[lo : lo + step]),
                                range(0, src.size, step)))
            else:
                np.copyto(dst, src)
            fresh[kind] = dst
        glob = {}
        for k in plan.keys:
            kind = plan.key_group[k]
            s = plan.key_segment[k]
            arr = fresh[kind][s.offset : s.offset + s.numel].reshape(s.shape)
            if out_dtype_override is not None:
                arr = arr.astype(out_dtype_override, copy=False)
            if as_torch:
                glob[k] = torch.from_numpy(arr)
            elif s.shape == ():
                glob[k] = arr.dtype.type(arr[()])  # numpy returns scalars for 0-d math
            else:
                glob[k] = arr
        return glob
