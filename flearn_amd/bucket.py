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

import collections
import concurrent.futures
import ctypes
import math
import os
import threading
from dataclasses import dataclass, field
from functools import reduce

import numpy as np
import torch

from . import _native as na
from .semantics import KIND_F32, KIND_F64, KIND_I64, Numerics, resolve

ALIGN = 64  # elements: 256 B for fp32, 512 B for 8-byte kinds
SMALL_BYTES = 4 << 20  # below this, host packing / unpacking runs on the calling thread

_STORE = {KIND_F32: np.float32, KIND_F64: np.float64, KIND_I64: np.int64}
_TORCH = {np.float32: torch.float32, np.float64: torch.float64, np.int64: torch.int64}
# device-upload dtypes a group's row table takes, and their fa_gather_rows_f64 source kind
_ROW_SOURCES = {torch.float64: {torch.float64: na.SRC_F64, torch.int64: na.SRC_I64, torch.float32: na.SRC_F32}}
_NP = {torch.float32: np.float32, torch.float64: np.float64, torch.int64: np.int64}
_FMT = {np.dtype(np.float32): ord("f"), np.dtype(np.float64): ord("d"), np.dtype(np.int64): ord("i")}


class AsyncPack:
    """Host copies run by native threads (csrc/fa_pyhost.c fa_py_pack_start / fa_pack_wait /
    fa_py_pack_end): `rows` is an int64 table, one row per piece: (index of the source dict,
    the value's size in bytes, format class, destination address, chunk, first byte, bytes).
    `start(dicts)` checks every value against the table under the GIL (all or nothing: None
    when a value is off the plan, nothing copied) and queues the copies in chunk order as jobs
    of SPLIT bytes; `wait(h, j)` returns (the GIL released) once chunk j's bytes are in, the
    waiting thread copying jobs of chunks <= j itself; `end(h)` waits for everything and drops
    the values.  No interpreter work per job: the Python pool's per-part GIL hand-offs kept the
    first chunk 0.5-0.9 ms from its launch in the client update."""

    SPLIT = 512 << 10  # bytes per native copy job

    def __init__(self, keys: tuple, rows: np.ndarray, nchunks: int, threads: int = 0):
        self.keys = keys
        self.desc = np.ascontiguousarray(rows.T).reshape(-1)
        self.nchunks = nchunks
        self.L = na.load_pyhost()
        if threads <= 0:
            try:
                cpus = len(os.sched_getaffinity(0))
            except (AttributeError, OSError):
                cpus = os.cpu_count() or 8
            threads = max(4, min(16, cpus))
        self.threads = threads

    def start(self, dicts):
        st = ctypes.c_int32(0)
        h = self.L.fa_py_pack_start(dicts, self.keys, len(self.keys), self.desc.ctypes.data, self.nchunks,
                                    self.SPLIT, self.threads, ctypes.byref(st))
        if not h:
            if st.value == 2:
                raise MemoryError("fa_py_pack_start: out of host memory")
            return None
        return h

    def wait(self, h, j: int) -> None:
        if self.L.fa_pack_wait(h, j) != 0:
            raise RuntimeError(f"fa_pack_wait({j}) failed")

    def end(self, h) -> None:
        self.L.fa_py_pack_end(h)


class _NativeRows:
    """Packs client rows through fa_py_pack_rows (csrc/fa_pyhost.c): one native call walks the
    clients' dicts and copies every piece into the pinned staging, the GIL released around the
    copies.  Built per pack call from the plan's pieces; `__call__(lo, hi)` returns False when a
    value is not a plain C-contiguous array of its planned dtype (torch tensors, views of other
    layouts...), and the caller then packs those rows from Python."""

    def __init__(self, pieces, hosts, w_local_lst, rows, memo=None):
        self.fn = na.load_pyhost().fa_py_pack_rows
        # plain dicts only (dict / OrderedDict, whose item lookup the C side reproduces)
        self.clients = [w if type(w) in (dict, collections.OrderedDict) else None for w in w_local_lst]
        hp = tuple((h.data_ptr(), h.stride(0)) for h in hosts)
        # keyed by the pieces list (memoized on the plan: one object per kind and shard layout)
        # AND the staging addresses: two kinds' stagings of different packers can occupy the same
        # pinned block in turn (the host caching allocator hands a freed block out again), and a
        # table keyed by addresses alone then packed one kind's keys into the other's stack
        key = ("native_rows", id(pieces), hp)
        cached = memo.get(key) if memo is not None else None
        if cached is None:
            # per piece: itemsize, numel, src lo, src hi, format, dst base, dst row stride
            # (elements), dst off -> the byte table fa_py_pack_rows reads (7 rows of pieces)
            t = np.array([(s.src_dtype.itemsize, s.numel, a, b, _FMT[s.src_dtype]) + hp[sh.index] + (d,)
                          for s, a, b, sh, d in pieces], dtype=np.int64).reshape(-1, 8).T
            item = t[0]
            table = np.concatenate([t[1] * item, t[2] * item, (t[3] - t[2]) * item, t[4], t[5],
                                    t[6] * item, t[7] * item])
            cached = (tuple(s.key for s, *_ in pieces), table)
            if memo is not None:
                memo[key] = cached
        self.keys, table = cached
        # ... then one skip flag per client row
        self.desc = np.concatenate([table, np.fromiter((r is not None for r in rows), dtype=np.int64, count=len(rows))])
        self.ptr = self.desc.ctypes.data

    @staticmethod
    def usable(pieces, hosts) -> bool:
        """Byte copies only: every source dtype is its bucket's storage dtype."""
        return bool(pieces) and all(
            h is not None and s.src_dtype in _FMT and np.dtype(_NP[h.dtype]) == s.src_dtype
            for s, _, _, sh, _ in pieces for h in (hosts[sh.index],))

    def __call__(self, lo: int, hi: int) -> bool:
        return self.fn(self.clients, self.keys, len(self.keys), self.ptr, lo, hi) == 0


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
    # derived per-plan data of the packer (pieces, native pack tables); plans are reused across
    # rounds (make_plan's cache), so this is computed once per model layout and staging buffer
    memo: dict = field(default_factory=dict, compare=False, repr=False)

    @property
    def f32(self):
        return self.groups.get(KIND_F32)


def _as_array_meta(v, where):
    """(dtype, shape, kind) of one uploaded value without copying it."""
    if isinstance(v, (np.ndarray, np.generic)):
        return v.dtype, v.shape, "numpy"
    if isinstance(v, torch.Tensor):
        if v.layout != torch.strided:
            # sparse / mkldnn / nested uploads: client data the engine does not take (TypeError ->
            # the server_exception route), never a torch error from deep inside the pack
            raise TypeError(f"{where}: {v.layout} tensor uploads are not supported (dense tensors only)")
        return np.dtype(str(v.dtype).replace("torch.", "")), tuple(v.shape), "torch"
    raise TypeError(f"{where}: unsupported value type {type(v).__name__} (expected ndarray or Tensor)")


def _raw_signature(w, keys):
    """(type, dtype, shape, layout) of every selected value, as the objects report them (no
    normalisation): equal signatures mean equal metadata, so only the first client needs the
    per-key checks (10,200 of them for 100 ResNet-18 uploads)."""
    try:
        return tuple((type(v), v.dtype, v.shape, getattr(v, "layout", None)) for v in map(w.__getitem__, keys))
    except (AttributeError, KeyError):
        return None


def _plain_dicts(w_local_lst) -> bool:
    """Every upload is a dict / OrderedDict, whose item lookup the native walks reproduce."""
    return all(type(w) in (dict, collections.OrderedDict) for w in w_local_lst)


def _same_signature_native(w_local_lst, keys, sig0=None) -> bool:
    """True when every client's (type, dtype, shape, layout) per key equals client 0's, read
    natively: numpy uploads through the buffer protocol (csrc/fa_pyhost.c fa_py_same_signature:
    type, format, itemsize, shape — numpy arrays are always strided), torch uploads from the
    tensors' TensorImpl (csrc/fa_torchmeta.cpp) — the same comparisons as _raw_signature without
    the per-attribute interpreter work; False when it differs or cannot tell (the caller then
    compares in Python)."""
    if len(w_local_lst) < 2 or not _plain_dicts(w_local_lst):
        return False
    lst = w_local_lst if type(w_local_lst) is list else list(w_local_lst)
    if sig0 is not None and sig0 and all(t[0] is np.ndarray for t in sig0):
        return na.load_pyhost().fa_py_same_signature(lst, tuple(keys)) == 1
    L = na.load_torchmeta()
    if L is None:
        return False
    return L.fa_tm_same_signature(lst, tuple(keys)) == 1


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
    k0 = w_local_lst[0].keys()
    if all(w.keys() == k0 for w in w_local_lst[1:]):  # the usual case: one model, same keys (C-level set compare)
        return list(k0)
    common = reduce(lambda a, b: a & b, [set(w.keys()) for w in w_local_lst])
    return [k for k in w_local_lst[0].keys() if k in common]


_PLANS: collections.OrderedDict = collections.OrderedDict()  # recent plans (read-only once built)
_PLANS_MAX = 8
_PLANS_LOCK = threading.Lock()


def make_plan(agg_weight_lst, w_local_lst, key_lst=None) -> BucketPlan:
    """The bucket plan of one aggregation.  A federated run aggregates the same model with the
    same weights round after round, so a plan is reused when the selected keys, every client's
    (type, dtype, shape, layout) per key, the client count and the weights (types and exact values, by
    repr: -0.0 and NaN included) all equal a recent call's."""
    if len(w_local_lst) == 0 or len(agg_weight_lst) == 0:
        raise IndexError("list index out of range")  # reference: agg_weight_lst[0] (strategy.py:123)
    if len(agg_weight_lst) != len(w_local_lst):
        raise ValueError("agg_weight_lst and w_local_lst differ in length")
    keys = sig0 = slow = None
    if key_lst is None and len(w_local_lst) > 1:
        # the usual round: client 0's keys, verified natively in every client together with their
        # metadata — a client missing one of them makes the native check give up (the general
        # intersection below then runs), so passing it proves the intersection is client 0's keys
        k0 = list(w_local_lst[0].keys())
        s0 = _raw_signature(w_local_lst[0], k0)
        if s0 is not None and _same_signature_native(w_local_lst, k0, s0):
            keys, sig0, slow = k0, s0, []
    if keys is None:
        keys = select_keys(w_local_lst, key_lst)
        sig0 = _raw_signature(w_local_lst[0], keys)
    if slow is not None:
        pass
    elif sig0 is not None and _same_signature_native(w_local_lst, keys, sig0):
        slow = []
    else:
        slow = [n for n in range(1, len(w_local_lst))
                if sig0 is None or _raw_signature(w_local_lst[n], keys) != sig0]
    ck = None
    if sig0 is not None and not slow:
        ck = (tuple(keys), sig0, len(w_local_lst), tuple(map(type, agg_weight_lst)), repr(list(agg_weight_lst)))
        try:
            with _PLANS_LOCK:
                plan = _PLANS.get(ck)
                if plan is not None:
                    _PLANS.move_to_end(ck)
                    return plan
        except TypeError:  # something unhashable in the metadata: plan afresh, uncached
            ck = None
    plan = _build_plan(agg_weight_lst, w_local_lst, keys, slow)
    if ck is not None:
        with _PLANS_LOCK:
            _PLANS[ck] = plan
            while len(_PLANS) > _PLANS_MAX:
                _PLANS.popitem(last=False)
    return plan


def _build_plan(agg_weight_lst, w_local_lst, keys, slow) -> BucketPlan:
    numerics_by_dtype = {}
    groups: dict = {}
    key_group = {}
    key_segment = {}
    input_kinds = set()
    for k in keys:
        dt, shape, ik = _as_array_meta(w_local_lst[0][k], f"client 0 key {k!r}")
        input_kinds.add(ik)
        for n in slow:  # clients whose metadata differs somewhere: find and report it
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
        elif g.numerics is not nm and not _same_numerics(g.numerics, nm):
            # (identity first: the dataclass __eq__ would compare the weight arrays elementwise
            # and raise for more than one client — a float64 model with int64 BN counters put
            # two dtypes' numerics into the f64 bucket and failed here)
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


@dataclass(frozen=True)
class Shard:
    """A column range [c0, c1) of the f32 bucket that lives on one device (multi-GPU ingest).
    Non-f32 buckets (f64 / i64: BN counters, a few bytes) always live on shard 0."""

    index: int
    device: torch.device
    c0: int
    c1: int

    @property
    def width(self) -> int:
        return self.c1 - self.c0


def rank_width(stride: int, world: int) -> int:
    """Columns per rank of a column-sharded process group: equal, ALIGN-aligned (the last ranks'
    ranges may be short or empty; the all-gather pads them)."""
    return -(-stride // (world * ALIGN)) * ALIGN


def split_columns(stride: int, devices) -> list:
    """Near-equal ALIGN-aligned column ranges of a stride-wide bucket, one per device."""
    k = len(devices)
    units = stride // ALIGN
    bounds = [ALIGN * (units * i // k) for i in range(k + 1)]
    bounds[-1] = stride
    return [Shard(i, torch.device(d), bounds[i], bounds[i + 1]) for i, d in enumerate(devices)]


class Packer:
    """Owns reusable pinned staging and device buckets; packs uploads, unpacks results.

    The f32 bucket is split by columns over `devices` (one Shard each): every device receives
    its columns of every client through its own PCIe link, reduces them, and sends its slice of
    the global model back — per-GPU parallel H2D/D2H.  With one device this is the plain path."""

    def __init__(self, devices, workers: int = 8):
        self.devices = [torch.device(d) for d in devices]
        self.device = self.devices[0]
        self.workers = workers
        self._pinned = {}
        self._pin_events = {}  # pinned staging key -> event after its last queued H2D
        self._dev = {}
        self._shards = {}
        self._pool = None
        self.last_wire_rows = 0
        self.last_wire_staged = 0
        self.last_row_tables = {}  # kind -> "slab" | "rows" | "gather" | "copy" for device-resident uploads
        #: device uploads carved from one allocation laid out as the bucket run as a stack
        #: (_slab_stack); False: always the pointer table (tools/rows_pmc.py measures that kernel)
        self.use_slabs = True
        self.rank_cols = None  # (rank, world): pack only this rank's columns of the f32 bucket
        #: host uploads packed by native threads in growing row chunks (AsyncPack); False: the
        #: Python pool packs ~8 equal chunks (also the fallback for values off the plan)
        self.native_async = True
        self.async_lookahead = 0  # chunks packed ahead of the DMA (0: all queued at once)
        self.async_threads = 0  # native pack threads (0: AsyncPack's default, <= 16)
        # kind -> how its last host pack ran: "serial" | "async" | "mixed" (some chunks packed
        # from Python: values off the plan) | "pool"
        self.last_pack_paths = {}
        #: one device: results stored into fresh pinned buffers by fa_copy kernels (zero-copy
        #: writes) and handed out as views; False: copy-engine D2H into staging + host copy into
        #: pageable memory.  The pinned buffers come from torch's pinned caching allocator, which
        #: keeps freed pages locked for reuse: a server that retains many rounds' w_glob (history,
        #: checkpoints) pins one model per retained round — set False there
        self.zero_copy_out = True

    def _executor(self) -> concurrent.futures.ThreadPoolExecutor:
        """One persistent pool per Packer: creating threads per call costs ~0.3 ms, which is the
        whole budget of a LeNet-sized round."""
        if self._pool is None:
            self._pool = concurrent.futures.ThreadPoolExecutor(self.workers, thread_name_prefix="fa-pack")
        return self._pool

    def _buf(self, cache, key, shape, dtype, **kw):
        t = cache.get(key)
        if t is None or t.numel() < math.prod(shape) or t.dtype != dtype:
            cache.pop(key, None)
            t = torch.zeros(math.prod(shape), dtype=dtype, **kw)
            cache[key] = t
        return t[: math.prod(shape)].view(shape)

    def hold(self, objs, device) -> None:
        """Keep `objs` (uploads read by queued launches) alive until the work queued so far on
        `device`'s current stream is done; earlier holds whose events completed are dropped."""
        self._held = [(e, o) for e, o in getattr(self, "_held", []) if not e.query()]
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        self._held.append((ev, objs))

    def device_bucket(self, tag, shape, dtype, device=None):
        """A reusable device buffer (contents undefined)."""
        dev = self.device if device is None else torch.device(device)
        return self._buf(self._dev, (tag, str(dev)), shape, dtype, device=dev)

    def shards(self, plan: BucketPlan, kind: str) -> list:
        g = plan.groups[kind]
        if kind != KIND_F32:
            return [Shard(0, self.device, 0, g.stride)]
        key = (g.stride, tuple(str(d) for d in self.devices), self.rank_cols)
        if key not in self._shards:
            if self.rank_cols is not None:  # one rank of a column-sharded process group
                rank, world = self.rank_cols
                w = rank_width(g.stride, world)
                c0 = min(rank * w, g.stride)
                self._shards[key] = [Shard(0, self.device, c0, min(c0 + w, g.stride))]
            else:
                self._shards[key] = split_columns(g.stride, self.devices)
        return self._shards[key]

    @staticmethod
    def _pieces(g: Group, shards) -> list:
        """(segment, src_lo, src_hi, shard, dst_lo): each key segment cut at shard boundaries."""
        out = []
        for s in g.segments:
            lo, hi = s.offset, s.offset + s.numel
            for sh in shards:
                a, b = max(lo, sh.c0), min(hi, sh.c1)
                if a < b:
                    out.append((s, a - lo, b - lo, sh, a - sh.c0))
        return out

    def pack(self, plan: BucketPlan, w_local_lst) -> dict:
        """Copy every client's selected tensors into the device buckets.
        Returns kind -> [(shard, device stack [N, shard.width])]."""
        out = {}
        self.last_wire_staged = 0
        self.last_row_tables = {}
        self.last_pack_paths = {}
        for kind, g in plan.groups.items():
            tdt = _TORCH[g.store_dtype]
            shards = self.shards(plan, kind)
            devs = [self.device_bucket(("in", kind, sh.index), (plan.n_clients, sh.width), tdt, sh.device)
                    for sh in shards]
            pk = ("pieces", kind, tuple((sh.index, sh.c0, sh.c1) for sh in shards))
            pieces = plan.memo.get(pk)
            if pieces is None:
                pieces = plan.memo[pk] = self._pieces(g, shards)
            if plan.input_kind == "torch" and all(w_local_lst[0][s.key].device.type == "cuda" for s in g.segments):
                rp = self._row_ptrs(plan, g, w_local_lst, shards)
                if rp is not None and kind == KIND_F32 and self.use_slabs:
                    slab = self._slab_stack(plan, g, w_local_lst, rp)
                    if slab is not None:  # one allocation laid out as the bucket: the stack itself
                        out[kind] = [(shards[0], slab)]
                        self.last_row_tables[kind] = "slab"
                        continue
                table = RowTable(self, plan, g, *rp, shards[0].device) if rp is not None else None
                if table is not None and kind == KIND_F32 and len(shards) == 1 and table.aligned:
                    out[kind] = [(shards[0], table)]  # read in place by fa_reduce_f32_rows
                    self.last_row_tables[kind] = "rows"
                    continue
                if table is not None and len(shards) == 1:
                    table.gather_into(devs[0])  # one launch for the whole bucket
                    self.last_row_tables[kind] = "gather"
                else:  # column shards over several devices: per-piece copies
                    self.last_row_tables[kind] = "copy"
                    for n, w in enumerate(w_local_lst):
                        for s, a, b, sh, d in pieces:
                            devs[sh.index][n, d : d + (b - a)].copy_(w[s.key].reshape(-1)[a:b])
            else:
                rows = self._wire_rows(g, w_local_lst) if kind == KIND_F32 else [None] * plan.n_clients
                if len(shards) == 1 and all(r is not None for r in rows):
                    staged = self._wire_stack(g, w_local_lst, shards[0].device)
                    if staged is not None:  # uploads already copied to the device at decode time
                        out[kind] = [(shards[0], staged)]
                        self.last_wire_staged = plan.n_clients
                        continue
                if all(r is not None for r in rows):
                    hosts = [None] * len(shards)  # every row already sits in pinned memory
                else:
                    hkeys = [("in", kind, sh.index) for sh in shards]
                    for hk in hkeys:  # the previous round's H2D from this staging must be done
                        ev = self._pin_events.pop(hk, None)
                        if ev is not None:
                            ev.synchronize()
                    hosts = [self._buf(self._pinned, hk, (plan.n_clients, sh.width), tdt, pin_memory=True)
                             for hk, sh in zip(hkeys, shards)]
                self.last_pack_paths[kind] = self._pack_pipelined(plan, pieces, w_local_lst, shards, hosts, devs, rows)
                if hosts[0] is not None:
                    for hk, sh in zip(hkeys, shards):
                        ev = torch.cuda.Event()
                        ev.record(torch.cuda.current_stream(sh.device))
                        self._pin_events[hk] = ev
            out[kind] = list(zip(shards, devs))
        return out

    def row_table(self, plan: BucketPlan, g: Group, w_local_lst, shards):
        """RowTable of device-resident uploads for bucket group g, or None when some value is
        not a contiguous tensor of an accepted dtype on the bucket's (single, whole-bucket)
        device.  Accepted: the store dtype; for the float64 group also int64 and float32 values
        (BN num_batches_tracked), which fa_gather_rows_f64 converts as numpy's promotion does."""
        rp = self._row_ptrs(plan, g, w_local_lst, shards)
        return None if rp is None else RowTable(self, plan, g, *rp, shards[0].device)

    @staticmethod
    def _slab_stack(plan: BucketPlan, g: Group, w_local_lst, rp):
        """The uploads as a [N, stride] stack view when every client's fp32 tensors sit in ONE
        allocation laid out exactly as this bucket — key k of client n at row_base + n * pitch +
        offset(k), the same pitch for every client (flearn_amd.device_state_dicts makes such
        uploads) — else None.  The stack kernel then reads them in place: no pointer table, and
        the translations of one allocation instead of one per (client, tensor) (the row-pointer
        kernel's 7-8% at NS)."""
        segs, ptrs, keep, _src = rp
        n = plan.n_clients
        if not segs or ptrs.shape[1] != n:
            return None
        off = np.array([s.offset for s in segs], dtype=np.int64) * 4
        base = ptrs[0] - off[0]  # each client's row start
        if not np.array_equal(ptrs - off[:, None], np.broadcast_to(base, ptrs.shape)):
            return None
        pitch = int(base[1] - base[0]) if n > 1 else g.stride * 4
        if n > 1 and not (np.diff(base) == pitch).all():
            return None
        if pitch < g.stride * 4 or pitch % 16 or int(base[0]) % 16:
            return None
        t0 = w_local_lst[0][segs[0].key]
        st = t0.untyped_storage()
        lo, hi = st.data_ptr(), st.data_ptr() + st.nbytes()
        first, end = int(base[0]), int(base[0]) + (n - 1) * pitch + g.stride * 4
        if first < lo or end > hi:  # the rows must lie inside that one allocation
            return None
        return torch.empty(0, dtype=torch.float32, device=t0.device).set_(
            st, (first - lo) // 4, (n, g.stride), (pitch // 4, 1))

    def _row_ptrs(self, plan: BucketPlan, g: Group, w_local_lst, shards):
        """(segments, pointer table [segments][clients], tensors kept, source kinds) of
        device-resident uploads — row_table's inputs — or None."""
        if len(shards) != 1 or shards[0].c0 != 0 or shards[0].c1 != g.stride:
            return None
        dev = shards[0].device
        store = _TORCH[g.store_dtype]
        accept = _ROW_SOURCES.get(store, {store: na.SRC_F64})
        segs = [s for s in g.segments if s.numel > 0]
        w0 = w_local_lst[0]
        dts = tuple(getattr(w0[s.key], "dtype", None) for s in segs)
        if any(d not in accept for d in dts):
            return None
        src = [accept[d] for d in dts]
        ptrs = np.empty((len(segs), plan.n_clients), dtype=np.int64)
        L = na.load_torchmeta()
        if L is not None and _plain_dicts(w_local_lst):  # TensorImpl reads (csrc/fa_torchmeta.cpp)
            keep = [None] * (len(segs) * plan.n_clients)
            lst = w_local_lst if type(w_local_lst) is list else list(w_local_lst)
            index = dev.index if dev.index is not None else torch.cuda.current_device()
            if L.fa_tm_tensor_ptrs(lst, tuple(s.key for s in segs), dts, index, ptrs.ctypes.data, keep) == 0:
                return segs, ptrs, keep, src
        keep = []
        for j, s in enumerate(segs):
            row = ptrs[j]
            for n, w in enumerate(w_local_lst):
                t = w[s.key]
                if t.dtype != dts[j] or t.device != dev or not t.is_contiguous():
                    return None
                row[n] = t.data_ptr()
                keep.append(t)
        return segs, ptrs, keep, src

    def _wire_stack(self, g: Group, w_local_lst, device):
        from .wire import wire_device_stack

        sig = tuple((s.key, s.shape, s.offset) for s in g.segments) + (g.stride,)
        return wire_device_stack(w_local_lst, sig, device)

    def _wire_rows(self, g: Group, w_local_lst) -> list:
        """Per client: the pinned row the wire codec decoded its fp32 params into, when that row
        is laid out exactly as this bucket (flearn_amd.wire.decode) — else None."""
        from .wire import wire_row

        sig = tuple((s.key, s.shape, s.offset) for s in g.segments) + (g.stride,)
        rows = [wire_row(w, sig) for w in w_local_lst]
        self.last_wire_rows = sum(r is not None for r in rows)
        return rows

    def _pack_pipelined(self, plan: BucketPlan, pieces, w_local_lst, shards, hosts, devs, rows=None):
        """Host ingest: client rows are packed into pinned staging by a thread pool, chunk by
        chunk, and each finished chunk's H2D copies (one per shard, on that device's stream) are
        queued at once, so the DMA of chunk k runs while the CPU packs chunk k+1 (flearn's
        uploads are pageable host arrays: they must be copied once into pinned memory before a
        DMA engine can read them).  Clients whose fp32 params the wire codec decoded straight
        into a pinned row of this layout (`rows[n]`) skip the pack and are DMA'd from there."""
        rows = rows if rows is not None else [None] * plan.n_clients
        host_np = [h.numpy() if h is not None else None for h in hosts]
        native = (_NativeRows(pieces, hosts, w_local_lst, rows, plan.memo)
                  if _NativeRows.usable(pieces, hosts) else None)

        def fill(n):
            if rows[n] is not None:
                return
            w = w_local_lst[n]
            cache = {}
            for s, a, b, sh, d in pieces:
                src = cache.get(s.key)
                if src is None:
                    v = w[s.key]
                    if isinstance(v, torch.Tensor):
                        v = v.detach().cpu().numpy()
                    src = cache[s.key] = np.asarray(v).reshape(-1)
                host_np[sh.index][n, d : d + (b - a)] = src[a:b]

        def fill_rows(lo, hi):
            if native is None or not native(lo, hi):
                for r in range(lo, hi):
                    fill(r)

        def ship(lo, hi):
            for sh, h, dv in zip(shards, hosts, devs):
                with torch.cuda.device(sh.device):
                    r = lo
                    while r < hi:
                        if rows[r] is not None:
                            dv[r].copy_(rows[r][sh.c0 : sh.c1], non_blocking=True)
                            r += 1
                            continue
                        e = r
                        while e < hi and rows[e] is None:
                            e += 1
                        dv[r:e].copy_(h[r:e], non_blocking=True)
                        r = e

        n = plan.n_clients
        workers = max(1, min(self.workers, n))
        nbytes = sum(int(d.numel()) * d.element_size() for d in devs)
        if workers == 1 or nbytes < SMALL_BYTES or all(r is not None for r in rows):
            fill_rows(0, n)
            ship(0, n)
            return "serial"
        if self.native_async and native is not None and _plain_dicts(w_local_lst):
            aps, bounds = self._async_rows(plan, pieces, hosts, rows)
            lst = w_local_lst if type(w_local_lst) is list else list(w_local_lst)
            ahead = len(aps) if self.async_lookahead <= 0 else self.async_lookahead
            started = collections.deque()  # (chunk, handle or None: that chunk packs in Python)
            path = "async"
            try:
                for j in range(min(ahead, len(aps))):
                    started.append((j, aps[j].start(lst)))
                for j, (lo, hi) in enumerate(bounds):
                    _, h = started[0]
                    if h is None:  # a value off the plan in this chunk: the _NativeRows / Python pack
                        fill_rows(lo, hi)
                        path = "mixed"
                    else:
                        aps[j].wait(h, 0)
                        aps[j].end(h)
                    started.popleft()  # only once its copies are done (the finally ends the rest)
                    ship(lo, hi)
                    if j + ahead < len(aps):
                        started.append((j + ahead, aps[j + ahead].start(lst)))
            finally:
                for j, h in started:  # only after an error: no copy may outlive the call
                    if h is not None:
                        aps[j].end(h)
            return path
        chunk = max(workers, -(-n // 8))  # ~8 chunks, at least one row per worker
        ex = self._executor()
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            list(ex.map(lambda r: fill_rows(r, r + 1), range(lo, hi)))
            ship(lo, hi)
        return "pool"

    def _async_rows(self, plan: BucketPlan, pieces, hosts, rows):
        """([AsyncPack per chunk], [(lo, hi)]): chunks of rows that grow 1, 2, 4, ... up to
        ~n/12 (the first DMA starts after one row is packed, ~0.5 ms for ResNet-18, where ~8
        equal chunks of a pool pack held it back by a whole chunk); each chunk's packed rows'
        pieces in row order.  Cached on the plan per staging address and wire-row pattern."""
        n = plan.n_clients
        skip = tuple(r is not None for r in rows)
        hp = tuple((h.data_ptr(), h.stride(0) * h.element_size()) if h is not None else (0, 0) for h in hosts)
        key = ("async_rows", id(pieces), hp, skip, self.async_threads)
        hit = plan.memo.get(key)
        if hit is not None:
            return hit
        cap = max(1, -(-n // 12))
        bounds, lo, size = [], 0, 1
        while lo < n:
            hi = min(n, lo + size)
            bounds.append((lo, hi))
            lo, size = hi, min(cap, size * 2)
        # per piece: value bytes, format, row-0 destination, row stride, first byte, bytes
        item = np.array([s.src_dtype.itemsize for s, *_ in pieces], dtype=np.int64)
        total = np.array([s.numel for s, *_ in pieces], dtype=np.int64) * item
        fmt = np.array([_FMT[s.src_dtype] for s, *_ in pieces], dtype=np.int64)
        dst0 = np.array([hp[sh.index][0] for _s, _a, _b, sh, _d in pieces], dtype=np.int64) + \
            np.array([d for *_x, d in pieces], dtype=np.int64) * item
        rstride = np.array([hp[sh.index][1] for _s, _a, _b, sh, _d in pieces], dtype=np.int64)
        lo_b = np.array([a for _s, a, *_x in pieces], dtype=np.int64) * item
        nb = np.array([b - a for _s, a, b, *_x in pieces], dtype=np.int64) * item
        pkeys = tuple(s.key for s, *_ in pieces)
        p = len(pieces)
        aps = []
        for lo, hi in bounds:
            r = np.array([i for i in range(lo, hi) if not skip[i]], dtype=np.int64)[:, None]
            m = len(r)
            table = np.stack([np.broadcast_to(r, (m, p)), np.broadcast_to(total, (m, p)), np.broadcast_to(fmt, (m, p)),
                              dst0 + r * rstride, np.zeros((m, p), dtype=np.int64), np.broadcast_to(lo_b, (m, p)),
                              np.broadcast_to(nb, (m, p))], axis=-1).reshape(-1, 7)
            aps.append(AsyncPack(pkeys * m, table, 1, threads=self.async_threads))
        out = plan.memo[key] = (aps, bounds)
        return out

    def unpack(self, plan: BucketPlan, results: dict, as_torch: bool, out_dtype_override=None) -> dict:
        """results: kind -> [(shard, device tensor [shard.width])].  Returns {key: fresh value} in
        plan order with the reference's types: ndarray (numpy scalar for 0-d keys) or torch CPU
        tensor, views of ONE freshly allocated buffer per kind — nothing returned is shared with
        staging or with later calls."""
        if self.zero_copy_out and len({sh.device for parts in results.values() for sh, _ in parts}) == 1:
            fresh = self._unpack_zero_copy(plan, results)
        else:
            fresh = self._unpack_staged(plan, results)
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

    def _unpack_zero_copy(self, plan: BucketPlan, results: dict) -> dict:
        """One device: fa_copy kernels store each result straight into a fresh pinned buffer per
        kind over PCIe (~53 GB/s; the copy engine's D2H ran at ~30 GB/s)
        and the values handed out are views of it — no staging, no host copy.  The buffer comes
        from torch's pinned caching allocator and goes back to it when the views die (it stays
        page-locked in torch's cache: `zero_copy_out`)."""
        L = na.lib()
        fresh, dev = {}, None
        for kind, parts in results.items():
            buf = torch.empty(plan.groups[kind].stride, dtype=parts[0][1].dtype, pin_memory=True)
            for sh, t in parts:
                dev = sh.device
                src = t[: sh.width]
                dst = buf[sh.c0 : sh.c0 + sh.width]
                with torch.cuda.device(sh.device):
                    rc = -2
                    if src.is_contiguous() and src.is_cuda:
                        rc = L.fa_copy(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(),
                                       torch.cuda.current_stream(sh.device).cuda_stream)
                    if rc == na.FA_ERR_ALIGN:
                        dst.copy_(src, non_blocking=True)
                    else:
                        na.check(rc, "fa_copy")
            fresh[kind] = buf.numpy()
        if dev is not None:
            torch.cuda.current_stream(dev).synchronize()
        return fresh

    def _unpack_staged(self, plan: BucketPlan, results: dict) -> dict:
        """Each shard's D2H goes to reusable pinned staging on its device's stream (all links in
        parallel); the slices are then copied, by a thread pool, into ONE freshly allocated buffer
        per kind."""
        staged = []
        for kind, parts in results.items():
            for sh, t in parts:
                h = self._buf(self._pinned, ("out", kind, sh.index, t.dtype), (sh.width,), t.dtype, pin_memory=True)
                with torch.cuda.device(sh.device):
                    h.copy_(t[: sh.width], non_blocking=True)
                staged.append((kind, sh, h))
        for d in {sh.device for _, sh, _ in staged}:
            torch.cuda.current_stream(d).synchronize()
        fresh = {kind: np.empty(plan.groups[kind].stride, dtype=_NP[parts[0][1].dtype])
                 for kind, parts in results.items()}
        step = 1 << 22  # 4M elements per copy task
        tasks = []
        for kind, sh, h in staged:
            src = h.numpy()
            for lo in range(0, sh.width, step):
                hi = min(sh.width, lo + step)
                tasks.append((fresh[kind], sh.c0 + lo, src, lo, hi))

        def copy(t):
            dst, d0, src, lo, hi = t
            np.copyto(dst[d0 : d0 + (hi - lo)], src[lo:hi])

        nbytes = sum(int(h.numel()) * h.element_size() for _, _, h in staged)
        if len(tasks) > 1 and self.workers > 1 and nbytes >= SMALL_BYTES:
            list(self._executor().map(copy, tasks))
        else:
            for t in tasks:
                copy(t)
        return fresh


class RowTable:
    """Device-resident uploads read where they lie (flearn's run2 path hands the server torch
    tensors, flearn/server/Communicator.py:287-292): a device table of per-(key, client) tensor
    pointers, [segments][clients], plus the bucket's piece table (fa_rows_plan, cached on the
    plan).  fa_reduce_f32_rows reads every upload once in one launch, with no pack copy; the
    8-byte kinds (BN counters) and unaligned fp32 tensors take one fa_gather_rows launch into a
    device stack instead of N*K copy kernels.  `shape` = (clients, stride) like a stack.

    The tensors are referenced until the launches that read them have completed (an event
    recorded after them is checked at the next use of the packer), so the caching allocator
    cannot hand their memory to another stream meanwhile."""

    def __init__(self, packer: Packer, plan: BucketPlan, g: Group, segs, ptrs: np.ndarray, keep, src, device):
        self.packer, self.plan, self.group, self.segs = packer, plan, g, segs
        self.src = tuple(src) if src is not None else (na.SRC_F64,) * len(segs)  # per segment
        self.converts = any(k != na.SRC_F64 for k in self.src)  # some segment is not the store dtype
        self.device = torch.device(device)
        self.shape = (plan.n_clients, g.stride)
        self.aligned = bool(ptrs.size == 0 or not (ptrs % 16).any())
        self.n_pieces = 0
        self.pieces = None
        itemsize = np.dtype(g.store_dtype).itemsize
        self.elem_size = itemsize
        # the pointer table: reused pinned staging (waited on before it is rewritten), then H2D
        key = ("rows", g.kind, str(self.device))
        ev = packer._pin_events.pop(key, None)
        if ev is not None:
            ev.synchronize()
        host = packer._buf(packer._pinned, key, (max(ptrs.size, 1),), torch.int64, pin_memory=True)
        host[: ptrs.size].numpy()[:] = ptrs.reshape(-1)
        self.ptrs = packer.device_bucket(key, (max(ptrs.size, 1),), torch.int64, self.device)
        self.ptrs.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        packer._pin_events[key] = ev
        self.keep = keep
        self.work = packer.device_bucket(("rows_work", str(self.device)), (1,), torch.int32, self.device)

    def piece_table(self, op: int):
        """(device fa_piece array, slot count, grid) for this bucket layout and epilogue, cached
        on the plan."""
        mk = ("row_pieces", self.group.kind, int(op), str(self.device))
        hit = self.plan.memo.get(mk)
        if hit is None:
            L = na.load()
            cols = np.array([s.offset for s in self.segs], dtype=np.int64)
            lens = np.array([s.numel for s in self.segs], dtype=np.int64)
            cnt, grid = ctypes.c_int64(), ctypes.c_int32()
            with torch.cuda.device(self.device):  # the default grid follows this device's CUs
                na.check(L.fa_rows_plan(len(self.segs), cols.ctypes.data, lens.ctypes.data, int(op), 0, None, 0,
                                        ctypes.byref(cnt), ctypes.byref(grid)), "fa_rows_plan")
                arr = np.zeros((max(cnt.value, 1), ctypes.sizeof(na.Piece)), dtype=np.uint8)
                na.check(L.fa_rows_plan(len(self.segs), cols.ctypes.data, lens.ctypes.data, int(op), grid.value,
                                        arr.ctypes.data, cnt.value, ctypes.byref(cnt), ctypes.byref(grid)),
                         "fa_rows_plan")
            dev = torch.from_numpy(arr.reshape(-1)).to(self.device)  # once per layout
            hit = self.plan.memo[mk] = (dev, cnt.value, grid.value)
        return hit

    def gather_into(self, stack: torch.Tensor) -> None:
        """One launch: every (key, client) tensor into its segment of the device stack [N, stride]
        (converted to float64 per segment when the float64 group holds int64 / float32 values)."""
        L = na.load()
        mk = ("row_segs", self.group.kind, str(self.device), self.src)
        segs = self.plan.memo.get(mk)
        if segs is None:
            cols = [s.offset for s in self.segs] + [s.numel for s in self.segs]
            t = np.array(cols + (list(self.src) if self.converts else []), dtype=np.int64)
            segs = self.plan.memo[mk] = torch.from_numpy(t).to(self.device)
        if self.converts:
            na.check(L.fa_gather_rows_f64(stack.data_ptr(), stack.stride(0), self.shape[0], self.ptrs.data_ptr(),
                                          segs.data_ptr(), len(self.segs), na.stream_handle(self.device)),
                     "fa_gather_rows_f64")
        else:
            na.check(L.fa_gather_rows(stack.data_ptr(), stack.stride(0), self.shape[0], self.elem_size,
                                      self.ptrs.data_ptr(), segs.data_ptr(), len(self.segs),
                                      na.stream_handle(self.device)), "fa_gather_rows")
        self.release()

    def release(self) -> None:
        """Call after the launches that read the uploads are queued: the packer keeps them alive
        until those launches have completed."""
        self.packer.hold(self.keep, self.device)
        self.keep = []
