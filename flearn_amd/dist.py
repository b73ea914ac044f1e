"""Multi-GPU aggregation: element-range sharding of the bucket + RCCL all-gather over xGMI.

One process per GPU (torch.distributed, backend "nccl" = RCCL).  The aggregation is independent
per element, so the flattened fp32 bucket is split by COLUMNS: every rank holds its columns of
all N clients and reduces them with the same fused kernel; the only exchange is reassembling the
global model.  Layer-granular sharding (what the north star's wording suggests) would cap
ResNet-18 at ~5x on 8 GPUs because fc/layer4 tensors are up to 20% of the model; columns
balance exactly.

Column layout (block-cyclic, `stripes` stripes of per-rank widths S_c, multiples of 64):
    O_c = S_0 + ... + S_{c-1};  P_pad = W * (S_0 + ... + S_{last})
    stripe c covers global columns [W*O_c, W*(O_c + S_c)); rank r owns [W*O_c + r*S_c, +S_c)
    rank r's local stack is [N, sum S_c]: local column O_c + j <-> global W*O_c + r*S_c + j
so the all-gather of stripe c writes one contiguous range of the global bucket, and stripe c's
gather (on RCCL's stream) overlaps the reduce of stripe c+1 (on the compute stream).
Optionally the plan ends in a REPLICATED tail of `rep` columns, [W*sum(S), W*sum(S) + rep) =
[n_cols - rep, n_cols): every rank holds those columns of all N clients and reduces them itself,
after its stripes, while the last gathers are in flight — redundant compute instead of
communication, worth it where the all-gather, not the reduce, sets the step (few GPUs, one xGMI
link per peer: at G = 2 every GPU receives half the model over ONE link).  The rank's local
columns are then [stripes..., tail]; the tail's results are written straight into the global
bucket (bit-identical on every rank: same data, same kernel, same order).
Optimizer state (prev, v_t) is sharded the same way and never communicated.

The stripe widths come from a two-stage pipeline model (`StripeModel`, `plan_stripes`,
`plan_shards`): stripe c's reduce costs a_r + b_r*S_c on the compute stream, its gather
a_g + b_g*S_c on RCCL's, a gather starts when its stripe is reduced and the previous gather is
done, the replicated tail's reduce follows the last stripe's; the plan with the smallest simulated
makespan over tail sizes, stripe counts and geometric width ratios wins.  bench.py fits the four
coefficients on the running job (one full-width and one narrow launch of each) before it plans,
so the schedule follows the node's measured HBM and xGMI rates.

The same code runs on the gloo backend (CPU tests, and two processes sharing one GPU on a
1-GPU box, where RCCL refuses two ranks on one device): device tensors are then staged through
host memory around the collective (`all_gather_into`).
"""
from __future__ import annotations

import ctypes
import warnings
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .streams import side_stream

ALIGN = 64
MAX_PUSH_RANKS = 8  # fa_push's destination count: one MI355X node

#: how a push is ordered after its stripe's reduce: "host" (the host waits for the reduce, then
#: issues the push with no device-side cross-stream wait), "producer" (the push's streams wait on
#: an event of the reduce's stream) or "chain" (round 5: an event of the pusher's stream after its
#: wait on the reduce's).  "auto", the product's: the copy-engine push in host order — with
#: device-side waits its legs (and its own-copy kernel) started before the reduce had finished,
#: 1-30% of rank-steps among eight processes on one GPU — and the kernel push in producer order:
#: never wrong in the same probes (0 of 6,656 rank-steps, tests/push_order_probe.py), and host
#: order costs it a host round trip per stripe (100 x 3.2 M columns, a rank's share of NS at G = 8,
#: 4 stripes: 0.32-0.40 ms per step against 0.275)
_PUSH_ORDER = "auto"


def push_order(mode: str) -> str:
    """The order a PushGather of `mode` uses now (_PUSH_ORDER resolved)."""
    if _PUSH_ORDER != "auto":
        return _PUSH_ORDER
    return "producer" if mode == "kernel" else "host"


def peer_stream(device) -> torch.cuda.Stream:
    """A copy-engine leg's stream (normal priority; tests/push_order_probe.py overrides it)."""
    return torch.cuda.Stream(device)


def _host_staged(t: torch.Tensor, group) -> bool:
    """gloo cannot be trusted with device tensors for every collective: stage them on the host."""
    return t.device.type != "cpu" and dist.get_backend(group) == "gloo"


def all_gather_into(dst: torch.Tensor, src: torch.Tensor, group=None, async_op: bool = False):
    """dist.all_gather_into_tensor(dst, src), host-staged on gloo for device tensors (then
    synchronous: returns None).  On RCCL it is the collective itself (async when asked)."""
    if not _host_staged(src, group):
        return dist.all_gather_into_tensor(dst, src, group=group, async_op=async_op)
    hsrc = src.detach().to("cpu")
    hdst = torch.empty(dst.shape, dtype=dst.dtype)
    dist.all_gather_into_tensor(hdst, hsrc, group=group)
    dst.copy_(hdst)
    return None


#: exported buckets released by their users, handed out again by DeviceBuffer.get (see
#: DeviceBuffer); per device they are kept within PARK_CAP x the largest bucket the device has
#: exported — beyond that the smallest are freed
_PARKED: list = []
PARK_CAP = 2
_LARGEST: dict = {}  # device -> bytes of the largest bucket it has exported
_TRIMMED = [0, 0]  # exported buckets freed to keep within the cap: (count, bytes)


def size_class(nbytes: int) -> int:
    """Bucket sizes come in four classes per octave (2^k, 1.25, 1.5, 1.75 x 2^k; at least 4 KiB):
    requests a few percent apart share one class, so released buckets fit the next job's."""
    nbytes = max(int(nbytes), 4096)
    step = 1 << max(nbytes.bit_length() - 3, 0)
    return -(-nbytes // step) * step


class DeviceBuffer:
    """A device allocation of its own (C ABI fa_dev_alloc), outside torch's caching allocator:
    what the push gather exports.  A caching-allocator tensor lives inside a segment that other
    tensors share and that torch recycles (empty_cache frees it), and hipIpcGetMemHandle exports
    the whole segment; this is one bucket, one export.

    Once exported (`exported`), `free()` parks a bucket and `DeviceBuffer.get` hands it out again
    (re-exporting the same memory).  With several processes on one GPU, an exporter that freed
    imported memory and exported again made 13-34% of later imports map the wrong allocation;
    with nothing exported freed, and a barrier after every unmap, 0 of 1,920 imports were wrong
    (profiles/r05/ipc/).  Parking is bounded: per device the parked bytes
    stay within PARK_CAP x the largest bucket the device has exported, the smallest parked
    buckets beyond that are freed (`trimmed()` counts them) — a later import that maps the wrong
    allocation is still refused by the token check of every mapping (_map_peers), so the cost of
    a trim is at worst a refused push set-up (RCCL's all-gather then), never a wrong bucket.
    `tensor()` views it (torch keeps this object alive while any view does); an unexported buffer
    is freed by `free()` or when the last view dies."""

    def __init__(self, nbytes: int, device):
        from . import _native as na

        self.L, self.na = na.lib(), na
        self.nbytes, self.device = int(nbytes), torch.device(device)
        self._exported = False
        self._typestr = "<f4"
        self.ptr = self._alloc()

    def _alloc(self) -> int:
        p = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            self.na.check(self.L.fa_dev_alloc(self.nbytes, ctypes.byref(p)), "fa_dev_alloc")
        return p.value

    def _release(self, ptr: int):
        with torch.cuda.device(self.device):
            self.na.check(self.L.fa_dev_free(ptr), "fa_dev_free")

    @property
    def exported(self) -> bool:
        """Set when peers may map it: from then on free() parks it."""
        return self._exported

    @exported.setter
    def exported(self, value: bool):
        if value and not self._exported:
            key = str(self.device)
            _LARGEST[key] = max(_LARGEST.get(key, 0), self.nbytes)
        self._exported = bool(value)

    @classmethod
    def get(cls, nbytes: int, device) -> "DeviceBuffer":
        """A parked (previously exported, released) buffer of at least nbytes on `device` — the
        smallest that fits — or a new one of nbytes' size class."""
        dev = torch.device(device)
        fits = [b for b in _PARKED if b.device == dev and b.nbytes >= nbytes]
        if fits:
            b = min(fits, key=lambda x: x.nbytes)
            _PARKED.remove(b)
            return b
        return cls(size_class(nbytes), dev)

    @staticmethod
    def parked_bytes(device=None) -> int:
        return sum(b.nbytes for b in _PARKED if device is None or b.device == torch.device(device))

    @staticmethod
    def park_cap(device) -> int:
        return PARK_CAP * _LARGEST.get(str(torch.device(device)), 0)

    @staticmethod
    def trimmed() -> dict:
        return {"buckets": _TRIMMED[0], "bytes": _TRIMMED[1]}

    @staticmethod
    def _trim(device):
        """Free the smallest parked buckets of `device` until the parked bytes fit the cap."""
        cap = DeviceBuffer.park_cap(device)
        parked = sorted((b for b in _PARKED if b.device == device), key=lambda b: b.nbytes)
        total = sum(b.nbytes for b in parked)
        for b in parked:
            if total <= cap:
                break
            _PARKED.remove(b)
            total -= b.nbytes
            ptr, b.ptr = b.ptr, None
            b._release(ptr)
            _TRIMMED[0] += 1
            _TRIMMED[1] += b.nbytes

    @property
    def __cuda_array_interface__(self):
        if not self.ptr:
            raise RuntimeError("DeviceBuffer already freed")
        item = int(self._typestr[-1])
        return {"shape": (self.nbytes // item,), "typestr": self._typestr, "data": (self.ptr, False),
                "version": 2, "strides": None}

    def tensor(self, dtype=torch.float32) -> torch.Tensor:
        """A 1-D view of the whole buffer (float32 or int32)."""
        self._typestr = {torch.float32: "<f4", torch.int32: "<i4"}[dtype]
        t = torch.as_tensor(self, device=self.device)
        if t.data_ptr() != self.ptr or t.device != self.device:
            raise RuntimeError("DeviceBuffer view does not alias its allocation")
        return t

    def free(self):
        """Release: an exported buffer is parked for reuse (freed only beyond the parking cap), any
        other freed."""
        if not self.ptr:
            return
        if self.exported:
            if self not in _PARKED:
                _PARKED.append(self)
                DeviceBuffer._trim(self.device)
            return
        ptr, self.ptr = self.ptr, None
        self._release(ptr)

    def __del__(self):
        try:
            if not self.exported:
                self.free()
        except Exception:  # noqa: BLE001 - interpreter shutdown: nothing left to report to
            pass


def _all_ok(pg, ok: int) -> bool:
    t = torch.tensor([ok], dtype=torch.int32, device=pg.device if pg.nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pg.group)
    return bool(t.item())


class HipIpc:
    """The IPC transport of the push gather: HIP IPC handles of device allocations (C ABI
    fa_ipc_*), read back through a copy engine.  `_IPC` is the one in use; the CPU tests put a
    shared-memory stand-in there to run the pool's collective protocol, token checks included,
    over gloo (tests/test_recv_pool.py)."""

    @staticmethod
    def accepts(device) -> bool:
        return torch.device(device).type == "cuda"

    @staticmethod
    def sync(device):
        torch.cuda.synchronize(device)

    @staticmethod
    def handle(ptr: int):
        """(handle bytes, byte offset of ptr in its allocation), or None."""
        from . import _native as na

        h, off = ctypes.create_string_buffer(64), ctypes.c_int64(0)
        if na.lib().fa_ipc_handle(ptr, h, ctypes.byref(off)) != 0:
            return None
        return bytes(h.raw), int(off.value)

    @staticmethod
    def open(hb: bytes):
        """The base address a peer's handle maps at here, or None."""
        from . import _native as na

        base = ctypes.c_void_p()
        if na.lib().fa_ipc_open(hb, ctypes.byref(base)) != 0 or not base.value:
            return None
        return base.value

    @staticmethod
    def read16(probe: torch.Tensor, addr: int) -> bool:
        """The 16 bytes at a mapped address into `probe` (4 int32, same device)."""
        from . import _native as na

        s = torch.cuda.current_stream(probe.device)
        if na.lib().fa_copy_dma(probe.data_ptr(), addr, 16, s.cuda_stream) != 0:
            return False
        s.synchronize()
        return True

    @staticmethod
    def close(base: int):
        from . import _native as na

        na.lib().fa_ipc_close(base)

    @staticmethod
    def last_error() -> bytes:
        from . import _native as na

        return na.lib().fa_last_error()


_IPC = HipIpc


def _map_peers(pg, full: torch.Tensor):
    """Collective: register `full` (IPC handle of its allocation + offset) and map every peer's;
    (opened bases, per-rank device address of each rank's buffer, stale peers).  A token written
    into the buffer's first 16 bytes (the caller's bytes there are saved and put back) is read
    back through every mapping: an import that maps some other allocation than the one exported
    is refused instead of pushed into (the stale imports of round 4).  Every
    rank raises RuntimeError (nothing left mapped) if any rank cannot map or validate a peer."""
    ipc = _IPC
    bases, dsts, stale = [], [], []
    ok = 1
    mine = None
    saved = None
    if pg.world > MAX_PUSH_RANKS or not ipc.accepts(full.device) or not full.is_contiguous() or full.numel() < 4:
        ok = 0
    else:
        head = full.view(torch.int32)[:4]
        saved = head.clone()
        token = torch.randint(-2**31, 2**31 - 1, (4,), dtype=torch.int32)
        head.copy_(token)
        ipc.sync(full.device)
        got = ipc.handle(full.data_ptr())
        if got is not None:
            mine = (got[0], got[1], token.tolist())
        else:
            ok = 0
    infos = [None] * pg.world
    dist.all_gather_object(infos, mine, group=pg.group)
    if ok and all(i is not None for i in infos):
        probe = torch.empty(4, dtype=torch.int32, device=full.device)
        for r, (hb, off, tok) in enumerate(infos):
            if r == pg.rank:
                dsts.append(full.data_ptr())
                continue
            base = ipc.open(hb)
            if base is None:
                ok = 0
                break
            bases.append(base)
            dsts.append(base + off)
            if not ipc.read16(probe, base + off):
                ok = 0
                break
            if probe.tolist() != tok:
                stale.append(r)
                ok = 0
    else:
        ok = 0
    agreed = _all_ok(pg, ok)  # every rank has read every token it reads: the heads may go back
    if saved is not None:
        full.view(torch.int32)[:4].copy_(saved)
    if not agreed:
        for b in bases:
            ipc.close(b)
        dist.barrier(group=pg.group)  # nobody exports again while a peer is still closing
        err = ipc.last_error()
        why = (f" (here: the mappings of ranks {stale} did not hold their tokens)" if stale else
               f" (here: {err.decode(errors='replace')})" if err and not ok else "")
        raise RuntimeError("PushGather: a rank could not map its peers' receive buffers" + why)
    return bases, dsts, stale


def _unmap_all(bases, group):
    """Collective: close this rank's imports, then a barrier — after it no peer is still closing
    an import when any rank exports again (exporting while a peer closes made a third of the
    probe's imports map the wrong allocation: DESIGN.md section 6)."""
    for b in bases:
        _IPC.close(b)
    dist.barrier(group=group)


def _resolve_group(group):
    return group if group is not None else dist.distributed_c10d._get_default_group()


def _group_alive(g) -> bool:
    try:
        return g in dist.distributed_c10d._world.pg_map
    except Exception:  # noqa: BLE001 - a torch without the registry: assume alive
        return True


class _RecvPool:
    """Receive buckets of the one-shot push, per (device, process group): each an allocation of
    its own (DeviceBuffer), exported once and mapped once by every peer, handed out to job after
    job (`take` / `give`: a few ms of collective set-up and token checks saved per job — the
    bench's plan trials build a dozen jobs).  Released collectively: `shutdown_push(group)`
    (call it before destroying the group) has every peer close its imports, then a barrier, and
    the buckets are parked (DeviceBuffer: exported memory is parked for re-export, freed only
    beyond the parking cap — freeing imported memory is what made later imports map the wrong
    allocation) for the next pool to re-export.  A `take` that finds no free bucket large enough first releases
    the free ones (same protocol) and takes a parked one that fits or a new one of the request's
    size class (DeviceBuffer.get), so the buckets held stay near the largest set in use at once
    and the parked ones within DeviceBuffer's cap.  Every rank takes and gives in the
    same order, so the slots agree across ranks (checked at each take).

    Keyed by the group OBJECT (held, so its id cannot be reused by a later group): a destroyed and
    re-created default group gets a new pool.  A pool whose group was destroyed without
    shutdown_push is dropped locally the next time any pool is looked up (imports closed with no
    barrier possible any more — the unordered unmap the token check at the next set-up guards
    against — buckets parked)."""

    _pools: dict = {}

    def __init__(self, device, gobj):
        self.device, self.gobj = device, gobj
        self.slots = []  # [DeviceBuffer, fp32 view, per-rank device addresses, opened peer bases, busy]

    @classmethod
    def get(cls, device, group):
        g = _resolve_group(group)
        for key in [k for k, p in cls._pools.items() if not _group_alive(p.gobj)]:
            cls._pools.pop(key)._drop_local()
        key = (str(device), id(g))
        p = cls._pools.get(key)
        if p is None:
            p = cls._pools[key] = _RecvPool(device, g)
        return p

    @classmethod
    def bytes_held(cls) -> int:
        return sum(s[0].nbytes for p in cls._pools.values() for s in p.slots)

    def _retire(self, pg, idx):
        """Collective: every rank closes its imports of the slots `idx`, a barrier, then the
        buckets are parked (same indices on every rank)."""
        if not idx:
            return
        _unmap_all([b for i in idx for b in self.slots[i][3]], pg.group)
        for i in sorted(idx, reverse=True):
            buf = self.slots.pop(i)[0]
            buf.free()  # exported: parked for reuse (within the parking cap)

    def take(self, pg, cols: int):
        i = next((j for j, s in enumerate(self.slots) if not s[4] and s[1].numel() >= cols), None)
        picks = [None] * pg.world
        dist.all_gather_object(picks, (i, len(self.slots)), group=pg.group)
        if len(set(picks)) != 1:
            raise RuntimeError(f"PushGather: the ranks' receive pools disagree ({picks})")
        if i is None:  # retire the free buckets that are too small, then a new one (collective)
            self._retire(pg, [j for j, s in enumerate(self.slots) if not s[4]])
            if not _IPC.accepts(self.device):  # refused on every rank together
                pg.device = torch.device(self.device)
                _map_peers(pg, torch.empty(4))
            want = max(cols, 4)
            buf = DeviceBuffer.get(-(-want // ALIGN) * ALIGN * 4, self.device)
            view = buf.tensor(torch.float32)
            pg.full, pg.device = view, self.device
            buf.exported = True  # from here on parked when released
            try:
                bases, dsts, _stale = _map_peers(pg, view)
            except RuntimeError:
                del view
                buf.free()  # parked; every peer closed its imports (and barriered) before the raise
                raise
            self.slots.append([buf, view, dsts, bases, False])
            i = len(self.slots) - 1
        self.slots[i][4] = True
        return i, self.slots[i][1], self.slots[i][2]

    def give(self, i: int):
        self.slots[i][4] = False

    def shutdown(self, pg):
        """Collective: unmap every bucket on every rank, barrier, park."""
        busy = [j for j, s in enumerate(self.slots) if s[4]]
        if busy:
            warnings.warn(f"shutdown_push: {len(busy)} receive bucket(s) still in use by a reducer that was "
                          "not released; their results are overwritten by the next push job", stacklevel=3)
        self._retire(pg, list(range(len(self.slots))))

    def _drop_local(self):
        for s in self.slots:
            for b in s[3]:
                _IPC.close(b)
            s[0].free()
        self.slots = []


def shutdown_push(group=None, device=None):
    """Collective over `group`: release the push gather's receive buckets of this process for
    that group — every peer's mapping closed, then a barrier, then each rank parks its own
    (DeviceBuffer.get hands them to the next pool; beyond the parking cap the smallest are
    freed).  Call it
    before dist.destroy_process_group; the next push job maps its buckets afresh."""
    g = _resolve_group(group)
    for key in [k for k, p in _RecvPool._pools.items() if p.gobj is g
                and (device is None or k[0] == str(torch.device(device)))]:
        pool = _RecvPool._pools.pop(key)
        pool.shutdown(type("_Ctx", (), {"group": group})())


class PushGather:
    """One-shot all-gather over xGMI by direct peer stores (C ABI fa_ipc_* / fa_push).

    Every rank registers its receive buffer `full` once (IPC handles exchanged with
    all_gather_object) and maps its peers' buffers; a reduced stripe is then pushed by ONE kernel
    into every rank's `full` at the same offset — each peer's copy crosses that peer's own xGMI
    link, nothing is forwarded, received data is never re-read, and the receiving GPU spends no
    kernel on it (RCCL's all-gather forwards chunks along rings and copies them out of its
    buffers on every GPU: HBM traffic that competes with the reduce).
    Ordering, all on this object's stream: `begin()` — a barrier after this rank's earlier work on
    the compute stream (no peer may overwrite a `full` its owner is still reading); `push()` after
    the stripe's reduce; `end()` — a barrier after the pushes, which the compute stream then waits
    for: once every rank has passed it, every peer's stores into this rank's `full` are complete
    (each push kernel ends with a system-scope release).  On RCCL the barriers are 1-element
    all_reduces ordered on the stream; on gloo (several processes sharing one GPU in the tests)
    host synchronisations plus dist.barrier.
    Construction is collective and all-or-nothing: if any rank cannot map a peer, every rank
    raises RuntimeError (nothing stays mapped) and the caller keeps RCCL's all-gather."""

    def __init__(self, full: torch.Tensor | None, group=None, mode: str = "kernel", cols: int = 0, device=None):
        """full: the receive buffer to register (exported and mapped for this object, unmapped by
        close()) — a DeviceBuffer (its fp32 view becomes `self.full`; once exported it is never
        freed: `free()` parks it), or a tensor, whose whole caching-allocator segment is exported
        (the caller must then keep that memory allocated for the process's lifetime: a freed
        exported segment makes later imports unreliable); or None with
        `cols` / `device`: a bucket of at least `cols` fp32 columns from the process's receive
        pool (_RecvPool: mapped once by every peer, reused until shutdown_push)."""
        from . import _native as na

        if mode not in ("kernel", "dma"):
            raise ValueError(f"PushGather mode {mode!r}")
        self.mode = mode
        self.na, self.L = na, na.lib()
        self.group = group
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"
        self.pool_slot = None
        if full is None:
            self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            self.pool = _RecvPool.get(self.device, group)
            self.pool_slot, buf, self.dst = self.pool.take(self, cols)
            self.full, self.bases, self.stale = buf[:cols], [], []
        else:
            if isinstance(full, DeviceBuffer):  # exported from here on: parked when released
                full.exported = True
                self.owner, full = full, full.tensor(torch.float32)
            self.full, self.device = full, full.device
            self.bases, self.dst, self.stale = _map_peers(self, full)
        # a high-priority stream, whose hardware queue is apart from the compute stream's — on a
        # shared queue the push kernels run in queue order with the next stripes' reduces instead
        # of beside them (streams.py)
        self.stream = side_stream(self.device)
        self.flag = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.grid = 0  # fa_push blocks (0: the library's default)
        # mode "dma": one stream per peer, each leg a copy-engine copy (fa_copy_dma) — copies on
        # one stream would run one after the other, one link at a time
        self.peer_streams = [peer_stream(self.device) for _ in range(self.world - 1)] if mode == "dma" else []
        self._pending = None  # host order: the last stripe whose push is not issued yet
        self._peer_handles = (ctypes.c_void_p * max(1, len(self.peer_streams)))(
            *[s.cuda_stream for s in self.peer_streams]) if self.peer_streams else None

    def _barrier(self):
        if self.nccl:
            with torch.cuda.stream(self.stream):
                dist.all_reduce(self.flag, group=self.group)
        else:
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)

    def begin(self):
        # a step abandoned between its pushes (an exception before end()) leaves its last stripe
        # pending: never issue it into this step's buckets
        self._pending = None
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self._barrier()

    def push(self, src: torch.Tensor, elem_offset: int):
        """Stores src (this rank's reduced slice) into every rank's `full` at elem_offset."""
        n = src.numel() * src.element_size()
        if n == 0:
            return
        off = elem_offset * self.full.element_size()
        if elem_offset < 0 or off + n > self.full.numel() * self.full.element_size():
            raise ValueError("push outside the receive buffer")
        cur = torch.cuda.current_stream(self.device)
        order = push_order(self.mode)
        if order == "host":
            # (the copy-engine push) the push of stripe c is issued once the host has seen stripe
            # c's reduce complete — at push(c+1), after reduce c+1 is queued — and needs no
            # device-side wait.  With device-side waits (an event of the reduce's stream,
            # "producer"; round 5's event on the pusher's stream, "chain"), eight processes sharing
            # a GPU with the copy-engine legs' streams on hardware queues of their own copied
            # stripes before their reduce had finished — the own-copy KERNEL on the pusher's stream
            # included (tests/push_order_probe.py --forensic).  The kernel push
            # (no copy-engine streams) takes the device-side order below: see _PUSH_ORDER
            ev = torch.cuda.Event()
            ev.record(cur)
            prev, self._pending = self._pending, (ev, src, off, n)
            if prev is not None:
                self._issue(*prev)
            return
        self.stream.wait_stream(cur)
        if self.mode == "kernel":
            self._push_kernel(src, off, n)
            return
        after = self.stream if order == "chain" else cur
        peers = (ctypes.c_void_p * (self.world - 1))(*[d + off for r, d in enumerate(self.dst) if r != self.rank])
        self.na.check(self.L.fa_push_dma(src.data_ptr(), n, peers, self.world - 1, self._peer_handles,
                                         after.cuda_stream), "fa_push_dma")
        self.na.check(self.L.fa_copy(self.dst[self.rank] + off, src.data_ptr(), n, self.stream.cuda_stream), "fa_copy")

    def _push_kernel(self, src, off, n):
        dsts = (ctypes.c_void_p * self.world)(*[d + off for d in self.dst])
        self.na.check(self.L.fa_push(src.data_ptr(), n, dsts, self.world, self.grid, self.stream.cuda_stream), "fa_push")

    def _issue(self, ev, src, off, n):
        """Host order: wait on the host for the stripe's reduce, then push it — the push kernel on
        the pusher's stream, or the copy-engine legs on theirs and this rank's own copy."""
        ev.synchronize()
        if self.mode == "kernel":
            self._push_kernel(src, off, n)
            return
        peers = [d + off for r, d in enumerate(self.dst) if r != self.rank]
        for d, s in zip(peers, self.peer_streams):
            self.na.check(self.L.fa_copy_dma(d, src.data_ptr(), n, s.cuda_stream), "fa_copy_dma")
        self.na.check(self.L.fa_copy(self.dst[self.rank] + off, src.data_ptr(), n, self.stream.cuda_stream), "fa_copy")

    def join(self):
        """Every push of the step is issued and the copy-engine legs are complete before the
        closing barrier: in host order the pending stripe is pushed and the host waits for the
        legs' streams; otherwise the pusher's stream waits on them (a pending stripe left by a
        switch of _PUSH_ORDER mid-step is flushed either way)."""
        if push_order(self.mode) == "host" or self._pending is not None:
            if self._pending is not None:
                pending, self._pending = self._pending, None
                self._issue(*pending)
            for s in self.peer_streams:
                s.synchronize()
            return
        if self.peer_streams:
            self.na.check(self.L.fa_stream_join(self.stream.cuda_stream, self._peer_handles, len(self.peer_streams)),
                          "fa_stream_join")

    def end(self):
        self.join()
        self._barrier()
        torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def gather(self, src: torch.Tensor, elem_offset: int):
        """A whole all-gather of one slice: begin, push, end."""
        self.begin()
        self.push(src, elem_offset)
        self.end()

    def close(self):
        """Collective: after every rank's pushes are done (a barrier), a pool bucket goes back to
        the pool, still mapped; an explicitly registered `full` is unmapped by every peer and a
        second barrier follows, so no rank frees or re-exports its buffer while a peer still maps
        it."""
        if self.dst:
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)
            if self.pool_slot is not None:
                self.pool.give(self.pool_slot)
                self.pool_slot, self.dst = None, []
            else:
                _unmap_all(self.bases, self.group)
                self.bases, self.dst = [], []


@dataclass(frozen=True)
class StripeModel:
    """Per-stripe cost model of one rank (seconds; widths in columns per rank).
    reduce(S) = a_r + b_r*S on the compute stream; gather(S) = a_g + b_g*S on the collective's
    stream (a stripe of S columns per rank is an all-gather of world*S columns).
    Contention: a reduce that runs beside a gather streams (1 + c_r) times slower, a gather that
    runs beside a reduce (1 + c_g) times slower — they share the CUs and the HBM.  Measured on one
    MI355X with a copy kernel standing in for the gather (tools/overlap_probe.py);
    0 = the optimistic model (perfect overlap)."""

    a_r: float
    b_r: float
    a_g: float
    b_g: float
    c_r: float = 0.0
    c_g: float = 0.0

    @staticmethod
    def assumed(n_clients: int, world: int, hbm_bytes_s: float = 7.0e12, link_bytes_s: float = 50e9,
                launch_s: float = 10e-6, collective_s: float = 30e-6) -> "StripeModel":
        """A priori coefficients: the reduce streams N*4 B per column at the measured 1-GPU rate
        (~7 TB/s); an all-gather brings (world-1)*4 B per column into each GPU over
        its world-1 xGMI links (one per peer on an MI355X node) at an assumed per-link rate.
        bench.py replaces them with measured ones."""
        ingress = max(world - 1, 1) * link_bytes_s
        return StripeModel(launch_s, n_clients * 4.0 / hbm_bytes_s, collective_s,
                           max(world - 1, 0) * 4.0 / ingress)

    @staticmethod
    def fit(w_big: int, w_small: int, r_big: float, r_small: float, g_big: float, g_small: float,
            c_r: float = 0.0, c_g: float = 0.0) -> "StripeModel":
        """Coefficients from two widths' measured reduce and gather times (non-negative), plus
        the contention terms (measured separately)."""
        def line(tb, ts):
            b = max((tb - ts) / max(w_big - w_small, 1), 0.0)
            return max(ts - b * w_small, 0.0), b

        a_r, b_r = line(r_big, r_small)
        a_g, b_g = line(g_big, g_small)
        return StripeModel(a_r, b_r, a_g, b_g, max(c_r, 0.0), max(c_g, 0.0))

    def with_contention(self, c_r: float, c_g: float) -> "StripeModel":
        return StripeModel(self.a_r, self.b_r, self.a_g, self.b_g, max(c_r, 0.0), max(c_g, 0.0))

    def makespan(self, widths, rep: int = 0) -> tuple:
        """(step time, reduce-stream busy time, exposed gather time) of a stripe plan; `rep`
        replicated columns are reduced after the stripes, with no gather.  Every stripe's reduce
        but the first runs beside the previous stripe's gather, and every gather but one that
        finds the reduce stream idle runs beside a reduce: those streaming terms carry the
        contention factors (1 + c_r) and (1 + c_g)."""
        t_red = t_gat = 0.0
        last = len(widths) - 1
        for c, w in enumerate(widths):
            t_red += self.a_r + self.b_r * w * (1.0 + (self.c_r if c > 0 else 0.0))
            busy_after = c < last or rep > 0  # a reduce (next stripe or the tail) runs beside it
            t_gat = max(t_red, t_gat) + self.a_g + self.b_g * w * (1.0 + (self.c_g if busy_after else 0.0))
        if rep:
            t_red += self.a_r + self.b_r * rep * (1.0 + (self.c_r if widths else 0.0))
        step = max(t_gat, t_red)
        return step, t_red, step - t_red


def plan_stripes(local_cols: int, model: StripeModel, max_stripes: int = 8, rep: int = 0) -> tuple:
    """Stripe widths (multiples of ALIGN summing to >= local_cols) minimising the model's makespan
    (followed by `rep` replicated columns).
    Candidates: k = 1..max_stripes stripes with geometric widths S_c ~ q**c for q on a grid
    (q < 1: big stripes first, the usual choice when the reduce dominates; q > 1: a small first
    stripe so the gathers start early, when the collective dominates)."""
    units = max(1, -(-local_cols // ALIGN))
    best = ((units * ALIGN,), model.makespan((units * ALIGN,), rep)[0])
    for k in range(2, min(max_stripes, units) + 1):
        for q in (0.125, 0.25, 0.35, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0, 1.15, 1.3, 1.5, 2.0, 3.0, 4.0):
            raw = [q**c for c in range(k)]
            tot = sum(raw)
            u = [max(1, int(units * x / tot)) for x in raw]
            u[0 if q <= 1 else -1] += units - sum(u)  # the remainder goes to the big end
            if min(u) < 1:
                continue
            widths = tuple(x * ALIGN for x in u)
            t = model.makespan(widths, rep)[0]
            if t < best[1] - 1e-12:
                best = (widths, t)
    return best[0]


#: replicated-tail sizes plan_shards tries, as fractions of the bucket
REP_FRACTIONS = (0.0, 0.01, 0.02, 0.03, 0.05, 0.075, 0.1, 0.125, 0.15, 0.175, 0.2, 0.25, 0.3, 0.35, 0.4,
                 0.45, 0.5, 0.55, 0.6)


def plan_shards(n_cols: int, world: int, model: StripeModel, max_stripes: int = 8,
                fractions=REP_FRACTIONS) -> tuple:
    """(stripe widths, replicated tail columns) minimising the model's makespan for an n_cols
    bucket on `world` ranks: the padded plan with no tail, against plans whose stripes cover
    exactly world*sum(widths) = n_cols - rep columns and whose last `rep` columns every rank
    reduces itself (ShardPlan.rep).  A tail pays where the gather dominates: each replicated
    column costs every rank one column of reduce and saves (world-1)/world of a column of
    gather ingress."""
    lc = -(-max(n_cols, 1) // max(world, 1))
    w0 = plan_stripes(lc, model, max_stripes)
    best = (w0, 0, model.makespan(w0)[0])
    if world < 2:
        return best[0], 0
    for f in fractions:
        units = int(n_cols * (1.0 - f)) // (world * ALIGN)
        rep = n_cols - world * units * ALIGN
        if units < 1 or rep <= 0:
            continue
        w = plan_stripes(units * ALIGN, model, max_stripes, rep=rep)
        t = model.makespan(w, rep)[0]
        if t < best[2] - 1e-12:
            best = (w, rep, t)
    return best[0], best[1]


#: the reduce's and a concurrent all-gather stand-in's slowdowns measured on one MI355X
#: (tools/overlap_probe.py, profiles/r04/overlap/: a 32-64-block copy at 0.3-0.55 TB/s beside the
#: default-grid reduce) — the prior for the contended candidate plans
CONTENTION_PRIOR = (0.37, 0.82)


def shard_candidates(n_cols: int, world: int, model: StripeModel, max_stripes: int = 8,
                     contention=CONTENTION_PRIOR) -> list:
    """The plans a measured trial chooses among (bench.py times each for a few steps on the
    running job): plan_shards' best, the best plan with no replicated tail, and the best with
    half and with 1.5x the best's tail; then the best plan of the same model with the measured
    one-GPU contention terms (RCCL's kernels and the reduce share CUs and HBM: a concurrent
    gather slows the reduce by ~1/3 and itself ~1.8x, profiles/r04/overlap/) and the plain
    serial plan — one stripe, no overlap at all.  The model's overlap is the optimistic end; the
    measured step picks."""
    best = plan_shards(n_cols, world, model, max_stripes)
    out = [best]
    if world < 2:
        return out

    def with_tail(rep_target):
        units = int(n_cols - rep_target) // (world * ALIGN)
        rep = n_cols - world * units * ALIGN
        if units < 1 or rep <= 0:
            return None
        return plan_stripes(units * ALIGN, model, max_stripes, rep=rep), rep

    cands = [(plan_stripes(-(-max(n_cols, 1) // world), model, max_stripes), 0)]
    if best[1] >= 4 * world * ALIGN:
        cands += [with_tail(best[1] // 2), with_tail(min(int(best[1] * 1.5), int(n_cols * 0.75)))]
    if contention is not None and (model.c_r, model.c_g) == (0.0, 0.0):
        cands.append(plan_shards(n_cols, world, model.with_contention(*contention), max_stripes))
    lc = -(-max(n_cols, 1) // world)
    cands.append(((-(-lc // ALIGN) * ALIGN,), 0))  # serial: reduce everything, then one gather
    for c in cands:
        if c is not None and c not in out:
            out.append(c)
    return out


@dataclass(frozen=True)
class ShardPlan:
    n_cols: int  # real global columns (parameters)
    world: int
    rank: int
    widths: tuple  # S_c: columns per (stripe c, rank) slice, each a multiple of ALIGN
    rep: int = 0  # replicated tail: global columns [n_cols - rep, n_cols), reduced by every rank

    @staticmethod
    def make(n_cols: int, world: int, rank: int, stripes: int = 4, weights=None) -> "ShardPlan":
        """Equal stripes by default; `weights` (one per stripe) sizes them unevenly, e.g. (3, 1):
        the gather of the big first stripe hides behind the small last stripe's reduce and only
        the last stripe's gather stays exposed."""
        if world < 1 or not 0 <= rank < world or stripes < 1:
            raise ValueError("bad world / rank / stripes")
        if weights is None:
            per = -(-max(n_cols, 1) // (world * stripes))
            return ShardPlan(n_cols, world, rank, (-(-per // ALIGN) * ALIGN,) * stripes)
        weights = tuple(float(x) for x in weights)
        if len(weights) != stripes or min(weights) <= 0:
            raise ValueError("need one positive weight per stripe")
        if stripes == 1:
            return ShardPlan.make(n_cols, world, rank, 1)
        total = -(-max(n_cols, 1) // world)  # columns per rank
        total = -(-total // ALIGN) * ALIGN
        widths, acc = [], 0
        for c in range(stripes - 1):
            w = -(-int(total * weights[c] / sum(weights)) // ALIGN) * ALIGN
            w = max(ALIGN, min(w, total - acc - ALIGN * (stripes - 1 - c)))
            widths.append(w)
            acc += w
        widths.append(max(ALIGN, total - acc))
        return ShardPlan(n_cols, world, rank, tuple(widths))

    @staticmethod
    def from_widths(n_cols: int, world: int, rank: int, widths, rep: int = 0) -> "ShardPlan":
        """A plan with explicit per-rank stripe widths (e.g. from plan_stripes / plan_shards);
        rep > 0: the stripes cover exactly the first n_cols - rep columns (no padding) and every
        rank reduces the last rep itself."""
        widths = tuple(int(w) for w in widths)
        rep = int(rep)
        if not widths or any(w <= 0 or w % ALIGN for w in widths):
            raise ValueError("stripe widths must be positive multiples of ALIGN")
        if rep < 0 or (rep and world * sum(widths) + rep != n_cols):
            raise ValueError("a replicated tail needs stripes covering exactly n_cols - rep columns")
        if world * sum(widths) + rep < n_cols:
            raise ValueError("stripes do not cover the bucket")
        if world < 1 or not 0 <= rank < world:
            raise ValueError("bad world / rank")
        return ShardPlan(n_cols, world, rank, widths, rep)

    @property
    def stripes(self) -> int:
        return len(self.widths)

    @property
    def shard(self) -> int:
        """The slice width when all stripes are equal."""
        if len(set(self.widths)) != 1:
            raise ValueError("stripes differ in width: use shard_of(stripe)")
        return self.widths[0]

    def shard_of(self, stripe: int) -> int:
        return self.widths[stripe]

    @property
    def padded(self) -> int:
        """Global columns the stripes cover (the gathered range; padding included when rep == 0)."""
        return self.world * sum(self.widths)

    @property
    def full_cols(self) -> int:
        """Columns of the reassembled bucket: the gathered range and the replicated tail."""
        return self.padded + self.rep

    @property
    def local_stripes(self) -> int:
        """Local columns of the stripes (the tail's local columns follow them)."""
        return sum(self.widths)

    @property
    def local_cols(self) -> int:
        return sum(self.widths) + self.rep

    @property
    def local_stride(self) -> int:
        """Row stride of the rank's local stack and state (local_cols rounded up to ALIGN, so
        every row stays 16-B aligned whatever the tail's width)."""
        return -(-self.local_cols // ALIGN) * ALIGN

    def segments(self):
        """(local begin, global begin, width) of every local column range: the stripes, then the
        replicated tail."""
        out = [(self.local_begin(c), self.global_begin(c), self.widths[c]) for c in range(self.stripes)]
        if self.rep:
            out.append((self.local_stripes, self.padded, self.rep))
        return out

    def local_begin(self, stripe: int) -> int:
        return sum(self.widths[:stripe])

    def global_begin(self, stripe: int, rank: int | None = None) -> int:
        r = self.rank if rank is None else rank
        return self.world * self.local_begin(stripe) + r * self.widths[stripe]

    def local_to_global(self, local_col: int) -> int:
        for lo, g0, w in self.segments():
            if lo <= local_col < lo + w:
                return g0 + (local_col - lo)
        raise IndexError(local_col)

    def real_cols_in_slice(self, stripe: int, rank: int | None = None) -> int:
        """Columns of this slice that are real parameters (the tail slices may be padding)."""
        g0 = self.global_begin(stripe, rank)
        return max(0, min(self.widths[stripe], self.n_cols - g0))


class PingPong:
    """Double-buffered state of a fused server step on one rank's columns (FedAVGM / FedOPT):
    step k reads (prev[k % 2], v[k % 2]) and writes the global model and v_t into the other pair,
    so the kernel's epilogue stores never land on the lines it has just loaded (in place costs
    1-3% per launch, DESIGN.md §4 finding 20).  `out` is where the current step writes the fp32
    model (the next step's prev); `flip()` advances after every stripe of a step is launched."""

    def __init__(self, prev: torch.Tensor, v: torch.Tensor):
        self.prev = [prev, torch.empty_like(prev)]
        self.v = [v, torch.empty_like(v)]
        self.cur = 0

    @property
    def out(self) -> torch.Tensor:
        return self.prev[1 - self.cur]

    def window(self, c0: int, n: int):
        """(prev, v, v_out) of local columns [c0, c0 + n) for the current step."""
        i, o = self.cur, 1 - self.cur
        return self.prev[i][c0 : c0 + n], self.v[i][c0 : c0 + n], self.v[o][c0 : c0 + n]

    def flip(self):
        self.cur ^= 1


class ShardedReducer:
    """Runs one aggregation step on this rank's shard and reassembles the full bucket.

    reduce_fn(col_begin, n_cols, out_slice) reduces local columns [col_begin, +n_cols) into
    out_slice — on a GPU it is the HIP kernel (aggregator.reduce_stack); the CPU tests inject
    the oracle to check the sharding and gather logic with gloo.
    """

    def __init__(self, plan: ShardPlan, reduce_fn, device, group=None, local_out=None, gather=None, state=None,
                 push: bool | str = False, push_grid: int = 0):
        self.plan = plan
        self.reduce_fn = reduce_fn
        self.device = torch.device(device)
        self.group = group
        # gather=None: all-gather only when there is more than one rank; True forces the
        # collective path (a 1-rank RCCL group exercises the exact multi-GPU call sequence)
        self.gather = plan.world > 1 if gather is None else gather
        # state: the PingPong of a fused optimizer — each step writes into its `out` buffer;
        # local_out may alias the sharded `prev` of a fused optimizer updated in place
        self.state = state
        self._local_out = (None if state is not None else
                           torch.empty(plan.local_stride, dtype=torch.float32, device=self.device)
                           if local_out is None else local_out)
        # the replicated tail goes straight into the global bucket unless its local results are
        # state (a fused optimizer's next prev): then it is reduced locally and copied across
        self._tail_direct = state is None and local_out is None
        # one rank: local columns ARE the global columns, nothing to reassemble
        # push: False (RCCL's all-gather), True / "kernel" (fa_push stores) or "dma" (copy engines):
        # reassemble with direct peer stores (PushGather) into a bucket from the process's receive
        # pool (mapped by the peers once); RuntimeError on every rank if some rank cannot map a peer
        self.pusher = (PushGather(None, group, mode="dma" if push == "dma" else "kernel", cols=plan.full_cols,
                                  device=self.device) if self.gather and push else None)
        self.full = (self.pusher.full if self.pusher is not None else
                     torch.empty(plan.full_cols, dtype=torch.float32, device=self.device) if self.gather else None)
        if self.pusher is not None:
            self.pusher.grid = push_grid

    def release(self):
        """Collective when pushing: after every rank's pushes, the bucket goes back to the receive
        pool.  The tensor step() returned is a view of that bucket: the next pushing job reuses it,
        and shutdown_push frees it — copy a result out before releasing if it must outlive the
        job."""
        if self.pusher is not None:
            self.pusher.close()
            self.pusher = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()
        return False

    def __del__(self):
        if getattr(self, "pusher", None) is not None:
            # release() is collective: it cannot run here; the bucket stays taken until
            # shutdown_push frees the pool
            try:
                warnings.warn("ShardedReducer with a push gather dropped without release(): its receive bucket "
                              "stays in use until shutdown_push", ResourceWarning, stacklevel=2)
            except Exception:  # noqa: BLE001 - interpreter shutdown: nothing left to warn
                pass

    @property
    def local_out(self) -> torch.Tensor:
        """Where the current step writes this rank's columns."""
        return self.state.out if self.state is not None else self._local_out

    def step(self) -> torch.Tensor:
        p = self.plan
        works = []
        out = self.local_out
        pg = self.pusher
        if pg is not None:
            pg.begin()
        for c in range(p.stripes):
            lo, sc = p.local_begin(c), p.shard_of(c)
            self.reduce_fn(lo, sc, out[lo : lo + sc])
            if pg is not None:  # this rank's slice of stripe c, into every rank's bucket
                pg.push(out[lo : lo + sc], p.world * lo + p.rank * sc)
            elif self.gather:
                g0 = p.world * lo  # stripe c's contiguous range of the global bucket
                dst = self.full[g0 : g0 + p.world * sc]
                w = all_gather_into(dst, out[lo : lo + sc], group=self.group, async_op=True)
                if w is not None:
                    works.append(w)
        if p.rep:  # the replicated tail, while the last gathers are in flight
            lo, g0 = p.local_stripes, p.padded
            if self.gather and self._tail_direct:
                self.reduce_fn(lo, p.rep, self.full[g0 : g0 + p.rep])
            else:
                self.reduce_fn(lo, p.rep, out[lo : lo + p.rep])
                if self.gather:
                    self.full[g0 : g0 + p.rep].copy_(out[lo : lo + p.rep])
        if self.state is not None:
            self.state.flip()
        if pg is not None:
            pg.end()
        for w in works:
            w.wait()
        return self.full[: p.n_cols] if self.gather else out[: p.n_cols]


def hip_reduce_fn(stack, weights, mode, denom, reorder=False, state: PingPong | None = None, **epilogue):
    """reduce_fn over a device-resident local stack [N, local_cols] with the fused HIP kernel.
    Epilogue state: a PingPong (double-buffered: the step reads its current pair, writes the
    model into out_slice — the PingPong's `out` — and v_t into the other v), or prev / v
    local-column tensors updated in place.  reorder: allow the split-N kernel
    (aggregator.reduce_stack)."""
    from .aggregator import reduce_stack

    prev, v = epilogue.pop("prev", None), epilogue.pop("v", None)

    def fn(col_begin, n_cols, out_slice):
        kw = dict(epilogue)
        if state is not None:
            p_in, v_in, v_out = state.window(col_begin, n_cols)
            kw.update(prev=p_in, v=v_in, v_out=v_out)
        elif prev is not None:
            kw.update(prev=prev[col_begin : col_begin + n_cols], v=v[col_begin : col_begin + n_cols])
        reduce_stack(stack, weights, mode, denom, col_begin=col_begin, n_cols=n_cols, out32=out_slice, reorder=reorder,
                     **kw)

    return fn


def gather_columns(local: torch.Tensor, width: int, stride: int, group=None) -> torch.Tensor:
    """Reassemble a column-sharded bucket (Aggregator(group=...)): rank r holds columns
    [r*width, r*width + local.numel()) of a `stride`-wide bucket (the last ranks' ranges may be
    short or empty).  One all_gather_into_tensor of `width` padded columns per rank; returns the
    first `stride` columns of the gathered buffer (on every rank)."""
    world = dist.get_world_size(group)
    if local.numel() == width:
        src = local
    else:
        src = torch.zeros(width, dtype=local.dtype, device=local.device)
        src[: local.numel()] = local
    full = torch.empty(world * width, dtype=local.dtype, device=local.device)
    all_gather_into(full, src, group=group)
    return full[:stride]
