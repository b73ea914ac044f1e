"""The push gather's receive pool (flearn_amd.dist._RecvPool) on CPU, gloo world 2.

The GPU parts are stubbed (the bucket allocation, `_map_peers`' IPC export / import, the unmaps),
the collective protocol is real: buckets are mapped once and handed out again, the first free
slot that fits is reused, a slot in use is never handed out twice, a larger request retires the
free buckets (every peer unmaps, barrier, park) before it maps a new one, ranks whose pools
disagree all raise, `shutdown_push` empties the pools with every import closed before any bucket
is parked, the next pool re-exports a parked bucket, and a destroyed and re-created default group
maps its buckets afresh.  `test_parked_buckets_stay_within_the_cap` runs the real DeviceBuffer and
`_map_peers` over a shared-memory stand-in for HIP IPC: growing then shrinking requests keep the
parked bytes within the cap, and every mapping is token-checked (a wrong one refused)."""
import os
import tempfile
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _FakeL:
    def __init__(self, events):
        self.events = events

    def fa_ipc_close(self, b):
        self.events.append(("close", b))
        return 0


def _install_stubs(fd, events):
    L = _FakeL(events)
    counter = [0]
    parked = []

    class FakeBuf:
        def __init__(self, nbytes, device):
            self.nbytes, self.L, self.exported = nbytes, L, False
            self.t = torch.zeros(nbytes // 4)
            counter[0] += 1
            self.id = counter[0]
            events.append(("alloc", self.id))

        @classmethod
        def get(cls, nbytes, device):
            fits = [b for b in parked if b.nbytes >= nbytes]
            if fits:
                b = min(fits, key=lambda x: x.nbytes)
                parked.remove(b)
                events.append(("reuse", b.id))
                return b
            return cls(nbytes, device)

        @staticmethod
        def parked_bytes():
            return sum(b.nbytes for b in parked)

        def tensor(self, dtype=torch.float32):
            return self.t

        def free(self):  # exported: parked, never freed
            assert self.exported
            parked.append(self)
            events.append(("park", self.id))

    def fake_map(pg, full):
        dist.barrier(group=pg.group)  # collective like the real one
        events.append(("map", full.numel()))
        return [1000 + full.numel()], [full.data_ptr()] * pg.world, []

    fd.DeviceBuffer = FakeBuf
    fd._map_peers = fake_map
    fd._IPC = types.SimpleNamespace(close=L.fa_ipc_close, accepts=lambda d: torch.device(d).type == "cuda")
    fd._RecvPool._pools.clear()
    from flearn_amd import _native as na

    na.lib = lambda: L  # shutdown_push binds the library
    return L, FakeBuf


def _cols(want):  # the pool's request: ALIGN-rounded (DeviceBuffer.get applies the size class)
    return -(-want // 64) * 64


def _worker(rank, world, init):
    from flearn_amd import dist as fd

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    ev = []
    L, FB = _install_stubs(fd, ev)
    try:
        # the pool's device is named cuda:0 (a CPU device is refused collectively, as the GPU-only
        # IPC path requires); every GPU call is stubbed, so no GPU is touched
        pg = types.SimpleNamespace(world=world, rank=rank, group=None, nccl=False, device=torch.device("cpu"), L=L)
        pool = fd._RecvPool.get("cuda:0", None)
        assert fd._RecvPool.get(torch.device("cuda:0"), None) is pool
        i, buf, dsts = pool.take(pg, 1000)
        assert i == 0 and buf.numel() == _cols(1000) and len(dsts) == world
        j, buf2, _ = pool.take(pg, 500)  # slot 0 is busy: a second bucket
        assert j == 1
        pool.give(i)
        k, buf3, _ = pool.take(pg, 800)  # fits slot 0 again: no new mapping
        assert k == 0 and buf3.data_ptr() == buf.data_ptr()
        assert [e for e in ev if e[0] == "map"] == [("map", _cols(1000)), ("map", _cols(500))]
        pool.give(k)
        pool.give(j)
        ev.clear()
        # larger than every slot: the free ones are released first (every import closed, then a
        # barrier, then parked — never freed), and a new bucket is mapped
        k, _b, _ = pool.take(pg, 2000)
        assert ev == [("close", 1000 + _cols(1000)), ("close", 1000 + _cols(500)), ("park", 2), ("park", 1),
                      ("alloc", 3), ("map", _cols(2000))], ev
        assert k == 0 and len(pool.slots) == 1
        assert fd._RecvPool.bytes_held() == _cols(2000) * 4
        pool.give(k)
        k, _b, _ = pool.take(pg, 3)  # first free slot that fits
        assert k == 0
        pool.give(k)
        # rank 1 holds slot 0 while rank 0 does not: the picks differ, every rank raises
        if rank == 1:
            pool.slots[0][4] = True
        with pytest.raises(RuntimeError, match="disagree"):
            pool.take(pg, 10)
        pool.slots[0][4] = False
        dist.barrier()
        # shutdown: every import closed (and a barrier) before anything is parked; the pools hold
        # nothing, the parked buckets wait for reuse
        ev.clear()
        fd.shutdown_push()
        assert ev == [("close", 1000 + _cols(2000)), ("park", 3)], ev
        assert fd._RecvPool.bytes_held() == 0 and not fd._RecvPool._pools
        assert FB.parked_bytes() == 4 * (_cols(1000) + _cols(500) + _cols(2000))
        # the next pool re-exports the smallest parked bucket that fits (no new allocation)
        p2 = fd._RecvPool.get("cuda:0", None)
        ev.clear()
        p2.take(pg, 64)
        assert ev == [("reuse", 2), ("map", _cols(500))], ev
        # a pool whose group is destroyed without shutdown: dropped locally at the next lookup
        # (imports closed, bucket parked), and the re-created group maps its buckets afresh
        old = id(p2)
        dist.destroy_process_group()
        dist.init_process_group("gloo", init_method=init + "_2", rank=rank, world_size=world)
        ev.clear()
        p3 = fd._RecvPool.get("cuda:0", None)
        assert id(p3) != old and not p3.slots
        assert ev == [("close", 1000 + _cols(500)), ("park", 2)], ev
        i, _b, _ = p3.take(pg, 64)
        assert i == 0 and ev[-1] == ("map", _cols(500))
        p3.give(i)
        fd.shutdown_push()
        assert fd._RecvPool.bytes_held() == 0
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_recv_pool_lifecycle():
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_pool_"), "pg")
    mp.spawn(_worker, args=(2, init), nprocs=2, join=True)


class _ShmIpc:
    """HIP IPC's stand-in on CPU: a DeviceBuffer is a POSIX shared-memory segment, its handle the
    segment's name, a peer's import an attachment of it; read16 copies through the mapping, as
    the token check reads through a copy engine."""

    def __init__(self, events, wrong_open=None):
        from multiprocessing import shared_memory

        self.sm, self.events, self.wrong_open = shared_memory, events, wrong_open
        self.own = {}  # address -> SharedMemory (this rank's allocations)
        self.attached = {}  # address -> SharedMemory (imports)

    @staticmethod
    def _addr(shm):
        import ctypes

        return ctypes.addressof(ctypes.c_char.from_buffer(shm.buf))

    def alloc(self, nbytes):
        shm = self.sm.SharedMemory(create=True, size=nbytes)
        a = self._addr(shm)
        self.own[a] = shm
        return a

    def release(self, ptr):
        shm = self.own.pop(ptr)
        try:
            shm.close()
        except BufferError:  # a tensor view still alive: the mapping goes with the process
            pass
        shm.unlink()
        self.events.append(("freed", ptr))

    def view(self, ptr, dtype):
        return torch.frombuffer(self.own[ptr].buf, dtype=dtype)

    def accepts(self, device):
        return torch.device(device).type == "cpu"

    def sync(self, device):
        pass

    def handle(self, ptr):
        for a, shm in self.own.items():
            if a <= ptr < a + shm.size:
                return shm.name.encode().ljust(64, b"\0"), ptr - a
        return None

    def open(self, hb):
        name = hb.rstrip(b"\0").decode()
        if self.wrong_open is not None:  # an import that maps some other allocation
            name, self.wrong_open = self.wrong_open, None
        shm = self.sm.SharedMemory(name=name)
        a = self._addr(shm)
        self.attached[a] = shm
        return a

    def read16(self, probe, addr):
        import ctypes

        ctypes.memmove(probe.data_ptr(), addr, 16)
        self.events.append(("token_read", addr))
        return True

    def close(self, base):
        shm = self.attached.pop(base)
        try:
            shm.close()
        except BufferError:
            pass
        self.events.append(("close", base))

    def last_error(self):
        return b""


def _cap_worker(rank, world, init):
    from flearn_amd import dist as fd

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    ev = []
    ipc = _ShmIpc(ev)
    fd._IPC = ipc
    fd._RecvPool._pools.clear()
    fd.DeviceBuffer._alloc = lambda self: ipc.alloc(self.nbytes)
    fd.DeviceBuffer._release = lambda self, ptr: ipc.release(ptr)
    fd.DeviceBuffer.tensor = lambda self, dtype=torch.float32: ipc.view(self.ptr, dtype)

    def init_buf(self, nbytes, device):  # the real constructor minus the native library
        self.L, self.na = None, None
        self.nbytes, self.device = int(nbytes), torch.device(device)
        self._exported = False
        self._typestr = "<f4"
        self.ptr = self._alloc()

    fd.DeviceBuffer.__init__ = init_buf
    try:
        pg = types.SimpleNamespace(world=world, rank=rank, group=None, nccl=False, device=torch.device("cpu"))
        pool = fd._RecvPool.get("cpu", None)
        maps = 0
        # growing by ~25% per request: each larger request retires the free bucket and maps a new
        # one, so without the cap the parked bytes would reach ~4x the largest bucket
        for cols in (100_000, 125_000, 160_000, 200_000, 250_000, 320_000, 400_000):
            n0 = sum(1 for e in ev if e[0] == "token_read")
            i, buf, dsts = pool.take(pg, cols)
            maps += 1
            # the new bucket's mapping read every peer's token through the mapping
            assert sum(1 for e in ev if e[0] == "token_read") - n0 == world - 1
            buf.fill_(float(rank + 1))
            dist.barrier()
            peer = (rank + 1) % world
            probe = torch.empty(4, dtype=torch.float32)
            ipc.read16(probe, dsts[peer])  # the mapping reaches the peer's bucket
            assert probe.tolist() == [float(peer + 1)] * 4
            dist.barrier()
            pool.give(i)
            assert fd.DeviceBuffer.parked_bytes("cpu") <= fd.DeviceBuffer.park_cap("cpu")
        assert fd.DeviceBuffer.trimmed()["buckets"] > 0  # the cap did bind
        assert any(e[0] == "freed" for e in ev)
        # shrinking: smaller requests reuse the free bucket, no new mapping
        n0 = sum(1 for e in ev if e[0] == "token_read")
        for cols in (300_000, 20_000, 64):
            i, buf, _ = pool.take(pg, cols)
            pool.give(i)
        assert sum(1 for e in ev if e[0] == "token_read") == n0
        fd.shutdown_push()
        assert fd.DeviceBuffer.parked_bytes("cpu") <= fd.DeviceBuffer.park_cap("cpu")
        # a mapping of the wrong allocation is refused on every rank (the token check)
        pool = fd._RecvPool.get("cpu", None)
        if rank == 0:
            victim = next(iter(ipc.own.values())).name  # rank 0's own segment, not the peer's
            ipc.wrong_open = victim
        with pytest.raises(RuntimeError, match="did not hold their tokens" if rank == 0 else "could not map"):
            pool.take(pg, 450_000)
        dist.barrier()
    finally:
        dist.destroy_process_group()
        for a in list(ipc.own):
            ipc.release(a)


def test_parked_buckets_stay_within_the_cap():
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_cap_"), "pg")
    mp.spawn(_cap_worker, args=(2, init), nprocs=2, join=True)


def test_size_classes():
    from flearn_amd.dist import size_class

    assert size_class(1) == 4096 and size_class(4096) == 4096
    for n in (4097, 10_000, 123_457, 10**9 + 7):
        c = size_class(n)
        assert n <= c < n * 1.25 + 4096 and c % 256 == 0
        assert size_class(c) == c  # a class is its own class
    # requests a few percent apart share a class
    assert size_class(1_000_000) == size_class(1_030_000)
