"""The push gather's receive pool (flearn_amd.dist._RecvPool) on CPU, gloo world 2.

The GPU parts are stubbed (the bucket allocation, `_map_peers`' IPC export / import, the unmaps),
the collective protocol is real: buckets are mapped once and handed out again, the first free
slot that fits is reused, a slot in use is never handed out twice, a larger request retires the
free buckets (every peer unmaps, barrier, free) before it maps a new one, ranks whose pools
disagree all raise, `shutdown_push` returns the pool's memory to zero with every import closed
before any bucket is freed, and a destroyed and re-created default group gets fresh buckets."""
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

    class FakeBuf:
        def __init__(self, nbytes, device):
            self.nbytes, self.L = nbytes, L
            self.t = torch.zeros(nbytes // 4)
            counter[0] += 1
            self.id = counter[0]
            events.append(("alloc", self.id))

        def tensor(self, dtype=torch.float32):
            return self.t

        def free(self):
            events.append(("free", self.id))

    def fake_map(pg, full):
        dist.barrier(group=pg.group)  # collective like the real one
        events.append(("map", full.numel()))
        return [1000 + full.numel()], [full.data_ptr()] * pg.world, []

    fd.DeviceBuffer = FakeBuf
    fd._map_peers = fake_map
    fd._RecvPool._pools.clear()
    from flearn_amd import _native as na

    na.lib = lambda: L  # shutdown_push binds the library for the unmaps
    return L


def _worker(rank, world, init):
    from flearn_amd import dist as fd

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    ev = []
    L = _install_stubs(fd, ev)
    try:
        pg = types.SimpleNamespace(world=world, rank=rank, group=None, nccl=False, device=torch.device("cpu"), L=L)
        pool = fd._RecvPool.get("cpu", None)
        assert fd._RecvPool.get(torch.device("cpu"), None) is pool
        i, buf, dsts = pool.take(pg, 1000)
        assert i == 0 and buf.numel() == 1000 and len(dsts) == world
        j, buf2, _ = pool.take(pg, 500)  # slot 0 is busy: a second buffer
        assert j == 1
        pool.give(i)
        k, buf3, _ = pool.take(pg, 800)  # fits slot 0 again: no new mapping
        assert k == 0 and buf3.data_ptr() == buf.data_ptr()
        assert [e for e in ev if e[0] == "map"] == [("map", 1000), ("map", 500)]
        pool.give(k)
        pool.give(j)
        ev.clear()
        k, _b, _ = pool.take(pg, 2000)  # larger than every slot: the free ones retire first
        assert ev == [("close", 2000), ("close", 1500), ("free", 2), ("free", 1), ("alloc", 3), ("map", 2000)], ev
        assert k == 0 and len(pool.slots) == 1
        assert fd._RecvPool.bytes_held() == 8000
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
        # shutdown: every import closed (and a barrier) before any bucket is freed; memory zero
        ev.clear()
        fd.shutdown_push()
        assert ev == [("close", 3000), ("free", 3)], ev
        assert fd._RecvPool.bytes_held() == 0 and not fd._RecvPool._pools
        # a pool whose group is destroyed without shutdown: dropped locally at the next lookup,
        # and the re-created group maps fresh buckets
        p2 = fd._RecvPool.get("cpu", None)
        p2.take(pg, 64)
        old = id(p2)
        dist.destroy_process_group()
        dist.init_process_group("gloo", init_method=init + "_2", rank=rank, world_size=world)
        ev.clear()
        p3 = fd._RecvPool.get("cpu", None)
        assert id(p3) != old and not p3.slots
        assert ("free", 4) in ev and ("close", 1064) in ev
        i, _b, _ = p3.take(pg, 64)
        assert i == 0 and ev[-1] == ("map", 64)
        p3.give(i)
        fd.shutdown_push()
        assert fd._RecvPool.bytes_held() == 0
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_recv_pool_lifecycle():
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_pool_"), "pg")
    mp.spawn(_worker, args=(2, init), nprocs=2, join=True)
