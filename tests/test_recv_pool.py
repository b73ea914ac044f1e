"""The push gather's receive pool (flearn_amd.dist._RecvPool) on CPU, gloo world 2.

The GPU parts are stubbed (the bucket allocation, `_map_peers`' IPC export / import, the unmaps),
the collective protocol is real: buckets are mapped once and handed out again, the first free
slot that fits is reused, a slot in use is never handed out twice, a larger request retires the
free buckets (every peer unmaps, barrier, park) before it maps a new one, ranks whose pools
disagree all raise, `shutdown_push` empties the pools with every import closed before any bucket
is parked (exported memory is never freed: DESIGN.md section 6), the next pool re-exports a
parked bucket, and a destroyed and re-created default group maps its buckets afresh."""
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
    fd._RecvPool._pools.clear()
    from flearn_amd import _native as na

    na.lib = lambda: L  # shutdown_push binds the library for the unmaps
    return L, FakeBuf


def _cols(want):  # the pool's bucket size: 1/8 headroom, ALIGN-rounded
    return (want + want // 8 + 64) // 64 * 64


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
