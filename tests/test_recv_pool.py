"""The push gather's receive pool (flearn_amd.dist._RecvPool) on CPU, gloo world 2: buffers are
mapped once (the collective `_map_peers`, stubbed here: it needs the GPU) and handed out again,
the first free slot that fits is reused, a slot in use is never handed out twice, a larger
request maps a new buffer, and ranks whose pools disagree all raise instead of pushing into
different buckets."""
import os
import tempfile
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, init):
    from flearn_amd import dist as fd

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        maps = []

        def fake_map(pg, full):
            dist.barrier(group=pg.group)  # collective like the real one
            maps.append(full.numel())
            return [], [full.data_ptr()] * pg.world, []

        fd._map_peers = fake_map
        fd._RecvPool._pools.clear()
        pg = types.SimpleNamespace(world=world, rank=rank, group=None, nccl=False, device=torch.device("cpu"))
        pool = fd._RecvPool.get("cpu", None)
        assert fd._RecvPool.get(torch.device("cpu"), None) is pool
        i, buf, dsts = pool.take(pg, 1000)
        assert i == 0 and buf.numel() == 1000 and maps == [1000] and len(dsts) == world
        j, buf2, _ = pool.take(pg, 500)  # slot 0 is busy: a second buffer
        assert j == 1 and maps == [1000, 500]
        pool.give(i)
        k, buf3, _ = pool.take(pg, 800)  # fits slot 0 again: no new mapping
        assert k == 0 and buf3.data_ptr() == buf.data_ptr() and maps == [1000, 500]
        pool.give(k)
        pool.give(j)
        k, _b, _ = pool.take(pg, 2000)  # larger than every slot: a third buffer
        assert k == 2 and maps == [1000, 500, 2000]
        pool.give(k)
        k, _b, _ = pool.take(pg, 3)  # first free slot that fits
        assert k == 0 and maps == [1000, 500, 2000]
        pool.give(k)
        # rank 1 holds slot 0 while rank 0 does not: the picks differ, every rank raises
        if rank == 1:
            pool.slots[0][2] = True
        with pytest.raises(RuntimeError, match="disagree"):
            pool.take(pg, 10)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_recv_pool_reuses_and_agrees():
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_pool_"), "pg")
    mp.spawn(_worker, args=(2, init), nprocs=2, join=True)
