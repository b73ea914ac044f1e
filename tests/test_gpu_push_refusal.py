"""PushGather's agreement protocol (gloo, world 2, on the GPU box: the library needs a device to
load): a rank that cannot register or map its receive buffer — here every rank, since the
buffers are host tensors — makes EVERY rank raise RuntimeError with nothing left mapped, so no
rank goes on to push while another falls back to RCCL; ShardedReducer(push=True) surfaces the
same error."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, init):
    from flearn_amd.dist import PushGather, ShardedReducer, ShardPlan

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        with pytest.raises(RuntimeError, match="could not map"):
            PushGather(torch.zeros(4096))
        plan = ShardPlan.make(10_000, world, rank, 1)
        with pytest.raises(RuntimeError, match="could not map"):
            ShardedReducer(plan, lambda c0, n, out: None, "cpu", gather=True, push=True)
        with pytest.raises(ValueError):
            PushGather(torch.zeros(64), mode="rdma")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_every_rank_refuses_together(cuda):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="fa_push_"), "pg")
    mp.spawn(_worker, args=(2, init), nprocs=2, join=True)
