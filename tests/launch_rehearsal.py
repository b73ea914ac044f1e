"""CPU rehearsal of bench.py's launcher path (run by tests/test_launch.py, never on its own).

    python tests/launch_rehearsal.py N [FAIL_RANK]

The parent goes through flearn_amd.launch.ensure_ranks exactly as `bench.py --gpus N` does (N
fresh children via torch.distributed.run on 127.0.0.1); only the device count is stubbed (CPU
container) and each rank reduces its element-range shard with the C oracle instead of the HIP
kernel, then reassembles the bucket with the gloo all-gather of flearn_amd.dist.ShardedReducer.
Rank 0 prints one JSON line with n_gpus = dist.get_world_size(), like bench.py.
"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from flearn_amd import launch  # noqa: E402


def main():
    n = int(sys.argv[1])
    fail_rank = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    rc = launch.ensure_ranks(n, __file__, sys.argv[1:], device_count=lambda: n, timeout=240)
    if rc is not None:
        sys.exit(rc)
    rank, _, world = launch.rank_env()
    if rank == fail_rank:
        sys.exit(3)

    import numpy as np
    import torch
    import torch.distributed as dist

    import oracle
    from flearn_amd.dist import ShardedReducer, ShardPlan

    dist.init_process_group("gloo")  # env:// from torch.distributed.run
    clients, p, seed = 9, 70_001, 5
    plan = ShardPlan.make(p, world, rank, 2, weights=(3, 1))
    local = np.zeros((clients, plan.local_cols), np.float32)
    for c in range(plan.stripes):
        lo, width = plan.local_begin(c), plan.real_cols_in_slice(c)
        if width:
            local[:, lo : lo + width] = oracle.fill_uniform(clients, width, seed, col0=plan.global_begin(c))
    w = np.ones(clients, np.float32)
    denom = float(np.sum([1.0] * clients))

    def fn(col_begin, ncols, out_slice):
        g = oracle.c_reduce(oracle.MODE_W32_DIV64, local[:, col_begin : col_begin + ncols], w, denom)
        out_slice.copy_(torch.from_numpy(g.astype(np.float32)))

    full = ShardedReducer(plan, fn, "cpu").step().numpy()
    ref = oracle.c_reduce(oracle.MODE_W32_DIV64, oracle.fill_uniform(clients, p, seed), w, denom)
    same = bool(np.array_equal(full.view(np.uint32), ref.astype(np.float32).view(np.uint32)))
    flags = torch.tensor([int(same)])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(json.dumps({"n_gpus": dist.get_world_size(), "bit_exact": bool(flags.item())}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if flags.item() else 1)


if __name__ == "__main__":
    main()
