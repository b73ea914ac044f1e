"""Self-check of a column-sharded aggregation step on the hardware it ran on.

`bench.py --gpus N` (and any caller of `flearn_amd.dist.ShardedReducer`) can prove that the
global model the ranks reassembled — each rank's column slices, moved by the RCCL all-gather
over xGMI into one contiguous bucket, plus a replicated tail every rank reduced itself — is what
the unsharded reduce computes (the reference's `Strategy.server_ensemble`, strategy.py:123-129,
as `Server.ensemble` calls it, Server.py:140).

How: windows of columns are placed on every boundary the sharding introduces — each
(stripe, rank) slice start, i.e. every gather destination and every rank boundary; the
replicated tail's two edges; the bucket's two ends — plus evenly spread windows up to a count.
For each window the caller regenerates all N clients' columns of that window (inputs that depend
only on (seed, client, global column), like `fa_fill_uniform_f32`'s) and reduces them UNSHARDED
with the same kernel; the gathered bucket must match bit for bit.  The fused optimizers' state
(v_t) is never gathered: each rank checks its own slices of it the same way, on windows at both
edges of every local segment.  Mismatch counts are summed over the ranks, so every rank learns
the verdict.  Nothing here compares against a restatement: it is the product kernel against
itself, unsharded.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

#: process exit status of a run whose reassembled bucket failed the check
EXIT_MISMATCH = 3

_INT_VIEW = {torch.float32: torch.int32, torch.float64: torch.int64}


def bits_equal(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Bitwise equality of two float tensors (NaN payloads and signed zeros included)."""
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    a = a.contiguous()
    b = b.to(a.device).contiguous()
    return bool(torch.equal(a.view(_INT_VIEW[a.dtype]), b.view(_INT_VIEW[b.dtype])))


def boundary_windows(plan, width: int = 4096, count: int = 64) -> list:
    """[(first global column, width)] of the windows to check for a ShardPlan: one straddling
    every (stripe, rank) slice start and end, the replicated tail's edges and the bucket's ends,
    then evenly spread ones until there are `count` (fewer only when the bucket is too narrow
    for that many distinct windows).  Every window lies inside [0, plan.n_cols)."""
    n = plan.n_cols
    if n <= 0:
        return []
    w = min(width, n)
    starts = set()

    def around(c):
        starts.add(c - w // 2)

    for c in range(plan.stripes):
        for r in range(plan.world):
            g0 = plan.global_begin(c, r)
            around(g0)
            around(g0 + plan.widths[c])
    if plan.rep:
        around(plan.padded)
    starts |= {0, n - w}
    starts = {max(0, min(s, n - w)) for s in starts}
    i = 0
    spread = max(count, 2)
    while len(starts) < count and i < spread:
        starts.add(i * (n - w) // (spread - 1))
        i += 1
    return [(s, w) for s in sorted(starts)]


def segment_windows(plan, width: int = 4096) -> list:
    """[(local column, global column, width)]: windows at both edges of each of this rank's
    local segments (stripe slices and the replicated tail), inside their real columns — where a
    sharded state buffer (v_t) has its slice boundaries."""
    out = set()
    for lo, g0, seg in plan.segments():
        real = max(0, min(seg, plan.n_cols - g0))
        if real == 0:
            continue
        w = min(width, real)
        out.add((lo, g0, w))
        out.add((lo + real - w, g0 + real - w, w))
    return sorted(out)


def check_step(plan, full: torch.Tensor, expect, state: torch.Tensor | None = None, group=None,
               width: int = 4096, count: int = 64, compare=None, local_model: bool = False) -> dict:
    """Check one reassembled step.

    full   : the global fp32 bucket the step returned (at least plan.n_cols columns)
    expect : expect(g0, w) -> (model [w], state [w] or None): the unsharded reduce of the
             regenerated window (state only when `state` is given)
    state  : this rank's local state buffer after the step (a fused optimizer's v_t) or None
    compare: compare(got, want) -> bool (default: bitwise)
    local_model: `full` holds only this rank's local columns (no gather: bench.py --emulate-world);
             the model is then checked on the local segment windows, like the state
    Returns {"windows" (model windows, checked on every rank), "state_windows" and
    "mismatched_windows" (summed over the ranks of `group` when torch.distributed is
    initialised), "first_mismatches" (this rank's), "verified"}."""
    cmp = compare or bits_equal
    bad = []
    if local_model:
        wins = segment_windows(plan, width)
        for lo, g0, w in wins:
            want, _ = expect(g0, w)
            if not cmp(full[lo : lo + w], want[:w]):
                bad.append(("model", g0))
    else:
        wins = boundary_windows(plan, width, count)
        for g0, w in wins:
            want, _ = expect(g0, w)
            if not cmp(full[g0 : g0 + w], want[:w]):
                bad.append(("model", g0))
    swins = segment_windows(plan, width) if state is not None else []
    for lo, g0, w in swins:
        _, want_v = expect(g0, w)
        if not cmp(state[lo : lo + w], want_v[:w]):
            bad.append(("state", g0))
    counts, ranks = [len(swins), len(bad)], 1
    if dist.is_available() and dist.is_initialized():
        on = full.device if dist.get_backend(group) == "nccl" else "cpu"
        t = torch.tensor(counts, dtype=torch.int64, device=on)
        dist.all_reduce(t, group=group)
        counts = [int(x) for x in t.tolist()]
        ranks = dist.get_world_size(group)
    return {"windows": len(wins), "window_cols": min(width, plan.n_cols), "ranks_checked": ranks,
            "state_windows": counts[0], "mismatched_windows": counts[1],
            "first_mismatches": [f"{k}@{g0}" for k, g0 in bad[:8]], "verified": counts[1] == 0}
