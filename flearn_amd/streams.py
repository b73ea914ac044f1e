"""A stream for kernels meant to run BESIDE the caller's stream (the kernel push gather's).

HIP spreads a process's streams over GPU_MAX_HW_QUEUES (4 on the MI355X boxes) hardware queues per
priority, round-robin; two streams on one hardware queue run their work in queue order, whatever
their events say.  Round 5 traced the stripe pipeline (tools/trace_pipeline.py,
profiles/r05/pipeline_queues/): the push gather's stream and RCCL's internal stream, both of normal
priority, landed on the compute stream's queue and ran 0% of their time beside a reduce.  A
high-priority stream is taken from the other priority's queues, so it never shares the (normal
priority) compute stream's: the same pipeline then ran 91-93% of its gather time beside a reduce
(the kernel push; RCCL's stream from the high-priority pool).
Priority also lets the gather's small kernels be dispatched ahead of the reduce's blocks, which
suits work on the step's critical path.

Used for KERNEL work beside the compute stream only.  Copy-engine transfers (hipMemcpyAsync ...
NoCU) run on the copy engines whatever queue their stream has, and with high-priority streams a
rank's slice was wrong in the buckets after the step's closing barrier — half of the wrong values
the previous step's, half the bucket's older contents: tests/push_order_probe.py, eight processes,
the copy-engine push with in-place Adagrad, 32 of 576 rank-steps wrong with high-priority streams
and 0 of 576 with normal ones (the kernel push: 0 of 576 either way;
profiles/r05/pipeline_queues/).  RCCL's internal stream stays in torch's normal pool (the process
group's default): a high-priority one would give the all-gather its own queue too, but the line
bench.py must not lose runs on it, and one GPU cannot test RCCL between ranks.
"""
from __future__ import annotations

import torch

HIGH = -1  # torch's high stream priority on ROCm (the only other level is 0)


def side_stream(device) -> torch.cuda.Stream:
    """A high-priority stream: its hardware queue is never one a normal-priority stream uses."""
    return torch.cuda.Stream(device, priority=HIGH)
