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

The push gathers' pusher stream (both forms): its push kernels or own copies run beside the next
stripe's reduce.  The copy-engine legs' streams stay at normal priority (flearn_amd.dist.peer_stream).
Round 5 saw wrong buckets with the copy-engine push's streams at high priority; round 6 found the
cause — device-side cross-queue event waits that let copies start before their reduce finished,
with several processes' streams on queues of their own — and removed the copy-engine push's
reliance on them (its legs are host-ordered); the kernel push, never wrong
with its device-side wait in the same probes, keeps it.  RCCL's internal stream stays in torch's
normal pool (the process group's default).
"""
from __future__ import annotations

import torch

HIGH = -1  # torch's high stream priority on ROCm (the only other level is 0)


def side_stream(device) -> torch.cuda.Stream:
    """A high-priority stream: its hardware queue is never one a normal-priority stream uses."""
    return torch.cuda.Stream(device, priority=HIGH)
