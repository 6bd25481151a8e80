"""One process-wide set of compute streams.

HIP binds each new stream to one of GPU_MAX_HW_QUEUES (4 by default)
hardware queues; once the pool is full a new stream shares the least-used
queue, so two streams created late (after RCCL's, torch's and earlier
phases' streams) can land on ONE queue and run their kernels strictly in turn
(seen in a rocprofv3 trace of bench.py: both streaming-phase streams on queue
4, no overlap; profiles/lab2_conv.md). The set is created as early as
possible — ``parallel.init`` makes the first two right after selecting the
device, before any communicator exists — and every user takes its streams
from it.
"""
from typing import List

import torch

_POOL: dict = {}


def compute_streams(device: torch.device, k: int) -> List[torch.cuda.Stream]:
    """The first ``k`` streams of this process's set on ``device``, created on
    first use."""
    key = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    pool = _POOL.setdefault(key, [])
    while len(pool) < k:
        pool.append(torch.cuda.Stream(torch.device("cuda", key)))
    return pool[:k]
