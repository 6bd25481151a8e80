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
import ctypes
import os
from typing import List, Optional

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


_WAIT_FLAGS = {"auto": 0, "spin": 1, "yield": 2}
_WAIT_IN_FORCE: dict = {}


def wait_policy_in_force(device: torch.device) -> str:
    """The policy the last ``host_wait_policy`` call set on ``device``."""
    return _WAIT_IN_FORCE.get(torch.device(device).index, "auto")


def host_wait_policy(device: torch.device, mode: Optional[str] = None) -> str:
    """How host waits on this device (``torch.cuda.synchronize``, event
    waits) detect completion: ``hipSetDeviceFlags`` schedule flag. HIP's
    ``auto`` picks *yield* whenever the machine has more logical CPUs than HIP
    contexts — the waiting thread then sleeps on a completion interrupt after a
    short active-wait window, and wakes up late. ``spin`` polls the completion
    signal on the waiting thread (one CPU core while it waits). ``mode``
    defaults to ``MPX_HIP_WAIT`` (auto | spin | yield). Returns the policy in
    force."""
    mode = (mode or os.environ.get("MPX_HIP_WAIT", "auto")).lower()
    if mode not in _WAIT_FLAGS:
        raise ValueError(f"MPX_HIP_WAIT must be one of {sorted(_WAIT_FLAGS)}, not {mode!r}")
    if torch.device(device).type != "cuda":
        return "auto"
    if mode == "auto" and torch.device(device).index not in _WAIT_IN_FORCE:
        return "auto"  # the runtime's own choice, untouched
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
    idx = torch.device(device).index
    prev = ctypes.c_int()
    hip.hipGetDevice(ctypes.byref(prev))
    if idx is not None:
        hip.hipSetDevice(idx)
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(_WAIT_FLAGS[mode]))
    hip.hipSetDevice(prev.value)
    res = mode if rc == 0 else f"auto (hipSetDeviceFlags({mode}) returned {rc})"
    if mode == "auto" and rc == 0:
        _WAIT_IN_FORCE.pop(idx, None)
    else:
        _WAIT_IN_FORCE[idx] = res
    return res
