"""Multi-GPU tier: one process per MI355X, torch.distributed over RCCL/xGMI."""

from .collectives import (all_gather_floats, all_gather_object, all_reduce_max, all_reduce_sum, all_reduce_sum_host,
                          broadcast_object, gather_slabs, max_over_ranks, scatter_rows)
from .dist import DistContext, context, init, shutdown
from .fault import EXIT_HUNG, FaultInjected, Watchdog, fault_hook
from .halo import HaloExchange
from .native_comm import NativeComm, P2PPlan
from .slab import Slab, max_rows_per_gpu, min_ranks_for

__all__ = [
    "all_gather_floats",
    "all_gather_object",
    "all_reduce_max",
    "all_reduce_sum_host",
    "all_reduce_sum",
    "broadcast_object",
    "gather_slabs",
    "max_over_ranks",
    "scatter_rows",
    "DistContext",
    "EXIT_HUNG",
    "FaultInjected",
    "Watchdog",
    "fault_hook",
    "context",
    "init",
    "shutdown",
    "HaloExchange",
    "NativeComm",
    "P2PPlan",
    "Slab",
    "max_rows_per_gpu",
    "min_ranks_for",
]
