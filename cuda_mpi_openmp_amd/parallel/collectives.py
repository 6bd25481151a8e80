"""Global reductions and slab assembly over torch.distributed (RCCL on GPU).

The reference's only "global reduction" is the harness's median over runs; the
distributed tier needs real ones: a residual max for Jacobi, a max over ranks
for step timing, a gather of output slabs for verification, and a broadcast of
lab3 class parameters computed on one rank.
"""

from __future__ import annotations

import os
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from .dist import DistContext
from .slab import Slab


def _native_ok(x: torch.Tensor, ctx: DistContext) -> bool:
    return ctx.native is not None and x.is_cuda and x.is_contiguous() and x.dtype in (
        torch.float64, torch.float32, torch.int32)


def _scalar_device(ctx: DistContext, site: str):
    """Where a host scalar's tensor goes for a collective: the rank's GPU under
    RCCL (it takes device tensors only), the host under gloo.
    ``MPX_CONTRACT_INJECT=<site>`` puts it on the host anyway — a test hook
    that the nccl contract (parallel/contract.py) must catch at ``site``."""
    if ctx.backend != "nccl" or os.environ.get("MPX_CONTRACT_INJECT") == site:
        return "cpu"
    return ctx.device


def _host_staged(x: torch.Tensor, ctx: DistContext) -> bool:
    """A GPU tensor on a gloo control plane (one-GPU rehearsal): reduce a host copy."""
    return x.is_cuda and ctx.backend != "nccl"


def _all_reduce(x: torch.Tensor, ctx: DistContext, op, native_op: str) -> torch.Tensor:
    if ctx.is_distributed:
        if _native_ok(x, ctx):
            ctx.native.all_reduce_(x, native_op)
        elif _host_staged(x, ctx):
            h = x.cpu()
            dist.all_reduce(h, op=op)
            x.copy_(h)
        else:
            dist.all_reduce(x, op=op)
    return x


def all_reduce_max(x: torch.Tensor, ctx: DistContext) -> torch.Tensor:
    """In-place MAX over ranks, ordered on the current stream (native RCCL tier
    when available, torch.distributed otherwise)."""
    return _all_reduce(x, ctx, dist.ReduceOp.MAX, "max")


def all_reduce_sum(x: torch.Tensor, ctx: DistContext) -> torch.Tensor:
    return _all_reduce(x, ctx, dist.ReduceOp.SUM, "sum")


def max_over_ranks(value: float, ctx: DistContext) -> float:
    """Max of a host scalar over ranks (e.g. each rank's step time)."""
    if not ctx.is_distributed:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_scalar_device(ctx, "max_over_ranks"))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(value: float, ctx: DistContext) -> List[float]:
    """Every rank's host scalar, in rank order (e.g. per-rank step times)."""
    if not ctx.is_distributed:
        return [float(value)]
    dev = _scalar_device(ctx, "all_gather_floats")
    mine = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    every = [torch.empty_like(mine) for _ in range(ctx.world)]
    dist.all_gather(every, mine)
    return [float(t.item()) for t in every]


def all_reduce_sum_host(value: float, ctx: DistContext) -> float:
    """Sum of a host scalar over ranks."""
    if not ctx.is_distributed:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_scalar_device(ctx, "all_reduce_sum_host"))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def all_gather_object(obj: Any, ctx: DistContext) -> List[Any]:
    """Every rank's picklable host object, in rank order."""
    if not ctx.is_distributed:
        return [obj]
    every: List[Any] = [None] * ctx.world
    dist.all_gather_object(every, obj)
    return every


def broadcast_object(obj: Any, ctx: DistContext, src: int = 0) -> Any:
    if not ctx.is_distributed:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src, device=ctx.device if ctx.backend == "nccl" else None)
    return box[0]


def gather_slabs(own: torch.Tensor, slab: Slab, ctx: DistContext, dst: int = 0) -> Optional[torch.Tensor]:
    """Assemble every rank's owned rows into the full array on ``dst``.

    Slabs differ by at most one row, so each rank pads to the largest slab and
    a single all_gather moves everything; ``dst`` trims and concatenates.
    """
    if not ctx.is_distributed:
        return own
    if _host_staged(own, ctx):
        own = own.cpu()  # gloo control plane: the assembled array comes back on the host
    maxr = max(slab.rows_of(r) for r in range(slab.world))
    pad = torch.zeros((maxr,) + tuple(own.shape[1:]), dtype=own.dtype, device=own.device)
    pad[: own.shape[0]] = own
    parts: List[torch.Tensor] = [torch.empty_like(pad) for _ in range(slab.world)]
    dist.all_gather(parts, pad)
    if ctx.rank != dst:
        return None
    return torch.cat([parts[r][: slab.rows_of(r)] for r in range(slab.world)], dim=0)


def scatter_rows(full: Optional[torch.Tensor], slab: Slab, ctx: DistContext, like: torch.Tensor,
                 src: int = 0) -> torch.Tensor:
    """Inverse of gather_slabs: rank ``src`` holds the full array, every rank
    receives its owned rows (broadcast of the whole array, then slice: fine for
    test-sized data; production runs generate slabs in place)."""
    if not ctx.is_distributed:
        return full[slab.row0: slab.row0 + slab.rows].clone()
    shape = (slab.global_rows,) + tuple(like.shape[1:])
    buf = full.to(like.device).contiguous() if ctx.rank == src else torch.empty(shape, dtype=like.dtype,
                                                                                  device=like.device)
    dist.broadcast(buf, src=src)
    return buf[slab.row0: slab.row0 + slab.rows].clone()
