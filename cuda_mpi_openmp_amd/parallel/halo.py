"""Halo exchange between vertically adjacent row slabs over torch.distributed.

With the ``nccl`` backend (RCCL) the four transfers of a rank (send/recv to
the rank above and below) are issued as ONE grouped ``batch_isend_irecv`` —
RCCL point-to-point over the direct xGMI link between the two GPUs. The call
makes RCCL's stream wait only for work already queued on the current stream,
so a caller can queue the halo-independent interior compute right after
:meth:`HaloExchange.start` and overlap it with the transfer; :meth:`wait`
then orders the current stream after the transfer.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

from .dist import DistContext
from ..utils import trace
from .slab import Slab


class HaloExchange:
    """``start``/``wait`` pair; with ``ctx.native`` (the libmpx RCCL tier) the
    same op list runs as one grouped send/recv from C on a comm stream forked
    from the current stream, otherwise through ``batch_isend_irecv``."""

    def __init__(self, slab: Slab, ctx: DistContext):
        self.slab = slab
        self.ctx = ctx
        self._works: List = []
        self._plans: Dict[Tuple[int, Tuple[int, ...]], object] = {}
        self._native_pending = False

    def _ops(self, buf: torch.Tensor):
        s = self.slab
        o = s.own_offset
        ops = []
        if s.has_up and (s.halo_up or s.halo_down):
            up = self.ctx.rank - 1
            if s.halo_down:  # the rank above reads my first halo_down rows
                ops.append(dist.P2POp(dist.isend, buf[o:o + s.halo_down], up))
            if s.halo_up:  # I read its last halo_up rows
                ops.append(dist.P2POp(dist.irecv, buf[0:s.halo_up], up))
        if s.has_down and (s.halo_up or s.halo_down):
            down = self.ctx.rank + 1
            if s.halo_up:  # the rank below reads my last halo_up rows
                ops.append(dist.P2POp(dist.isend, buf[o + s.rows - s.halo_up:o + s.rows], down))
            if s.halo_down:
                ops.append(dist.P2POp(dist.irecv, buf[o + s.rows:o + s.rows + s.halo_down], down))
        return ops

    def start(self, buf: torch.Tensor) -> None:
        if buf.shape[0] != self.slab.buffer_rows:
            raise ValueError("buffer rows do not match the slab")
        if not self.ctx.is_distributed:
            self._works = []
            return
        nc = self.ctx.native
        if nc is not None and buf.is_cuda:
            nc.p2p_start(self._plan(buf))
            self._native_pending = True
            return
        ops = self._ops(buf)
        self._works = dist.batch_isend_irecv(ops) if ops else []

    def wait(self) -> None:
        if self._native_pending:
            self.ctx.native.p2p_wait()
            self._native_pending = False
        for w in self._works:
            w.wait()
        self._works = []

    def exchange(self, buf: torch.Tensor) -> None:
        """Blocking-in-stream exchange: later work on the current stream sees the
        halos. Natively this is one grouped send/recv on the current stream."""
        with trace.range("halo.exchange"):
            nc = self.ctx.native
            if nc is not None and buf.is_cuda:
                nc.p2p(self._plan(buf))
                return
            self.start(buf)
            self.wait()

    def _plan(self, buf: torch.Tensor):
        key = (buf.data_ptr(), tuple(buf.shape))
        plan = self._plans.get(key)
        if plan is None:
            from .native_comm import plan_from_p2p_ops

            plan = self._plans[key] = plan_from_p2p_ops(self._ops(buf))
        return plan
