"""One-sided halo transport: neighbours' slab rows read directly over xGMI.

The 8 MI355X of a node form a full xGMI mesh with load/store access between
peers. Instead of a two-sided RCCL send/recv per step (a separate RCCL kernel,
~9 µs of launch and handshake for a few tens of KB, profiles/comm_step.md),
each rank maps its neighbours' slab allocations (IPC handles, dmabuf on this
stack) once, and the convolution kernel itself reads the halo rows from the
neighbour's HBM on every step (``mpx_conv_peer``: a wave-uniform row-source
select in the load path). The bytes that cross xGMI per step are the same
2 x halo rows as with send/recv; the extra kernel and its queue slot are gone.

Consistency: a neighbour's rows are read while the step runs, so slab inputs
must be published before the step that reads them — :meth:`publish` (device
sync + barrier), which ``SlabEdgeDetector.load``/``fill_random`` call.
Reference: no multi-GPU code exists there; the decomposition is
the BASELINE north star.
"""

from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native
from .dist import DistContext
from .slab import Slab


class PeerHalo:
    """IPC-mapped neighbour slabs of one rank.

    ``own`` is this rank's owned rows (a (rows, ...) CUDA tensor view whose row
    0 is logical row 0). After construction ``up_ptr`` / ``dn_ptr`` are the
    biased device addresses ``mpx_conv_peer`` takes: logical row g < 0 lives at
    ``up_ptr + g * row_bytes`` (the upper neighbour's last rows), g >= rows at
    ``dn_ptr + g * row_bytes`` (the lower neighbour's first rows).
    """

    def __init__(self, ctx: DistContext, slab: Slab, own: torch.Tensor):
        if not own.is_cuda or not own.is_contiguous():
            raise ValueError("peer halos need a contiguous CUDA slab")
        self.ctx = ctx
        self.slab = slab
        self.own = own
        self.row_bytes = own[0].numel() * own.element_size()
        self._bases: List[int] = []
        L = _native.lib()
        n = L.mpx_ipc_handle_size()
        h = (ctypes.c_char * n)()
        off = ctypes.c_int64()
        _native.check(L.mpx_ipc_get_handle(own.data_ptr(), h, ctypes.byref(off)))
        mine = (bytes(h), int(off.value), slab.rows, self.row_bytes)
        every: List[Optional[tuple]] = [None] * ctx.world
        dist.all_gather_object(every, mine)
        self.up_ptr = own.data_ptr()
        self.dn_ptr = own.data_ptr()
        r = ctx.rank
        try:
            if slab.has_up:
                hb, o, rows_up, rb = every[r - 1]
                assert rb == self.row_bytes, "neighbour row pitch differs"
                self.up_ptr = self._open(hb) + o + rows_up * rb
            if slab.has_down:
                hb, o, _rows, rb = every[r + 1]
                assert rb == self.row_bytes, "neighbour row pitch differs"
                self.dn_ptr = self._open(hb) + o - slab.rows * rb
        except Exception:
            self.close()
            raise

    def _open(self, handle: bytes) -> int:
        L = _native.lib()
        base = ctypes.c_void_p()
        _native.check(L.mpx_ipc_open(handle, ctypes.byref(base)))
        self._bases.append(int(base.value))
        return int(base.value)

    def rows_ptr(self, g: int) -> int:
        """Device address of logical row ``g`` (own or a neighbour's)."""
        if g < 0:
            return self.up_ptr + g * self.row_bytes
        if g >= self.slab.rows:
            return self.dn_ptr + g * self.row_bytes
        return self.own.data_ptr() + g * self.row_bytes

    def pull(self, buf: torch.Tensor) -> None:
        """Copy the halo rows into ``buf`` (a slab buffer with resident halo rows,
        own rows at ``slab.own_offset``) on the current stream — for CPU-side
        verification and for consumers that need a local copy."""
        s = self.slab
        L = _native.lib()
        st = _native.stream_of(buf)
        base = buf.data_ptr() + s.own_offset * self.row_bytes
        for g in list(range(-s.halo_up, 0)) if s.has_up else []:
            _native.check(L.mpx_memcpy_d2d(base + g * self.row_bytes, self.rows_ptr(g), self.row_bytes, st))
        for g in list(range(s.rows, s.rows + s.halo_down)) if s.has_down else []:
            _native.check(L.mpx_memcpy_d2d(base + g * self.row_bytes, self.rows_ptr(g), self.row_bytes, st))

    def verify(self) -> bool:
        """Collective: every rank reads its neighbours' boundary rows through the
        mapping and compares them with what the owners hold."""
        s = self.slab
        dev = self.own.device
        flat = self.own.view(torch.uint8).reshape(s.rows, -1)
        mine = (flat[: max(1, s.halo_down)].to(torch.int64).sum().item(),
                flat[s.rows - max(1, s.halo_up):].to(torch.int64).sum().item())
        every: List[Optional[tuple]] = [None] * self.ctx.world
        dist.all_gather_object(every, mine)
        ok = True
        tmp = torch.empty((max(1, s.halo_up, s.halo_down), self.row_bytes), dtype=torch.uint8, device=dev)
        L = _native.lib()
        st = _native.stream_of(tmp)
        if s.has_up and s.halo_up:
            _native.check(L.mpx_memcpy_d2d(tmp.data_ptr(), self.rows_ptr(-s.halo_up), s.halo_up * self.row_bytes, st))
            ok &= tmp[: s.halo_up].to(torch.int64).sum().item() == every[self.ctx.rank - 1][1]
        if s.has_down and s.halo_down:
            _native.check(L.mpx_memcpy_d2d(tmp.data_ptr(), self.rows_ptr(s.rows), s.halo_down * self.row_bytes, st))
            ok &= tmp[: s.halo_down].to(torch.int64).sum().item() == every[self.ctx.rank + 1][0]
        votes: List[Optional[bool]] = [None] * self.ctx.world
        dist.all_gather_object(votes, bool(ok))
        return all(votes)

    def publish(self) -> None:
        """Make this rank's slab writes visible to the neighbours' next step."""
        torch.cuda.synchronize(self.own.device)
        self.ctx.barrier()

    def close(self) -> None:
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []


def try_peer_halo(ctx: DistContext, slab: Slab, own: torch.Tensor) -> Optional[PeerHalo]:
    """Collective: a verified PeerHalo on every rank, or None on every rank
    (any rank failing to map or read its neighbours -> everyone keeps RCCL)."""
    if ctx.world < 2 or not own.is_cuda or not dist.is_initialized():
        return None
    ph, err = None, None
    try:
        ph = PeerHalo(ctx, slab, own)
    except Exception as e:  # noqa: BLE001 - reported below, then everyone falls back
        err = f"{type(e).__name__}: {e}"
    votes: List[Optional[bool]] = [None] * ctx.world
    dist.all_gather_object(votes, ph is not None)
    if not all(votes):
        if ph is not None:
            ph.close()
        if err is not None:
            import sys

            print(f"[peer-halo] rank {ctx.rank}: IPC mapping unavailable ({err}); using RCCL", file=sys.stderr)
        return None
    ph.publish()
    if not ph.verify():
        ph.close()
        return None
    return ph
