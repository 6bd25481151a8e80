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
import os
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


# --------------------------------------------------------------------------
# Jacobi: one-sided halos with device-side ordering
# --------------------------------------------------------------------------
def _dbg(ctx: DistContext, msg: str) -> None:
    if os.environ.get("MPX_DEBUG_PEER"):
        import sys
        import time

        print(f"[peer r{ctx.rank} {time.monotonic():.3f}] {msg}", file=sys.stderr, flush=True)


class _JacobiPeerDesc(ctypes.Structure):
    """ctypes mirror of ``mpx_jacobi_peer`` (native/include/mpx/capi.h)."""

    _fields_ = [("up_row", ctypes.c_void_p * 2), ("dn_row", ctypes.c_void_p * 2), ("up_flag", ctypes.c_void_p),
                ("dn_flag", ctypes.c_void_p), ("sync", ctypes.c_void_p), ("spin_limit", ctypes.c_uint)]


# hipIpcOpenMemHandle of one allocation above 2 GiB never returned on the
# MI355X box (ROCm 7 dmabuf path; 2048.5 MiB hung, 1152 MiB mapped in ~1 ms),
# so every IPC-shared allocation stays below this and larger slabs fall back
# to RCCL with a message instead of hanging.
IPC_MAX_BYTES = (2 << 30) - (64 << 20)


class JacobiPeerLink:
    """IPC links of one Jacobi rank to its neighbours' u/u_new buffers and
    completed-iteration words (``mpx_jacobi_peer_sweep``).

    ``storages`` are this rank's two allocations: the first holds ``bufs[0]``
    and the sync block, the second ``bufs[1]`` (each (rows + 2) x cols), each
    below IPC_MAX_BYTES. Each sweep's edge waves read the neighbours' boundary
    rows over xGMI and wait on / publish the iteration counters on the device —
    the host only launches one kernel per iteration (reference: none; SURVEY
    §2.6 / §7.2 step 7 north star).
    """

    def __init__(self, ctx: DistContext, slab: Slab, storages: List[torch.Tensor], bufs: List[torch.Tensor],
                 sync: torch.Tensor):
        self.ctx = ctx
        self.slab = slab
        self.bufs = bufs
        self.sync = sync
        self.row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        self._bases: List[int] = []
        for st in storages:
            nb = st.numel() * st.element_size()
            if nb > IPC_MAX_BYTES:
                raise ValueError(f"slab allocation of {nb / 2**20:.0f} MiB exceeds the {IPC_MAX_BYTES >> 20} MiB IPC "
                                 "mapping limit")
        L = _native.lib()
        mine = []
        for st, parts in ((storages[0], (bufs[0], sync)), (storages[1], (bufs[1],))):
            h = (ctypes.c_char * L.mpx_ipc_handle_size())()
            off = ctypes.c_int64()
            _native.check(L.mpx_ipc_get_handle(st.data_ptr(), h, ctypes.byref(off)))
            mine.append((bytes(h), int(off.value) + (parts[0].data_ptr() - st.data_ptr()),
                         (parts[1].data_ptr() - parts[0].data_ptr()) if len(parts) > 1 else None))
        mine = (mine, slab.rows, self.row_bytes)
        _dbg(ctx, "link: handles taken")
        every: List[Optional[tuple]] = [None] * ctx.world
        dist.all_gather_object(every, mine)
        _dbg(ctx, "link: handles exchanged")
        self._nb = {}
        try:
            for side, r in (("up", ctx.rank - 1), ("dn", ctx.rank + 1)):
                if 0 <= r < ctx.world:
                    (h0, b0, sy_rel), (h1, b1, _), rows, rb = every[r][0][0], every[r][0][1], every[r][1], every[r][2]
                    if rb != self.row_bytes:
                        raise ValueError("neighbour row pitch differs")
                    p0 = self._open(h0) + b0
                    p1 = self._open(h1) + b1
                    _dbg(ctx, f"link: opened {side} neighbour")
                    self._nb[side] = (p0, p1, p0 + sy_rel, rows)
        except Exception:
            self.close()
            raise
        self.desc = _JacobiPeerDesc()

    def _open(self, handle: bytes) -> int:
        L = _native.lib()
        base = ctypes.c_void_p()
        _native.check(L.mpx_ipc_open(handle, ctypes.byref(base)))
        self._bases.append(int(base.value))
        return int(base.value)

    def publish(self, u: torch.Tensor, iteration: int) -> None:
        """Collective, between sweeps: make this rank's buffers visible, set its
        completed-iteration word to ``iteration`` (every rank passes the same
        value) and rebuild the descriptor for the current u/u_new roles."""
        torch.cuda.synchronize(u.device)
        self.sync.zero_()
        self.sync[0] = iteration
        torch.cuda.synchronize(u.device)
        # which buffer is u at even iterations, per rank
        even = 0 if (u.data_ptr() == self.bufs[0].data_ptr()) == (iteration % 2 == 0) else 1
        every: List[Optional[int]] = [None] * self.ctx.world
        dist.all_gather_object(every, even)
        d = _JacobiPeerDesc()
        for side, r in (("up", self.ctx.rank - 1), ("dn", self.ctx.rank + 1)):
            if side not in self._nb:
                continue
            b0, b1, sy, rows = self._nb[side]
            bufs = (b0, b1) if every[r] == 0 else (b1, b0)
            row = rows if side == "up" else 1  # its last / first owned row
            ptrs = [b + row * self.row_bytes for b in bufs]
            if side == "up":
                d.up_row[0], d.up_row[1], d.up_flag = ptrs[0], ptrs[1], sy
            else:
                d.dn_row[0], d.dn_row[1], d.dn_flag = ptrs[0], ptrs[1], sy
        d.sync = self.sync.data_ptr()
        d.spin_limit = int(os.environ.get("MPX_PEER_SPIN_LIMIT", "0"))  # diagnostics: give up sooner
        self.desc = d
        self.ctx.barrier()

    def timed_out(self) -> bool:
        return bool(self.sync[64].item())

    def close(self) -> None:
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []


def try_jacobi_peer(ctx: DistContext, slab: Slab, storages: List[torch.Tensor], bufs: List[torch.Tensor],
                    sync: torch.Tensor, layout_ok: bool) -> Optional[JacobiPeerLink]:
    """Collective: a JacobiPeerLink on every rank, or None on every rank."""
    if ctx.world < 2 or not storages[0].is_cuda or not dist.is_initialized():
        return None
    link, err = None, None
    if not layout_ok:
        err = "columns are not a multiple of the 16-byte vector width"
    else:
        try:
            link = JacobiPeerLink(ctx, slab, storages, bufs, sync)
        except Exception as e:  # noqa: BLE001 - reported below, then everyone falls back
            err = f"{type(e).__name__}: {e}"
    votes: List[Optional[bool]] = [None] * ctx.world
    dist.all_gather_object(votes, link is not None)
    if not all(votes):
        if link is not None:
            link.close()
        if err is not None:
            import sys

            print(f"[peer-halo] rank {ctx.rank}: Jacobi IPC links unavailable ({err}); using RCCL", file=sys.stderr)
        return None
    return link
