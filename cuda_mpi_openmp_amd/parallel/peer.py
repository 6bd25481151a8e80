"""One-sided halo transports: neighbours' slab rows read directly over xGMI.

The 8 MI355X of a node form a full xGMI mesh with load/store access between
peers. Instead of a two-sided RCCL send/recv per step (a separate RCCL kernel,
~9 µs of launch and handshake for a few tens of KB, profiles/comm_step.md),
each rank maps its neighbours' slab allocations (IPC handles, dmabuf on this
stack) once, and the kernels read the halo rows from the neighbour's HBM:

* :class:`PeerHalo` — static slab inputs (the conv benchmark): the conv
  kernel itself reads the neighbours' boundary rows on every step
  (``mpx_conv_peer``: a wave-uniform row-source select in the load path);
* :class:`JacobiPeerLink` — device-signalled: per-iteration order comes from
  completed-iteration words in device memory (``mpx_jacobi_peer_sweep``);
* :class:`StreamHaloLink` — the streaming conv (input changes every step): a
  one-workgroup-per-side fetch kernel publishes this rank's step, waits for
  each neighbour to reach it and copies their boundary rows into the local
  halo rows (``mpx_halo_fetch_run``).

Set-up is collective and TIME-BOUNDED everywhere:

* every control-plane exchange runs on a dedicated gloo group with a
  ``MPX_PEER_SETUP_TIMEOUT`` (default 60 s) deadline — a rank that stops
  answering turns into a :class:`PeerSetupError` naming the phase on every
  other rank, never a hang;
* every ``hipIpcOpenMemHandle`` runs on a helper thread with a
  ``MPX_PEER_OPEN_TIMEOUT`` (default 20 s) deadline; a late open counts as a
  failure and every rank falls back to RCCL (the vote below);
* mappings are verified THROUGH THE KERNELS' OWN LOAD PATH before anything
  trusts them — a checksum kernel with the conv's 16-byte buffer loads
  (static rows), or the signalled probe kernel (pattern rows written with the
  production system-scope stores, a released counter, the production bounded
  wait and system-scope loads) — and any mismatch or timeout on any rank
  makes every rank fall back to RCCL, with a note on stderr;
* each phase is logged with a timestamp (``MPX_PEER_LOG_DIR``: one file per
  rank; ``MPX_DEBUG_PEER=1``: stderr), so a stall names its phase.

Fault injection (tests): ``MPX_PEER_INJECT=open_stall@R`` (rank R's IPC open
never returns), ``verify_corrupt@R`` (R reports a wrong checksum),
``probe_corrupt@R`` (R writes a wrong probe pattern).

Limitation of the open deadline: ``open_stall`` sleeps on the
helper thread BEFORE it calls into HIP, so the tests show the vote and the
RCCL fallback are time-bounded when an open is late, not when an open hangs
INSIDE the runtime (as hipIpcOpenMemHandle did for one allocation above 2 GiB,
``profiles/peer_setup.md``). A thread abandoned inside the runtime may hold
HIP or driver locks, and the in-process fallback (closing the other mappings,
RCCL initialisation) is then not shown to be bounded; the job watchdog
(``parallel/fault.py``) still ends such a job. Every allocation these
transports export stays below ``IPC_MAX_BYTES``, the size class that never
hung; a job that does hit an open timeout can be re-run with ``--halo rccl``.

Reference: no multi-GPU code exists there; the decomposition is
the BASELINE north star.
"""

from __future__ import annotations

import ctypes
import datetime
import os
import sys
import threading
import time
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import _native
from .dist import DistContext
from .slab import Slab

SYNC_BYTES = 512            # one sync block: word 0 step/iteration, 32 edge-wave counter, 64 error, 96 mismatches
PROBE_MAGIC = 0x40000000    # probe counter value; iteration / step counters never reach it
W_ERR, W_MISMATCH = 64, 96

# hipIpcOpenMemHandle of one allocation above 2 GiB never returned on the
# MI355X box (ROCm 7 dmabuf path; 2048.5 MiB hung, 1152 MiB mapped in ~1 ms).
# Every IPC-shared allocation stays below this; larger slabs use RCCL with a
# message, and the open itself is deadline-bounded besides (_open_bounded).
IPC_MAX_BYTES = (2 << 30) - (64 << 20)


class PeerSetupError(RuntimeError):
    """A collective step of the peer set-up failed or timed out (no agreement
    on a fallback is possible any more: the job stops loudly instead)."""


def _setup_timeout() -> float:
    return float(os.environ.get("MPX_PEER_SETUP_TIMEOUT", "60"))


def _open_timeout() -> float:
    return float(os.environ.get("MPX_PEER_OPEN_TIMEOUT", "20"))


def _injected(kind: str, rank: int) -> bool:
    spec = os.environ.get("MPX_PEER_INJECT", "")
    return any(tok.strip() == f"{kind}@{rank}" for tok in spec.split(",") if tok.strip())


# --------------------------------------------------------------------------
# phase log
# --------------------------------------------------------------------------
_last_phase: dict = {}


def phase(ctx: DistContext, msg: str) -> None:
    """Record a set-up phase: MPX_PEER_LOG_DIR/peer_rank<r>.log (append) and,
    with MPX_DEBUG_PEER=1, stderr."""
    t = time.monotonic()
    _last_phase[ctx.rank] = msg
    line = f"[peer r{ctx.rank} {t:.3f}] {msg}"
    d = os.environ.get("MPX_PEER_LOG_DIR")
    if d:
        try:
            with open(os.path.join(d, f"peer_rank{ctx.rank}.log"), "a") as f:
                f.write(line + "\n")
        except OSError:
            pass
    if os.environ.get("MPX_DEBUG_PEER"):
        print(line, file=sys.stderr, flush=True)


def last_phase(rank: int) -> Optional[str]:
    return _last_phase.get(rank)


# --------------------------------------------------------------------------
# bounded control plane
# --------------------------------------------------------------------------
_GROUP = {"g": None, "key": None}


def _setup_group(ctx: DistContext):
    """A gloo group with the set-up deadline (created collectively, once per
    process group)."""
    key = id(dist.group.WORLD)
    if _GROUP["g"] is None or _GROUP["key"] != key:
        phase(ctx, "setup group: create")
        _GROUP["g"] = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=_setup_timeout()))
        _GROUP["key"] = key
    return _GROUP["g"]


def _allgather(ctx: DistContext, obj, what: str) -> list:
    g = _setup_group(ctx)
    phase(ctx, f"{what}: all_gather enter")
    out: List[Optional[object]] = [None] * ctx.world
    try:
        dist.all_gather_object(out, obj, group=g)
    except Exception as e:  # noqa: BLE001 - timeouts and dead peers alike
        phase(ctx, f"{what}: all_gather FAILED ({type(e).__name__})")
        raise PeerSetupError(f"rank {ctx.rank}: peer set-up step '{what}' failed or timed out "
                             f"(deadline {_setup_timeout():.0f} s): {type(e).__name__}: {e}") from e
    phase(ctx, f"{what}: all_gather done")
    return out


def _agree(ctx: DistContext, ok: bool, what: str) -> bool:
    return all(bool(v) for v in _allgather(ctx, bool(ok), what))


def _note(ctx: DistContext, msg: str) -> None:
    phase(ctx, msg)
    print(f"[peer-halo] rank {ctx.rank}: {msg}", file=sys.stderr, flush=True)


# --------------------------------------------------------------------------
# IPC helpers
# --------------------------------------------------------------------------
def _get_handle(ptr: int) -> tuple:
    L = _native.lib()
    h = (ctypes.c_char * L.mpx_ipc_handle_size())()
    off = ctypes.c_int64()
    _native.check(L.mpx_ipc_get_handle(ptr, h, ctypes.byref(off)))
    return bytes(h), int(off.value)


def _open_bounded(ctx: DistContext, handle: bytes, device: int, what: str) -> int:
    """hipIpcOpenMemHandle on a helper thread, bounded by MPX_PEER_OPEN_TIMEOUT.
    A late open is abandoned (and closed by the helper if it ever returns)."""
    L = _native.lib()
    lock = threading.Lock()
    st: dict = {"done": False, "abandoned": False}
    stall = _injected("open_stall", ctx.rank)

    def work():
        if stall:
            time.sleep(3600.0)
        base = ctypes.c_void_p()
        rc = L.mpx_ipc_open_dev(device, handle, ctypes.byref(base))
        err = L.mpx_last_error() if rc else None  # thread-local message
        with lock:
            st.update(done=True, rc=rc, base=base.value, err=err)
            late = st["abandoned"]
        if late and rc == 0:
            L.mpx_ipc_close(base)

    phase(ctx, f"ipc open {what}: start")
    t = threading.Thread(target=work, name=f"mpx-ipc-open-{what}", daemon=True)
    t.start()
    t.join(_open_timeout())
    with lock:
        if not st["done"]:
            st["abandoned"] = True
            phase(ctx, f"ipc open {what}: TIMED OUT after {_open_timeout():.0f} s")
            raise TimeoutError(f"hipIpcOpenMemHandle ({what}) did not return within {_open_timeout():.0f} s")
    if st["rc"]:
        raise _native.MpxError(st["err"].decode() if st["err"] else f"mpx_ipc_open_dev rc {st['rc']}")
    phase(ctx, f"ipc open {what}: done")
    return int(st["base"])


class SyncBlock:
    """A SYNC_BYTES device block for counters, IPC-exportable: uncached memory
    when the stack can export it (kind 2), else fine-grained (1), else coarse
    (0) — ``mpx_sync_alloc``."""

    KINDS = {2: "uncached", 1: "fine-grained", 0: "coarse-grained"}

    def __init__(self):
        L = _native.lib()
        p = ctypes.c_void_p()
        k = ctypes.c_int()
        _native.check(L.mpx_sync_alloc(SYNC_BYTES, ctypes.byref(p), ctypes.byref(k)))
        self.ptr = int(p.value)
        self.kind = self.KINDS.get(int(k.value), "?")

    def read(self, word: int) -> int:
        v = ctypes.c_uint()
        _native.check(_native.lib().mpx_sync_read(self.ptr, word, ctypes.byref(v)))
        return int(v.value)

    def write(self, word: int, value: int) -> None:
        _native.check(_native.lib().mpx_sync_write(self.ptr, word, value))

    def clear(self) -> None:
        _native.check(_native.lib().mpx_sync_clear(self.ptr, SYNC_BYTES))

    def free(self) -> None:
        if self.ptr:
            _native.lib().mpx_sync_free(self.ptr)
            self.ptr = 0


class _ProbeDesc(ctypes.Structure):
    """ctypes mirror of ``mpx_peer_probe`` (native/include/mpx/capi.h)."""

    _fields_ = [("own_rows", ctypes.c_void_p * 4), ("nb_rows", (ctypes.c_void_p * 2) * 2),
                ("flag", ctypes.c_void_p * 2), ("sync", ctypes.c_void_p), ("row_bytes", ctypes.c_int64),
                ("rank", ctypes.c_int), ("magic", ctypes.c_uint), ("spin_limit", ctypes.c_uint)]


def _signalled_probe(ctx: DistContext, device: torch.device, sync: SyncBlock, own_rows: Sequence[Optional[int]],
                     nb_rows: dict, nb_flags: dict, row_bytes: int) -> bool:
    """Run the signalled probe kernel on this rank (collective in effect: it
    waits for the neighbours' probe counters) and return this rank's verdict.
    nb_rows/nb_flags: {"up"|"dn": ([row of buffer 0, row of buffer 1], flag ptr)}."""
    d = _ProbeDesc()
    for q, r in enumerate(own_rows):
        d.own_rows[q] = r or None
    for s, side in enumerate(("up", "dn")):
        if side in nb_rows:
            d.nb_rows[s][0], d.nb_rows[s][1] = nb_rows[side][0], nb_rows[side][1]
            d.flag[s] = nb_flags[side]
    d.sync = sync.ptr
    d.row_bytes = row_bytes
    # an injected corruption writes another rank's pattern: the neighbours must see it
    d.rank = ctx.rank + (1000 if _injected("probe_corrupt", ctx.rank) else 0)
    d.magic = PROBE_MAGIC
    d.spin_limit = int(os.environ.get("MPX_PEER_SPIN_LIMIT", "0"))
    phase(ctx, "probe: launch")
    with torch.cuda.device(device):
        _native.check(_native.lib().mpx_peer_probe_run(ctypes.byref(d), torch.cuda.current_stream(device).cuda_stream))
        torch.cuda.synchronize(device)
    err, bad = sync.read(W_ERR), sync.read(W_MISMATCH)
    phase(ctx, f"probe: done (timeout={err}, mismatched words={bad})")
    if err or bad:
        _note(ctx, f"signalled probe failed (wait gave up: {bool(err)}, mismatched words: {bad})")
    return not err and not bad


def _rows_checksum(ptr: int, row_bytes: int, nrows: int, device: torch.device) -> int:
    out = torch.zeros(1, dtype=torch.int64, device=device)
    _native.check(_native.lib().mpx_rows_checksum(ptr, row_bytes, nrows, row_bytes, 0, out.data_ptr(),
                                                  torch.cuda.current_stream(device).cuda_stream))
    return int(out.item()) & (2**64 - 1)


# --------------------------------------------------------------------------
# static slabs (conv)
# --------------------------------------------------------------------------
class PeerHalo:
    """IPC-mapped neighbour slabs of one rank (static inputs).

    ``own`` is this rank's owned rows (a (rows, ...) CUDA tensor view whose row
    0 is logical row 0). After construction ``up_ptr`` / ``dn_ptr`` are the
    biased device addresses ``mpx_conv_peer`` takes: logical row g < 0 lives at
    ``up_ptr + g * row_bytes`` (the upper neighbour's last rows), g >= rows at
    ``dn_ptr + g * row_bytes`` (the lower neighbour's first rows).

    Construction maps (locally bounded) after a handle exchange the caller has
    done; :func:`try_peer_halo` is the collective entry point.
    """

    def __init__(self, ctx: DistContext, slab: Slab, own: torch.Tensor, every: list):
        self.ctx = ctx
        self.slab = slab
        self.own = own
        self.row_bytes = own[0].numel() * own.element_size()
        self._bases: List[int] = []
        self.up_ptr = own.data_ptr()
        self.dn_ptr = own.data_ptr()
        r = ctx.rank
        dev = own.device.index
        try:
            if slab.has_up:
                if every[r - 1] is None:
                    raise RuntimeError("upper neighbour exported no handle")
                hb, o, rows_up, rb = every[r - 1]
                if rb != self.row_bytes:
                    raise ValueError("neighbour row pitch differs")
                self.up_ptr = self._open(hb, dev, "up") + o + rows_up * rb
            if slab.has_down:
                if every[r + 1] is None:
                    raise RuntimeError("lower neighbour exported no handle")
                hb, o, _rows, rb = every[r + 1]
                if rb != self.row_bytes:
                    raise ValueError("neighbour row pitch differs")
                self.dn_ptr = self._open(hb, dev, "down") - slab.rows * rb + o
        except Exception:
            self.close()
            raise

    def _open(self, handle: bytes, device: int, what: str) -> int:
        base = _open_bounded(self.ctx, handle, device, what)
        self._bases.append(base)
        return base

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
        """Collective: every rank reads its neighbours' boundary rows through
        the mapping with the conv kernels' 16-byte buffer loads (checksum
        kernel) and compares with the owners' checksums of the same rows."""
        s = self.slab
        dev = self.own.device
        nd, nu = max(1, s.halo_down), max(1, s.halo_up)
        torch.cuda.synchronize(dev)
        first = _rows_checksum(self.own.data_ptr(), self.row_bytes, min(nd, s.rows), dev)
        last = _rows_checksum(self.own.data_ptr() + (s.rows - min(nu, s.rows)) * self.row_bytes, self.row_bytes,
                              min(nu, s.rows), dev)
        if _injected("verify_corrupt", self.ctx.rank):
            first, last = first ^ 1, last ^ 1
        every = _allgather(self.ctx, (first, last), "verify: owner checksums")
        ok = True
        if s.has_up and s.halo_up:
            got = _rows_checksum(self.rows_ptr(-s.halo_up), self.row_bytes, s.halo_up, dev)
            ok &= got == every[self.ctx.rank - 1][1]
        if s.has_down and s.halo_down:
            got = _rows_checksum(self.rows_ptr(s.rows), self.row_bytes, s.halo_down, dev)
            ok &= got == every[self.ctx.rank + 1][0]
        phase(self.ctx, f"verify: kernel-path checksums {'match' if ok else 'DIFFER'}")
        return _agree(self.ctx, ok, "verify: vote")

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
    (any rank failing to export, map — within its deadline — or read its
    neighbours through the kernel load path -> everyone keeps RCCL)."""
    if ctx.world < 2 or not own.is_cuda or not dist.is_initialized():
        return None
    phase(ctx, "conv peer set-up: begin")
    mine, err = None, None
    try:
        if not own.is_contiguous():
            raise ValueError("peer halos need a contiguous CUDA slab")
        hb, off = _get_handle(own.data_ptr())
        mine = (hb, off, slab.rows, own[0].numel() * own.element_size())
    except Exception as e:  # noqa: BLE001 - reported below, then everyone falls back
        err = f"{type(e).__name__}: {e}"
    every = _allgather(ctx, mine, "conv: handles")
    ph = None
    if mine is not None:
        try:
            ph = PeerHalo(ctx, slab, own, every)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    if not _agree(ctx, ph is not None, "conv: map vote"):
        if ph is not None:
            ph.close()
        _note(ctx, f"IPC mapping unavailable ({err or 'a neighbour failed'}); using RCCL")
        return None
    ph.publish()
    if not ph.verify():
        ph.close()
        _note(ctx, "kernel-path verification of the mapped halo rows failed; using RCCL")
        return None
    phase(ctx, "conv peer set-up: ok")
    return ph


# --------------------------------------------------------------------------
# Jacobi: one-sided halos with device-side ordering
# --------------------------------------------------------------------------
class _JacobiPeerDesc(ctypes.Structure):
    """ctypes mirror of ``mpx_jacobi_peer`` (native/include/mpx/capi.h)."""

    _fields_ = [("up_row", ctypes.c_void_p * 2), ("dn_row", ctypes.c_void_p * 2), ("up_flag", ctypes.c_void_p),
                ("dn_flag", ctypes.c_void_p), ("sync", ctypes.c_void_p), ("spin_limit", ctypes.c_uint)]


class JacobiPeerLink:
    """IPC links of one Jacobi rank to its neighbours' u/u_new buffers and
    completed-iteration words (``mpx_jacobi_peer_sweep``).

    ``storages`` are this rank's two buffer allocations (``bufs[0]`` and
    ``bufs[1]``, each (rows + 2) x cols), each below IPC_MAX_BYTES; the
    iteration words live in a separate :class:`SyncBlock` (uncached memory
    where exportable). Each sweep's edge waves read the neighbours' boundary
    rows over xGMI and wait on / publish the iteration counters on the device
    — the host only launches one kernel per iteration (reference: none;
    SURVEY §2.6 / §7.2 step 7 north star). Built by :func:`try_jacobi_peer`.
    """

    def __init__(self, ctx: DistContext, slab: Slab, bufs: List[torch.Tensor], sync: SyncBlock, every: list):
        self.ctx = ctx
        self.slab = slab
        self.bufs = bufs
        self.sync = sync
        self.row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        self._bases: List[int] = []
        self._nb = {}
        dev = bufs[0].device.index
        try:
            for side, r in (("up", ctx.rank - 1), ("dn", ctx.rank + 1)):
                if 0 <= r < ctx.world:
                    if every[r] is None:
                        raise RuntimeError(f"{side} neighbour exported no handles")
                    (h0, b0), (h1, b1), (hs, bs), rows, rb = every[r]
                    if rb != self.row_bytes:
                        raise ValueError("neighbour row pitch differs")
                    p0 = self._open(h0, dev, f"{side} u0") + b0
                    p1 = self._open(h1, dev, f"{side} u1") + b1
                    ps = self._open(hs, dev, f"{side} sync") + bs
                    self._nb[side] = (p0, p1, ps, rows)
        except Exception:
            self.close(free_sync=False)
            raise
        self.desc = _JacobiPeerDesc()

    def _open(self, handle: bytes, device: int, what: str) -> int:
        base = _open_bounded(self.ctx, handle, device, what)
        self._bases.append(base)
        return base

    def probe(self) -> bool:
        """Signalled kernel-path probe over both buffers' shared rows (this
        rank's verdict; the caller votes). Scribbles on rows 1 and n of both
        buffers: run before the field is initialised."""
        rb, n = self.row_bytes, self.slab.rows
        own = [self.bufs[0].data_ptr() + rb, self.bufs[0].data_ptr() + n * rb,
               self.bufs[1].data_ptr() + rb, self.bufs[1].data_ptr() + n * rb]
        nb_rows, nb_flags = {}, {}
        for side, (p0, p1, ps, rows) in self._nb.items():
            row = rows if side == "up" else 1  # its last / first owned row
            nb_rows[side] = [p0 + row * rb, p1 + row * rb]
            nb_flags[side] = ps
        self.sync.clear()
        return _signalled_probe(self.ctx, self.bufs[0].device, self.sync, own, nb_rows, nb_flags, rb)

    def publish(self, u: torch.Tensor, iteration: int) -> None:
        """Collective, between sweeps (every rank's earlier sweeps finished —
        the caller synchronised and passed a barrier): reset this rank's sync
        words, set its completed-iteration word to ``iteration`` (every rank
        passes the same value) and rebuild the descriptor for the current
        u/u_new roles."""
        torch.cuda.synchronize(u.device)
        self.sync.clear()
        self.sync.write(0, iteration)
        # which buffer is u at even iterations, per rank
        even = 0 if (u.data_ptr() == self.bufs[0].data_ptr()) == (iteration % 2 == 0) else 1
        every = _allgather(self.ctx, even, "jacobi: publish parity")
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
        d.sync = self.sync.ptr
        d.spin_limit = int(os.environ.get("MPX_PEER_SPIN_LIMIT", "0"))  # diagnostics: give up sooner
        self.desc = d
        _agree(self.ctx, True, "jacobi: publish done")

    def timed_out(self) -> bool:
        return bool(self.sync.read(W_ERR))

    def close(self, free_sync: bool = True) -> None:
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []
        if free_sync:
            self.sync.free()


def try_jacobi_peer(ctx: DistContext, slab: Slab, storages: List[torch.Tensor], bufs: List[torch.Tensor],
                    layout_ok: bool) -> Optional[JacobiPeerLink]:
    """Collective: a mapped AND probed JacobiPeerLink on every rank, or None on
    every rank (export, bounded map, or the signalled kernel-path probe
    failing anywhere -> everyone keeps RCCL)."""
    if ctx.world < 2 or not storages[0].is_cuda or not dist.is_initialized():
        return None
    phase(ctx, "jacobi peer set-up: begin")
    mine, err, sync = None, None, None
    try:
        if not layout_ok:
            raise ValueError("columns are not a multiple of the 16-byte vector width")
        for st in storages:
            nb = st.numel() * st.element_size()
            if nb > IPC_MAX_BYTES:
                raise ValueError(f"slab allocation of {nb / 2**20:.0f} MiB exceeds the {IPC_MAX_BYTES >> 20} MiB "
                                 "IPC mapping limit")
        sync = SyncBlock()
        parts = []
        for st, t in ((storages[0], bufs[0]), (storages[1], bufs[1])):
            h, off = _get_handle(st.data_ptr())
            parts.append((h, off + (t.data_ptr() - st.data_ptr())))
        parts.append(_get_handle(sync.ptr))
        row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        mine = (parts[0], parts[1], parts[2], slab.rows, row_bytes)
        phase(ctx, f"jacobi: sync block is {sync.kind} memory")
    except Exception as e:  # noqa: BLE001 - reported below, then everyone falls back
        err = f"{type(e).__name__}: {e}"
    every = _allgather(ctx, mine, "jacobi: handles")
    link = None
    if mine is not None:
        try:
            link = JacobiPeerLink(ctx, slab, bufs, sync, every)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    if not _agree(ctx, link is not None, "jacobi: map vote"):
        if link is not None:
            link.close()
        elif sync is not None:
            sync.free()
        _note(ctx, f"Jacobi IPC links unavailable ({err or 'a neighbour failed'}); using RCCL")
        return None
    ok = link.probe()
    agreed = _agree(ctx, ok, "jacobi: probe vote")
    for b in bufs:  # the probe wrote patterns into the shared rows (either outcome)
        b.zero_()
    if not agreed:
        link.close()
        _note(ctx, "signalled kernel-path probe failed on some rank; using RCCL")
        return None
    phase(ctx, "jacobi peer set-up: ok")
    return link


# --------------------------------------------------------------------------
# streaming conv: device-signalled halo fetch per step
# --------------------------------------------------------------------------
class _HaloFetchDesc(ctypes.Structure):
    """ctypes mirror of ``mpx_halo_fetch`` (native/include/mpx/capi.h)."""

    _fields_ = [("src", ctypes.c_void_p * 2), ("dst", ctypes.c_void_p * 2), ("bytes", ctypes.c_int64 * 2),
                ("flag", ctypes.c_void_p * 2), ("sync", ctypes.c_void_p), ("step", ctypes.c_uint),
                ("spin_limit", ctypes.c_uint)]


class StreamHaloLink:
    """Per-step halo fetch for a slab whose input changes every step (two
    ping-pong input buffers, each (buffer_rows, ...) with the owned rows at
    ``slab.own_offset``). Step k (1-based) reads buffer (k-1) % 2: the fetch
    kernel publishes k, waits until each neighbour published k (it finished
    step k-1, so its rows of this buffer are written, and it finished its
    fetch of step k-1, so it no longer reads ours of the buffer this step
    overwrites — a one-sided window waits on the side it does not read from
    for exactly this), then copies the neighbours' boundary rows into this
    rank's halo rows. Built by :func:`try_stream_halo`."""

    def __init__(self, ctx: DistContext, slab: Slab, bufs: List[torch.Tensor], sync: SyncBlock, every: list):
        self.ctx = ctx
        self.slab = slab
        self.bufs = bufs
        self.sync = sync
        self.row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        self._bases: List[int] = []
        self._nb = {}
        dev = bufs[0].device.index
        try:
            for side, r in (("up", ctx.rank - 1), ("dn", ctx.rank + 1)):
                if 0 <= r < ctx.world:
                    if every[r] is None:
                        raise RuntimeError(f"{side} neighbour exported no handles")
                    (h0, b0), (h1, b1), (hs, bs), rows, own_off, rb = every[r]
                    if rb != self.row_bytes:
                        raise ValueError("neighbour row pitch differs")
                    p0 = self._open(h0, dev, f"{side} buf0") + b0
                    p1 = self._open(h1, dev, f"{side} buf1") + b1
                    ps = self._open(hs, dev, f"{side} sync") + bs
                    self._nb[side] = (p0, p1, ps, rows, own_off)
        except Exception:
            self.close(free_sync=False)
            raise
        self._descs: List[_HaloFetchDesc] = []
        s, rb = slab, self.row_bytes
        any_halo = s.halo_up > 0 or s.halo_down > 0
        for k in range(2):  # one descriptor per buffer parity; only `step` changes
            d = _HaloFetchDesc()
            if "up" in self._nb and any_halo:
                p0, p1, ps, rows, off = self._nb["up"]
                d.flag[0] = ps  # waited on even without rows to copy (it may read ours)
                if s.halo_up:
                    d.src[0] = (p0, p1)[k] + (off + rows - s.halo_up) * rb  # its last halo_up owned rows
                    d.dst[0] = bufs[k].data_ptr() + (s.own_offset - s.halo_up) * rb
                    d.bytes[0] = s.halo_up * rb
            if "dn" in self._nb and any_halo:
                p0, p1, ps, rows, off = self._nb["dn"]
                d.flag[1] = ps
                if s.halo_down:
                    d.src[1] = (p0, p1)[k] + off * rb  # its first halo_down owned rows
                    d.dst[1] = bufs[k].data_ptr() + (s.own_offset + s.rows) * rb
                    d.bytes[1] = s.halo_down * rb
            d.sync = sync.ptr
            d.spin_limit = int(os.environ.get("MPX_PEER_SPIN_LIMIT", "0"))
            self._descs.append(d)

    def _open(self, handle: bytes, device: int, what: str) -> int:
        base = _open_bounded(self.ctx, handle, device, what)
        self._bases.append(base)
        return base

    def probe(self) -> bool:
        rb, s = self.row_bytes, self.slab
        own = [b.data_ptr() + (s.own_offset + r) * rb for b in self.bufs for r in (0, s.rows - 1)]
        nb_rows, nb_flags = {}, {}
        for side, (p0, p1, ps, rows, off) in self._nb.items():
            row = off + rows - 1 if side == "up" else off
            nb_rows[side] = [p0 + row * rb, p1 + row * rb]
            nb_flags[side] = ps
        self.sync.clear()
        ok = _signalled_probe(self.ctx, self.bufs[0].device, self.sync, own, nb_rows, nb_flags, rb)
        return ok

    def reset(self) -> None:
        """Collective between runs: every rank's step word back to 0 (callers
        synchronise and pass a barrier first)."""
        torch.cuda.synchronize(self.bufs[0].device)
        self.sync.clear()
        _agree(self.ctx, True, "stream: reset")

    def fetch(self, step: int, stream: int) -> None:
        """Halo rows of buffer (step - 1) % 2 for step ``step`` (1-based)."""
        d = self._descs[(step - 1) % 2]
        d.step = step
        _native.check(_native.lib().mpx_halo_fetch_run(ctypes.byref(d), stream))

    def timed_out(self) -> bool:
        return bool(self.sync.read(W_ERR))

    def close(self, free_sync: bool = True) -> None:
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []
        if free_sync:
            self.sync.free()


def try_stream_halo(ctx: DistContext, slab: Slab, bufs: List[torch.Tensor]) -> Optional[StreamHaloLink]:
    """Collective: a mapped and probed StreamHaloLink on every rank, or None on
    every rank (-> RCCL halos)."""
    if ctx.world < 2 or not bufs[0].is_cuda or not dist.is_initialized():
        return None
    phase(ctx, "stream peer set-up: begin")
    mine, err, sync = None, None, None
    rb = bufs[0][0].numel() * bufs[0].element_size()
    try:
        sync = SyncBlock()
        mine = (_get_handle(bufs[0].data_ptr()), _get_handle(bufs[1].data_ptr()), _get_handle(sync.ptr),
                slab.rows, slab.own_offset, rb)
        phase(ctx, f"stream: sync block is {sync.kind} memory")
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    every = _allgather(ctx, mine, "stream: handles")
    link = None
    if mine is not None:
        try:
            link = StreamHaloLink(ctx, slab, bufs, sync, every)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    if not _agree(ctx, link is not None, "stream: map vote"):
        if link is not None:
            link.close()
        elif sync is not None:
            sync.free()
        _note(ctx, f"streaming peer halos unavailable ({err or 'a neighbour failed'}); using RCCL")
        return None
    ok = link.probe()
    agreed = _agree(ctx, ok, "stream: probe vote")
    for b in bufs:  # the probe wrote patterns into the shared rows (either outcome)
        b.zero_()
    if not agreed:
        link.close()
        _note(ctx, "signalled kernel-path probe failed on some rank; using RCCL")
        return None
    link.reset()
    phase(ctx, "stream peer set-up: ok")
    return link
