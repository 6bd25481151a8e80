"""One-sided halo transports: neighbours' boundary rows read directly over xGMI.

The 8 MI355X of a node form a full xGMI mesh with load/store access between
peers. Instead of a two-sided RCCL send/recv per step (a separate RCCL kernel,
~9 µs of launch and handshake for a few tens of KB, profiles/comm_step.md),
each rank exports ONE small :class:`Mailbox` (its step / iteration words plus
two parity slots of its boundary rows; IPC handles, dmabuf on this stack), its
neighbours map it once, and the kernels read the halo rows from the
neighbour's HBM. The slabs themselves are never shared, so their size is not
bounded by any IPC limit:

* :class:`PeerHalo` — static slab inputs (the conv benchmark): the conv
  kernel itself reads the neighbours' mailbox rows on every step
  (``mpx_conv_peer``: a wave-uniform row-source select in the load path);
* :class:`JacobiPeerLink` — device-signalled: per-iteration order comes from
  completed-iteration words in the mailboxes (``mpx_jacobi_peer_sweep``); the
  edge waves write their new edge rows write-through into the mailbox;
* :class:`StreamHaloLink` — the streaming conv (input changes every step):
  fused into the band kernel (one launch per step; only edge waves wait) or,
  for other shapes, a one-workgroup-per-side fetch kernel.

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
``probe_corrupt@R`` (R writes a wrong probe pattern), ``map_fail@R`` (R's
mapping of its neighbours' mailboxes fails — in every set-up: conv, streaming
conv and Jacobi —, so every rank must agree on RCCL).

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
# Only mailboxes are exported now (tens to hundreds of KiB), far below it; the
# open itself is deadline-bounded besides (_open_bounded).
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

    def __init__(self, nbytes: int = SYNC_BYTES):
        L = _native.lib()
        p = ctypes.c_void_p()
        k = ctypes.c_int()
        _native.check(L.mpx_sync_alloc(nbytes, ctypes.byref(p), ctypes.byref(k)))
        self.ptr = int(p.value)
        self.nbytes = nbytes
        self.kind = self.KINDS.get(int(k.value), "?")

    def read(self, word: int) -> int:
        v = ctypes.c_uint()
        _native.check(_native.lib().mpx_sync_read(self.ptr, word, ctypes.byref(v)))
        return int(v.value)

    def write(self, word: int, value: int) -> None:
        _native.check(_native.lib().mpx_sync_write(self.ptr, word, value))

    def clear(self) -> None:
        """Zero the counter words (the first SYNC_BYTES)."""
        _native.check(_native.lib().mpx_sync_clear(self.ptr, SYNC_BYTES))

    def free(self) -> None:
        if self.ptr:
            _native.lib().mpx_sync_free(self.ptr)
            self.ptr = 0


def _mb_first(base: int, p: int, rb: int, nf: int, nl: int) -> int:
    """Address of slot ``p``'s first-rows region of a mailbox at ``base``."""
    return base + SYNC_BYTES + p * (nf + nl) * rb


def _mb_last(base: int, p: int, rb: int, nf: int, nl: int) -> int:
    return _mb_first(base, p, rb, nf, nl) + nf * rb


class Mailbox(SyncBlock):
    """This rank's exported mailbox: ONE small allocation
    holding the sync block (counters) followed by two parity slots, each with
    this rank's first ``n_first`` rows (read by the rank above) and last
    ``n_last`` rows (read by the rank below). The neighbours IPC-map only the
    mailbox, never the slab, so the one-sided transports work for slabs of
    any size (sized for 288 GB of HBM) and the >2 GiB IPC-open hang of round 2
    (``profiles/peer_setup.md``) cannot be reached: a mailbox is tens to
    hundreds of KiB. Region sizes are at least one row (the start-up probe
    writes one row into each). The memory is the sync block's: uncached where
    exportable, so the protocol's write-through stores and system-scope loads
    never meet a stale cache line."""

    def __init__(self, row_bytes: int, n_first: int, n_last: int):
        self.rb = int(row_bytes)
        self.nf = max(1, int(n_first))
        self.nl = max(1, int(n_last))
        super().__init__(SYNC_BYTES + 2 * (self.nf + self.nl) * self.rb)

    def first(self, p: int) -> int:
        return _mb_first(self.ptr, p, self.rb, self.nf, self.nl)

    def last(self, p: int) -> int:
        return _mb_last(self.ptr, p, self.rb, self.nf, self.nl)

    def export(self) -> tuple:
        """(IPC handle, offset, row bytes, first rows, last rows) for the neighbours."""
        h, off = _get_handle(self.ptr)
        return (h, off, self.rb, self.nf, self.nl)

    def put(self, p: int, first_src: Optional[int], last_src: Optional[int], n_first: int, n_last: int,
            stream: int) -> None:
        """Stream-ordered copies of this rank's boundary rows into slot ``p``."""
        L = _native.lib()
        if first_src is not None and n_first > 0:
            _native.check(L.mpx_memcpy_d2d(self.first(p), first_src, n_first * self.rb, stream))
        if last_src is not None and n_last > 0:
            _native.check(L.mpx_memcpy_d2d(self.last(p), last_src, n_last * self.rb, stream))


class MappedMailbox:
    """A neighbour's mailbox, mapped into this process (same layout)."""

    def __init__(self, base: int, rb: int, nf: int, nl: int):
        self.base, self.rb, self.nf, self.nl = base, rb, nf, nl
        self.sync = base

    def first(self, p: int) -> int:
        return _mb_first(self.base, p, self.rb, self.nf, self.nl)

    def last(self, p: int) -> int:
        return _mb_last(self.base, p, self.rb, self.nf, self.nl)


def _retire(ctx: DistContext, device: torch.device, what: str) -> None:
    """Before a rank frees its mailbox: its own queued work is done and every
    rank has reached the same point (a neighbour's last step may still read
    the mailbox). Bounded (the set-up group's deadline); on a timeout the
    caller frees anyway — the job is failing already."""
    torch.cuda.synchronize(device)
    try:
        _agree(ctx, True, f"{what}: retire")
    except PeerSetupError:
        pass


def _map_neighbours(ctx: DistContext, every: list, rb: int, opener) -> dict:
    """{"up"|"dn": MappedMailbox} for the ranks above / below (``opener(handle,
    what)`` maps an IPC handle, bounded)."""
    out = {}
    for side, r in (("up", ctx.rank - 1), ("dn", ctx.rank + 1)):
        if 0 <= r < ctx.world:
            if every[r] is None:
                raise RuntimeError(f"{side} neighbour exported no mailbox")
            h, off, nrb, nf, nl = every[r]
            if nrb != rb:
                raise ValueError("neighbour row pitch differs")
            out[side] = MappedMailbox(opener(h, f"{side} mailbox") + off, nrb, nf, nl)
    return out


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
    """Mailbox-backed neighbour rows of one rank (static inputs).

    ``own`` is this rank's owned rows (a (rows, ...) CUDA tensor view whose row
    0 is logical row 0). :meth:`publish` copies its boundary rows into this
    rank's mailbox (slot 0); after construction ``up_ptr`` / ``dn_ptr`` are the
    biased device addresses ``mpx_conv_peer`` takes: logical row g < 0 lives at
    ``up_ptr + g * row_bytes`` (the upper neighbour's last rows, in ITS
    mailbox), g >= rows at ``dn_ptr + g * row_bytes`` (the lower neighbour's
    first rows).

    Construction maps (locally bounded) after a handle exchange the caller has
    done; :func:`try_peer_halo` is the collective entry point.
    """

    def __init__(self, ctx: DistContext, slab: Slab, own: torch.Tensor, mailbox: Mailbox, every: list):
        self.ctx = ctx
        self.slab = slab
        self.own = own
        self.mailbox = mailbox
        self.row_bytes = own[0].numel() * own.element_size()
        self._bases: List[int] = []
        self.up_ptr = own.data_ptr()
        self.dn_ptr = own.data_ptr()
        try:
            self._nb = _map_neighbours(ctx, every, self.row_bytes,
                                       lambda h, what: self._open(h, own.device.index, what))
            if "up" in self._nb:
                m = self._nb["up"]
                if m.nl < slab.halo_up:
                    raise ValueError("upper neighbour's mailbox holds fewer rows than the halo")
                self.up_ptr = m.last(0) + slab.halo_up * self.row_bytes
            if "dn" in self._nb:
                m = self._nb["dn"]
                if m.nf < slab.halo_down:
                    raise ValueError("lower neighbour's mailbox holds fewer rows than the halo")
                self.dn_ptr = m.first(0) - slab.rows * self.row_bytes
        except Exception:
            self.close(collective=False)
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
        """Make this rank's slab writes visible to the neighbours' next step:
        its boundary rows into the mailbox, then every rank synchronised."""
        s, rb = self.slab, self.row_bytes
        st = _native.stream_of(self.own)
        nf, nl = min(s.halo_down, s.rows), min(s.halo_up, s.rows)
        self.mailbox.put(0, self.own.data_ptr() if s.has_up else None,
                         self.own.data_ptr() + (s.rows - nl) * rb if s.has_down else None, nf, nl, st)
        torch.cuda.synchronize(self.own.device)
        self.ctx.barrier()

    def close(self, collective: bool = True) -> None:
        """Unmap the neighbours and free the mailbox; ``collective`` (every
        rank calls it) first waits until no rank can still be reading it."""
        if collective and self.mailbox is not None and self._bases:
            _retire(self.ctx, self.own.device, "conv")
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []
        if self.mailbox is not None:
            self.mailbox.free()
            self.mailbox = None


def try_peer_halo(ctx: DistContext, slab: Slab, own: torch.Tensor) -> Optional[PeerHalo]:
    """Collective: a verified PeerHalo on every rank, or None on every rank
    (any rank failing to export, map — within its deadline — or read its
    neighbours through the kernel load path -> everyone keeps RCCL)."""
    if ctx.world < 2 or not own.is_cuda or not dist.is_initialized():
        return None
    phase(ctx, "conv peer set-up: begin")
    mine, err, mb = None, None, None
    try:
        if not own.is_contiguous():
            raise ValueError("peer halos need a contiguous CUDA slab")
        rb = own[0].numel() * own.element_size()
        mb = Mailbox(rb, slab.halo_down, slab.halo_up)
        mine = mb.export()
        phase(ctx, f"conv: mailbox of {mb.nbytes} B ({mb.kind} memory)")
    except Exception as e:  # noqa: BLE001 - reported below, then everyone falls back
        err = f"{type(e).__name__}: {e}"
    every = _allgather(ctx, mine, "conv: handles")
    ph = None
    if mine is not None:
        if _injected("map_fail", ctx.rank):  # fault hook: this rank cannot map its neighbours
            err = "RuntimeError: injected mapping failure (MPX_PEER_INJECT map_fail)"
        else:
            try:
                ph = PeerHalo(ctx, slab, own, mb, every)
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
                mb = None  # freed by the failed PeerHalo
    if not _agree(ctx, ph is not None, "conv: map vote"):
        if ph is not None:
            ph.close(collective=False)  # nobody launched a kernel on the mailboxes
        elif mb is not None:
            mb.free()
        _note(ctx, f"IPC mapping unavailable ({err or 'a neighbour failed'}); using RCCL")
        return None
    ph.publish()
    if not ph.verify():
        ph.close(collective=False)  # verify() ended in a collective vote: every rank is here
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
                ("dn_flag", ctypes.c_void_p), ("sync", ctypes.c_void_p), ("spin_limit", ctypes.c_uint),
                ("mb_first", ctypes.c_void_p * 2), ("mb_last", ctypes.c_void_p * 2)]


class JacobiPeerLink:
    """Mailbox links of one Jacobi rank to its neighbours (``mpx_jacobi_peer_sweep``).

    Each rank exports one :class:`Mailbox` (its completed-iteration word plus
    two parity slots of its first and last owned rows); the sweep's edge waves
    wait on the neighbours' words, read their edge rows of u^(t) from their
    mailboxes over xGMI, and store their own new edge rows write-through into
    this rank's mailbox slot for u^(t+1) — the slab buffers themselves are
    never shared, so slabs of any size keep the transport (reference: none;
    SURVEY §2.6 / §7.2 step 7 north star). Built by :func:`try_jacobi_peer`.
    """

    def __init__(self, ctx: DistContext, slab: Slab, bufs: List[torch.Tensor], mailbox: Mailbox, every: list):
        self.ctx = ctx
        self.slab = slab
        self.bufs = bufs
        self.sync = mailbox
        self.row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        self._bases: List[int] = []
        dev = bufs[0].device.index
        try:
            self._nb = _map_neighbours(ctx, every, self.row_bytes, lambda h, what: self._open(h, dev, what))
        except Exception:
            self.close(free_sync=False)
            raise
        d = _JacobiPeerDesc()
        if "up" in self._nb:
            m = self._nb["up"]
            d.up_row[0], d.up_row[1], d.up_flag = m.last(0), m.last(1), m.sync
            d.mb_first[0], d.mb_first[1] = mailbox.first(0), mailbox.first(1)
        if "dn" in self._nb:
            m = self._nb["dn"]
            d.dn_row[0], d.dn_row[1], d.dn_flag = m.first(0), m.first(1), m.sync
            d.mb_last[0], d.mb_last[1] = mailbox.last(0), mailbox.last(1)
        d.sync = mailbox.ptr
        d.spin_limit = int(os.environ.get("MPX_PEER_SPIN_LIMIT", "0"))  # diagnostics: give up sooner
        self.desc = d

    def _open(self, handle: bytes, device: int, what: str) -> int:
        base = _open_bounded(self.ctx, handle, device, what)
        self._bases.append(base)
        return base

    def probe(self) -> bool:
        """Signalled kernel-path probe over both mailbox slots (this rank's
        verdict; the caller votes)."""
        mb = self.sync
        own = [mb.first(0), mb.last(0), mb.first(1), mb.last(1)]
        nb_rows, nb_flags = {}, {}
        for side, m in self._nb.items():
            nb_rows[side] = [m.last(0), m.last(1)] if side == "up" else [m.first(0), m.first(1)]
            nb_flags[side] = m.sync
        self.sync.clear()
        return _signalled_probe(self.ctx, self.bufs[0].device, self.sync, own, nb_rows, nb_flags, self.row_bytes)

    def publish(self, u: torch.Tensor, iteration: int) -> None:
        """Collective, between sweeps (every rank's earlier sweeps finished —
        the caller synchronised and passed a barrier): reset this rank's sync
        words, set its completed-iteration word to ``iteration`` (every rank
        passes the same value) and put u's edge rows into mailbox slot
        ``iteration % 2``. The descriptor does not depend on the u / u_new roles
        (captured graphs stay valid)."""
        n, rb = self.slab.rows, self.row_bytes
        st = _native.stream_of(u)
        self.sync.put(iteration % 2, u.data_ptr() + rb if "up" in self._nb else None,
                      u.data_ptr() + n * rb if "dn" in self._nb else None, 1, 1, st)
        torch.cuda.synchronize(u.device)
        self.sync.clear()
        self.sync.write(0, iteration)
        _agree(self.ctx, True, "jacobi: publish done")

    def timed_out(self) -> bool:
        return bool(self.sync.read(W_ERR))

    def close(self, free_sync: bool = True, collective: bool = False) -> None:
        """Unmap the neighbours (and free this rank's mailbox with
        ``free_sync``); ``collective`` first waits until no rank can still be
        reading the mailbox."""
        if collective and free_sync and self._bases:
            _retire(self.ctx, self.bufs[0].device, type(self).__name__)
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []
        if free_sync:
            self.sync.free()


def try_jacobi_peer(ctx: DistContext, slab: Slab, bufs: List[torch.Tensor], layout_ok: bool) -> Optional[JacobiPeerLink]:
    """Collective: a mapped AND probed JacobiPeerLink on every rank, or None on
    every rank (export, bounded map, or the signalled kernel-path probe
    failing anywhere -> everyone keeps RCCL). Only the small mailboxes are
    exported: the u / u_new slabs may be any size."""
    if ctx.world < 2 or not bufs[0].is_cuda or not dist.is_initialized():
        return None
    phase(ctx, "jacobi peer set-up: begin")
    mine, err, mb = None, None, None
    try:
        if not layout_ok:
            raise ValueError("columns are not a multiple of the 16-byte vector width")
        row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        mb = Mailbox(row_bytes, 1, 1)
        mine = mb.export()
        phase(ctx, f"jacobi: mailbox of {mb.nbytes} B ({mb.kind} memory)")
    except Exception as e:  # noqa: BLE001 - reported below, then everyone falls back
        err = f"{type(e).__name__}: {e}"
    every = _allgather(ctx, mine, "jacobi: handles")
    link = None
    if mine is not None:
        try:
            if _injected("map_fail", ctx.rank):
                raise RuntimeError("injected mapping failure (MPX_PEER_INJECT map_fail)")
            link = JacobiPeerLink(ctx, slab, bufs, mb, every)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    if not _agree(ctx, link is not None, "jacobi: map vote"):
        if link is not None:
            link.close()
        elif mb is not None:
            mb.free()
        _note(ctx, f"Jacobi IPC links unavailable ({err or 'a neighbour failed'}); using RCCL")
        return None
    ok = link.probe()
    agreed = _agree(ctx, ok, "jacobi: probe vote")
    if not agreed:
        link.close()
        _note(ctx, "signalled kernel-path probe failed on some rank; using RCCL")
        return None
    phase(ctx, "jacobi peer set-up: ok")
    return link


# --------------------------------------------------------------------------
# streaming conv: fused halo (band kernel) or a device-signalled fetch per step
# --------------------------------------------------------------------------
class _HaloFetchDesc(ctypes.Structure):
    """ctypes mirror of ``mpx_halo_fetch`` (native/include/mpx/capi.h)."""

    _fields_ = [("src", ctypes.c_void_p * 2), ("dst", ctypes.c_void_p * 2), ("bytes", ctypes.c_int64 * 2),
                ("flag", ctypes.c_void_p * 2), ("sync", ctypes.c_void_p), ("step", ctypes.c_uint),
                ("spin_limit", ctypes.c_uint), ("own_src", ctypes.c_void_p * 2), ("mb_dst", ctypes.c_void_p * 2),
                ("mb_bytes", ctypes.c_int64 * 2)]


class _StreamPeerDesc(ctypes.Structure):
    """ctypes mirror of ``mpx_conv_stream_peer`` (native/include/mpx/capi.h)."""

    _fields_ = [("up_src", ctypes.c_void_p * 2), ("dn_src", ctypes.c_void_p * 2), ("up_flag", ctypes.c_void_p),
                ("dn_flag", ctypes.c_void_p), ("mb_first", ctypes.c_void_p * 2), ("mb_last", ctypes.c_void_p * 2),
                ("sync", ctypes.c_void_p), ("n_first", ctypes.c_int), ("n_last", ctypes.c_int),
                ("n_edge", ctypes.c_int), ("spin_limit", ctypes.c_uint)]


def stream_fused_ok(w: int, rows: int, filt) -> bool:
    """The fused streaming halo needs the band kernel's shape."""
    if os.environ.get("MPX_STREAM_FUSED", "1") == "0":  # A/B: the fetch-kernel path
        return False
    return bool(_native.lib().mpx_conv_stream_peer_ok(w, w, rows, filt.k, filt.anchor, filt.mode))


class StreamHaloLink:
    """Per-step halos for a slab whose input changes every step (two ping-pong
    input buffers, each (buffer_rows, ...) with the owned rows at
    ``slab.own_offset``; step k (1-based) reads buffer (k-1) % 2 = frame k-1).
    Every rank exports one :class:`Mailbox`; frame t's boundary rows live in
    its slot t % 2. Two forms:

    * ``fused`` (band-kernel shapes, the flagship): ONE launch per step
      (:meth:`conv`, ``mpx_conv_stream_peer_run``) — the conv's edge waves wait
      on the neighbours' step words, read their mailbox rows, write their own
      output boundary rows into this rank's mailbox and publish the step;
      interior waves never wait;
    * fetch (other shapes): :meth:`fetch` runs the one-workgroup-per-side
      kernel (own rows into the mailbox, publish, wait, copy the neighbours'
      mailbox rows into the local halo rows) before the ordinary conv launch.

    Built by :func:`try_stream_halo`."""

    def __init__(self, ctx: DistContext, slab: Slab, bufs: List[torch.Tensor], mailbox: Mailbox, every: list,
                 filt=None, fused: bool = False):
        self.ctx = ctx
        self.slab = slab
        self.bufs = bufs
        self.sync = mailbox
        self.filt = filt
        self.fused = fused
        self.row_bytes = bufs[0][0].numel() * bufs[0].element_size()
        self._bases: List[int] = []
        dev = bufs[0].device.index
        try:
            self._nb = _map_neighbours(ctx, every, self.row_bytes, lambda h, what: self._open(h, dev, what))
        except Exception:
            self.close(free_sync=False)
            raise
        s, rb = slab, self.row_bytes
        nf, nl = min(s.halo_down, s.rows), min(s.halo_up, s.rows)  # rows the neighbours read from this rank
        spin = int(os.environ.get("MPX_PEER_SPIN_LIMIT", "0"))
        any_halo = s.halo_up > 0 or s.halo_down > 0
        self._descs: List[_HaloFetchDesc] = []
        for a in range(2):  # fetch form: one descriptor per frame parity; only `step` changes
            d = _HaloFetchDesc()
            own = bufs[a].data_ptr() + s.own_offset * rb
            if "up" in self._nb and any_halo:
                m = self._nb["up"]
                d.flag[0] = m.sync  # waited on even without rows to copy (it reads our mailbox)
                if s.halo_up:
                    d.src[0] = m.last(a)  # its last halo_up rows of frame a
                    d.dst[0] = own - s.halo_up * rb
                    d.bytes[0] = s.halo_up * rb
                if nf:
                    d.own_src[0], d.mb_dst[0], d.mb_bytes[0] = own, mailbox.first(a), nf * rb
            if "dn" in self._nb and any_halo:
                m = self._nb["dn"]
                d.flag[1] = m.sync
                if s.halo_down:
                    d.src[1] = m.first(a)
                    d.dst[1] = own + s.rows * rb
                    d.bytes[1] = s.halo_down * rb
                if nl:
                    d.own_src[1], d.mb_dst[1], d.mb_bytes[1] = own + (s.rows - nl) * rb, mailbox.last(a), nl * rb
            d.sync = mailbox.ptr
            d.spin_limit = spin
            self._descs.append(d)
        sp = _StreamPeerDesc()  # fused form
        if "up" in self._nb:
            m = self._nb["up"]
            sp.up_flag = m.sync
            for p in range(2):
                sp.up_src[p] = m.last(p) + s.halo_up * rb
                sp.mb_first[p] = mailbox.first(p)
        if "dn" in self._nb:
            m = self._nb["dn"]
            sp.dn_flag = m.sync
            for p in range(2):
                sp.dn_src[p] = m.first(p) - s.rows * rb
                sp.mb_last[p] = mailbox.last(p)
        sp.sync = mailbox.ptr
        sp.n_first, sp.n_last = nf, nl
        sp.spin_limit = spin
        self._sp = sp
        self._nfl = (nf, nl)
        if fused:
            wx, wy = filt.c_taps()
            self._conv_args = [(bufs[a].data_ptr() + s.own_offset * rb, bufs[1 - a].data_ptr() + s.own_offset * rb,
                                bufs[0].shape[1], bufs[0].shape[1], s.rows, s.y_lo, s.y_hi, filt.k, filt.anchor,
                                filt.mode, wx, wy, ctypes.byref(sp)) for a in range(2)]
            self._keep = (wx, wy)

    def _open(self, handle: bytes, device: int, what: str) -> int:
        base = _open_bounded(self.ctx, handle, device, what)
        self._bases.append(base)
        return base

    def probe(self) -> bool:
        mb = self.sync
        own = [mb.first(0), mb.last(0), mb.first(1), mb.last(1)]
        nb_rows, nb_flags = {}, {}
        for side, m in self._nb.items():
            nb_rows[side] = [m.last(0), m.last(1)] if side == "up" else [m.first(0), m.first(1)]
            nb_flags[side] = m.sync
        self.sync.clear()
        return _signalled_probe(self.ctx, self.bufs[0].device, self.sync, own, nb_rows, nb_flags, self.row_bytes)

    def reset(self) -> None:
        """Collective between runs (callers synchronise and pass a barrier
        first): every rank's step word back to 0; the fused form also puts
        frame 0's boundary rows (buffer 0) into mailbox slot 0."""
        s, rb = self.slab, self.row_bytes
        if self.fused:
            own = self.bufs[0].data_ptr() + s.own_offset * rb
            nf, nl = self._nfl
            self.sync.put(0, own if "up" in self._nb else None,
                          own + (s.rows - nl) * rb if "dn" in self._nb else None, nf, nl,
                          _native.stream_of(self.bufs[0]))
        torch.cuda.synchronize(self.bufs[0].device)
        self.sync.clear()
        _agree(self.ctx, True, "stream: reset")

    def fetch(self, step: int, stream: int) -> None:
        """Fetch form: halo rows of buffer (step - 1) % 2 for step ``step`` (1-based)."""
        d = self._descs[(step - 1) % 2]
        d.step = step
        _native.check(_native.lib().mpx_halo_fetch_run(ctypes.byref(d), stream))

    def conv(self, step: int, stream: int) -> None:
        """Fused form: step ``step`` (1-based) in ONE launch — buffer (step-1) % 2
        convolved into the other buffer's owned rows, halos from the mailboxes."""
        rc = _native.lib().mpx_conv_stream_peer_run(*self._conv_args[(step - 1) % 2], stream)
        if rc:
            _native.check(rc)

    def pull(self, step: int) -> None:
        """Copy the neighbours' mailbox rows of frame ``step`` into the halo rows
        of buffer ``step % 2`` (the fused form never fills them; verification
        needs them). Call after every rank finished its steps up to ``step``."""
        s, rb = self.slab, self.row_bytes
        a = step % 2
        L = _native.lib()
        st = _native.stream_of(self.bufs[a])
        own = self.bufs[a].data_ptr() + s.own_offset * rb
        if "up" in self._nb and s.halo_up:
            _native.check(L.mpx_memcpy_d2d(own - s.halo_up * rb, self._nb["up"].last(a), s.halo_up * rb, st))
        if "dn" in self._nb and s.halo_down:
            _native.check(L.mpx_memcpy_d2d(own + s.rows * rb, self._nb["dn"].first(a), s.halo_down * rb, st))

    def timed_out(self) -> bool:
        return bool(self.sync.read(W_ERR))

    def close(self, free_sync: bool = True, collective: bool = False) -> None:
        """Unmap the neighbours (and free this rank's mailbox with
        ``free_sync``); ``collective`` first waits until no rank can still be
        reading the mailbox."""
        if collective and free_sync and self._bases:
            _retire(self.ctx, self.bufs[0].device, type(self).__name__)
        L = _native.lib()
        for b in self._bases:
            L.mpx_ipc_close(ctypes.c_void_p(b))
        self._bases = []
        if free_sync:
            self.sync.free()


def try_stream_halo(ctx: DistContext, slab: Slab, bufs: List[torch.Tensor], filt=None) -> Optional[StreamHaloLink]:
    """Collective: a mapped and probed StreamHaloLink on every rank, or None on
    every rank (-> RCCL halos). The fused form is used when every rank's shape
    fits the band kernel (``stream_fused_ok``)."""
    if ctx.world < 2 or not bufs[0].is_cuda or not dist.is_initialized():
        return None
    phase(ctx, "stream peer set-up: begin")
    mine, err, mb = None, None, None
    rb = bufs[0][0].numel() * bufs[0].element_size()
    fused = filt is not None and stream_fused_ok(int(bufs[0].shape[1]), slab.rows, filt)
    try:
        mb = Mailbox(rb, slab.halo_down, slab.halo_up)
        mine = mb.export()
        phase(ctx, f"stream: mailbox of {mb.nbytes} B ({mb.kind} memory)")
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    every = _allgather(ctx, (mine, fused), "stream: handles")
    fused = all(bool(f) for _, f in every)
    every = [m for m, _ in every]
    link = None
    if mine is not None:
        try:
            if _injected("map_fail", ctx.rank):
                raise RuntimeError("injected mapping failure (MPX_PEER_INJECT map_fail)")
            link = StreamHaloLink(ctx, slab, bufs, mb, every, filt, fused)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    if not _agree(ctx, link is not None, "stream: map vote"):
        if link is not None:
            link.close()
        elif mb is not None:
            mb.free()
        _note(ctx, f"streaming peer halos unavailable ({err or 'a neighbour failed'}); using RCCL")
        return None
    ok = link.probe()
    agreed = _agree(ctx, ok, "stream: probe vote")
    if not agreed:
        link.close()
        _note(ctx, "signalled kernel-path probe failed on some rank; using RCCL")
        return None
    link.reset()
    phase(ctx, f"stream peer set-up: ok ({'fused band kernel' if fused else 'fetch kernel'})")
    return link
