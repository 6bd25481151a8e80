"""2-D Jacobi solver for the Laplace equation on a row-slab decomposed grid —
the distributed-stencil north star of BASELINE.json ("MPI -> RCCL 2D Jacobi
stencil, 16384^2 grid domain-decomposed across 8 MI355X, halo exchange over
xGMI"). The reference has no such solver; this is its MI355X-native
form.

Halo transports (``halo=``):

* ``"peer"`` (GPU, default when available): one-sided and device-signalled.
  Each rank IPC-maps its neighbours' mailboxes (completed-iteration word and
  two parity slots of their edge rows; the slabs are never shared, so they
  may be any size) once; every iteration is ONE sweep kernel whose slab-edge
  waves wait on the neighbours' counters, read their edge rows over xGMI,
  write this rank's new edge rows write-through into its mailbox and publish
  its counter (native/src/kernels/jacobi.hip, ``parallel.peer.
  JacobiPeerLink``). No exchange kernel, no host round trip per iteration.
* ``"rccl"``: two-sided send/recv of the edge rows (below).

RCCL transport, per iteration and rank:
  1. sweep the two slab-edge rows (the only rows a neighbour needs);
  2. post the halo exchange of those freshly computed rows over RCCL
     (point-to-point on the xGMI link between neighbouring GPUs);
  3. sweep the interior rows while the exchange is in flight;
  4. wait for the halos, swap u <-> u_new.
Every ``check_every`` iterations the sweeps also fold max|u_new - u| into a
device scalar and one 8-byte all-reduce(MAX) produces the global residual (the
small-message latency over xGMI is paid once per check, not per iteration).

Global boundary: Dirichlet. Row 0 of rank 0's buffer is the top boundary, the
last buffer row of the last rank the bottom boundary; columns 0 and cols-1 are
fixed. A decomposed run is bit-identical to a one-rank run.
"""

from __future__ import annotations

import ctypes
from typing import Callable, Optional

import torch

from .. import ops
from ..parallel.collectives import all_reduce_max, gather_slabs
from ..parallel.dist import DistContext
from ..parallel.fault import FaultInjected, fault_hook as _fault_hook  # noqa: F401 (re-export)
from ..parallel.halo import HaloExchange
from ..parallel.slab import Slab


class SlabJacobi:
    def __init__(self, ctx: DistContext, global_rows: int, cols: int, dtype=torch.float64, check_every: int = 10,
                 overlap: bool | str = "auto", halo: str = "auto"):
        if cols < 3:
            raise ValueError("need at least 3 columns")
        self.ctx = ctx
        self.cols = cols
        self.dtype = dtype
        self.check_every = max(1, int(check_every))
        # "auto": in order with the native RCCL tier (a cross-queue join costs
        # ~10 us on MI355X, more than the 1-row halo transfer it would hide;
        # profiles/comm_step.md), overlapped on torch.distributed
        self.overlap = (ctx.native is None) if overlap == "auto" else bool(overlap)
        self.slab = Slab(global_rows, ctx.world, ctx.rank, halo_up=1, halo_down=1)
        self.halo = HaloExchange(self.slab, ctx)
        shape = (self.slab.buffer_rows, cols)
        dev = ctx.device
        if halo not in ("auto", "peer", "rccl", "none"):
            raise ValueError(f"unknown halo transport {halo!r}")
        # "none": benchmarking ablation only — ranks sweep their slabs with no
        # halo exchange at all (wrong answer, same per-rank work): the
        # difference to "peer" is the cost of the device-side ordering and the
        # xGMI halo reads
        self.no_halo = halo == "none"
        if self.no_halo:
            self.overlap = False
        self.peer = None
        if halo not in ("rccl", "none") and ctx.is_distributed and dev.type == "cuda":
            # only a small mailbox per rank is IPC-shared (its iteration word and
            # two parity slots of its edge rows: parallel.peer.Mailbox), so the
            # u / u_new slabs may be any size
            from ..parallel.peer import try_jacobi_peer

            self.u = torch.zeros(shape, dtype=dtype, device=dev)
            self.un = torch.zeros(shape, dtype=dtype, device=dev)
            es = self.u.element_size()
            nv = 16 // es
            layout_ok = cols % nv == 0 and self.u.data_ptr() % 16 == 0 and self.un.data_ptr() % 16 == 0
            self.peer = try_jacobi_peer(ctx, self.slab, [self.u, self.un], layout_ok)
            if self.peer is None and halo == "peer":
                raise RuntimeError("peer halo transport unavailable (IPC mapping failed or cols not a multiple of "
                                   f"{nv})")
        else:
            if halo == "peer" and ctx.is_distributed:
                raise RuntimeError("peer halos need GPU ranks (IPC-mapped device memory)")
            self.u = torch.zeros(shape, dtype=dtype, device=dev)
            self.un = torch.zeros(shape, dtype=dtype, device=dev)
        self.resid = torch.zeros(1, dtype=dtype, device=dev)
        self.iteration = 0
        self.last_residual: Optional[float] = None
        self._halos_valid = False  # u's halo rows hold the neighbours' current rows
        self._graphs: dict = {}  # (u pointer at cycle start, check_every) -> StepGraph of one cycle

    # ------------------------------------------------------------------ setup
    def set_boundary(self, top: float = 1.0, bottom: float = 0.0, left: float = 0.0, right: float = 0.0) -> None:
        for t in (self.u, self.un):
            t[:, 0] = left
            t[:, -1] = right
            if not self.slab.has_up:
                t[0, :] = top
            if not self.slab.has_down:
                t[-1, :] = bottom

    def fill(self, fn: Optional[Callable[[torch.Tensor, torch.Tensor], torch.Tensor]] = None, seed: int = 0) -> None:
        """Interior initial values: fn(global_row_index, col_index) or seeded noise."""
        self._quiesce()
        s = self.slab
        rows = torch.arange(s.row0, s.row0 + s.rows, device=self.u.device).unsqueeze(1)
        cols = torch.arange(1, self.cols - 1, device=self.u.device).unsqueeze(0)
        if fn is None:
            g = torch.Generator(device="cpu").manual_seed(seed + 7919 * self.ctx.rank)
            vals = torch.rand((s.rows, self.cols - 2), generator=g, dtype=torch.float64).to(self.u.device)
        else:
            vals = fn(rows, cols)
        self.u[1:1 + s.rows, 1:-1] = vals.to(self.dtype)
        self.un.copy_(self.u)
        self._halos_valid = False

    @property
    def transport(self) -> Optional[str]:
        if not self.ctx.is_distributed:
            return None
        if self.no_halo:
            return "none (ablation: no halo exchange)"
        if self.peer is not None:
            return "xgmi-peer-signalled"
        return "native-rccl" if self.ctx.native is not None else "torch.distributed"

    def _quiesce(self) -> None:
        """Peer mode, before any host write to the IPC-shared buffers: every
        rank's queued sweeps have finished (a neighbour's last untracked sweep
        may still be reading our edge rows or waiting on our iteration word)."""
        if self.peer is not None:
            torch.cuda.synchronize(self.u.device)
            self.ctx.barrier()

    def sync_halos(self) -> None:
        """Exchange u's slab-edge rows (needed once after (re)initialisation;
        afterwards every step refreshes the halos of the rows it computes).
        Peer mode: publish the buffers and reset every rank's iteration word.
        The captured cycle graphs hold the previous descriptor (the neighbours'
        buffer parity) by value, so they are dropped here."""
        if self.peer is not None or self.no_halo:
            if self.peer is not None:
                self._quiesce()
                self._graphs.clear()
            self.un.copy_(self.u)
            if self.peer is not None:
                self.peer.publish(self.u, self.iteration)
            self._halos_valid = True
            return
        self.halo.exchange(self.u)
        self.un.copy_(self.u)
        self._halos_valid = True

    def check_peer(self) -> None:
        """Raise when a device-side halo wait gave up (a neighbour stalled)."""
        if self.peer is not None and self.peer.timed_out():
            raise RuntimeError(f"rank {self.ctx.rank}: peer halo wait timed out at iteration ~{self.iteration}")

    @property
    def owned(self) -> torch.Tensor:
        return self.u[1:1 + self.slab.rows]

    # ------------------------------------------------------------------ stepping
    def _sweep(self, r0: int, r1: int, track: bool) -> None:
        if r1 <= r0:
            return
        if self.u.is_cuda:
            ops.jacobi_sweep(self.u, self.un, r0, r1, self.resid if track else None)
        else:
            r = ops.jacobi_sweep(self.u, self.un, r0, r1)
            if track:
                self.resid.fill_(max(float(self.resid.item()), r))

    def step(self) -> Optional[float]:
        corrupt = _fault_hook(self.ctx.rank, self.iteration)
        if not self._halos_valid:
            self.sync_halos()
        if corrupt:  # injected silent error: one value off by one.
            # Host-exchanged halos (RCCL / gloo): the received halo row itself — a
            # cross-rank halo error. Peer mailboxes: the neighbour reads
            # this rank's edge row from the mailbox slot the previous sweep wrote,
            # which the host cannot change without racing that read, so the error
            # goes into this rank's first owned row instead: it is wrong here at
            # once and reaches the upper neighbour one sweep later, through the
            # mailbox row this sweep writes (the update spreads it to the adjacent
            # columns). Either way the N-rank == one-device check must fail.
            row = 1 if self.peer is not None else 0 if self.slab.has_up else self.slab.rows + 1
            self.u[row, self.cols // 2] += 1.0
        track = (self.iteration + 1) % self.check_every == 0
        self._advance(track)
        if track:
            self.last_residual = float(self.resid.item())
            self.check_peer()
            return self.last_residual
        return None

    def _advance(self, track: bool) -> None:
        """One iteration's device work (sweeps, halo exchange, swap and, when
        tracking, the residual all-reduce) with no host synchronisation, so it
        can be captured into a HIP graph."""
        s = self.slab
        n = s.rows
        if track:
            self.resid.zero_()
        if self.peer is not None:
            from .. import _native

            _native.check(_native.lib().mpx_jacobi_peer_sweep(
                int(self.dtype == torch.float64), self.u.data_ptr(), self.un.data_ptr(), self.cols, self.cols, n,
                self.resid.data_ptr() if track else None, ctypes.byref(self.peer.desc), _native.stream_of(self.u)))
        elif self.ctx.is_distributed and self.overlap:
            edge = [1] if n == 1 else [1, n]
            for r in edge:
                self._sweep(r, r + 1, track)
            self.halo.start(self.un)      # RCCL waits for the edge rows only
            self._sweep(2, n, track)      # interior overlaps the transfer
            self.halo.wait()
        else:
            self._sweep(1, n + 1, track)
            if not self.no_halo:
                self.halo.exchange(self.un)
        self.u, self.un = self.un, self.u
        self.iteration += 1
        if track:
            all_reduce_max(self.resid, self.ctx)

    def run(self, iters: int, tol: Optional[float] = None, graph: bool = False) -> int:
        """``iters`` iterations (fewer once the residual drops below ``tol``).

        ``graph=True`` (GPU): the iterations run as replays of one HIP graph of
        a whole residual cycle — check_every iterations, doubled to an even
        count so u/un are back in place at the end of every replay — with the
        host reading the residual once per replay. Launch-bound sweeps (small
        slabs, many ranks) no longer wait on the host's per-launch cost.
        Falls back to eager steps when the step cannot be captured."""
        done = 0
        if graph and self.u.is_cuda:
            done = self._run_graph(iters, tol)
            if done < 0:  # tolerance reached inside the graphed part
                return self.iteration
        for _ in range(iters - done):
            r = self.step()
            if tol is not None and r is not None and r < tol:
                break
        return self.iteration

    def _cycle_graph(self):
        """The HIP graph of one residual cycle (check_every iterations) starting
        from the current u/un roles; with an odd check_every the roles
        alternate between cycles, so two graphs exist. Captured once, reused
        by every later run() (capture + instantiate cost milliseconds)."""
        from ..utils.graphs import try_step_graph

        key = (self.u.data_ptr(), self.check_every)
        if key in self._graphs:
            return self._graphs[key]
        state = (self.u, self.un, self.iteration)
        it = [0]

        def body():  # the last iteration of the cycle tracks the residual, as in step()
            it[0] += 1
            self._advance(it[0] == self.check_every)

        g = try_step_graph(body, self.check_every, self.u.device, warmup=0)
        self.u, self.un, self.iteration = state  # the capture recorded the cycle, it did not run it
        self._graphs[key] = g
        return g

    def _run_graph(self, iters: int, tol: Optional[float]) -> int:
        if not self._halos_valid:
            self.sync_halos()
        # align to a cycle boundary eagerly, so every replay starts a cycle
        done = 0
        while self.iteration % self.check_every and done < iters:
            r = self.step()
            done += 1
            if tol is not None and r is not None and r < tol:
                return -1
        while iters - done >= self.check_every:
            g = self._cycle_graph()
            if g is None:
                return done
            _fault_hook(self.ctx.rank, self.iteration)
            g.replay()
            if self.check_every % 2:
                self.u, self.un = self.un, self.u
            self.iteration += self.check_every
            done += self.check_every
            self.last_residual = float(self.resid.item())
            self.check_peer()
            if tol is not None and self.last_residual < tol:
                return -1
        return done

    # ------------------------------------------------------------------ I/O
    def gather(self) -> Optional[torch.Tensor]:
        return gather_slabs(self.owned.contiguous(), self.slab, self.ctx)

    def save_checkpoint(self, prefix: str) -> str:
        """One file per rank: owned rows (+ halos), iteration, residual."""
        path = f"{prefix}.rank{self.ctx.rank}.pt"
        torch.save({"u": self.u.cpu(), "iteration": self.iteration, "residual": self.last_residual,
                    "global_rows": self.slab.global_rows, "world": self.ctx.world, "cols": self.cols}, path)
        return path

    def close(self) -> None:
        """Collective in peer mode: unmap the neighbours' mailboxes and free this
        rank's once no rank can still be reading it."""
        if self.peer is not None:
            self.peer.close(collective=True)
            self.peer = None

    def load_checkpoint(self, prefix: str) -> None:
        ck = torch.load(f"{prefix}.rank{self.ctx.rank}.pt", weights_only=True)
        if (ck["global_rows"], ck["world"], ck["cols"]) != (self.slab.global_rows, self.ctx.world, self.cols):
            raise ValueError("checkpoint geometry does not match this solver")
        self._quiesce()
        self._graphs.clear()
        self.u.copy_(ck["u"].to(self.u.device, self.dtype))
        self.un.copy_(self.u)
        self.iteration = int(ck["iteration"])
        self.last_residual = ck["residual"]
        self._halos_valid = False
