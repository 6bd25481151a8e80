"""lab2 workload: edge detection / KxK convolution of RGBA8 images.

``EdgeDetector`` runs on one device. ``SlabEdgeDetector`` is the distributed
form: a global image of H rows is split into row slabs (one per rank); each
step refreshes the slab's halo rows from its neighbours over RCCL while the
halo-independent interior rows are already being convolved, then finishes the
few boundary rows (reference: single GPU only, lab2/src/main.cu; the
decomposition is the BASELINE north star "domain-decomposed halo exchange").
"""

from __future__ import annotations

from typing import Optional

import torch

from .. import ops
from ..ops.filters import Filter, get_filter
from ..parallel.dist import DistContext
from ..parallel.halo import HaloExchange
from ..parallel.slab import Slab
from ..utils import trace


class EdgeDetector:
    def __init__(self, filt: str | Filter = "roberts", geometry=None):
        self.filter = get_filter(filt) if isinstance(filt, str) else filt
        self.geometry = geometry

    def __call__(self, img: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.filter.name == "roberts" and self.geometry is not None:
            return ops.roberts(img, out, geometry=self.geometry)
        return ops.conv(img, self.filter, out)

    def reference(self, img: torch.Tensor) -> torch.Tensor:
        from ..ops import reference as ref

        return ref.conv(img, self.filter)


def stream_reference(full: torch.Tensor, filt: str | Filter, steps: int) -> torch.Tensor:
    """The streaming benchmark's frame sequence on ONE device over the whole
    image: ``steps`` iterated whole-image convolutions (step k convolves step
    k-1's output). The N-rank ``SlabEdgeDetector(stream=True)`` must equal it
    bit for bit."""
    f = get_filter(filt) if isinstance(filt, str) else filt
    a = full.contiguous().clone()
    b = torch.empty_like(a)
    for _ in range(steps):
        ops.conv(a, f, b)
        a, b = b, a
    return a


class SlabEdgeDetector:
    """One rank's share of a row-decomposed image convolution.

    ``overlap`` selects how a step's halo exchange meets its convolution:

    * ``False`` ("inorder"): exchange, then one launch for every row, both in
      order on the compute stream;
    * ``True`` ("overlap"): exchange on a second queue while the interior rows
      are convolved, then the boundary rows;
    * ``"pipeline"`` (native RCCL tier only): software-pipelined over steps —
      two input buffers; during step k the comm stream refreshes the halos of
      the buffer step k+1 will read while the compute stream convolves the
      buffer whose halos arrived during step k-1. Every step still performs a
      full exchange and a full convolution; the exchange simply runs one step
      ahead (a frame of latency, no loss of throughput), and the compute
      stream only ever waits on an exchange that finished a step earlier.
    * ``"auto"``: ``False`` with the native tier, ``True`` without (measured,
      profiles/comm_step.md).

    ``halo`` selects the transport of the halo rows:

    * ``"peer"``: one-sided — the neighbours' mailboxes (their boundary rows,
      copied there when the slab is loaded) are IPC-mapped once and the
      convolution kernel reads them over xGMI on every step (``parallel.peer``);
      no exchange kernel, one launch per step;
    * ``"rccl"``: two-sided send/recv (native RCCL tier, else torch.distributed),
      arranged by ``overlap``;
    * ``"auto"``: ``"peer"`` when every rank can map and verify its neighbours,
      else ``"rccl"``.

    ``stream=True`` makes the input change every step, so the halo rows a rank
    reads are new each step (a real inter-rank dependency): the
    filter is iterated — step k convolves step k-1's output — over two
    ping-pong input buffers. Step k's halo rows come from the neighbours'
    step k-1 output, via the mailboxes (``peer``, ``parallel.peer.
    StreamHaloLink``: fused into the band kernel — one launch per step, only
    the slab-edge waves wait on the neighbours and publish the step — or, for
    shapes the band kernel does not take, a device-signalled fetch kernel
    before the conv) or an in-order RCCL send/recv (``rccl``). Results equal a
    one-device run of the same frame sequence on the whole image.
    """

    def __init__(self, ctx: DistContext, global_h: int, w: int, filt: str | Filter = "sobel5",
                 overlap: bool | str = "auto", halo: str = "auto", stream: bool = False):
        self.ctx = ctx
        self.filter = get_filter(filt) if isinstance(filt, str) else filt
        self.w = w
        self.slab = Slab(global_h, ctx.world, ctx.rank, self.filter.halo_up, self.filter.halo_down)
        self.halo = HaloExchange(self.slab, ctx)
        # "auto": with the native RCCL tier the exchange runs in order on the
        # compute stream and one launch convolves every row — measured faster
        # than forking the transfer onto a second queue (the RCCL kernel then
        # shares the CUs with the convolution and each cross-queue join costs
        # 7-16 us; profiles/comm_step.md); torch.distributed keeps the overlap.
        if overlap == "auto":
            overlap = ctx.native is None
        self.stream = bool(stream)
        self.pipeline = (overlap == "pipeline" and ctx.native is not None and ctx.device.type == "cuda"
                         and not self.stream)
        self.overlap = bool(overlap) and not self.pipeline and overlap != "pipeline" and not self.stream
        dev = ctx.device
        nbuf = 2 if (self.pipeline or self.stream) else 1
        self.bufs = [torch.empty((self.slab.buffer_rows, w, 4), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        self.out = torch.empty((self.slab.rows, w, 4), dtype=torch.uint8, device=dev)
        # pre-validated launches for the three row ranges of a step
        s = self.slab
        mk = lambda b, lo, hi, peer=None: ops.ConvLauncher(b, self.out, self.filter,  # noqa: E731
                                                           src_row0=s.own_offset, out_row0=0, oy0=lo, oy1=hi,
                                                           y_lo=s.y_lo, y_hi=s.y_hi, peer=peer)
        self._all_b = [mk(b, 0, s.rows) for b in self.bufs]
        # the owned rows of each buffer, built once: a stream-mode step returns
        # one of them (a fresh slice per step costs microseconds of host time
        # against a ~23 us step)
        self._own_views = [b[s.own_offset: s.own_offset + s.rows] for b in self.bufs]
        self._all = self._all_b[0]
        self._interior = mk(self.bufs[0], *s.interior())
        self._boundary = [mk(self.bufs[0], a, b) for a, b in s.boundary()]
        self.peer = None
        self.slink = None
        self._sk = 0  # stream mode: steps done since the last load
        if halo not in ("auto", "peer", "rccl"):
            raise ValueError(f"unknown halo transport {halo!r}")
        if self.stream:
            # step reading buffer a writes the owned rows of buffer 1 - a
            self._stream_launch = [ops.ConvLauncher(self.bufs[a], self.bufs[1 - a], self.filter, src_row0=s.own_offset,
                                                    out_row0=s.own_offset, oy0=0, oy1=s.rows, y_lo=s.y_lo,
                                                    y_hi=s.y_hi) for a in range(2)]
            if halo != "rccl" and ctx.world > 1 and dev.type == "cuda":
                from ..parallel.peer import try_stream_halo

                self.slink = try_stream_halo(ctx, s, self.bufs, self.filter)
                if self.slink is None and halo == "peer":
                    raise RuntimeError("streaming peer halo transport unavailable (IPC mapping or probe failed)")
        elif halo != "rccl" and ctx.world > 1 and dev.type == "cuda":
            from ..parallel.peer import try_peer_halo

            self.peer = try_peer_halo(ctx, s, self.bufs[0][s.own_offset: s.own_offset + s.rows])
            if self.peer is None and halo == "peer":
                raise RuntimeError("peer halo transport unavailable (IPC mapping or verification failed)")
        if self.peer is not None:
            self.pipeline = self.overlap = False
            self._all = mk(self.bufs[0], 0, s.rows, self.peer)
        self._traced = trace.enabled()  # roctx ranges only when MPX_ROCTX=1
        self._k = 0          # steps issued (pipeline mode)
        self._primed = False
        if self.pipeline:
            self._ev_recv = [torch.cuda.Event(), torch.cuda.Event()]
            self._ev_conv = [torch.cuda.Event(), torch.cuda.Event()]

    @property
    def buf(self) -> torch.Tensor:
        """The input buffer the most recent (or next, before any step) step reads."""
        if self.stream:
            return self.bufs[(self._sk - 1) % 2] if self._sk else self.bufs[0]
        return self.bufs[(self._k - 1) % len(self.bufs)] if self._k else self.bufs[0]

    @property
    def stream_out(self) -> torch.Tensor:
        """Stream mode: the owned rows the most recent step wrote (its output,
        the next step's input)."""
        return self._own_views[self._sk % 2]

    @property
    def own(self) -> torch.Tensor:
        s = self.slab
        return self.buf[s.own_offset: s.own_offset + s.rows]

    def _drain_comm(self) -> None:
        if self.pipeline:
            self.ctx.native.comm_stream().synchronize()
            self._primed = False

    @property
    def transport(self) -> str:
        if not self.ctx.is_distributed:
            return "none"
        if self.slink is not None:
            return "xgmi-peer-fused" if self.slink.fused else "xgmi-peer-signalled-fetch"
        if self.peer is not None:
            return "xgmi-peer"
        return "native-rccl" if self.ctx.native is not None else "torch.distributed"

    def halo_filled(self) -> torch.Tensor:
        """The input buffer with its halo rows as the last step read them
        (peer modes copy them in from the neighbours' mailboxes first; the
        fused streaming form after every rank finished its steps)."""
        if self.peer is not None:
            self.peer.pull(self.bufs[0])
        if self.slink is not None and self.slink.fused and self._sk:
            torch.cuda.synchronize(self.bufs[0].device)
            self.ctx.barrier()
            self.slink.pull(self._sk - 1)
        return self.buf

    def _publish(self) -> None:
        if self.peer is not None:
            self.peer.publish()

    def _quiesce(self) -> None:
        """Stream + peer mode, before host writes to the shared buffers: every
        rank's queued steps (and so its fetches of our rows) have finished."""
        if self.slink is not None:
            torch.cuda.synchronize(self.bufs[0].device)
            self.ctx.barrier()

    def load(self, slab_rows: torch.Tensor) -> None:
        """Collective: set this rank's owned input rows (stream mode: frame 0)."""
        self._drain_comm()
        self._quiesce()
        s = self.slab
        for b in self.bufs:
            b[s.own_offset: s.own_offset + s.rows].copy_(slab_rows)
        self._restart()

    def fill_random(self, seed: int) -> None:
        self._drain_comm()
        self._quiesce()
        g = torch.Generator(device=self.bufs[0].device)
        g.manual_seed(seed)
        s = self.slab
        rows = torch.randint(0, 256, (s.rows, self.w, 4), dtype=torch.uint8, device=self.bufs[0].device, generator=g)
        for b in self.bufs:
            b[s.own_offset: s.own_offset + s.rows].copy_(rows)
        self._restart()

    def _restart(self) -> None:
        self._sk = 0
        if self.slink is not None:
            self.slink.reset()  # collective: step words back to 0
        self._publish()

    def _rows(self, a: int, b: int) -> None:
        s = self.slab
        ops.conv_rows(self.buf, self.out, self.filter, src_row0=s.own_offset, out_row0=0, oy0=a, oy1=b,
                      y_lo=s.y_lo, y_hi=s.y_hi)

    def cache_resident(self, flag: bool = True) -> None:
        """Hint that this detector's input stays cache-resident between steps
        (one small slab re-convolved): its static launches then load rows with
        the default cache policy instead of non-temporal loads (MPX_CONV_RESIDENT)."""
        twin = [self._twin[1]] if getattr(self, "_twin", None) else []
        for ln in [*self._all_b, self._all, self._interior, *self._boundary, *twin]:
            ln.resident = flag

    def step_twin(self, stream: int) -> torch.Tensor:
        """The static step into a second output slab, on ``stream``: with
        ``step`` on another stream, two steps of the SAME input run
        concurrently without a write race (the bench's cache-resident pass:
        one 64 MiB input + two outputs stay inside the 256 MiB MALL).
        Independent static steps only."""
        if self.stream or not self.independent_steps:
            raise RuntimeError("step_twin needs independent static steps (one rank or peer halos)")
        if getattr(self, "_twin", None) is None:
            s = self.slab
            out2 = torch.empty_like(self.out)
            ln = ops.ConvLauncher(self.bufs[0], out2, self.filter, src_row0=s.own_offset, out_row0=0, oy0=0,
                                  oy1=s.rows, y_lo=s.y_lo, y_hi=s.y_hi, peer=self.peer)
            ln.resident = self._all.resident
            self._twin = (out2, ln)
        self._twin[1](stream)
        return self._twin[0]

    @property
    def independent_steps(self) -> bool:
        """True when this detector's steps may run on any stream of the caller's
        choosing (``step(stream=...)``) while OTHER detectors run on other
        streams: no host-ordered collective is involved (one rank, static peer
        halos, or device-signalled streaming halos). A stream-mode detector's
        own steps still depend on each other, so the caller keeps each detector
        on ONE stream."""
        if self.pipeline:
            return False
        if self.stream:
            return not self.ctx.is_distributed or self.slink is not None
        return not self.ctx.is_distributed or self.peer is not None

    def step(self, stream: Optional[int] = None) -> torch.Tensor:
        """Exchange halos and convolve every owned row; returns the output slab.
        ``stream``: a raw HIP stream handle for the launch (independent steps
        only); default the current torch stream."""
        if self._traced:
            with trace.range("edge.step"):
                return self._step(stream)
        return self._step(stream)

    def _step(self, stream: Optional[int] = None) -> torch.Tensor:
        if self.stream:
            return self._step_stream(stream if self.independent_steps else None)
        if self.pipeline:
            return self._step_pipelined()
        if stream is not None and self.independent_steps:
            self._all(stream)
            return self.out
        st = torch.cuda.current_stream(self.buf.device).cuda_stream if self.buf.is_cuda else None
        if not self.ctx.is_distributed or self.peer is not None:
            self._all(st)  # peer mode: the kernel reads the neighbours' rows itself
            return self.out
        if self.overlap:
            self.halo.start(self.buf)       # RCCL waits only for work queued so far
            self._interior(st)              # overlaps the halo transfer
            self.halo.wait()                # current stream waits for the halo rows
            for launch in self._boundary:
                launch(st)
        else:
            self.halo.exchange(self.buf)
            self._all(st)
        return self.out

    def _step_stream(self, stream: Optional[int] = None) -> torch.Tensor:
        k = self._sk + 1
        a = (k - 1) % 2
        st = stream if stream is not None else (
            torch.cuda.current_stream(self.bufs[0].device).cuda_stream if self.bufs[0].is_cuda else None)
        if self.ctx.is_distributed:
            if self.slink is not None and self.slink.fused:
                self.slink.conv(k, st)            # ONE launch: the edge waves carry the halo protocol
                self._sk = k
                return self.stream_out
            if self.slink is not None:
                self.slink.fetch(k, st)           # device-ordered: no host round trip
            else:
                self.halo.exchange(self.bufs[a])  # in order on the current stream
        self._stream_launch[a](st)
        self._sk = k
        return self.stream_out

    def stream_timed_out(self) -> bool:
        """True when a device-side halo wait of the streaming fetch gave up."""
        return self.slink is not None and self.slink.timed_out()

    def check_stream(self) -> None:
        """Raise when a device-side halo wait of the streaming fetch gave up."""
        if self.stream_timed_out():
            raise RuntimeError(f"rank {self.ctx.rank}: streaming halo wait timed out near step {self._sk}")

    def _step_pipelined(self) -> torch.Tensor:
        nc = self.ctx.native
        cs = nc.comm_stream()
        compute = torch.cuda.current_stream(self.out.device)
        if not self._primed:
            # halos of the first buffer, in order; both buffers free to overwrite
            for ev in self._ev_conv:
                ev.record(compute)
            cs.wait_stream(compute)
            nc.p2p(self.halo._plan(self.bufs[self._k % 2]), cs)
            self._ev_recv[self._k % 2].record(cs)
            self._primed = True
        cur, nxt = self._k % 2, (self._k + 1) % 2
        # comm stream: refresh the next buffer's halos once the conv that last
        # read that buffer has finished (write-after-read on its halo rows)
        cs.wait_event(self._ev_conv[nxt])
        nc.p2p(self.halo._plan(self.bufs[nxt]), cs)
        self._ev_recv[nxt].record(cs)
        # compute stream: this step's buffer; its exchange was issued a step ago
        compute.wait_event(self._ev_recv[cur])
        self._all_b[cur](compute.cuda_stream)
        self._ev_conv[cur].record(compute)
        self._k += 1
        return self.out

    def close(self) -> None:
        """Unmap the neighbours' slabs (peer modes). Collective in stream+peer
        mode (no rank unmaps while a neighbour may still read its rows)."""
        if self.slink is not None:
            self._quiesce()
            self.slink.close()
            self.slink = None
        if self.peer is not None:
            self.peer.close(collective=True)
            self.peer = None

    def finish(self) -> None:
        """Join the comm stream into the current stream (end of a timed run)."""
        if self.pipeline and self._primed:
            torch.cuda.current_stream(self.out.device).wait_stream(self.ctx.native.comm_stream())
