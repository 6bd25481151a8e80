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


class SlabEdgeDetector:
    """One rank's share of a row-decomposed image convolution."""

    def __init__(self, ctx: DistContext, global_h: int, w: int, filt: str | Filter = "sobel5",
                 overlap: bool | str = "auto"):
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
        self.overlap = bool(overlap)
        dev = ctx.device
        self.buf = torch.empty((self.slab.buffer_rows, w, 4), dtype=torch.uint8, device=dev)
        self.out = torch.empty((self.slab.rows, w, 4), dtype=torch.uint8, device=dev)
        # pre-validated launches for the three row ranges of a step
        s = self.slab
        mk = lambda a, b: ops.ConvLauncher(self.buf, self.out, self.filter, src_row0=s.own_offset,  # noqa: E731
                                          out_row0=0, oy0=a, oy1=b, y_lo=s.y_lo, y_hi=s.y_hi)
        self._all = mk(0, s.rows)
        self._interior = mk(*s.interior())
        self._boundary = [mk(a, b) for a, b in s.boundary()]
        self._traced = trace.enabled()  # roctx ranges only when MPX_ROCTX=1

    @property
    def own(self) -> torch.Tensor:
        s = self.slab
        return self.buf[s.own_offset: s.own_offset + s.rows]

    def load(self, slab_rows: torch.Tensor) -> None:
        self.own.copy_(slab_rows)

    def fill_random(self, seed: int) -> None:
        g = torch.Generator(device=self.buf.device)
        g.manual_seed(seed)
        self.own.copy_(torch.randint(0, 256, self.own.shape, dtype=torch.uint8, device=self.buf.device, generator=g))

    def _rows(self, a: int, b: int) -> None:
        s = self.slab
        ops.conv_rows(self.buf, self.out, self.filter, src_row0=s.own_offset, out_row0=0, oy0=a, oy1=b,
                      y_lo=s.y_lo, y_hi=s.y_hi)

    def step(self) -> torch.Tensor:
        """Exchange halos and convolve every owned row; returns the output slab."""
        if self._traced:
            with trace.range("edge.step"):
                return self._step()
        return self._step()

    def _step(self) -> torch.Tensor:
        st = torch.cuda.current_stream(self.buf.device).cuda_stream if self.buf.is_cuda else None
        if not self.ctx.is_distributed:
            self._all(st)
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
