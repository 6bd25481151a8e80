"""lab3 workload: per-pixel Mahalanobis maximum-likelihood classification.

``PixelClassifier`` fits class statistics from training points (host fp64,
reference lab3/src/main.cu:102-152) and labels every pixel's alpha channel on
the GPU (direct FMA chain or the fp64-MFMA quadratic-form GEMM with exact
fallback). ``SlabPixelClassifier`` is the row-decomposed form: the training
pixels that fall in each rank's slab are all-gathered (a few KB) so every rank
computes bit-identical statistics with the reference's operation order, then
each rank classifies its own rows — no halo, embarrassingly parallel.
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..parallel.dist import DistContext
from ..parallel.slab import Slab


class PixelClassifier:
    def __init__(self, path: str = "auto"):
        self.path = path
        self.mu = None
        self.inv = None

    def fit(self, img: torch.Tensor, classes: Sequence[np.ndarray]) -> "PixelClassifier":
        self.mu, self.inv = ops.class_stats(img, classes)
        return self

    def __call__(self, img: torch.Tensor, grid: int = 0, block: int = 0) -> torch.Tensor:
        if self.mu is None:
            raise RuntimeError("fit() first")
        return ops.classify_(img, self.mu, self.inv, path=self.path, grid=grid, block=block)


class SlabPixelClassifier:
    def __init__(self, ctx: DistContext, global_h: int, w: int, path: str = "auto"):
        self.ctx = ctx
        self.w = w
        self.slab = Slab(global_h, ctx.world, ctx.rank)
        self.path = path
        self.img = torch.empty((self.slab.rows, w, 4), dtype=torch.uint8, device=ctx.device)
        self.mu = None
        self.inv = None

    def fit(self, classes: Sequence[np.ndarray]) -> None:
        """classes: per class an (n, 2) array of GLOBAL (x, y) points."""
        s = self.slab
        host = self.img.detach().cpu()
        pts = [np.asarray(c, dtype=np.int64).reshape(-1, 2) for c in classes]
        flat = np.concatenate(pts)
        mine = (flat[:, 1] >= s.row0) & (flat[:, 1] < s.row0 + s.rows)
        vals = np.zeros(len(flat), dtype=np.int64)
        if mine.any():
            loc = flat[mine]
            vals[mine] = host[loc[:, 1] - s.row0, loc[:, 0]].contiguous().view(torch.int32).numpy().astype(
                np.int64).reshape(-1) & 0xFFFFFFFF
        t = torch.from_numpy(vals).to(self.ctx.device if self.ctx.backend == "nccl" else "cpu")
        if self.ctx.is_distributed:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)  # each point is owned by exactly one rank
        train = t.cpu().numpy().astype(np.uint32)
        # a 1-row image of the training pixels in global point order: the
        # statistics see exactly the reference's summation order
        row = torch.from_numpy(train.view(np.uint8).reshape(1, -1, 4).copy())
        offs = np.cumsum([0] + [len(p) for p in pts])
        local = [np.stack([np.arange(offs[c], offs[c + 1]), np.zeros(len(pts[c]), dtype=np.int64)], 1)
                 for c in range(len(pts))]
        self.mu, self.inv = ops.class_stats(row, local)

    def classify(self) -> torch.Tensor:
        return ops.classify_(self.img, self.mu, self.inv, path=self.path)


def split_rows(full: torch.Tensor, slab: Slab) -> torch.Tensor:
    return full[slab.row0: slab.row0 + slab.rows]


def class_points_for(h: int, w: int, nc: int, npts: int, seed: int = 0) -> List[np.ndarray]:
    rng = np.random.default_rng(seed)
    return [np.stack([rng.integers(0, w, npts), rng.integers(0, h, npts)], 1) for _ in range(nc)]
