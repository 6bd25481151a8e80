"""lab1 workload: element-wise vector subtraction c = a - b.

``VectorSub`` runs on one device with an optional harness launch geometry.
``ShardedVectorSub`` splits the global vectors into contiguous shards, one per
rank (no halo: each element is independent); ``gather()`` reassembles the
result on rank 0.
"""

from __future__ import annotations

from typing import Optional

import torch

from .. import ops
from ..parallel.collectives import gather_slabs
from ..parallel.dist import DistContext
from ..parallel.slab import Slab


class VectorSub:
    def __init__(self, grid: int = 0, block: int = 0):
        self.grid, self.block = grid, block

    def __call__(self, a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return ops.vsub(a, b, out, grid=self.grid, block=self.block)


class ShardedVectorSub:
    def __init__(self, ctx: DistContext, n: int, dtype=torch.float64):
        self.ctx = ctx
        self.slab = Slab(n, ctx.world, ctx.rank)
        shape = (self.slab.rows,)
        self.a = torch.empty(shape, dtype=dtype, device=ctx.device)
        self.b = torch.empty(shape, dtype=dtype, device=ctx.device)
        self.c = torch.empty(shape, dtype=dtype, device=ctx.device)

    def fill_random(self, seed: int = 0) -> None:
        g = torch.Generator(device="cpu").manual_seed(seed + self.ctx.rank)
        self.a.copy_((torch.rand(self.a.shape, generator=g, dtype=torch.float64) * 2 - 1).to(self.a.dtype))
        self.b.copy_((torch.rand(self.b.shape, generator=g, dtype=torch.float64) * 2 - 1).to(self.b.dtype))

    def step(self) -> torch.Tensor:
        return ops.vsub(self.a, self.b, self.c)

    def gather(self) -> Optional[torch.Tensor]:
        return gather_slabs(self.c, self.slab, self.ctx)
