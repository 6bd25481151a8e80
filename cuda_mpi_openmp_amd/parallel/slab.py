"""Row-slab domain decomposition (the distributed analogue of the reference's
grid-stride loops: "scale the sequence" becomes "scale the grid").

A global array of ``global_rows`` rows is split into contiguous slabs, one per
rank, balanced to within one row. Each rank stores its slab with ``halo_up``
rows above and ``halo_down`` rows below it; interior ranks fill those from
their neighbours, edge ranks clamp (the kernels' y_lo / y_hi bounds), so a
decomposed run is bit-identical to a single-GPU run.
"""

from __future__ import annotations

from dataclasses import dataclass

# MI355X: 288 GB HBM3E per GPU (spec); leave headroom for the runtime, RCCL
# buffers and the allocator's caching.
HBM_BYTES_PER_GPU = 288 * 10**9
HBM_USABLE_FRACTION = 0.85


@dataclass(frozen=True)
class Slab:
    global_rows: int
    world: int
    rank: int
    halo_up: int = 0
    halo_down: int = 0

    def __post_init__(self):
        if self.world < 1 or not 0 <= self.rank < self.world:
            raise ValueError("bad rank/world")
        if self.global_rows < self.world:
            raise ValueError("fewer rows than ranks")
        if self.world > 1 and min(self.rows_of(r) for r in range(self.world)) < max(self.halo_up, self.halo_down, 1):
            raise ValueError("slabs thinner than the halo: use fewer ranks")

    def rows_of(self, r: int) -> int:
        base, extra = divmod(self.global_rows, self.world)
        return base + (1 if r < extra else 0)

    def row0_of(self, r: int) -> int:
        base, extra = divmod(self.global_rows, self.world)
        return r * base + min(r, extra)

    @property
    def rows(self) -> int:
        return self.rows_of(self.rank)

    @property
    def row0(self) -> int:
        """Global index of this rank's first owned row."""
        return self.row0_of(self.rank)

    @property
    def has_up(self) -> bool:
        return self.rank > 0

    @property
    def has_down(self) -> bool:
        return self.rank + 1 < self.world

    @property
    def buffer_rows(self) -> int:
        return self.halo_up + self.rows + self.halo_down

    @property
    def own_offset(self) -> int:
        """Buffer row holding owned row 0."""
        return self.halo_up

    @property
    def y_lo(self) -> int:
        """Lowest readable logical row: resident halo rows, or clamp at the global top."""
        return -self.halo_up if self.has_up else 0

    @property
    def y_hi(self) -> int:
        return self.rows - 1 + (self.halo_down if self.has_down else 0)

    def interior(self):
        """Owned output rows [a, b) whose window needs no halo from a neighbour."""
        a = self.halo_up if self.has_up else 0
        b = self.rows - self.halo_down if self.has_down else self.rows
        return a, max(a, b)

    def boundary(self):
        """Owned output rows that read neighbour halo rows, as [a, b) ranges."""
        a, b = self.interior()
        out = []
        if a > 0:
            out.append((0, a))
        if b < self.rows:
            out.append((b, self.rows))
        return out


def max_rows_per_gpu(bytes_per_row: int, buffers: int = 2, hbm_bytes: int = HBM_BYTES_PER_GPU,
                     usable: float = HBM_USABLE_FRACTION) -> int:
    """Largest slab (rows) that fits ``buffers`` row-arrays in one GPU's HBM."""
    return int(hbm_bytes * usable) // (bytes_per_row * buffers)


def min_ranks_for(global_rows: int, bytes_per_row: int, buffers: int = 2) -> int:
    """Fewest GPUs whose slabs fit in HBM (288 GB each on MI355X)."""
    cap = max_rows_per_gpu(bytes_per_row, buffers)
    return max(1, -(-global_rows // cap))
