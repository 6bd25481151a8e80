"""HIP graphs for launch-bound inner loops.

A distributed step is a handful of small launches (halo send/recv, a
convolution or a stencil sweep, a residual reduction); when a sweep takes
tens of microseconds the host's per-launch cost (ctypes + HIP enqueue, RCCL
group calls) becomes the bottleneck. :class:`StepGraph` records ``n`` calls of
a step function once into a ``torch.cuda.CUDAGraph`` — on ROCm a hipGraph,
RCCL calls included (RCCL supports stream capture) — and replays them with
one launch. Every replay performs exactly the recorded work: each step of the
loop still runs every kernel and every transfer it ran eagerly.

The step function must be capturable: no host synchronisation, no
``.item()``, no allocation that changes between calls, the same buffers every
time (libmpx entry points never allocate or synchronise: capi.h).
"""

from __future__ import annotations

from typing import Callable, Optional

import torch


class StepGraph:
    def __init__(self, step: Callable[[], object], n: int, device: torch.device, warmup: int = 1):
        if n < 1:
            raise ValueError("need at least one step per graph")
        if device.type != "cuda":
            raise ValueError("HIP graphs need a GPU device")
        self.n = n
        self.device = device
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            # lazy per-stream state (RCCL channels, code objects) before capture
            for _ in range(warmup):
                step()
        torch.cuda.current_stream(device).wait_stream(side)
        torch.cuda.synchronize(device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for _ in range(n):
                step()
        torch.cuda.synchronize(device)

    def replay(self) -> None:
        self.graph.replay()

    def reset(self) -> None:
        self.graph.reset()


def try_step_graph(step: Callable[[], object], n: int, device: torch.device,
                   warmup: int = 1) -> Optional[StepGraph]:
    """A StepGraph, or None when this step cannot be captured here (the caller
    then keeps launching eagerly). Capture failures are reported on stderr."""
    if device.type != "cuda" or n < 1:
        return None
    try:
        return StepGraph(step, n, device, warmup)
    except Exception as e:  # noqa: BLE001 - fall back to eager launches
        import sys

        print(f"[graphs] step capture failed, running eagerly: {type(e).__name__}: {e}", file=sys.stderr)
        torch.cuda.synchronize(device)
        return None
