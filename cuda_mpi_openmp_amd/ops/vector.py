"""lab1 operator: element-wise vector subtraction (reference lab1/src/main.cu:22-29)."""

from __future__ import annotations

from typing import Optional

import torch

from .. import _native


def vsub(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, grid: int = 0,
         block: int = 0) -> torch.Tensor:
    """``out = a - b`` for contiguous fp64/fp32 vectors (any shape, flattened).

    ``grid``/``block`` reproduce a harness launch shape on the GPU; 0/0 picks the
    MI355X-tuned streaming launch.
    """
    if a.shape != b.shape or a.dtype != b.dtype or a.device != b.device:
        raise ValueError("a and b must match in shape, dtype and device")
    if a.dtype not in (torch.float64, torch.float32):
        raise ValueError("vsub supports float64 and float32")
    if not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("inputs must be contiguous")
    if out is None:
        out = torch.empty_like(a)
    n = a.numel()
    L = _native.lib()
    f64 = a.dtype == torch.float64
    if a.is_cuda:
        fn = L.mpx_vsub_f64 if f64 else L.mpx_vsub_f32
        _native.check(fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), n, grid, block, _native.stream_of(a)))
    else:
        fn = L.mpx_cpu_vsub_f64 if f64 else L.mpx_cpu_vsub_f32
        fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), n)
    return out
