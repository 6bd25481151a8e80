"""2-D Jacobi sweep on a row slab with one halo row above and below.

Layout: ``u`` has shape (rows + 2, cols); row 0 and row rows+1 are halo rows
(neighbour data, or the fixed Dirichlet boundary at the global edges), columns
0 and cols-1 are Dirichlet boundary. A sweep writes owned rows [r0, r1)
(1-based) of ``un`` and optionally folds max|un - u| into ``resid``.
"""

from __future__ import annotations

from typing import Optional

import torch

from .. import _native


def jacobi_sweep(u: torch.Tensor, un: torch.Tensor, r0: int, r1: int,
                 resid: Optional[torch.Tensor] = None) -> Optional[float]:
    """GPU: enqueue the sweep (resid, a 1-element tensor zeroed by the caller,
    accumulates the max on device). CPU: run it and return the residual."""
    if u.shape != un.shape or u.dim() != 2 or u.dtype != un.dtype:
        raise ValueError("u/un must be matching 2-D tensors")
    if not (u.is_contiguous() and un.is_contiguous()):
        raise ValueError("u/un must be contiguous")
    rows2, cols = u.shape
    if not (1 <= r0 <= r1 <= rows2 - 1):
        raise ValueError("rows out of range")
    L = _native.lib()
    if u.is_cuda:
        rp = 0 if resid is None else resid.data_ptr()
        if resid is not None and (resid.dtype != u.dtype or resid.device != u.device):
            raise ValueError("resid must match u's dtype and device")
        if u.dtype == torch.float64:
            _native.check(L.mpx_jacobi_f64(u.data_ptr(), un.data_ptr(), cols, cols, r0, r1, rp, _native.stream_of(u)))
        elif u.dtype == torch.float32:
            _native.check(L.mpx_jacobi_f32(u.data_ptr(), un.data_ptr(), cols, cols, r0, r1, rp, _native.stream_of(u)))
        else:
            raise ValueError("jacobi supports float64/float32")
        return None
    if u.dtype != torch.float64:
        raise ValueError("CPU jacobi reference is float64")
    r = L.mpx_cpu_jacobi_f64(u.data_ptr(), un.data_ptr(), cols, cols, r0, r1)
    if resid is not None:
        resid.fill_(max(float(resid.item()), r))
    return r
