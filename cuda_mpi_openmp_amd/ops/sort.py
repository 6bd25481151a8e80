"""lab5 operator: ascending in-place sort of the reference's binary lab5
fixtures' element types (lab5/data/{int10,float10,uchar10}; SURVEY §4 — the
reference ships the inputs but no program, so the order contract is ours)."""

from __future__ import annotations

import numpy as np
import torch

from .. import _native

DTYPES = {torch.int32: 0, torch.float32: 1, torch.uint8: 2}
FIXTURE_DTYPES = {"int": np.int32, "float": np.float32, "uchar": np.uint8}


def sort_(x: torch.Tensor) -> torch.Tensor:
    """Sort a contiguous int32 / float32 / uint8 tensor ascending, in place
    (flattened). Floats follow the IEEE total order of their bit patterns
    (-NaN < -inf < -0.0 < +0.0 < +inf < +NaN). GPU tensors run the gfx950
    radix (int32/float32, bitonic for n <= 4096) / counting-sort (uint8)
    kernels with scratch from torch's caching allocator on the tensor's stream;
    CPU tensors run the C reference."""
    if x.dtype not in DTYPES:
        raise ValueError("sort_ supports int32, float32 and uint8")
    if not x.is_contiguous():
        raise ValueError("input must be contiguous")
    L = _native.lib()
    if x.is_cuda:
        dt = DTYPES[x.dtype]
        nbytes = int(L.mpx_sort_workspace_bytes(x.numel(), dt))
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=x.device) if nbytes else None
        _native.check(L.mpx_sort_ws(x.data_ptr(), x.numel(), dt, ws.data_ptr() if ws is not None else None, nbytes,
                                    _native.stream_of(x)))
    else:
        L.mpx_cpu_sort(x.data_ptr(), x.numel(), DTYPES[x.dtype])
    return x


def read_fixture(path: str, kind: str) -> np.ndarray:
    """A lab5 binary array: little-endian int32 n, then n elements of ``kind``
    (int / float / uchar)."""
    raw = open(path, "rb").read()
    n = int(np.frombuffer(raw[:4], dtype="<i4")[0])
    dt = np.dtype(FIXTURE_DTYPES[kind]).newbyteorder("<")
    if len(raw) != 4 + n * dt.itemsize:
        raise ValueError(f"{path}: size {len(raw)} does not match n = {n} of {kind}")
    return np.frombuffer(raw[4:], dtype=dt).astype(FIXTURE_DTYPES[kind])
