"""lab3 operators: class statistics (host, fp64) and per-pixel Mahalanobis
maximum-likelihood classification (reference lab3/src/main.cu:40-155)."""

from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from .edge import check_image

PATHS = {"direct": 0, "mfma": 1, "auto": 2, "fast": 3, "mfma64": 4, "mfma8": 5, "mfma16": 6}
PATH_NAMES = {v: k for k, v in PATHS.items()}
MAX_CLASSES = 32


def class_stats(img: torch.Tensor, classes: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
    """Per-class mean (nc, 3) and inverse covariance (nc, 3, 3) from (x, y) points.

    Mirrors the reference host code operation for operation (unbiased
    covariance, cofactor determinant, adjugate inverse), so a class with a
    single point produces the same NaN/inf statistics as the reference.
    """
    h, w = check_image(img)
    nc = len(classes)
    if not 1 <= nc <= MAX_CLASSES:
        raise ValueError(f"need 1 <= nc <= {MAX_CLASSES}")
    host = img.detach().to("cpu").contiguous()
    pts = [np.asarray(c, dtype=np.int64).reshape(-1, 2) for c in classes]
    np_arr = _native.i32_array([len(p) for p in pts])
    coords = _native.i32_array(np.concatenate(pts).reshape(-1).tolist())
    mu = (ctypes.c_double * (3 * nc))()
    inv = (ctypes.c_double * (9 * nc))()
    _native.check(_native.lib().mpx_class_stats(host.data_ptr(), w, h, nc, np_arr, coords, mu, inv))
    return np.array(mu[:], dtype=np.float64).reshape(nc, 3), np.array(inv[:], dtype=np.float64).reshape(nc, 3, 3)


def classify_(img: torch.Tensor, mu: np.ndarray, inv: np.ndarray, path: str = "auto", grid: int = 0,
              block: int = 0, ambiguous: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In place: alpha of every pixel = argmin_c (p - mu_c)^T inv_c (p - mu_c).

    ``path``:
      * ``direct`` — the reference fp64 FMA chain;
      * ``fast``   — fp32 packed-VALU distances;
      * ``mfma``   — fp32 MFMA distance GEMM (v_mfma_f32_32x32x2f32);
      * ``mfma64`` — fp64 MFMA distance GEMM (v_mfma_f64_16x16x4_f64);
      * ``mfma8``  — exact int8 MFMA distance GEMM (16-bit fixed-point weights
        in two int8 limbs, int32 keys): one pixel per lane on
        v_mfma_i32_4x4x4_16b_i8 up to 13 classes, v_mfma_i32_32x32x16_i8
        above;
      * ``mfma16`` — f16 MFMA distance GEMM (v_mfma_f32_32x32x16_f16, f16
        hi + lo weight limbs, exact integer features, fp32 keys): one pixel
        per lane with all of its classes in that lane;
      * ``auto``   — ``mfma16`` from 4 classes, ``fast`` below (each where
        its statistics permit a bound; else ``fast``, then ``direct``).
        Round-6 medians at 8192^2, µs, fast / mfma16: nc = 1 97 / 118,
        3 117 / 122, 4 127 / 121, 8 187 / 141, 16 297 / 174, 32 531 / 286
        (``mfma8`` never led by more than the box spread).
    The fp32/fp64-GEMM paths classify a pixel only when its best/second margin exceeds a
    rigorous bound on the fp32-vs-reference error and recompute every other
    pixel with the fp64 chain, so every path returns identical classes
    (statistics for which no bound can be proven run ``direct``). With
    ``ambiguous`` (a 1-element int32 device tensor) the number of pixels that
    took the exact fallback is added to it. CPU tensors use the OpenMP reference.
    """
    h, w = check_image(img)
    mu_c, inv_c, nc = _params(mu, inv)
    L = _native.lib()
    if img.is_cuda:
        amb = 0
        if ambiguous is not None:
            if not (ambiguous.is_cuda and ambiguous.dtype == torch.int32 and ambiguous.numel() >= 1):
                raise ValueError("ambiguous must be a 1-element int32 device tensor")
            amb = ambiguous.data_ptr()
        _native.check(L.mpx_classify_ex(img.data_ptr(), h * w, nc, mu_c.ptr, inv_c.ptr, grid, block, PATHS[path], amb,
                                        _native.stream_of(img)))
    else:
        L.mpx_cpu_classify(img.data_ptr(), h * w, nc, mu_c.ptr, inv_c.ptr)
    return img


class _F64:
    """A contiguous float64 view or copy and a ctypes array over its buffer
    (which the object keeps alive). ctypes arrays built from Python lists cost
    ~40 µs per call, a third of an 8192^2 classification; from_buffer ~1 µs."""

    __slots__ = ("arr", "ptr")

    def __init__(self, a: np.ndarray):
        arr = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
        if not arr.flags.writeable:
            arr = arr.copy()
        self.arr = arr
        self.ptr = (ctypes.c_double * max(1, arr.size)).from_buffer(arr) if arr.size else (ctypes.c_double * 1)()


def _params(mu: np.ndarray, inv: np.ndarray):
    m, i = _F64(mu), _F64(inv)
    nc = m.arr.size // 3
    if i.arr.size != 9 * nc or not 1 <= nc <= MAX_CLASSES:
        raise ValueError("mu must be (nc, 3) and inv (nc, 3, 3) with 1 <= nc <= 32")
    return m, i, nc


def plan(mu: np.ndarray, inv: np.ndarray, path: str = "auto") -> Tuple[str, float]:
    """(path actually run, fp32 decision margin) for these class statistics."""
    mu_c, inv_c, nc = _params(mu, inv)
    margin = ctypes.c_float(0.0)
    r = _native.lib().mpx_classify_plan(nc, mu_c.ptr, inv_c.ptr, PATHS[path], ctypes.byref(margin))
    _native.check(r if r < 0 else 0)
    return PATH_NAMES[r], float(margin.value)
