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
      * ``auto``   — ``mfma8`` below 9 classes, at 15-16 and from 20 (where it
        measured faster on MI355X, round-5 sweeps at 8192^2, µs: nc = 4 123
        vs 134, 8 172 vs 188, 15 262 vs 279, 16 260-267 vs 288-297, 32
        376-381 vs 505-524), else ``fast`` (the f32 MFMA shares the VALU's
        fp32 datapath on gfx950; at 9-14 the int8 forms' lead over fast32 is
        within the box-to-box spread or negative, and fast32 wins at 17-19).
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
        _native.check(L.mpx_classify_ex(img.data_ptr(), h * w, nc, mu_c, inv_c, grid, block, PATHS[path], amb,
                                        _native.stream_of(img)))
    else:
        L.mpx_cpu_classify(img.data_ptr(), h * w, nc, mu_c, inv_c)
    return img


def _params(mu: np.ndarray, inv: np.ndarray):
    mu = np.ascontiguousarray(mu, dtype=np.float64).reshape(-1)
    inv = np.ascontiguousarray(inv, dtype=np.float64).reshape(-1)
    nc = mu.size // 3
    if inv.size != 9 * nc or not 1 <= nc <= MAX_CLASSES:
        raise ValueError("mu must be (nc, 3) and inv (nc, 3, 3) with 1 <= nc <= 32")
    return _native.f64_array(mu.tolist()), _native.f64_array(inv.tolist()), nc


def plan(mu: np.ndarray, inv: np.ndarray, path: str = "auto") -> Tuple[str, float]:
    """(path actually run, fp32 decision margin) for these class statistics."""
    mu_c, inv_c, nc = _params(mu, inv)
    margin = ctypes.c_float(0.0)
    r = _native.lib().mpx_classify_plan(nc, mu_c, inv_c, PATHS[path], ctypes.byref(margin))
    _native.check(r if r < 0 else 0)
    return PATH_NAMES[r], float(margin.value)
