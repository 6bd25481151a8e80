"""The exact int8-MFMA lab3 path (MFMA8, native/src/kernels/classify.hip),
emulated on the CPU with the kernel's integer arithmetic: features as int8
limbs, the host's int8 weight limbs (mpx_classify_i8_params), int32 keys
((D_a << 8) + D_b) << 5 | class, the top-2 margin test. Every pixel the test
DECIDES must get the reference fp64 chain's class (the rest take the exact
fallback on the GPU); no key may overflow int32. GPU runs of the real kernel
are in tests/test_gpu_kernels.py / test_gpu_headline.py."""

import ctypes

import numpy as np
import pytest
import torch

from cuda_mpi_openmp_amd import _native, ops
from cuda_mpi_openmp_amd.ops import reference as ref

from .helpers import rand_img, smooth_img


def i8_params(mu, inv):
    nc = mu.shape[0]
    a = np.zeros((32, 16), np.int8)
    b = np.zeros((32, 16), np.int8)
    c = np.zeros(32, np.int32)
    t2 = ctypes.c_int32()
    m = np.ascontiguousarray(mu, np.float64)
    iv = np.ascontiguousarray(inv, np.float64)
    rc = _native.lib().mpx_classify_i8_params(nc, m.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                              iv.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.ctypes.data,
                                              b.ctypes.data, c.ctypes.data, ctypes.byref(t2))
    return rc, a, b, c, int(t2.value)


def features(img):
    """(npix, 16) int64: the kernel's K = 16 int8 feature slots per pixel."""
    px = img.reshape(-1, 4)[:, :3].numpy().astype(np.int64) - 128
    r, g, bl = px[:, 0], px[:, 1], px[:, 2]
    P = np.stack([r * r, g * g, bl * bl, r * g, r * bl, g * bl], 1)
    h = (P + 128) >> 8                 # byte 1 of P + 128
    lo = P - 256 * h                   # byte 0 of P, signed
    F = np.concatenate([h, r[:, None], g[:, None], lo, bl[:, None], np.zeros_like(r)[:, None]], 1)
    assert F.min() >= -128 and F.max() <= 127
    # the kernel packs bytes: check the byte identities it relies on
    assert np.array_equal(((P + 128) >> 8) & 0xFF, ((P + 128) & 0xFF00) >> 8)
    assert np.array_equal(lo & 0xFF, P & 0xFF)
    return F


def emulate(img, a, b, c, t2, nc):
    F = features(img)
    da = F @ a.astype(np.int64).T                      # (npix, 32)
    db = F @ b.astype(np.int64).T + c.astype(np.int64)[None, :]
    key = (((da << 8) + db) << 5) + np.arange(32)[None, :]
    assert key.max() < 2**31 and key.min() >= -2**31, "int32 key overflow"
    order = np.sort(key, 1)
    B, S = order[:, 0], order[:, 1]
    decided = ((S >> 5) - (B >> 5)) > t2
    return (B & 31), decided


def check(img, mu, inv, max_undecided):
    nc = mu.shape[0]
    rc, a, b, c, t2 = i8_params(mu, inv)
    assert rc == 0
    assert np.all(a[nc:] == 0) and np.all(b[nc:] == 0) and np.all(c[nc:] == (1 << 26) - 64)
    cls, decided = emulate(img, a, b, c, t2, nc)
    want = ref.classify(img, mu, inv)[..., 3].reshape(-1).numpy().astype(np.int64)
    bad = decided & (cls != want)
    assert not bad.any(), f"{bad.sum()} decided pixels differ from the fp64 chain"
    assert (~decided).mean() <= max_undecided, (~decided).mean()
    return (~decided).mean()


@pytest.mark.parametrize("nc", [1, 2, 4, 16, 32])
def test_i8_emulation_random_points(nc):
    img = rand_img(96, 96, seed=nc)
    rng = np.random.default_rng(nc)
    mu, inv = ops.class_stats(img, [rng.integers(0, 96, (64, 2)) for _ in range(nc)])
    # near-identical classes (uniform image, random points): the hard case
    check(img, mu, inv, max_undecided=0.25)


@pytest.mark.parametrize("nc", [3, 8, 24])
def test_i8_emulation_separated_classes(nc):
    """Natural-image-like data with spatially coherent classes: few
    undecided pixels."""
    img = smooth_img(120, 128, seed=nc)
    rng = np.random.default_rng(100 + nc)
    pts = []
    for _ in range(nc):
        y0, x0 = rng.integers(0, 110), rng.integers(0, 118)
        pts.append(np.stack([x0 + rng.integers(0, 10, 40), y0 + rng.integers(0, 10, 40)], 1))
    mu, inv = ops.class_stats(img, pts)
    check(img, mu, inv, max_undecided=0.15)


def test_i8_params_refuse_unprovable_statistics():
    """Non-finite statistics (a 1-point class: NaN covariance) have no bound:
    the path resolves to the fp64 chain."""
    img = rand_img(16, 16)
    mu, inv = ops.class_stats(img, [np.array([[1, 1]]), np.array([[2, 2], [3, 3], [4, 5]])])
    rc, *_ = i8_params(mu, inv)
    assert rc != 0
    assert ops.classify_plan(mu, inv, "mfma8")[0] == "direct"


def test_i8_plan_reports_margin():
    img = rand_img(64, 64, seed=2)
    rng = np.random.default_rng(2)
    mu, inv = ops.class_stats(img, [rng.integers(0, 64, (30, 2)) for _ in range(5)])
    path, margin = ops.classify_plan(mu, inv, "mfma8")
    assert path == "mfma8" and margin >= 1
