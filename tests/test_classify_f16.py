"""The f16-MFMA lab3 path (MFMA16, native/src/kernels/classify.hip), emulated
on the CPU: the kernel's exact f16 features (channel products split as
h = f16(P), l = P - h), the host's f16 weight limbs (mpx_classify_f16_params),
an fp32 accumulator fed in slot order (one of the orders the host bound
covers), fp32 keys with the class in the low 5 mantissa bits, and the FAST32
margin test. Every pixel the test DECIDES must get the reference fp64 chain's
class (the rest take the exact fallback on the GPU), every key must stay
positive, and the undecided share must be far below the int8 path's. GPU runs
of the real kernel are in tests/test_gpu_kernels.py."""

import ctypes

import numpy as np
import pytest

from cuda_mpi_openmp_amd import _native, ops
from cuda_mpi_openmp_amd.ops import reference as ref

from .helpers import rand_img, smooth_img


def f16_params(mu, inv):
    nc = mu.shape[0]
    w = np.zeros((32, 3, 8), np.uint16)
    c = np.zeros(32, np.float32)
    t2 = ctypes.c_float()
    m = np.ascontiguousarray(mu, np.float64)
    iv = np.ascontiguousarray(inv, np.float64)
    rc = _native.lib().mpx_classify_f16_params(nc, m.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                               iv.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), w.ctypes.data,
                                               c.ctypes.data, ctypes.byref(t2))
    return rc, w.view(np.float16).astype(np.float64), c, float(t2.value)


def features(img):
    """(npix, 2, 8) float64: the two K = 8 feature fragments B1, B3."""
    q = img.reshape(-1, 4)[:, :3].numpy().astype(np.float64) - 128
    r, g, b = q[:, 0], q[:, 1], q[:, 2]
    P = np.stack([r * r, g * g, b * b, r * b, r * g, b * g], 1)
    h = P.astype(np.float16).astype(np.float64)  # v_pk_mul_f16 (round to nearest even)
    lo = P - h                                   # v_pk_fma_f16(x, y, -h): exact
    assert np.abs(lo).max() <= 4 and np.array_equal(lo, lo.astype(np.float16).astype(np.float64))
    B1 = np.concatenate([h, r[:, None], g[:, None]], 1)
    B3 = np.concatenate([lo, b[:, None], b[:, None]], 1)
    return B1, B3


def emulate(img, w, c, t2, nc):
    B1, B3 = features(img)
    npix = B1.shape[0]
    acc = np.broadcast_to(c[None, :], (npix, 32)).astype(np.float32)
    for j, F in ((0, B1), (1, B1), (2, B3)):
        for s in range(8):
            prod = (w[None, :, j, s] * F[:, s, None]).astype(np.float32)  # exact: <= 22 significant bits
            acc = (acc + prod).astype(np.float32)
    assert np.all(acc[:, :nc] > 0), "a key lost its positivity bias"
    bits = acc.view(np.uint32)
    key = (bits & np.uint32(0xFFFFFFE0)) | np.arange(32, dtype=np.uint32)[None, :]
    order = np.sort(key, 1)
    B, S = order[:, 0], order[:, 1]
    vb = (B & np.uint32(0xFFFFFFE0)).view(np.float32).astype(np.float64)
    vs = (S & np.uint32(0xFFFFFFE0)).view(np.float32).astype(np.float64)
    rhs = np.float32(vs * 1.125 * 2.0**-17 + t2).astype(np.float64)
    decided = np.float32(vs - vb).astype(np.float64) > rhs
    return (B & 31).astype(np.int64), decided


def check(img, mu, inv, max_undecided):
    nc = mu.shape[0]
    rc, w, c, t2 = f16_params(mu, inv)
    assert rc == 0
    assert np.all(w[nc:] == 0) and np.all(c[nc:] == np.float32(3e38))
    cls, decided = emulate(img, w, c, t2, nc)
    want = ref.classify(img, mu, inv)[..., 3].reshape(-1).numpy().astype(np.int64)
    bad = decided & (cls != want)
    assert not bad.any(), f"{bad.sum()} decided pixels differ from the fp64 chain"
    assert (~decided).mean() <= max_undecided, (~decided).mean()
    return (~decided).mean()


@pytest.mark.parametrize("nc", [1, 2, 4, 16, 17, 32])
def test_f16_emulation_random_points(nc):
    img = rand_img(96, 96, seed=nc)
    rng = np.random.default_rng(nc)
    mu, inv = ops.class_stats(img, [rng.integers(0, 96, (64, 2)) for _ in range(nc)])
    # near-identical classes (uniform image, random points): the hard case;
    # the int8 path leaves ~1.2 % undecided at 32 classes, f16 limbs far fewer
    check(img, mu, inv, max_undecided=0.02)


@pytest.mark.parametrize("nc", [3, 8, 24])
def test_f16_emulation_separated_classes(nc):
    img = smooth_img(120, 128, seed=nc)
    rng = np.random.default_rng(100 + nc)
    pts = []
    for _ in range(nc):
        y0, x0 = rng.integers(0, 110), rng.integers(0, 118)
        pts.append(np.stack([x0 + rng.integers(0, 10, 40), y0 + rng.integers(0, 10, 40)], 1))
    mu, inv = ops.class_stats(img, pts)
    check(img, mu, inv, max_undecided=0.02)


def test_f16_margin_tighter_than_int8():
    """At 32 classes on uniform pixels the f16 limbs leave at least 5x fewer
    pixels to the fallback than the int8 limbs (the reason for the path)."""
    from .test_classify_i8 import check as check_i8

    img = rand_img(128, 128, seed=7)
    rng = np.random.default_rng(7)
    mu, inv = ops.class_stats(img, [rng.integers(0, 128, (64, 2)) for _ in range(32)])
    u16 = check(img, mu, inv, max_undecided=0.02)
    u8 = check_i8(img, mu, inv, max_undecided=0.25)
    assert u16 * 5 <= u8, (u16, u8)


def test_f16_params_refuse_unprovable_statistics():
    img = rand_img(16, 16)
    mu, inv = ops.class_stats(img, [np.array([[1, 1]]), np.array([[2, 2], [3, 3], [4, 5]])])
    rc, *_ = f16_params(mu, inv)
    assert rc != 0
    assert ops.classify_plan(mu, inv, "mfma16")[0] == "direct"


def test_f16_plan_reports_margin():
    img = rand_img(64, 64, seed=2)
    rng = np.random.default_rng(2)
    mu, inv = ops.class_stats(img, [rng.integers(0, 64, (30, 2)) for _ in range(5)])
    path, margin = ops.classify_plan(mu, inv, "mfma16")
    assert path == "mfma16" and margin > 0
