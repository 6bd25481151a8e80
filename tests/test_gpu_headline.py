"""Headline geometries, verified in full (VERDICT r1 "What's weak" #1).

The production kernels size their work from the image (segment lengths, rows
per wave, prefetch depth), so the small-shape tests do not reach the code
paths the benchmarks time. These run the BASELINE configurations themselves
and compare every output byte with the OpenMP CPU reference:

* lab2: sobel5 / gauss5 / Roberts at 4096 x 4096 (the flagship shape);
* lab3: the fast32, mfma32 and mfma64 classifiers at 8192 x 8192 with 4, 16
  and 32 classes (BASELINE config 4);
* Jacobi: one fp64 sweep of a 2048 x 16384 slab (a 16384^2 grid over 8 GPUs).
"""

import numpy as np
import pytest
import torch

from cuda_mpi_openmp_amd import ops

from .helpers import rand_img, smooth_img

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def img4096():
    return {"random": rand_img(4096, 4096, seed=21), "smooth": smooth_img(4096, 4096, seed=22)}


@pytest.mark.parametrize("kind", ["random", "smooth"])
@pytest.mark.parametrize("filt", ["sobel5", "gauss5", "roberts"])
def test_conv_4096_every_pixel(gpu, img4096, kind, filt):
    img = img4096[kind]
    g = ops.conv(img.to(gpu), filt).cpu()
    c = ops.conv(img, filt)
    assert torch.equal(g, c)


def test_roberts_kernel_4096_reference_geometries(gpu, img4096):
    """The lab2 Roberts kernel under the tuned launch and the reference's
    published launch geometries, every pixel against the CPU reference."""
    img = img4096["smooth"]
    c = ops.roberts(img)
    d = img.to(gpu)
    for geom in (None, ((32, 32), (16, 16)), ((16, 16), (32, 32)), ((32, 32), (64, 64))):
        assert torch.equal(ops.roberts(d, geometry=geom).cpu(), c), geom


@pytest.fixture(scope="module")
def lab3_8192():
    """8192^2 random pixels and the CPU (OpenMP, fp64 direct) classes for 4, 16
    and 32 classes — computed once for the module."""
    img = rand_img(8192, 8192, seed=31)
    rng = np.random.default_rng(32)
    out = {}
    for nc in (4, 16, 32):
        pts = [np.stack([rng.integers(0, 8192, 64), rng.integers(0, 8192, 64)], 1) for _ in range(nc)]
        mu, inv = ops.class_stats(img, pts)
        cpu = img.clone()
        ops.classify_(cpu, mu, inv)
        out[nc] = (mu, inv, cpu[..., 3].clone())
    return img, out


@pytest.mark.parametrize("nc", [4, 16, 32])
@pytest.mark.parametrize("path", ["fast", "mfma", "mfma64", "mfma8", "auto"])
def test_classify_8192_every_pixel(gpu, lab3_8192, nc, path):
    img, ref = lab3_8192
    mu, inv, cls = ref[nc]
    d = img.to(gpu)
    ops.classify_(d, mu, inv, path=path)
    out = d.cpu()
    assert torch.equal(out[..., 3], cls)
    assert torch.equal(out[..., :3], img[..., :3])  # RGB untouched (in-place alpha write only)


def test_jacobi_sweep_2048x16384_fp64(gpu):
    rows, cols = 2048, 16384
    g = torch.Generator().manual_seed(41)
    u = torch.rand((rows + 2, cols), generator=g, dtype=torch.float64)
    un_c = u.clone()
    r_cpu = ops.jacobi_sweep(u, un_c, 1, rows + 1)
    ud = u.to(gpu)
    un = ud.clone()
    res = torch.zeros(1, dtype=torch.float64, device=gpu)
    ops.jacobi_sweep(ud, un, 1, rows + 1, res)
    assert torch.equal(un.cpu(), un_c)
    assert res.item() == r_cpu
