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
@pytest.mark.parametrize("path", ["fast", "mfma", "mfma64", "mfma8", "mfma16", "auto"])
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


# ---------------------------------------------------------------------------
# Independent oracles at the headline shapes: plain torch
# fp32 (ops/reference.py: F.conv2d over the dense K x K window, one summation
# order of its own) for every named filter, and torch fp64 quadratic forms for
# lab3 — not the framework's own C reference.
# ---------------------------------------------------------------------------
from cuda_mpi_openmp_amd.ops import filters as _filters  # noqa: E402
from cuda_mpi_openmp_amd.ops import reference as _ref  # noqa: E402

# measured on these exact images (CPU native == GPU bit for bit): at most 154
# +-1 pixels of 16.8 M for any filter / image (gauss5 separable vs its dense
# oracle); the bound leaves 5x margin
_MAX_OFF_BY_ONE = 800


def _oracle_check(got: torch.Tensor, img: torch.Tensor, f) -> None:
    exp = _ref.conv(img, f)
    assert torch.equal(got[..., 3], exp[..., 3]), "alpha must pass through"
    assert torch.equal(got[..., 0], got[..., 1]) and torch.equal(got[..., 0], got[..., 2])
    d = (got[..., 0].to(torch.int16) - exp[..., 0].to(torch.int16)).abs()
    assert int(d.max()) <= 1, f"{f.name}: gray level off by {int(d.max())}"
    assert int((d == 1).sum()) <= _MAX_OFF_BY_ONE, f"{f.name}: {int((d == 1).sum())} pixels off by one"
    if f.base_mode == _filters.MODE_MAG2:
        # saturated (oracle magnitude >= 256) and zero gradients: exact
        y = _ref.luma(img)
        import torch.nn.functional as F

        up, dn = f.anchor, f.k - 1 - f.anchor
        yp = F.pad(y[None, None], (up, dn, up, dn), mode="replicate")
        wx, wy = f.dense()
        gx = F.conv2d(yp, torch.tensor(wx, dtype=torch.float32).reshape(1, 1, f.k, f.k))[0, 0]
        gy = F.conv2d(yp, torch.tensor(wy, dtype=torch.float32).reshape(1, 1, f.k, f.k))[0, 0]
        s = gx * gx + gy * gy
        sure = (s >= 256.0 ** 2) | (s == 0)
        assert torch.equal(got[..., 0][sure], exp[..., 0][sure]), f"{f.name}: saturated / zero gradient differs"


@pytest.fixture(scope="module")
def oracle_imgs(img4096):
    sat = rand_img(4096, 4096, seed=23)
    sat[..., :3] = (sat[..., :3] > 127).to(torch.uint8) * 255  # every channel 0 or 255: the v_med3 clamp ends
    return {"random": img4096["random"], "smooth": img4096["smooth"], "saturated": sat}


@pytest.mark.parametrize("kind", ["random", "smooth", "saturated"])
@pytest.mark.parametrize("name", _filters.list_filters())
def test_conv_4096_vs_torch_oracle(gpu, oracle_imgs, kind, name):
    img = oracle_imgs[kind]
    f = ops.get_filter(name)
    _oracle_check(ops.conv(img.to(gpu), f).cpu(), img, f)


def test_conv_4096_iterated_sobel5_vs_torch_oracle(gpu, img4096):
    """A 20-step iterated sobel5 frame (mostly 0 / 255: the streaming bench's
    frames) convolved once more, against the torch oracle."""
    f = ops.get_filter("sobel5")
    x = img4096["random"].to(gpu)
    for _ in range(20):
        x = ops.conv(x, f)
    frame = x.cpu()
    ext = ((frame[..., 0] == 0) | (frame[..., 0] == 255)).float().mean().item()
    assert ext > 0.5, f"iterated frame not saturation-heavy ({ext:.2f})"
    _oracle_check(ops.conv(x, f).cpu(), frame, f)


def test_classify_8192_nc32_vs_torch_fp64_oracle(gpu, lab3_8192):
    """8192^2, 32 classes, every GPU path against torch fp64 quadratic forms:
    disagreements only where the two classes' distances are a near-tie."""
    img, ref = lab3_8192
    mu, inv, _ = ref[32]
    px = img.reshape(-1, 4)
    n, chunk = px.shape[0], 1 << 22
    best = torch.empty(n, dtype=torch.uint8)
    for s0 in range(0, n, chunk):  # torch ops on the GPU, no framework kernel
        best[s0:s0 + chunk] = torch.argmin(_ref.classify_dist(px[s0:s0 + chunk], mu, inv, device=gpu), dim=1)
    for path in ("fast", "mfma", "mfma64", "mfma8", "mfma16", "auto"):
        d = img.to(gpu)
        ops.classify_(d, mu, inv, path=path)
        got = d.cpu()[..., 3].reshape(-1)
        bad = (got != best).nonzero().flatten()
        assert bad.numel() < 1e-4 * n, f"{path}: {bad.numel()} disagreements"
        if bad.numel():
            dist = _ref.classify_dist(px[bad], mu, inv, device=gpu)
            dg = dist.gather(1, got[bad].long()[:, None])[:, 0]
            db = dist.gather(1, best[bad].long()[:, None])[:, 0]
            rel = ((dg - db).abs() / db.abs().clamp_min(1e-300)).max().item()
            assert rel < 1e-9, f"{path}: a disagreement is not a near-tie (relative gap {rel:.3g})"
