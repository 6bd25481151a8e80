"""Numerics of the hand-written gfx950 kernels (run on a real MI355X).

Each HIP kernel is compared against (a) the native CPU reference, bit for bit,
and (b) a plain-PyTorch reference of the same op (fp32 for image ops, fp64
for lab1/lab3/Jacobi), per the test strategy of SURVEY §4.
"""

import os

import numpy as np
import pytest
import torch

from cuda_mpi_openmp_amd import ops
from cuda_mpi_openmp_amd.ops import reference as ref

from .helpers import LAB2_DATA, LAB2_GT, LAB3_CLASSES, LAB3_DATA, LAB3_GT, bytes_to_img, hex_bytes, img_to_bytes, rand_img, smooth_img

pytestmark = pytest.mark.gpu

GEOMS = [None, ((32, 32), (16, 16)), ((16, 16), (32, 32)), ((2, 2), (16, 16)), ((32, 32), (64, 64)),
         ((16, 16), (1024, 1024)), ((64, 4), (8, 8)), ((1, 1), (1, 1))]


@pytest.mark.parametrize("name", ["test_01", "test_02"])
@pytest.mark.parametrize("geom", GEOMS)
def test_roberts_ground_truth(gpu, name, geom):
    img = bytes_to_img(hex_bytes(os.path.join(LAB2_DATA, name + ".txt")))
    out = ops.roberts(img.to(gpu), geometry=geom)
    torch.cuda.synchronize()
    assert img_to_bytes(out) == hex_bytes(os.path.join(LAB2_GT, name + ".txt"))


@pytest.mark.parametrize("hw", [(1, 1), (1, 5), (5, 1), (3, 3), (4, 4), (17, 33), (64, 128), (129, 257), (480, 640),
                                (1000, 1003)])
@pytest.mark.parametrize("geom", [None, ((32, 8), (8, 8)), ((16, 16), (4, 4))])
def test_roberts_matches_cpu_and_torch(gpu, hw, geom):
    img = smooth_img(*hw, seed=hw[0] * 7 + hw[1])
    gpu_out = ops.roberts(img.to(gpu), geometry=geom).cpu()
    assert torch.equal(gpu_out, ops.roberts(img))  # native CPU, bit-exact
    assert torch.equal(gpu_out, ref.roberts(img))  # plain torch fp32, same op order


@pytest.mark.parametrize("filt", ["roberts", "sobel3", "prewitt3", "scharr3", "laplace3", "box3", "sharpen3", "sobel5",
                                  "gauss5", "log5", "sobel5_dense", "gauss5_dense"])
@pytest.mark.parametrize("hw", [(1, 1), (2, 7), (7, 2), (31, 129), (64, 128), (200, 300), (257, 260)])
def test_conv_matches_cpu_exact_and_torch(gpu, filt, hw):
    f = ops.get_filter(filt)
    img = smooth_img(*hw, seed=11)
    g = ops.conv(img.to(gpu), f).cpu()
    c = ops.conv(img, f)
    assert torch.equal(g, c)
    d = ops.conv(img.to(gpu), f, direct=True).cpu()
    assert torch.equal(d, c)
    t = ref.conv(img, f)
    diff = (g[..., :3].int() - t[..., :3].int()).abs()
    assert int(diff.max()) <= 1
    assert torch.equal(g[..., 3], img[..., 3])


@pytest.mark.parametrize("filt", ["roberts", "sobel3", "sobel5", "gauss5", "log5", "sobel5_dense"])
@pytest.mark.parametrize("w", [4, 8, 252, 256, 260, 512, 516, 1028])
def test_conv_band_kernel_strip_edges(gpu, filt, w):
    """The band kernel (256-column strips, 8-B aprons at the strip edges,
    clamp-to-edge by the lane's own pixel at x = 0 and x = w), forced onto small
    aligned images: partial strips, exactly one strip, one lane, every segment
    height; then the default size threshold (wave kernel) gives the same bytes."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    f = ops.get_filter(filt)
    old = L.mpx_conv_set_band_min(0)
    try:
        for h in (1, 2, 5, 17, 33, 70):
            img = rand_img(h, w, seed=w + h)
            assert torch.equal(ops.conv(img.to(gpu), f).cpu(), ops.conv(img, f)), (h, w)
    finally:
        L.mpx_conv_set_band_min(old)
    assert old >= 1 << 20
    img = rand_img(33, w, seed=w)
    assert torch.equal(ops.conv(img.to(gpu), f).cpu(), ops.conv(img, f))


@pytest.mark.parametrize("filt", ["sobel5", "gauss5", "sobel5_dense", "gauss5_dense", "log5"])
def test_conv_vertical_share_kernel(gpu, filt):
    """Band mode 4 (conv_band16v_kernel: 16 vertically consecutive segments per
    workgroup, shared halo rows handed over through LDS) on every 5-row window:
    whole 16-segment groups, partial groups, a short last segment (its
    neighbours fall back to memory halos), several strips, slab launches with
    resident halo rows; every byte against the CPU reference."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    f = ops.get_filter(filt)
    old_min, old_mode = L.mpx_conv_set_band_min(0), L.mpx_conv_set_band_mode(4)
    try:
        for h, w in ((4096, 4096), (512, 260), (16 * 16 + 7, 516), (16 * 3, 1024), (19, 256), (5, 64), (300, 8)):
            img = rand_img(h, w, seed=h + w)
            assert torch.equal(ops.conv(img.to(gpu), f).cpu(), ops.conv(img, f)), (h, w)
        # a slab launch: logical rows [0, 200) of a buffer with 2 resident halo rows each side
        buf = rand_img(204, 516, seed=9)
        out_g = torch.empty((200, 516, 4), dtype=torch.uint8, device=gpu)
        ops.conv_rows(buf.to(gpu), out_g, f, src_row0=2, out_row0=0, oy0=0, oy1=200, y_lo=-2, y_hi=201)
        out_c = torch.empty((200, 516, 4), dtype=torch.uint8)
        ops.conv_rows(buf, out_c, f, src_row0=2, out_row0=0, oy0=0, oy1=200, y_lo=-2, y_hi=201)
        assert torch.equal(out_g.cpu(), out_c)
    finally:
        L.mpx_conv_set_band_mode(old_mode)
        L.mpx_conv_set_band_min(old_min)


@pytest.mark.parametrize("filt", ["roberts", "sobel3", "prewitt3", "scharr3", "laplace3", "sharpen3", "sobel5_dense",
                                  "log5"])
def test_conv_named_taps_equal_runtime_taps(gpu, filt):
    # named filters run compile-time tap classes; -0.0 in place of the zero taps
    # defeats the bit-exact match, so the same operator runs with runtime taps
    f = ops.get_filter(filt)
    nz = lambda t: tuple(-0.0 if v == 0.0 else v for v in t)  # noqa: E731
    rt = ops.Filter(filt + "_rt", f.k, f.anchor, f.mode, nz(f.wx), nz(f.wy))
    img = rand_img(131, 390, seed=5).to(gpu)
    assert torch.equal(ops.conv(img, f).cpu(), ops.conv(img, rt).cpu())


def test_conv_roberts_equals_roberts_kernel(gpu):
    img = rand_img(333, 517, seed=3)
    a = ops.conv(img.to(gpu), "roberts").cpu()
    b = ops.roberts(img.to(gpu), geometry=((32, 8), (4, 4))).cpu()
    assert torch.equal(a, b)


def test_conv_custom_7x7_and_odd_anchor(gpu):
    rng = np.random.default_rng(0)
    f7 = ops.Filter.custom(7, rng.standard_normal(49).tolist(), rng.standard_normal(49).tolist())
    f4 = ops.Filter.custom(4, rng.standard_normal(16).tolist(), anchor=1, mode="abs1")
    img = smooth_img(150, 201, seed=5)
    for f in (f7, f4):
        assert torch.equal(ops.conv(img.to(gpu), f).cpu(), ops.conv(img, f))


def test_conv_separable_custom(gpu):
    """Runtime separable factors (wave kernel for k = 3/5/7, direct for k = 4 and
    abs1): GPU == CPU bit for bit, within one level of the dense torch sum."""
    rng = np.random.default_rng(7)
    img = smooth_img(203, 330, seed=6)
    fs = [ops.Filter.separable_custom(rng.standard_normal(k).tolist(), rng.standard_normal(k).tolist(), 0.5,
                                      rng.standard_normal(k).tolist(), rng.standard_normal(k).tolist(), 0.25)
          for k in (3, 5, 7, 4)]
    fs.append(ops.Filter.separable_custom([1, 4, 6, 4, 1], [1, 4, 6, 4, 1], 1.0 / 256, mode="lin1"))  # == gauss5, runtime
    fs.append(ops.Filter.separable_custom([1, 2, 1], [-1, 0, 1], 1.0, mode="abs1"))
    for f in fs:
        c = ops.conv(img, f)
        assert torch.equal(ops.conv(img.to(gpu), f).cpu(), c), f
        assert torch.equal(ops.conv(img.to(gpu), f, direct=True).cpu(), c), f
        assert int((c[..., 0].int() - ref.conv(img, f)[..., 0].int()).abs().max()) <= 1
    assert torch.equal(ops.conv(img.to(gpu), fs[4]).cpu(), ops.conv(img, "gauss5"))


@pytest.mark.parametrize("filt", ["roberts", "sobel5", "sobel3", "gauss5"])
def test_conv_rows_slab_equals_full_image(gpu, filt):
    """A slab with resident halo rows reproduces the full-image result."""
    f = ops.get_filter(filt)
    H, W = 300, 260
    img = smooth_img(H, W, seed=9)
    full = ops.conv(img, f)
    for r0, r1 in ((0, 100), (100, 217), (217, 300)):
        up = f.halo_up if r0 > 0 else 0
        dn = f.halo_down if r1 < H else 0
        buf = img[r0 - up: r1 + dn].contiguous().to(gpu)
        out = torch.empty((r1 - r0, W, 4), dtype=torch.uint8, device=gpu)
        ops.conv_rows(buf, out, f, src_row0=up, out_row0=0, oy0=0, oy1=r1 - r0, y_lo=-up, y_hi=r1 - r0 - 1 + dn)
        assert torch.equal(out.cpu(), full[r0:r1])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n", [0, 1, 3, 1000, 4097, 1 << 20])
@pytest.mark.parametrize("geom", [(0, 0), (1, 32), (4, 64), (32, 128), (512, 512), (1024, 1024)])
def test_vsub(gpu, dtype, n, geom):
    g = torch.Generator().manual_seed(n)
    a = (torch.rand(n, generator=g, dtype=torch.float64) * 2e100 - 1e100).to(dtype)
    b = (torch.rand(n, generator=g, dtype=torch.float64) * 2e100 - 1e100).to(dtype)
    if dtype == torch.float32:
        a, b = a.clamp(-1e30, 1e30), b.clamp(-1e30, 1e30)
    out = ops.vsub(a.to(gpu), b.to(gpu), grid=geom[0], block=geom[1]).cpu()
    assert torch.equal(out, a - b)


def test_vsub_unaligned_views(gpu):
    a = torch.arange(1001, dtype=torch.float64, device=gpu)[1:]
    b = torch.ones(1001, dtype=torch.float64, device=gpu)[1:]
    assert torch.equal(ops.vsub(a, b).cpu(), (a - b).cpu())


def test_classify_ground_truth(gpu):
    img = bytes_to_img(hex_bytes(os.path.join(LAB3_DATA, "test_01_lab3.txt")))
    mu, inv = ops.class_stats(img, LAB3_CLASSES)
    gt = hex_bytes(os.path.join(LAB3_GT, "test_01_lab3.txt"))
    for path in CLS_PATHS:
        d = img.to(gpu)
        ops.classify_(d, mu, inv, path=path)
        assert img_to_bytes(d) == gt, path


CLS_PATHS = ("direct", "fast", "mfma", "mfma64", "mfma8", "mfma16", "auto")


def _random_classes(img, nc, npts, seed):
    rng = np.random.default_rng(seed)
    h, w = img.shape[:2]
    return [np.stack([rng.integers(0, w, npts), rng.integers(0, h, npts)], 1) for _ in range(nc)]


@pytest.mark.parametrize("nc", [1, 2, 5, 16, 17, 24, 25, 32])
@pytest.mark.parametrize("path", CLS_PATHS)
def test_classify_matches_cpu(gpu, nc, path):
    img = smooth_img(193, 211, seed=nc)  # 40723 pixels: not a multiple of 4 or 128 (tail path)
    mu, inv = ops.class_stats(img, _random_classes(img, nc, 40, nc))
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    d = img.to(gpu)
    ops.classify_(d, mu, inv, path=path)
    assert torch.equal(d.cpu(), cpu)
    t = ref.classify(img, mu, inv)
    assert (t[..., 3] != cpu[..., 3]).float().mean() < 1e-3  # torch's summation order differs on near-ties


@pytest.mark.parametrize("path", ["direct", "fast"])
@pytest.mark.parametrize("geom", [(1024, 1024), (4096, 64), (3, 32), (1, 1)])
def test_classify_oversized_geometry(gpu, path, geom):
    """Caller grids far larger than the work: the empty workgroups are not
    launched (useful_grid), and the result equals the CPU reference either way."""
    img = smooth_img(37, 53, seed=5)  # 1961 pixels: vector body + 1-pixel tail
    mu, inv = ops.class_stats(img, _random_classes(img, 5, 20, 5))
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    d = img.to(gpu)
    ops.classify_(d, mu, inv, path=path, grid=geom[0], block=geom[1])
    assert torch.equal(d.cpu(), cpu)


@pytest.mark.parametrize("hw", [(7, 9), (300, 301), (1000, 1003), (1000, 1004)])
@pytest.mark.parametrize("geom", [((16, 16), (1024, 1024)), ((3, 5), (700, 900)), ((64, 4), (2, 4096))])
def test_roberts_oversized_geometry(gpu, hw, geom):
    """Grids with more blocks than tiles (scalar and 16-B kernels)."""
    img = smooth_img(*hw, seed=hw[1])
    assert torch.equal(ops.roberts(img.to(gpu), geometry=geom).cpu(), ops.roberts(img))


def test_geometry_literal_launch_matches(gpu, tmp_path):
    """MPX_GEOM_LITERAL=1 (the caller's grid as given) produces the same bytes
    as the default launch with the empty workgroups dropped."""
    import subprocess
    import sys
    code = (
        "import torch, sys\n"
        "from cuda_mpi_openmp_amd import ops\n"
        "from tests.helpers import smooth_img\n"
        "img = smooth_img(300, 301, seed=3)\n"
        "a = torch.arange(1003, dtype=torch.float64); b = torch.ones(1003, dtype=torch.float64)\n"
        "r = ops.roberts(img.cuda(), geometry=((16, 16), (1024, 1024))).cpu()\n"
        "v = ops.vsub(a.cuda(), b.cuda(), grid=1024, block=1024).cpu()\n"
        "torch.save({'r': r, 'v': v}, sys.argv[1])\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for lit in ("0", "1"):
        p = tmp_path / f"o{lit}.pt"
        env = dict(os.environ, MPX_GEOM_LITERAL=lit, PYTHONPATH=root)
        subprocess.run([sys.executable, "-c", code, str(p)], check=True, cwd=root, env=env, timeout=120)
        outs.append(torch.load(p, weights_only=True))
    assert torch.equal(outs[0]["r"], outs[1]["r"]) and torch.equal(outs[0]["v"], outs[1]["v"])
    assert torch.equal(outs[0]["v"], torch.arange(1003, dtype=torch.float64) - 1)


@pytest.mark.parametrize("path", CLS_PATHS)
def test_classify_random_pixels_and_fallback_rate(gpu, path):
    """Uniform random pixels (the bench's input): identical classes; the exact
    fallback stays rare."""
    img = rand_img(512, 640, seed=11)
    nc = 24
    mu, inv = ops.class_stats(img, _random_classes(img, nc, 64, 3))
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    d = img.to(gpu)
    amb = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.classify_(d, mu, inv, path=path, ambiguous=amb)
    assert torch.equal(d.cpu(), cpu)
    if path != "direct":
        # mfma8's integer keys carry 16-bit weights: its bound is ~100x the fp32
        # one, so ~1-2% of these near-identical classes' pixels re-rank exactly
        limit = 0.04 if path == "mfma8" else 0.01
        assert amb.item() < limit * img.shape[0] * img.shape[1]
    else:
        assert amb.item() == 0


@pytest.mark.parametrize("nc", [1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13])
def test_classify_mfma8_small_class_counts(gpu, nc):
    """mfma8 up to 13 classes runs the one-pixel-per-lane 4x4x4 int8 MFMA form
    (classify_mfma8s_kernel, every row-set count 1-7): uniform random pixels,
    classes identical to the CPU reference, the exact fallback rare."""
    img = rand_img(517, 643, seed=nc)  # 332431 pixels: vector body + 3-pixel tail
    mu, inv = ops.class_stats(img, _random_classes(img, nc, 64, 100 + nc))
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    assert ops.classify_plan(mu, inv, "mfma8")[0] == "mfma8"
    d = img.to(gpu)
    amb = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.classify_(d, mu, inv, path="mfma8", ambiguous=amb)
    assert torch.equal(d.cpu(), cpu)
    assert amb.item() < 0.04 * img.shape[0] * img.shape[1]


@pytest.mark.parametrize("path", ["fast", "mfma", "mfma64", "mfma8", "mfma16"])
def test_classify_exact_ties_all_fall_back(gpu, path):
    """Duplicated classes tie exactly on every pixel: every pixel must take the
    fp64 chain and keep the lowest class index (reference strict '<')."""
    img = smooth_img(64, 96, seed=4)
    pts = _random_classes(img, 2, 30, 5)
    mu, inv = ops.class_stats(img, [pts[0], pts[1], pts[0]])
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    d = img.to(gpu)
    amb = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.classify_(d, mu, inv, path=path, ambiguous=amb)
    assert torch.equal(d.cpu(), cpu)
    assert (cpu[..., 3] != 2).all()
    assert amb.item() >= int((cpu[..., 3] == 0).sum())  # every class-0 pixel tied with class 2


@pytest.mark.parametrize("nc", [1, 2, 3, 4, 5, 8, 11, 16, 17, 20, 23, 28, 32])
def test_classify_mfma16_class_counts(gpu, nc):
    """mfma16 (f16 MFMA, one pixel per lane): every ranked-register count on
    both the one-shot kernel (whole 1024-vector blocks, device deferral list +
    fix-up kernel) and the looped tail (the rest of the image): uniform random
    pixels, classes identical to the CPU reference, the fallback rare."""
    img = rand_img(517, 643, seed=nc)  # 332431 pixels: 81 one-shot blocks + a looped tail + 3 scalar pixels
    mu, inv = ops.class_stats(img, _random_classes(img, nc, 64, 200 + nc))
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    assert ops.classify_plan(mu, inv, "mfma16")[0] == "mfma16"
    d = img.to(gpu)
    amb = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.classify_(d, mu, inv, path="mfma16", ambiguous=amb)
    assert torch.equal(d.cpu(), cpu)
    assert amb.item() < 0.01 * img.shape[0] * img.shape[1]


def test_classify_mfma16_list_reuse_and_overflow(gpu):
    """The device deferral list is reused across calls on one stream (counter
    sets alternate; the fix-up zeroes the next call's set): a large image, a
    small one (no list), an image whose every pixel ties (the list overflows
    into the in-wave re-ranking), then large again — every result identical
    to the CPU reference."""
    big = rand_img(1024, 1536, seed=1)
    small = rand_img(31, 29, seed=2)
    mu, inv = ops.class_stats(big, _random_classes(big, 20, 64, 9))
    pts = _random_classes(big, 2, 30, 5)
    mu_t, inv_t = ops.class_stats(big, [pts[0], pts[1], pts[0]])
    tied = rand_img(2048, 2560, seed=3)  # 5.2M tied pixels: more entries than a sub-list holds
    for img, m, iv in ((big, mu, inv), (small, mu, inv), (tied, mu_t, inv_t), (big, mu, inv), (big, mu_t, inv_t)):
        cpu = img.clone()
        ops.classify_(cpu, m, iv)
        d = img.to(gpu)
        ops.classify_(d, m, iv, path="mfma16")
        assert torch.equal(d.cpu(), cpu)


def test_classify_unaligned_view(gpu):
    img = smooth_img(33, 65, seed=6)
    mu, inv = ops.class_stats(img, _random_classes(img, 3, 20, 6))
    flat = img.reshape(-1, 4)
    cpu = flat[1:].clone()
    ops.classify_(cpu.reshape(1, -1, 4), mu, inv)
    dev = flat.to(gpu)
    view = dev[1:].reshape(1, -1, 4)  # 4-byte offset: not 16-B aligned -> direct kernel
    for path in CLS_PATHS:  # classification ignores alpha, so re-running in place is idempotent
        ops.classify_(view, mu, inv, path=path)
        assert torch.equal(view.reshape(-1, 4).cpu(), cpu), path


def test_classify_near_ties_fall_back_exactly(gpu):
    """Two nearly identical classes: the fp32 paths must reproduce the direct chain."""
    img = smooth_img(128, 128, seed=1)
    pts = _random_classes(img, 1, 50, 0)[0]
    mu, inv = ops.class_stats(img, [pts, pts, pts[:-1]])
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    for path in ("fast", "mfma", "mfma64", "mfma8"):
        d = img.to(gpu)
        ops.classify_(d, mu, inv, path=path)
        assert torch.equal(d.cpu(), cpu), path


def test_classify_single_point_class_nan(gpu):
    """np = 1 -> zero covariance -> inf/NaN statistics; reference semantics kept."""
    img = smooth_img(32, 32, seed=2)
    mu, inv = ops.class_stats(img, [np.array([[0, 0]]), np.array([[1, 1], [2, 2], [5, 7]])])
    cpu = img.clone()
    ops.classify_(cpu, mu, inv)
    for path in CLS_PATHS:
        d = img.to(gpu)
        ops.classify_(d, mu, inv, path=path)
        assert torch.equal(d.cpu(), cpu)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
# (2413, 4096) / (4822, 4096): 4 rows per wave (fp64) / 8 (fp32) with tails;
# (1003, 16384): the production 8 rows per wave, odd row blocks walking up, and
# a 3-row tail in a bottom block that walks up (125 full blocks + 3 rows)
@pytest.mark.parametrize("shape", [(3, 3), (10, 7), (66, 130), (257, 1001), (2413, 4096), (4822, 4096),
                                   (1003, 16384)])
def test_jacobi_sweep(gpu, dtype, shape):
    rows, cols = shape
    g = torch.Generator().manual_seed(rows)
    u = torch.rand((rows + 2, cols), generator=g, dtype=torch.float64)
    un_ref = ref.jacobi(u, 1, rows + 1)
    ud = u.to(dtype).to(gpu)
    un = torch.zeros_like(ud)
    res = torch.zeros(1, dtype=dtype, device=gpu)
    ops.jacobi_sweep(ud, un, 1, rows + 1, res)
    torch.cuda.synchronize()
    got = un.cpu()[1:rows + 1]
    if dtype == torch.float64:
        assert torch.equal(got, un_ref[1:rows + 1])
        uc = u.clone()
        unc = torch.zeros_like(uc)
        r_cpu = ops.jacobi_sweep(uc, unc, 1, rows + 1)
        assert float(res.item()) == r_cpu
    else:
        assert torch.allclose(got.double(), un_ref[1:rows + 1], rtol=1e-6, atol=1e-6)


def test_fast_sqrt_exhaustive(gpu, capsys):
    """Every fp32 magnitude^2 in [0, 65025]: the production fast magnitude
    (v_sqrt_f32 + fract margin + exact fallback) equals the correctly rounded
    sqrtf + truncation of the reference. Also reports how many inputs the bare
    v_sqrt_f32 truncation would get wrong (the reason the margin exists)."""
    from cuda_mpi_openmp_amd import _native

    L = _native.tune_lib()  # the self-test entry point lives in the tuning library
    counts = []
    for raw in (0, 1):
        bad = torch.zeros(1, dtype=torch.int64, device=gpu)
        _native.check(L.mpx_selftest_fast_sqrt(bad.data_ptr(), raw, 0))
        torch.cuda.synchronize()
        counts.append(int(bad.item()))
    # the paired production path (mag2_to_gray: v_med3 clamp, margin test on
    # both lanes) over every float in [0, +inf], each paired with another value
    # and the band kernels' four-pixel form (mag4_to_gray: gray level from the
    # low byte of 2^23 + n, no conversion), every value with three partners
    for raw in (2, 3):
        bad = torch.zeros(1, dtype=torch.int64, device=gpu)
        _native.check(L.mpx_selftest_fast_sqrt(bad.data_ptr(), raw, 0))
        torch.cuda.synchronize()
        counts.append(int(bad.item()))
    with capsys.disabled():
        print(f"\nfast sqrt mismatches over all fp32 in [0, 65025]: production {counts[0]}, bare v_sqrt {counts[1]}; "
              f"over [0, inf]: paired path {counts[2]}, four-pixel path {counts[3]}")
    assert counts[0] == 0 and counts[2] == 0 and counts[3] == 0


@pytest.mark.parametrize("hw", [(5, 64), (23, 130), (47, 260), (200, 300), (1001, 517), (4096, 4096)])
@pytest.mark.parametrize("seg", [0, 8, 11])
def test_conv_alternating_segments_exact(gpu, hw, seg):
    """Separable sobel5 with odd segments walking their rows upwards (tuning
    variant kind 3, p2 = 2000) is bit-identical to the CPU reference, segment
    tails and image edges included."""
    import ctypes

    from cuda_mpi_openmp_amd import _native

    L = _native.tune_lib()
    f = ops.get_filter("sobel5")
    wx, wy = f.c_taps()
    img = smooth_img(*hw, seed=hw[0] + seg)
    d = img.to(gpu)
    out = torch.empty_like(d)
    _native.check(L.mpx_conv_variant(d.data_ptr(), out.data_ptr(), hw[1], hw[0], 5, 3, seg, 2000, 1, wx, wy, 0))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ops.conv(img, f))


def test_roberts_rgb_gpu_pins_reference_sample(gpu):
    """Per-channel Roberts (L1) on the device: byte-exact against the
    reference's lenna_out.data sample."""
    d = os.path.join(os.path.dirname(LAB2_DATA), "test_data")
    with open(os.path.join(d, "lenna.data"), "rb") as f:
        src = bytes_to_img(f.read())
    with open(os.path.join(d, "lenna_out.data"), "rb") as f:
        want = bytes_to_img(f.read())
    assert torch.equal(ops.roberts_rgb(src.to(gpu)).cpu(), want)


@pytest.mark.parametrize("hw", [(1, 1), (3, 5), (17, 64), (130, 257), (1024, 1000), (4096, 4096)])
def test_roberts_rgb_gpu_matches_cpu(gpu, hw):
    """Both launch forms (16-B quads when w % 4 == 0, per pixel otherwise),
    image edges included, against the native CPU reference."""
    img = rand_img(*hw, seed=hw[0] + hw[1])
    assert torch.equal(ops.roberts_rgb(img.to(gpu)).cpu(), ops.roberts_rgb(img))


@pytest.mark.parametrize("fname", ["sobel5", "gauss5", "roberts", "sobel5_dense"])
def test_conv_resident_hint_same_bytes(gpu, fname):
    """MPX_CONV_RESIDENT (ops.conv(..., resident=True), ConvLauncher.resident)
    changes only the band kernel's load policy: the bytes equal the default
    launch's and the CPU reference's (2048^2: above the band kernel's 4 Mpx
    threshold)."""
    img = rand_img(2048, 2048, seed=21)
    d = img.to(gpu)
    a = ops.conv(d, fname)
    b = ops.conv(d, fname, resident=True)
    assert torch.equal(a, b)
    assert torch.equal(a.cpu(), ops.conv(img, fname))
    out = torch.empty_like(d)
    ln = ops.ConvLauncher(d, out, ops.get_filter(fname), src_row0=0, out_row0=0, oy0=0, oy1=2048, y_lo=0, y_hi=2047)
    ln.resident = True
    assert ln.resident
    ln()
    torch.cuda.synchronize()
    assert torch.equal(out, a)
    ln.resident = False
    assert not ln.resident


def test_tune_library_variants_match_production(gpu):
    """The tuning entry points that live in libmpx_tune.so (round 6: the
    Jacobi and vsub variants left libmpx) compute what the production kernels
    compute: vsub kinds 0-3 against ops.vsub, Jacobi wave variants against
    ops.jacobi_sweep, interior rows bit-exact."""
    from cuda_mpi_openmp_amd import _native

    T = _native.tune_lib()
    for dt in (torch.float32, torch.float64):
        a = torch.rand(1 << 20, dtype=dt, device=gpu)
        b = torch.rand(1 << 20, dtype=dt, device=gpu)
        want = ops.vsub(a, b)
        for kind in range(4):
            c = torch.full_like(a, float("nan"))
            _native.check(T.mpx_vsub_variant(a.data_ptr(), b.data_ptr(), c.data_ptr(), a.numel(),
                                             int(dt == torch.float64), kind, 0, None))
            torch.cuda.synchronize()
            assert torch.equal(c, want), (dt, kind)
        n = 512
        u = torch.rand((n + 2, n), dtype=dt, device=gpu)
        ref = torch.empty_like(u)
        ops.jacobi_sweep(u, ref, 1, n + 1)
        for R, aux in ((8, 0), (8, 18), (5, 2), (16, 22)):
            un = torch.zeros_like(u)
            _native.check(T.mpx_jacobi_variant(u.data_ptr(), un.data_ptr(), n, n, 1, n + 1, None,
                                               int(dt == torch.float64), R, aux, None))
            torch.cuda.synchronize()
            assert torch.equal(un[1:n + 1, 1:-1], ref[1:n + 1, 1:-1]), (dt, R, aux)
