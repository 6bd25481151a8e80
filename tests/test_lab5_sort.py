"""lab5: ascending sort of the reference's binary lab5/data fixtures.

The reference ships only the inputs (int10, float10, uchar10) and no program,
so parity is unpinned: the oracle is numpy's sort (and, for floats, the IEEE
total order of the bit patterns, which numpy's sort does not define for NaN
and -0.0). GPU results are compared byte for byte with the C reference.
"""
import os
import subprocess

import numpy as np
import pytest
import torch

from cuda_mpi_openmp_amd import ops
from cuda_mpi_openmp_amd.ops.sort import read_fixture

from .helpers import ROOT

LAB5_DATA = os.path.join(ROOT, "labs", "lab5", "data")
KINDS = {"int": (np.int32, torch.int32), "float": (np.float32, torch.float32), "uchar": (np.uint8, torch.uint8)}


def total_order_sorted(a: np.ndarray) -> np.ndarray:
    """Reference order: int/uint8 numerically; float32 by the IEEE total order."""
    if a.dtype != np.float32:
        return np.sort(a, kind="stable")
    u = a.view(np.uint32)
    key = np.where(u >> 31 == 1, ~u, u | np.uint32(0x80000000))
    return a[np.argsort(key, kind="stable")]


def random_array(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "int":
        a = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        if n > 4:
            a[:4] = [-2**31, 2**31 - 1, 0, -1]
        return a
    if kind == "uchar":
        return rng.integers(0, 256, n, dtype=np.int64).astype(np.uint8)
    a = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    if n > 8:
        a[:8] = [np.inf, -np.inf, 0.0, -0.0, np.nan, -np.nan, 1e-45, -1e-45]
    return a


def fixture_bytes(kind, a):
    return np.int32(a.size).tobytes() + a.astype(KINDS[kind][0]).tobytes()


@pytest.mark.parametrize("kind", list(KINDS))
def test_fixtures_parse(kind):
    a = read_fixture(os.path.join(LAB5_DATA, kind + "10"), kind)
    assert a.size == 10
    expected = {"int": [0, 9, 8, 7, 6, 5, 4, 3, 2, 1], "float": [0, 9, 8, 7, 6, 5, 4, 3, 2, 1],
                "uchar": [1, 2, 3, 1, 2, 3, 1, 2, 3, 4]}[kind]
    assert a.tolist() == expected


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("n", [0, 1, 2, 3, 10, 1000, 4097, 200_003])
def test_cpu_sort_matches_total_order(kind, n):
    """libmpx's CPU path is the OpenMP build: n >= 2^16 takes the parallel
    run-sort + pairwise-merge path (uint8: per-thread histograms)."""
    a = random_array(kind, n, seed=n)
    t = torch.from_numpy(a.copy())
    ops.sort_(t)
    assert t.numpy().tobytes() == total_order_sorted(a).tobytes()


@pytest.mark.parametrize("exe", ["cpu_exe", "cpu_omp_exe"])
@pytest.mark.parametrize("kind", list(KINDS))
def test_lab5_cpu_program_on_fixtures(exe, kind):
    path = os.path.join(LAB5_DATA, kind + "10")
    with open(path, "rb") as f:
        r = subprocess.run([os.path.join(ROOT, "labs/lab5/src", exe), kind], stdin=f, capture_output=True,
                           timeout=60)
    assert r.returncode == 0, r.stderr
    head, _, payload = r.stdout.partition(b"\n")
    assert head.startswith(b"CPU execution time: <")
    a = read_fixture(path, kind)
    assert payload == np.sort(a).tobytes()


@pytest.mark.parametrize("exe", ["cpu_exe", "cpu_omp_exe"])
@pytest.mark.parametrize("kind", list(KINDS))
def test_lab5_cpu_program_large(exe, kind):
    """Serial -O0 and OpenMP builds agree with the total order on an array
    large enough for the parallel merge path."""
    a = random_array(kind, 300_007, seed=11)
    r = subprocess.run([os.path.join(ROOT, "labs/lab5/src", exe), kind], input=fixture_bytes(kind, a),
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.partition(b"\n")[2] == total_order_sorted(a).tobytes()


def test_lab5_cpu_program_rejects_short_input():
    r = subprocess.run([os.path.join(ROOT, "labs/lab5/src/cpu_exe"), "int"], input=np.int32(5).tobytes() + b"\0" * 8,
                       capture_output=True, timeout=60)
    assert r.returncode != 0 and b"expected 5 binary elements" in r.stderr


def test_sort_rejects_bad_dtype():
    with pytest.raises(ValueError):
        ops.sort_(torch.zeros(4, dtype=torch.float64))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("n", [0, 1, 2, 3, 10, 4095, 4096, 4097, 8191, 8192, 8193, 12289, 100_003, (1 << 20) + 7,
                               (1 << 22) + 3])
def test_gpu_sort_matches_cpu(gpu, kind, n):
    """Path and tile boundaries: the one-launch LDS bitonic network up to 4096
    keys, the radix sort above (8192-key tiles: a partial last tile, exactly
    one and just over one tile), and multi-thousand-tile look-back chains."""
    a = random_array(kind, n, seed=n + 1)
    d = torch.from_numpy(a.copy()).to(gpu)
    ops.sort_(d)
    assert d.cpu().numpy().tobytes() == total_order_sorted(a).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int_uniform", "int_range", "float_normal"])
def test_gpu_sort_auto_at_2_26(gpu, kind):
    """AUTO at 2^26 + 5 keys: 16384-key tiles (variant 22, one 1024-thread
    block per CU), a partial last tile, hot-digit ranking on the skewed
    passes — equal to torch.sort (no NaN / signed zeros in these inputs, where
    torch's order and the IEEE total order agree)."""
    n = (1 << 26) + 5
    g = torch.Generator(device=gpu)
    g.manual_seed(26)
    if kind == "int_uniform":
        x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=gpu, generator=g)
    elif kind == "int_range":
        x = torch.randint(0, 1000, (n,), dtype=torch.int32, device=gpu, generator=g)
    else:
        x = torch.randn(n, device=gpu, generator=g)
    ref = torch.sort(x).values
    ops.sort_(x)
    assert torch.equal(x.view(torch.int32), ref.view(torch.int32))


@pytest.mark.gpu
def test_gpu_sort_lane_order_probe(gpu):
    """the production ranking's stability premise (same-address
    returning LDS adds in ascending lane order) is probed once per device;
    gfx950 satisfies it, so AUTO keeps the returning-add variants."""
    from cuda_mpi_openmp_amd import _native

    assert _native.lib().mpx_sort_lane_order_ok(_native.stream_of(torch.empty(1, device=gpu))) == 1


@pytest.mark.gpu
def test_gpu_sort_matches_torch_and_handles_duplicates(gpu):
    x = torch.randint(-50, 50, (300_001,), dtype=torch.int32, device=gpu)
    ref = torch.sort(x).values
    ops.sort_(x)
    assert torch.equal(x, ref)
    f = torch.randn(1 << 18, device=gpu)
    ref = torch.sort(f).values
    ops.sort_(f)
    assert torch.equal(f, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("exe", ["to_plot_hip_exe", "hip_exe"])
@pytest.mark.parametrize("kind", list(KINDS))
def test_lab5_gpu_program(exe, kind):
    a = random_array(kind, 50_000, seed=7)
    for data in (fixture_bytes(kind, a), open(os.path.join(LAB5_DATA, kind + "10"), "rb").read()):
        r = subprocess.run([os.path.join(ROOT, "labs/lab5/src", exe), kind], input=data, capture_output=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        src = np.frombuffer(data[4:], dtype=KINDS[kind][0])
        payload = r.stdout
        if exe == "to_plot_hip_exe":
            head, _, payload = r.stdout.partition(b"\n")
            assert head.startswith(b"HIP execution time: <")
        assert payload == total_order_sorted(src).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", list(KINDS))
def test_gpu_sort_twice_in_place(gpu, kind):
    """The CLI's warm timing sorts the same buffer again: re-sorting sorted
    data (every wave hitting one histogram bin for uint8) must be a no-op."""
    a = random_array(kind, 50_000, seed=7)
    d = torch.from_numpy(a.copy()).to(gpu)
    for _ in range(3):
        ops.sort_(d)
        torch.cuda.synchronize()
        assert d.cpu().numpy().tobytes() == total_order_sorted(a).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("offset", [1, 3, 15, 16])
@pytest.mark.parametrize("n", [5, 17, 40_000, 1 << 20])
def test_gpu_sort_u8_unaligned(gpu, offset, n):
    """uint8 views that start off a 16-B boundary: bytewise head, 16-B body,
    bytewise tail; the bytes before the view stay untouched."""
    a = random_array("uchar", n + offset, seed=n + offset)
    d = torch.from_numpy(a.copy()).to(gpu)
    ops.sort_(d[offset:])
    got = d.cpu().numpy()
    assert got[:offset].tobytes() == a[:offset].tobytes()
    assert got[offset:].tobytes() == np.sort(a[offset:]).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [33, 1_000, 65_537, 1 << 22, 50_000_017])
def test_gpu_sort_u8_skewed(gpu, n):
    """uint8 counting sort on skewed bytes: most bins empty, one bin holding
    most keys, single-key bins, bucket edges inside a 16-B piece and across
    the per-wave runs of the fill."""
    rng = np.random.default_rng(n)
    a = rng.choice(np.array([0, 1, 7, 128, 200, 255], dtype=np.uint8), n, p=[0.02, 0.6, 0.1, 0.25, 0.02, 0.01])
    a[rng.integers(0, n, 3)] = [3, 99, 254]
    d = torch.from_numpy(a.copy()).to(gpu)
    ops.sort_(d)
    assert d.cpu().numpy().tobytes() == np.sort(a).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", ["equal", "sorted", "reversed", "two_values", "high_byte_only"])
def test_gpu_radix_sort_patterns(gpu, pattern):
    """Radix-specific digit distributions: a single digit value in every pass
    (all keys in one bucket: the look-back carries whole-tile counts), already
    sorted / reversed input (stability of the per-wave ranking), keys that
    differ only in the top byte (three passes are pure stable copies)."""
    n = 300_007
    rng = np.random.default_rng(5)
    if pattern == "equal":
        a = np.full(n, -7, dtype=np.int32)
    elif pattern == "sorted":
        a = np.sort(rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32))
    elif pattern == "reversed":
        a = np.sort(rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32))[::-1].copy()
    elif pattern == "two_values":
        a = rng.choice(np.array([3, -3], dtype=np.int32), n)
    else:
        a = (rng.integers(0, 256, n, dtype=np.int64) << 24).astype(np.uint32).view(np.int32)
    d = torch.from_numpy(a.copy()).to(gpu)
    ops.sort_(d)
    assert d.cpu().numpy().tobytes() == np.sort(a).tobytes()


@pytest.mark.gpu
def test_gpu_sort_is_stable_on_float_ties(gpu):
    """-0.0 and +0.0 are distinct keys; equal bit patterns keep their order —
    checked through the byte patterns of a tie-heavy float array."""
    n = 200_003
    rng = np.random.default_rng(9)
    a = rng.choice(np.array([0.0, -0.0, 1.5, -1.5, np.inf], dtype=np.float32), n)
    d = torch.from_numpy(a.copy()).to(gpu)
    ops.sort_(d)
    assert d.cpu().numpy().tobytes() == total_order_sorted(a).tobytes()


@pytest.mark.gpu
def test_gpu_sorts_on_two_streams_do_not_share_scratch(gpu):
    """Scratch comes from the caller (torch's caching allocator on each
    tensor's stream): two sorts in flight on different streams stay
    independent (round-1 advisor finding on the shared per-device scratch)."""
    xs = [torch.randint(0, 256, (3_000_000,), dtype=torch.uint8, device=gpu),
          torch.randint(-2**31, 2**31 - 1, (3_000_000,), dtype=torch.int32, device=gpu),
          torch.randint(0, 256, (2_000_001,), dtype=torch.uint8, device=gpu),
          torch.randint(-2**31, 2**31 - 1, (2_000_001,), dtype=torch.int32, device=gpu)]
    refs = [torch.sort(x).values for x in xs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(gpu) for _ in xs]
    for x, st in zip(xs, streams):
        with torch.cuda.stream(st):
            for _ in range(3):
                ops.sort_(x)
    torch.cuda.synchronize()
    for x, r in zip(xs, refs):
        assert torch.equal(x, r)


@pytest.mark.gpu
def test_gpu_sort_workspace_contract(gpu):
    """mpx_sort_ws refuses a workspace smaller than mpx_sort_workspace_bytes."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    n = 100_000
    need = int(L.mpx_sort_workspace_bytes(n, 0))
    assert need >= 4 * n
    assert int(L.mpx_sort_workspace_bytes(4096, 0)) == 0  # single-tile bitonic path needs none
    x = torch.zeros(n, dtype=torch.int32, device=gpu)
    ws = torch.empty(need - 16, dtype=torch.uint8, device=gpu)
    rc = L.mpx_sort_ws(x.data_ptr(), n, 0, ws.data_ptr(), need - 16, _native.stream_of(x))
    assert rc != 0 and b"workspace" in L.mpx_last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [1, 2, 4, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22])
@pytest.mark.parametrize("kind", ["int", "float"])
@pytest.mark.parametrize("n", [4097, 8193, 100_003, (1 << 20) + 7, (1 << 23) + 5])
def test_gpu_radix_variants(gpu, variant, kind, n):
    """Every radix schedule (1 onesweep look-back, 2 reduce-then-scan, 4 / 7 / 8
    the same with persistent prefetching scatters, 9 the lean scatter ranked by
    returning LDS adds — stable only if one instruction's same-address lanes
    apply in lane order, which this checks) against the total order,
    independent of which one AUTO picks at this size."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    dt = {"int": 0, "float": 1}[kind]
    a = random_array(kind, n, seed=n + variant)
    d = torch.from_numpy(a.copy()).to(gpu)
    nb = int(L.mpx_sort_workspace_bytes(n, dt))
    ws = torch.empty(nb, dtype=torch.uint8, device=gpu)
    _native.check(_native.tune_lib().mpx_sort_variant(d.data_ptr(), n, dt, ws.data_ptr(), nb, variant, _native.stream_of(d)))
    assert d.cpu().numpy().tobytes() == total_order_sorted(a).tobytes()
    _native.check(L.mpx_sort_ws_status(ws.data_ptr(), n, dt))  # no look-back wait gave up


def skewed_array(kind, n, seed):
    """Digit distributions with hot digits (at least 1/32 of the keys on one
    digit value in some pass): what RANK 3 ranks by ballot."""
    rng = np.random.default_rng(seed)
    if kind == "float_normal":  # top byte: a handful of sign / exponent values
        return rng.standard_normal(n).astype(np.float32)
    if kind == "float_unit":  # [0, 1): top byte 0x3f / 0x3e / ... (few), the rest uniform
        return rng.random(n, dtype=np.float32)
    if kind == "int_range":  # passes 2 and 3: one digit; pass 1: four
        return rng.integers(0, 1000, n, dtype=np.int64).astype(np.int32)
    if kind == "int_mix":  # 60 % one value, the rest uniform: one hot digit in every pass
        a = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        a[rng.random(n) < 0.6] = 0x12345678
        return a
    # "int_many_hot": eight top bytes of 1/8 each — more hot digits than
    # kHotMax, so four take ballots and four the returning add in one pass
    hi = rng.integers(0, 8, n, dtype=np.int64) * 29 + 3
    return ((hi << 24) | rng.integers(0, 1 << 24, n, dtype=np.int64)).astype(np.uint32).view(np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [12, 13, 18, 19, 20, 21, 22])
@pytest.mark.parametrize("kind", ["float_normal", "float_unit", "int_range", "int_mix", "int_many_hot"])
@pytest.mark.parametrize("n", [8193, (1 << 20) + 7, (1 << 23) + 5])
def test_gpu_radix_variants_skewed_digits(gpu, variant, kind, n):
    """Hot digits: the returning-add ranking (12 / 13) serialises same-address
    lanes, RANK 3 (18 / 19) ranks up to four hot digits per pass by ballot and
    the rest by returning adds. Both must stay stable (the lower passes' order
    survives every later pass) — checked against the total order."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    a = skewed_array(kind, n, seed=n + variant)
    dt = 1 if kind.startswith("float") else 0
    d = torch.from_numpy(a.copy()).to(gpu)
    nb = int(L.mpx_sort_workspace_bytes(n, dt))
    ws = torch.empty(nb, dtype=torch.uint8, device=gpu)
    _native.check(_native.tune_lib().mpx_sort_variant(d.data_ptr(), n, dt, ws.data_ptr(), nb, variant, _native.stream_of(d)))
    assert d.cpu().numpy().tobytes() == total_order_sorted(a).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 2, 4, 7, 8])
def test_gpu_sort_ws_status_ignores_stale_workspace(gpu, variant):
    """A recycled workspace full of 0xff bytes must not make mpx_sort_ws_status
    report a look-back give-up after a reduce-then-scan sort (which never
    waits): every schedule clears the flag it reads."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    n = (1 << 18) + 1001  # above the onesweep crossover: AUTO picks reduce-then-scan
    a = random_array("int", n, seed=77)
    d = torch.from_numpy(a.copy()).to(gpu)
    nb = int(L.mpx_sort_workspace_bytes(n, 0))
    ws = torch.full((nb,), 0xFF, dtype=torch.uint8, device=gpu)
    _native.check(_native.tune_lib().mpx_sort_variant(d.data_ptr(), n, 0, ws.data_ptr(), nb, variant, _native.stream_of(d)))
    torch.cuda.synchronize()
    assert d.cpu().numpy().tobytes() == total_order_sorted(a).tobytes()
    _native.check(L.mpx_sort_ws_status(ws.data_ptr(), n, 0))


def test_retired_sort_variants_are_refused():
    """Variants 3 (ballot peer masks), 5 (reverse tile walk) and 6 (six
    barriers per tile) were measured slower and removed (profiles/lab5_sort.md):
    the tuning entry refuses them before touching any memory."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    for v in (3, 5, 6, 23, -1):
        assert _native.tune_lib().mpx_sort_variant(None, 1 << 20, 0, None, 0, v, None) != 0
        assert b"sort variant" in L.mpx_last_error()


def test_scatter_probe_refuses_bad_args():
    """The tuning probe (tools/experiments/sort_probe.py) checks its inputs
    before any launch: unknown knock masks and missing workspaces."""
    from cuda_mpi_openmp_amd import _native

    L = _native.lib()
    assert _native.tune_lib().mpx_sort_scatter_probe(None, 1 << 20, None, 0, 0, None) != 0
    assert b"probe" in L.mpx_last_error()


def test_sort_experiments_live_in_the_tuning_library():
    """VERDICT r5 Next #3: libmpx exports only the production sort entry points;
    the variant table and the scatter probe are in libmpx_tune.so."""
    from cuda_mpi_openmp_amd import _native

    import ctypes

    raw = ctypes.CDLL(_native.lib()._name)  # a fresh handle: no attributes bound by _native
    T = _native.tune_lib()
    for name in ("mpx_sort_variant", "mpx_sort_scatter_probe"):
        assert hasattr(T, name)
        assert not hasattr(raw, name), f"{name} still exported by libmpx"
    assert hasattr(raw, "mpx_sort_ws") and hasattr(raw, "mpx_sort_lane_order_ok")
