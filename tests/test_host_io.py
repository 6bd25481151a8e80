"""lab1 host text I/O (reference lab1/src/main.cu:46-52 scanf, :82-84 printf):
the parallel parser / formatter in libmpx (mpx_parse_doubles, mpx_format_e10)
must give exactly the serial strtod / "%.10e " results."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from cuda_mpi_openmp_amd import _native

from .helpers import ROOT

libc = ctypes.CDLL(None)
libc.strtod.restype = ctypes.c_double
libc.strtod.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]


def _parse(text: bytes, count: int, pos: int = 0):
    L = _native.lib()
    L.mpx_parse_doubles.restype = ctypes.c_int64
    L.mpx_parse_doubles.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
    out = np.zeros(max(count, 1), dtype=np.float64)
    end = ctypes.c_size_t(0)
    got = L.mpx_parse_doubles(text, len(text), pos, count, out.ctypes.data, ctypes.byref(end))
    return got, out[:count], end.value


def _serial(tokens):
    return np.array([libc.strtod(t, None) for t in tokens], dtype=np.float64)


@pytest.mark.parametrize("n", [1, 7, 5000, 200_003])
def test_parse_matches_serial_strtod(n):
    rng = np.random.default_rng(n)
    vals = rng.uniform(-1e100, 1e100, n) * 10.0 ** rng.integers(-200, 100, n)
    special = [b"-0", b"+5", b"1e308", b"4.9e-324", b"inf", b"-inf", b"0x1p3", b"1.0000000001e+100", b"3"]
    toks = [np.format_float_scientific(v, precision=int(rng.integers(1, 17))).encode() for v in vals]
    toks[: min(n, len(special))] = special[: min(n, len(special))]
    seps = [b" ", b"\n", b"\t ", b"  \r\n"]
    text = b"\n  " + b"".join(t + seps[i % 4] for i, t in enumerate(toks)) + b"999 trailing"
    got, out, end = _parse(text, n)
    assert got == n
    ref = _serial(toks)
    assert out.tobytes() == ref.tobytes()  # bit-identical, NaN/inf/-0 included
    assert text[end - len(toks[-1]):end] == toks[-1]


def test_parse_reports_first_bad_token():
    text = b"1 2 3 x4 5 6" + b" 7" * 70000
    got, _, _ = _parse(text, 10)
    assert got == 3
    got, _, _ = _parse(b"1 2 3.5e", 3)
    assert got == 2
    got, out, _ = _parse(b"1 2", 5)  # too few tokens
    assert got == 2 and list(out[:2]) == [1.0, 2.0]


def test_format_matches_printf():
    L = _native.lib()
    L.mpx_format_e10.restype = ctypes.c_void_p
    L.mpx_format_e10.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_size_t)]
    rng = np.random.default_rng(3)
    v = np.concatenate([rng.uniform(-1e100, 1e100, 100_000), [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-310]])
    n = ctypes.c_size_t(0)
    p = L.mpx_format_e10(v.ctypes.data, v.size, ctypes.byref(n))
    got = ctypes.string_at(p, n.value)
    libc.free(ctypes.c_void_p(p))
    want = b"".join(b"%.10e " % x for x in v)
    assert got == want


def test_lab1_cpu_programs_agree_on_large_input():
    """cpu_exe (serial scanf/printf, -O0) and cpu_omp_exe (parallel parse and
    format) print the same bytes."""
    rng = np.random.default_rng(1)
    n = 300_001
    a, b = rng.uniform(-1e100, 1e100, n), rng.uniform(-1e100, 1e100, n)
    text = (f"{n}\n" + " ".join(f"{x:.10e}" for x in a) + "\n" + " ".join(repr(float(x)) for x in b)).encode()
    outs = []
    for exe in ("cpu_exe", "cpu_omp_exe"):
        r = subprocess.run([os.path.join(ROOT, "labs", "lab1", "src", exe)], input=text, capture_output=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.split(b"\n", 1)[1])
    assert outs[0] == outs[1]
    a10 = np.array([float(f"{x:.10e}") for x in a])  # the values the programs read
    assert outs[1] == b"".join(b"%.10e " % x for x in (a10 - b))


def _format(v):
    L = _native.lib()
    L.mpx_format_e10.restype = ctypes.c_void_p
    L.mpx_format_e10.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_size_t)]
    v = np.ascontiguousarray(v, dtype=np.float64)
    n = ctypes.c_size_t(0)
    p = L.mpx_format_e10(v.ctypes.data, v.size, ctypes.byref(n))
    got = ctypes.string_at(p, n.value)
    libc.free(ctypes.c_void_p(p))
    return got


def test_format_random_bit_patterns_exact():
    """The fast %.10e path (one 64x128-bit product with a truncated power of
    ten, exact-or-fallback) over random bit patterns of the whole double range
    — subnormals, powers of ten, round-half cases included — equals printf."""
    rng = np.random.default_rng(11)
    bits = rng.integers(0, 2**63, 400_000, dtype=np.uint64) | (rng.integers(0, 2, 400_000, dtype=np.uint64) << 63)
    v = bits.view(np.float64)
    v = v[np.isfinite(v)]
    edge = np.array([5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, 1e23, 9.99999999995e22,
                     1.00000000005, 1.00000000015, 0.5, 2.5e-5, 123456789012.5, 99999999999.5, 9.999999999950001])
    ints = rng.integers(1, 10**15, 100_000).astype(np.float64)                   # exact integers: halves, ties
    halves = (rng.integers(10**10, 10**11, 50_000) * 2 + 1).astype(np.float64) / 2  # exact ...5 ties at digit 11
    v = np.concatenate([v, -v[:1000], edge, -edge, ints, halves, np.ldexp(1.0, np.arange(-1074, 1024))])
    assert _format(v) == b"".join(b"%.10e " % x for x in v)


def test_parse_random_values_exact():
    """The fast parse (Clinger / Eisel-Lemire with exact fallback) equals
    strtod bit for bit on random doubles of the whole range written with
    1..17 significant digits in several styles, and on near-halfway inputs."""
    rng = np.random.default_rng(12)
    bits = rng.integers(0, 2**63, 200_000, dtype=np.uint64)
    vals = bits.view(np.float64)
    vals = vals[np.isfinite(vals)]
    toks = []
    for i, x in enumerate(vals):
        st = i % 5
        if st == 0:
            toks.append(repr(float(x)).encode())
        elif st == 1:
            toks.append(b"%.*e" % (int(rng.integers(0, 17)), x))
        elif st == 2:
            toks.append(b"%.*g" % (int(rng.integers(1, 18)), x))
        elif st == 3:
            toks.append(b"-%.10e" % x)
        else:
            toks.append(b"%.17g" % x)
    # halfway points between neighbouring doubles, written with 17-19 digits
    for x in rng.uniform(1, 1e10, 2000):
        mid = (float(x) + float(np.nextafter(x, np.inf))) / 2
        toks.append(b"%.19g" % mid)
        toks.append(b"%.17e" % mid)
    toks += [b"0.000000", b"-0.0", b"007", b"1e-400", b"1e400", b"4.9e-324", b"2.4703282292062328e-324",
             b"123456789012345678901234567890", b"0.1e1", b".5", b"5.", b"+.5e-3", b"9007199254740993"]
    text = b" ".join(toks) + b"\n"
    got, out, _ = _parse(text, len(toks))
    assert got == len(toks)
    assert out.tobytes() == _serial(toks).tobytes()


def test_lab1_host_io_speedup_and_identical(tmp_path):
    """the OpenMP lab1 program (fast exact parse / format,
    parallel) spends >= 5x less wall time than the serial scanf / printf path
    on a large input, with byte-identical output."""
    import time

    rng = np.random.default_rng(2)
    n = 1 << 21
    a, b = rng.uniform(-1e100, 1e100, n), rng.uniform(-1e100, 1e100, n)
    inp = tmp_path / "in.txt"
    inp.write_bytes(b"%d\n" % n + _format(a) + b"\n" + _format(b))
    outs, wall = [], {}
    for exe in ("cpu_exe", "cpu_omp_exe"):
        with open(inp, "rb") as f:
            t0 = time.perf_counter()
            r = subprocess.run([os.path.join(ROOT, "labs", "lab1", "src", exe)], stdin=f, capture_output=True,
                               timeout=600)
            wall[exe] = time.perf_counter() - t0
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.split(b"\n", 1)[1])
    assert outs[0] == outs[1]
    assert wall["cpu_exe"] >= 5.0 * wall["cpu_omp_exe"], wall
