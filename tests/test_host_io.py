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
