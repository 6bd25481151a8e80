"""Host-only AddressSanitizer / UBSan runs of the native CPU programs
(``make sanitize``; SURVEY §5 "race detection / sanitizers"). GPU ASan needs
xnack+ code objects, which the MI355X pool does not run, so the sanitizers
cover the host code: CPU references, .data I/O, stdin parsers."""

import os
import subprocess

import pytest

from .helpers import LAB2_DATA, LAB2_GT, LAB3_DATA, LAB3_GT, ROOT, hex_bytes

SAN = os.path.join(ROOT, "build", "san")


@pytest.fixture(scope="module", autouse=True)
def sanitized_build():
    r = subprocess.run(["make", "-C", ROOT, "-j", "8", "sanitize"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


def run(name, stdin):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="4")
    r = subprocess.run([os.path.join(SAN, name)], input=stdin, text=True, capture_output=True, env=env, timeout=300)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-3000:]
    assert "ERROR: LeakSanitizer" not in r.stderr, r.stderr[-3000:]
    return r


@pytest.mark.parametrize("exe", ["lab1_cpu_exe", "lab1_cpu_omp_exe"])
def test_lab1(exe):
    r = run(exe, "3\n1 2 3\n4 5 6")
    assert r.returncode == 0 and r.stdout.endswith("-3.0000000000e+00 -3.0000000000e+00 -3.0000000000e+00 ")
    r = run(exe, "3\n1 2 3\n4 5")  # truncated input: clean error, no overflow
    assert r.returncode != 0


@pytest.mark.parametrize("exe", ["lab2_cpu_exe", "lab2_cpu_omp_exe"])
def test_lab2(exe, tmp_path):
    src = tmp_path / "in.data"
    src.write_bytes(hex_bytes(os.path.join(LAB2_DATA, "test_01.txt")))
    out = tmp_path / "out.data"
    r = run(exe, f"{src}\n{out}")
    assert r.returncode == 0
    assert out.read_bytes() == hex_bytes(os.path.join(LAB2_GT, "test_01.txt"))
    r = run(exe, f"{os.path.join(LAB2_DATA, '96.data')}\n{out}")  # a real image through the sanitizer
    assert r.returncode == 0
    bad = tmp_path / "bad.data"
    bad.write_bytes(b"\x05\x00\x00\x00\x05\x00\x00\x00\x01\x02")  # header promises 25 px, holds 2 bytes
    r = run(exe, f"{bad}\n{out}")
    assert r.returncode != 0


@pytest.mark.parametrize("exe", ["lab3_cpu_exe", "lab3_cpu_omp_exe"])
def test_lab3(exe, tmp_path):
    src = tmp_path / "in.data"
    src.write_bytes(hex_bytes(os.path.join(LAB3_DATA, "test_01_lab3.txt")))
    out = tmp_path / "out.data"
    r = run(exe, f"{src}\n{out}\n2\n4 1 2 1 0 2 2 2 1\n4 0 0 0 1 1 1 2 0")
    assert r.returncode == 0
    assert out.read_bytes() == hex_bytes(os.path.join(LAB3_GT, "test_01_lab3.txt"))
    for bad in ("0", "2\n4 1 2 1 0 2 2 2", "1\n2 0 0 9 9", "1\n" + "600 " + "1 1 " * 600):
        r = run(exe, f"{src}\n{out}\n{bad}")  # clean errors (and one realloc growth), no leaks
        assert r.returncode != 0 or bad.startswith("1\n600")


def test_small_programs():
    assert run("hw1", "1 -3 2").returncode == 0
    assert run("hw2", "4\n3 1 2 0").stdout.startswith("0.000000e+00")
    assert run("lab3_read_input_exe", "2\n4 1 2 1 0 2 2 2 1\n4 0 0 0 1 1 1 2 0").returncode == 0
