"""The native command-line programs and their stdin/stdout contracts
(SURVEY Appendix A): CPU builds run here, GPU builds on the MI355X."""

import os
import subprocess

import numpy as np
import pytest

from .helpers import LAB2_DATA, LAB2_GT, LAB3_DATA, LAB3_GT, ROOT, hex_bytes


def run(exe, stdin, env=None, args=()):
    e = dict(os.environ)
    if env:
        e.update(env)
    return subprocess.run([os.path.join(ROOT, exe), *args], input=stdin, text=True, capture_output=True, env=e,
                          timeout=120)


def write_hex_as_data(src, dst):
    with open(dst, "wb") as f:
        f.write(hex_bytes(src))
    return dst


@pytest.mark.parametrize("exe", ["labs/lab1/src/cpu_exe", "labs/lab1/src/cpu_omp_exe"])
def test_lab1_cpu_contract(exe):
    r = run(exe, "3\n1 2 3\n4 5 6")
    assert r.returncode == 0
    head, _, body = r.stdout.partition("\n")
    assert head.startswith("CPU execution time: <") and head.endswith(" ms>")
    assert body == "-3.0000000000e+00 -3.0000000000e+00 -3.0000000000e+00 "


def test_lab1_cpu_truncated_input_fails():
    r = run("labs/lab1/src/cpu_exe", "3\n1 2 3\n4 5")
    assert r.returncode != 0 and "expected" in r.stderr


@pytest.mark.parametrize("exe", ["labs/lab2/src/cpu_exe", "labs/lab2/src/cpu_omp_exe"])
@pytest.mark.parametrize("name", ["test_01", "test_02"])
def test_lab2_cpu_ground_truth(exe, name, tmp_path):
    src = write_hex_as_data(os.path.join(LAB2_DATA, name + ".txt"), tmp_path / "in.data")
    out = tmp_path / "out.data"
    r = run(exe, f"{src}\n{out}")
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("CPU execution time: <")
    assert out.read_bytes() == hex_bytes(os.path.join(LAB2_GT, name + ".txt"))


def test_lab2_cpu_missing_input(tmp_path):
    r = run("labs/lab2/src/cpu_exe", f"{tmp_path}/nope.data\n{tmp_path}/o.data")
    assert r.returncode != 0 and "Error opening input file" in r.stderr


def test_lab2_cpu_other_filter(tmp_path):
    src = os.path.join(LAB2_DATA, "96.data")
    r = run("labs/lab2/src/cpu_omp_exe", f"{src}\n{tmp_path}/o.data", env={"MPX_LAB2_OP": "sobel3"})
    assert r.returncode == 0, r.stderr
    r = run("labs/lab2/src/cpu_omp_exe", f"{src}\n{tmp_path}/o.data", args=("--op", "nope"))
    assert r.returncode != 0


@pytest.mark.parametrize("exe", ["labs/lab3/src/cpu_exe", "labs/lab3/src/cpu_omp_exe"])
def test_lab3_cpu_ground_truth(exe, tmp_path):
    src = write_hex_as_data(os.path.join(LAB3_DATA, "test_01_lab3.txt"), tmp_path / "in.data")
    out = tmp_path / "out.data"
    r = run(exe, f"{src}\n{out}\n2\n4 1 2 1 0 2 2 2 1\n4 0 0 0 1 1 1 2 0")
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == hex_bytes(os.path.join(LAB3_GT, "test_01_lab3.txt"))


def test_lab3_read_input_probe():
    r = run("labs/lab3/src/read_input_exe", "2\n4 1 2 1 0 2 2 2 1\n4 0 0 0 1 1 1 2 0")
    assert r.returncode == 0
    assert "Class 1:" in r.stdout and "(2, 1)" in r.stdout and "Pixel count: 4" in r.stdout


@pytest.mark.parametrize("stdin,expect", [
    ("1 -3 2", "2.000000 1.000000\n"),
    ("0 0 0", "any\n"),
    ("0 0 5", "incorrect\n"),
    ("0 2 -4", "2.000000\n"),
    ("1 2 1", "-1.000000\n"),
    ("1 0 1", "imaginary\n"),
])
def test_hw1_quadratic(stdin, expect):
    assert run("bin/hw1", stdin).stdout == expect


def test_hw2_bubble_sort():
    vals = np.random.default_rng(0).normal(size=50).astype(np.float32)
    r = run("bin/hw2", f"{len(vals)} " + " ".join(map(str, vals)))
    got = np.array(r.stdout.split(), dtype=np.float32)
    assert np.allclose(got, np.sort(vals), rtol=1e-6)
    assert r.stdout.endswith(" \n")


# ---------------------------------------------------------------- GPU builds
@pytest.mark.gpu
@pytest.mark.parametrize("geom", ["0\n0", "1\n32", "512\n512", "1024\n1024"])
def test_lab1_gpu_contract(geom):
    r = run("labs/lab1/src/to_plot_hip_exe", f"{geom}\n3\n1 2 3\n4 5 6")
    assert r.returncode == 0, r.stderr
    head, _, body = r.stdout.partition("\n")
    assert head.startswith("HIP execution time: <")
    assert body == "-3.0000000000e+00 -3.0000000000e+00 -3.0000000000e+00 "
    r2 = run("labs/lab1/src/hip_exe", "3\n1 2 3\n4 5 6")
    assert r2.stdout == "-3.0000000000e+00 -3.0000000000e+00 -3.0000000000e+00 "


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["test_01", "test_02"])
@pytest.mark.parametrize("geom", ["32\n32\n16\n16", "16\n16\n1024\n1024", "2\n2\n16\n16", "0\n0\n0\n0"])
def test_lab2_gpu_ground_truth(name, geom, tmp_path):
    src = write_hex_as_data(os.path.join(LAB2_DATA, name + ".txt"), tmp_path / "in.data")
    out = tmp_path / "out.data"
    r = run("labs/lab2/src/to_plot_hip_exe", f"{geom}\n{src}\n{out}")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0].startswith("HIP execution time: <") and lines[-1] == "FINISHED!"
    assert out.read_bytes() == hex_bytes(os.path.join(LAB2_GT, name + ".txt"))
    r2 = run("labs/lab2/src/hip_exe", f"{src}\n{out}")
    assert r2.returncode == 0 and r2.stdout == ""
    assert out.read_bytes() == hex_bytes(os.path.join(LAB2_GT, name + ".txt"))


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["direct", "mfma", "mfma64", "mfma8", "auto"])
def test_lab3_gpu_ground_truth(path, tmp_path):
    src = write_hex_as_data(os.path.join(LAB3_DATA, "test_01_lab3.txt"), tmp_path / "in.data")
    out = tmp_path / "out.data"
    r = run("labs/lab3/src/to_plot_hip_exe", f"256\n256\n{src}\n{out}\n2\n4 1 2 1 0 2 2 2 1\n4 0 0 0 1 1 1 2 0",
            env={"MPX_LAB3_PATH": path})
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("HIP execution time: <")
    assert out.read_bytes() == hex_bytes(os.path.join(LAB3_GT, "test_01_lab3.txt"))


@pytest.mark.gpu
def test_gpu_info():
    r = run("bin/gpu_info", "")
    assert r.returncode == 0
    assert "gfx950" in r.stdout and "Multiprocessors count : 256" in r.stdout


@pytest.mark.gpu
def test_lab2_gpu_timing_policies(tmp_path):
    src = os.path.join(LAB2_DATA, "96.data")
    ms = {}
    for pol in ("cold", "cold-lazy", "warm", "median:5"):
        r = run("labs/lab2/src/to_plot_hip_exe", f"32\n32\n16\n16\n{src}\n{tmp_path}/o.data", env={"MPX_TIMING": pol})
        assert r.returncode == 0 and r.stdout.startswith("HIP execution time: <")
        assert "unknown MPX_TIMING" not in r.stderr
        ms[pol] = float(r.stdout.split("<")[1].split()[0])
    # cold-lazy also times the code object's lazy load (~0.25 ms per module)
    assert ms["cold-lazy"] > ms["cold"]


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ["conv", "--size", "1024", "--steps", "5", "--warmup", "1"],
    ["conv", "--size", "1000", "--steps", "3", "--warmup", "1", "--filter", "roberts"],
    ["jacobi", "--size", "2048", "--iters", "20", "--warmup", "2", "--check-every", "5"],
    ["jacobi", "--size", "1024", "--iters", "10", "--warmup", "1", "--fp32"],
    ["vsub", "--n", "1000003", "--steps", "5", "--warmup", "1"],
    ["vsub", "--n", "65536", "--steps", "5", "--warmup", "1", "--fp64"],
])
def test_mpx_mgpu_single_gpu(args):
    """Native multi-GPU runtime (one process, one thread + RCCL communicator per
    device) on the one GPU of the test box; every workload self-verifies."""
    import json

    r = run("bin/mpx_mgpu", "", args=[*args, "--gpus", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert rec.get("verified_bit_exact", rec.get("verified")) is True


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,extra", [(1, []), (2, []), (3, ["--fp32"]), (4, ["--rows", "805"])])
def test_mpx_mgpu_jacobi_peer_shared(ranks, extra):
    """Native runtime, one-sided device-signalled halos: up to 4 ranks (one
    stream each) rehearse on the one GPU; per-rank self-verification plus no
    device-side wait may time out."""
    import json

    r = run("bin/mpx_mgpu", "", args=["jacobi", "--halo", "peer", "--shared", "--gpus", str(ranks), "--size", "1024",
                                      "--iters", "40", "--warmup", "3", "--check-every", "10", *extra])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == ranks and rec["halo"] == "peer-signalled" and rec["verified"] is True
    assert rec["peer_probe"] == "ok"
    # N > 1: the gathered field equals ONE device running the same sweeps
    assert rec["one_device_equal"] is (True if ranks > 1 else None)


@pytest.mark.gpu
def test_mpx_mgpu_catches_injected_halo_corruption():
    """A silently corrupted halo value on one rank (MPX_FAULT_INJECT) must fail
    the N-rank == one-device check with exit code 3."""
    import json

    r = run("bin/mpx_mgpu", "", env={"MPX_FAULT_INJECT": "halo:1:7"},
            args=["jacobi", "--halo", "peer", "--shared", "--gpus", "3", "--size", "1024", "--iters", "20",
                  "--warmup", "2", "--check-every", "10"])
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["one_device_equal"] is False and rec["verified"] is False


def test_mpx_mgpu_usage_errors():
    assert run("bin/mpx_mgpu", "").returncode == 2
    assert run("bin/mpx_mgpu", "", args=["conv", "--bogus"]).returncode == 2
    assert run("bin/mpx_mgpu", "", args=["jacobi", "--halo", "carrier-pigeon"]).returncode == 2
    assert run("bin/mpx_mgpu", "", args=["conv", "--shared", "--gpus", "2"]).returncode == 2


def _png_to_data(png, dst):
    from cuda_mpi_openmp_amd.utils import ImgData

    dst.write_bytes(open(ImgData(str(png), cache_dir=str(dst.parent)).data_path, "rb").read())
    return dst


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["roberts", "sobel5", "gauss5"])
def test_lab2_gpu_multi_part_matches_cpu(op, tmp_path):
    """MPX_NGPUS=3: three row slabs (on the box's one GPU) with halo rows from
    the host image must reproduce the CPU program byte for byte."""
    src = _png_to_data(os.path.join(ROOT, "labs", "lab2", "metric_calc", "large", "doom.png"), tmp_path / "in.data")
    ref, got = tmp_path / "ref.data", tmp_path / "got.data"
    assert run("labs/lab2/src/cpu_omp_exe", f"{src}\n{ref}", env={"MPX_LAB2_OP": op}).returncode == 0
    r = run("labs/lab2/src/to_plot_hip_exe", f"0\n0\n0\n0\n{src}\n{got}", env={"MPX_LAB2_OP": op, "MPX_NGPUS": "3",
                                                                           "MPX_WARMUP": "2", "MPX_ALLOW_SHARED": "1"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("HIP execution time: <")
    assert got.read_bytes() == ref.read_bytes()


@pytest.mark.gpu
def test_multi_part_refuses_missing_devices():
    """MPX_NGPUS=N on fewer devices must not report an N-GPU time."""
    r = run("labs/lab1/src/to_plot_hip_exe", "0\n0\n5\n1 2 3 4 5\n5 4 3 2 1", env={"MPX_NGPUS": "64"})
    assert r.returncode == 2 and "MPX_ALLOW_SHARED" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
def test_lab1_gpu_multi_part():
    r = run("labs/lab1/src/to_plot_hip_exe", "0\n0\n5\n1 2 3 4 5\n5 4 3 2 1",
            env={"MPX_NGPUS": "3", "MPX_ALLOW_SHARED": "1"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.split("\n", 1)[1] == ("-4.0000000000e+00 -2.0000000000e+00 0.0000000000e+00 "
                                          "2.0000000000e+00 4.0000000000e+00 ")


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["direct", "fast"])
def test_lab3_gpu_multi_part_matches_cpu(path, tmp_path):
    src = _png_to_data(os.path.join(ROOT, "labs", "lab2", "metric_calc", "medium", "lenna.png"), tmp_path / "in.data")
    classes = "3\n4 10 10 20 20 30 30 40 40\n4 100 200 110 210 120 220 130 230\n5 400 50 410 60 420 70 430 80 500 500"
    ref, got = tmp_path / "ref.data", tmp_path / "got.data"
    assert run("labs/lab3/src/cpu_omp_exe", f"{src}\n{ref}\n{classes}").returncode == 0
    r = run("labs/lab3/src/to_plot_hip_exe", f"0\n0\n{src}\n{got}\n{classes}",
            env={"MPX_NGPUS": "5", "MPX_LAB3_PATH": path, "MPX_ALLOW_SHARED": "1"})
    assert r.returncode == 0, r.stderr
    assert got.read_bytes() == ref.read_bytes()
