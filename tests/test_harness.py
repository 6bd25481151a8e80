"""The run_test.py / tester.py compatible harness, driven with the CPU binaries
(GPU binaries in the gpu-marked tests)."""

import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

from cuda_mpi_openmp_amd.harness import args as hargs
from cuda_mpi_openmp_amd.harness import core
from cuda_mpi_openmp_amd.harness.processors import Lab1Processor
from cuda_mpi_openmp_amd.utils import imgdata

from .helpers import LAB2_DATA, LAB2_GT, ROOT, hex_bytes


def test_passthrough_kwargs_coercion():
    kw = hargs.passthrough_kwargs(["--a", "true", "--b", "3", "--c", "2.5", "--d", "x", "--flag",
                                   "--links", '["u1","u2"]', "--e=7"])
    assert kw == {"a": True, "b": 3, "c": 2.5, "d": "x", "flag": True, "links": ["u1", "u2"], "e": 7}


def test_timing_line_and_geometry():
    assert core.parse_timing("HIP execution time: <0.012345 ms>") == pytest.approx(0.012345)
    assert core.parse_timing("CPU execution time: <3.000000 ms>") == 3.0
    assert core.parse_timing("no timing") is None
    assert core.geometry_prefix([32, 32], [16, 16]) == "32\n32\n16\n16\n"
    assert core.geometry_prefix(512, 512) == "512\n512\n"
    assert core.geometry_prefix(None, None) == ""
    assert core.device_tag("/x/to_plot_hip_exe", [32, 32], [16, 16]) == "to_plot_hip_exe__32_32___16_16_"
    st = core.time_stats([1.0, 2.0, 3.0, None])
    assert st["median"] == 2.0 and st["min"] == 1.0 and st["max"] == 3.0


def test_imgdata_roundtrip(tmp_path):
    img = np.random.default_rng(0).integers(0, 256, (7, 9, 4), dtype=np.uint8)
    raw = imgdata.encode_data(img)
    assert np.array_equal(imgdata.decode_data(raw), img)
    p = tmp_path / "x.data"
    p.write_bytes(raw)
    d = imgdata.ImgData(str(p))
    assert d.width == 9 and d.height == 7 and d.data_path == str(p)
    assert imgdata.parse_hex(d.hex) == raw
    gt = open(os.path.join(LAB2_GT, "test_01.txt")).read()
    assert imgdata.hex_groups(hex_bytes(os.path.join(LAB2_GT, "test_01.txt")), row_pixels=3).upper() == gt.strip()
    # PNG: alpha forced to 255, converted copy written to the cache dir only
    png = os.path.join(LAB2_DATA, "lenna.png")
    before = set(os.listdir(LAB2_DATA))
    d = imgdata.ImgData(png, cache_dir=str(tmp_path / "cache"))
    assert d.pixels.shape == (512, 512, 4) and (d.pixels[..., 3] == 255).all()
    assert os.path.exists(d.data_path) and set(os.listdir(LAB2_DATA)) == before


def test_lab1_processor_roundtrip():
    p = Lab1Processor(min_vector_size=1500, max_vector_size=1600)
    stdin, kw, dbg = p.pre_process(device_info="x")
    n = dbg["vector_size"]
    lines = stdin.split("\n")
    a = np.array(lines[1].split(), dtype=np.float64)
    assert int(lines[0]) == n and a.size == n and np.array_equal(a, kw["first_vector"])  # exact round trip
    res = p.get_task_result(" ".join(f"{v:.10e}" for v in kw["first_vector"] - kw["second_vector"]) + " ")
    assert p.verify_result(res, **kw)
    assert not p.verify_result(res * 1.001, **kw)


def _copy_lab(tmp_path, lab):
    dst = tmp_path / "labs" / lab
    shutil.copytree(os.path.join(ROOT, "labs", lab, "src"), dst / "src",
                    ignore=shutil.ignore_patterns("*.csv", "*.png"))
    for sub in ("data", "data_out_gt"):
        if os.path.isdir(os.path.join(ROOT, "labs", lab, sub)):
            shutil.copytree(os.path.join(ROOT, "labs", lab, sub), dst / sub)
    return dst


def _run_test(args, cwd, env=None):
    return subprocess.run([sys.executable, os.path.join(ROOT, "run_test.py"), *args], cwd=cwd, capture_output=True,
                          text=True, timeout=600, env=dict(os.environ, **(env or {})))


def test_harness_lab2_cpu_binaries(tmp_path):
    lab = _copy_lab(tmp_path, "lab2")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--binary_path_cpu",
                   str(lab / "src" / "cpu_exe"), "--k_times", "3", "--kernel_sizes", "[[null, null]]",
                   "--metadata_columns2plot", '["filename"]'], tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "SUCCESS" in r.stdout and "FAILED" not in r.stdout
    df = pd.read_csv(lab / "src" / "stats_cpu_omp_exe.csv")
    for col in ("idx_run_time", "bin_name", "kernel_size", "test_verification_result", "time_kernel_exe_ms",
                "status", "err", "precision_array", "atol", "filename", "time_exe_ms_from_start_run_time_bin_name"):
        assert col in df.columns
    assert len(df) == 3 and df["test_verification_result"].all()
    assert os.path.exists(lab / "src" / "median_execution_time.png")
    # the CPU/GPU speedup of every GPU group is persisted, not only printed
    sp = pd.read_csv(lab / "src" / "speedup_cpu_omp_exe.csv")
    for col in ("device", "kernel_size", "n_gpus", "gpu_median_ms", "cpu_median_ms", "speedup_vs_cpu"):
        assert col in sp.columns
    assert len(sp) == 1 and sp["gpu_runs"][0] == 3 and sp["cpu_runs"][0] == 3
    assert abs(sp["speedup_vs_cpu"][0] - sp["cpu_median_ms"][0] / sp["gpu_median_ms"][0]) < 1e-9
    # outputs land under data_out/<bin>_<k1>_<k2>/, inputs untouched
    assert os.path.isdir(lab / "data_out" / "cpu_omp_exe_None_None")
    assert sorted(os.listdir(lab / "data")) == sorted(os.listdir(os.path.join(ROOT, "labs", "lab2", "data")))


def test_harness_lab2_detects_wrong_output(tmp_path):
    lab = _copy_lab(tmp_path, "lab2")
    # a "binary" that copies its input: test_01/test_02 must fail verification
    fake = lab / "src" / "fake_exe"
    fake.write_text("#!/bin/sh\nread a\nread b\ncp \"$a\" \"$b\"\necho 'CPU execution time: <1.0 ms>'\n")
    fake.chmod(0o755)
    r = _run_test(["--binary_path_cuda", str(fake), "--k_times", "5", "--kernel_sizes", "[[null, null]]"], tmp_path)
    assert "FAILED" in r.stdout
    assert os.path.exists(lab / "src" / "failed_fake_exe.csv")


def test_harness_verify_cpu_catches_one_lsb(tmp_path):
    """Images without GT are checked against the OpenMP CPU reference program
    (--verify cpu), not passed unconditionally: a 1-LSB corruption of one
    pixel of the metric_calc/large images fails; the honest program passes."""
    lab = _copy_lab(tmp_path, "lab2")
    shutil.copytree(os.path.join(ROOT, "labs", "lab2", "metric_calc"), lab / "metric_calc")
    shutil.rmtree(lab / "metric_calc" / "large_out_gt")  # no GT: the CPU oracle decides
    real = os.path.join(ROOT, "labs", "lab2", "src", "cpu_omp_exe")
    fake = lab / "src" / "lsb_exe"
    fake.write_text(f"""#!{sys.executable}
import subprocess, sys
stdin = sys.stdin.read()
r = subprocess.run([{real!r}], input=stdin, capture_output=True, text=True)
out = stdin.split()[1]
b = bytearray(open(out, "rb").read())
b[8 + 4 * (len(b) // 8)] ^= 1  # one LSB of one pixel's R channel
open(out, "wb").write(bytes(b))
sys.stdout.write(r.stdout)
""")
    fake.chmod(0o755)
    large = str(lab / "metric_calc" / "large")
    r = _run_test(["--binary_path_cuda", str(fake), "--k_times", "3", "--kernel_sizes", "[[null, null]]",
                   "--dir_to_data", large, "--verify", "cpu"], tmp_path)
    assert "FAILED" in r.stdout and "vs CPU reference" in r.stdout, r.stdout[-2000:]
    assert os.path.exists(lab / "src" / "failed_lsb_exe.csv")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--k_times", "3", "--kernel_sizes",
                   "[[null, null]]", "--dir_to_data", large, "--verify", "cpu"], tmp_path)
    assert r.returncode == 0 and "SUCCESS" in r.stdout and "FAILED" not in r.stdout, r.stdout[-2000:]


def test_harness_lab1_cpu(tmp_path):
    lab = _copy_lab(tmp_path, "lab1")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--k_times", "2", "--kernel_sizes",
                   "[[null, null]]", "--min_vector_size", "2000", "--max_vector_size", "2100"], tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    df = pd.read_csv(lab / "src" / "stats_cpu_omp_exe.csv")
    assert df["test_verification_result"].all() and (df["vector_size"] >= 2000).all()


def test_harness_lab3_cpu_random_classes(tmp_path):
    lab = _copy_lab(tmp_path, "lab3")
    shutil.copytree(os.path.join(ROOT, "labs", "lab3", "data"), lab / "data", dirs_exist_ok=True)
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--binary_path_cpu",
                   str(lab / "src" / "cpu_exe"), "--k_times", "2", "--kernel_sizes", "[[null, null]]",
                   "--metadata_columns2plot", '["filename", "stat_init_pts"]'], tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--k_times", "1", "--kernel_sizes",
                   "[[null, null]]", "--count_classes", "5", "--count_pts", "20", "--synthetic", "64x48"], tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.gpu
def test_harness_lab2_gpu_vs_cpu(tmp_path):
    lab = _copy_lab(tmp_path, "lab2")
    shutil.copytree(os.path.join(ROOT, "labs", "lab2", "metric_calc"), lab / "metric_calc")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "to_plot_hip_exe"), "--binary_path_cpu",
                   str(lab / "src" / "cpu_exe"), "--k_times", "4", "--kernel_sizes",
                   json.dumps([[[32, 32], [16, 16]], [[16, 16], [32, 32]], [[0, 0], [0, 0]]]),
                   "--metadata_columns2plot", '["filename"]', "--dir_to_data", str(lab / "metric_calc" / "large")],
                  tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "[Speedup]" in r.stdout
    df = pd.read_csv(lab / "src" / "stats_to_plot_hip_exe.csv")
    assert df["test_verification_result"].all() and (df["gpixel_per_s"] > 0).all()


@pytest.mark.gpu
def test_harness_lab2_gpu_n_gpus_warmup(tmp_path):
    """--n_gpus / --warmup reach the GPU binary (MPX_NGPUS / MPX_WARMUP) and the
    CSV records n_gpus."""
    lab = _copy_lab(tmp_path, "lab2")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "to_plot_hip_exe"), "--k_times", "2", "--kernel_sizes",
                   json.dumps([[[0, 0], [0, 0]]]), "--n_gpus", "2", "--warmup", "2", "--synthetic", "640x480"],
                  tmp_path, env={"MPX_ALLOW_SHARED": "1"})  # the one-GPU box rehearses 2 parts on one device
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    df = pd.read_csv(lab / "src" / "stats_to_plot_hip_exe.csv")
    assert df["test_verification_result"].all() and (df["n_gpus"] == 2).all()
    assert (df["devices_used"] == 1).all()  # ...and the CSV says so


def test_harness_refuses_n_gpus_beyond_visible(tmp_path):
    """--n_gpus N with fewer visible GPUs refuses to run (exit
    2) instead of writing an N-GPU row measured on fewer devices."""
    from cuda_mpi_openmp_amd.parallel.launch import visible_devices

    lab = _copy_lab(tmp_path, "lab2")
    n = max(2, visible_devices() + 1)
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--k_times", "1", "--kernel_sizes",
                   "[[null, null]]", "--n_gpus", str(n)], tmp_path, env={"MPX_ALLOW_SHARED": "0"})
    assert r.returncode == 2 and "refusing" in r.stderr, r.stderr[-2000:]
    assert not list((lab / "src").glob("stats_*.csv"))


def test_visible_devices_from_sysfs(tmp_path, monkeypatch):
    """The launcher counts GPUs from the KFD topology (no HIP runtime)."""
    from cuda_mpi_openmp_amd.parallel import launch

    for i, ver in enumerate([0, 90500, 90500, 0, 90500]):  # CPU nodes report 0
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 4\ngfx_target_version {ver}\nsimd_count 8\n")
    assert launch._kfd_gpu_count(str(tmp_path)) == 3
    assert launch._kfd_gpu_count(str(tmp_path / "missing")) is None
    # sysfs lists every GPU of the host; only render nodes this
    # process can open count (nodes 1 and 4 -> renderD128 / renderD131)
    dri = tmp_path / "dri"
    dri.mkdir()
    for i, minor in ((1, 128), (2, 129), (4, 131)):
        (tmp_path / str(i) / "properties").write_text(f"gfx_target_version 90500\ndrm_render_minor {minor}\n")
    (dri / "renderD128").write_text("")
    (dri / "renderD131").write_text("")
    assert launch._kfd_gpu_count(str(tmp_path), str(dri)) == 2
    (dri / "renderD131").chmod(0o000)
    if not os.access(dri / "renderD131", os.R_OK):  # (root ignores the mode bits)
        assert launch._kfd_gpu_count(str(tmp_path), str(dri)) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert launch._visible_filter(3) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert launch._visible_filter(3) == 0


@pytest.mark.parametrize("elem_type", ["int", "float", "uchar"])
def test_harness_lab5_cpu(tmp_path, elem_type):
    """lab5 through run_test.py: binary stdin/stdout, fixture + random arrays,
    byte-exact verification; the default --kernel_sizes geometry is not sent."""
    lab = _copy_lab(tmp_path, "lab5")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "cpu_omp_exe"), "--binary_path_cpu",
                   str(lab / "src" / "cpu_exe"), "--k_times", "3", "--elem_type", elem_type, "--max_size", "5000",
                   "--metadata_columns2plot", '["filename"]'], tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    df = pd.read_csv(lab / "src" / "stats_cpu_omp_exe.csv")
    assert len(df) == 3 and df["test_verification_result"].all()
    assert (df["elem_type"] == elem_type).all() and df["filename"].iloc[0] == f"{elem_type}10"


def test_harness_lab5_detects_unsorted(tmp_path):
    lab = _copy_lab(tmp_path, "lab5")
    fake = lab / "src" / "fake_exe"  # echoes its input unsorted
    fake.write_text("#!/bin/sh\necho 'CPU execution time: <1.0 ms>'\ntail -c +5\n")
    fake.chmod(0o755)
    r = _run_test(["--binary_path_cuda", str(fake), "--k_times", "2", "--n_random", "1"], tmp_path)
    assert "FAILED" in r.stdout
    assert os.path.exists(lab / "src" / "failed_fake_exe.csv")


@pytest.mark.gpu
def test_harness_lab5_gpu_vs_cpu(tmp_path):
    lab = _copy_lab(tmp_path, "lab5")
    r = _run_test(["--binary_path_cuda", str(lab / "src" / "to_plot_hip_exe"), "--binary_path_cpu",
                   str(lab / "src" / "cpu_exe"), "--k_times", "3", "--elem_type", "float", "--max_size", "200000"],
                  tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    df = pd.read_csv(lab / "src" / "stats_to_plot_hip_exe.csv")
    assert df["test_verification_result"].all() and (df["time_kernel_exe_ms"] >= 0).all()


def test_metric_calc_ground_truth_matches_cpu_reference():
    """The committed metric_calc GT (tools/make_metric_gt.py) is exactly the C
    reference's output on every bucket image."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_metric_gt.py"), "--check"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok ") == 13
