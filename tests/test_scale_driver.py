"""tools/scale.py: the 1/2/4/8 scaling driver, dry-run on the CPU (gloo)."""
import json
import os
import subprocess
import sys

from .helpers import ROOT


def test_scale_driver_cpu_dry_run(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale.py"), "--device", "cpu", "--gpus", "1,2",
                        "--only", "conv", "--out", str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    data = json.load(open(tmp_path / "scaling.json"))
    runs = {(x["name"], x["n"]): x for x in data["runs"]}
    one, two = runs[("conv/peer", 1)], runs[("conv/rccl", 2)]
    assert one["status"] == "ok" and one["efficiency"] == 1.0, one
    assert two["status"] == "ok" and two["n_reported"] == 2 and two["verified"] is True, two
    assert two["efficiency"] is not None and two["world_size_seen"]["torch_distributed"] == 2, two
    assert runs[("conv/peer", 2)]["status"] == "skipped" and runs[("conv/peer", 2)]["reason"]
    # the streaming conv (bench.py value_streaming) is its own curve, verified N-rank == one-device
    st1, st2 = runs[("conv-stream/peer", 1)], runs[("conv-stream/rccl", 2)]
    assert st1["status"] == "ok" and st1["efficiency"] == 1.0 and st1["verified"] is True, st1
    assert st2["status"] == "ok" and st2["verified"] is True and st2["efficiency"] is not None, st2
    assert (tmp_path / "scaling.csv").exists() and (tmp_path / "scaling.png").exists()


def test_scale_driver_cpu_lab1_lab3(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale.py"), "--device", "cpu", "--gpus", "1,2",
                        "--only", "lab", "--out", str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    runs = {(x["name"], x["n"]): x for x in json.load(open(tmp_path / "scaling.json"))["runs"]}
    for name in ("lab1/vsub", "lab3/classify"):
        for n in (1, 2):
            x = runs[(name, n)]
            assert x["status"] == "ok" and x["n_reported"] == n and x["verified"] is True, x
        assert runs[(name, 2)]["efficiency"] is not None
