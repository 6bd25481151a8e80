"""bench.py's own N-rank launch on the GPU box: two ranks rehearsed on the one
GPU (gloo control plane, peer halos over IPC), the path the driver's 1/2/4/8
scaling run takes with one rank per GPU."""
import json
import os
import subprocess
import sys

import pytest

from .helpers import ROOT

pytestmark = pytest.mark.gpu


def test_bench_self_launch_two_ranks_peer(gpu):
    env = dict(os.environ, MPX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--rotate", "2", "--size", "512", "--no-cpu-baseline", "--halo", "peer"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 2 and rec["world_size_seen"]["torch_distributed"] == 2
    assert rec["verified_bit_exact"] is True and rec["verified_pixels"] == 2 * 2 * 512 * 512
    assert rec["config"]["transport"] == "xgmi-peer"
    assert len(rec["per_rank_ms_per_step"]) == 2


@pytest.mark.parametrize("workload,extra", [("vsub", ["--elems", str(1 << 20)]), ("classify", ["--size", "512"])])
def test_bench_workloads_two_ranks(gpu, workload, extra):
    """lab1 / lab3 weak-scaling jobs of tools/scale.py, two ranks rehearsed on the
    one GPU: every rank's output verified."""
    env = dict(os.environ, MPX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_workloads.py"), "--workload", workload,
                        "--gpus", "2", "--steps", "3", "--warmup", "1", *extra],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 2 and rec["verified"] is True and len(rec["per_rank_ms_per_step"]) == 2 and rec["job_span_ms"] >= rec["max_rank_span_ms"]


def test_bench_two_ranks_peer_map_failure_falls_back_everywhere(gpu):
    """VERDICT r5 Next #7: rank 1 cannot map its neighbour's mailboxes
    (MPX_PEER_INJECT=map_fail@1): every rank takes the fallback transport in
    the static AND the streaming phase, every pixel still verified, rc 0."""
    env = dict(os.environ, MPX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", MPX_PEER_INJECT="map_fail@1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--rotate", "2", "--size", "512", "--no-cpu-baseline", "--steady-ms", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["status"] == "ok"
    assert rec["config"]["peer_probe"] == "fallback" and "peer" not in rec["config"]["transport"]
    assert rec["verified_bit_exact"] is True
    assert rec["value_streaming"] is not None and "peer" not in rec["transport_streaming"]
    assert rec["verified_bit_exact_streaming"] is True
    assert "using RCCL" in r.stderr


def test_bench_two_ranks_streaming_timeout_is_recorded(gpu):
    """A halo wait that gives up in the timed streaming steps on rank 1
    (MPX_BENCH_INJECT_STREAM_TIMEOUT=1): the run ends (no hang), the record
    says streaming_failed with value_streaming null, the static value stands
    verified, rc 0 (non-zero with --strict-streaming: each rank exits 3, the
    self-launch's torch.distributed.run reports that as 1)."""
    env = dict(os.environ, MPX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", MPX_BENCH_INJECT_STREAM_TIMEOUT="1")
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
            "--rotate", "2", "--size", "512", "--no-cpu-baseline", "--steady-ms", "0"]
    for strict in (False, True):
        r = subprocess.run(args + (["--strict-streaming"] if strict else []), cwd=ROOT, env=env,
                           capture_output=True, text=True, timeout=110)
        assert (r.returncode != 0) == strict, r.stderr[-2000:]
        if strict:
            assert "exitcode  : 3" in r.stderr
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        assert rec["status"] == "streaming_failed" and rec["value_streaming"] is None
        assert rec["verified_bit_exact"] is True and rec["value"] > 0
