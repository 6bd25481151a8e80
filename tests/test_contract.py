"""nccl-contract mode (parallel/contract.py): one-GPU
multi-rank rehearsals take the framework's ``backend == "nccl"`` branches,
and every tensor a collective receives must be on the rank's own device.

CPU tests check the wrapper and the plumbing (the rank's "device" is then the
CPU, so the device checks pass); the GPU tests run bench.py, the Jacobi bench
and the scaling rehearsal at 2 and 4 ranks on one GPU under the contract, and
show that a host tensor injected into one collective fails with its call site.
"""

import json
import os
import subprocess
import sys

import pytest
import torch

from cuda_mpi_openmp_amd.parallel import contract

from .helpers import ROOT
from .test_bench_contract import _port


def test_check_tensor_names_call_site():
    contract._DEV = torch.device("cuda", 0)
    try:
        with pytest.raises(contract.ContractError) as ei:
            contract.check_tensor(torch.zeros(3), "all_reduce")
        msg = str(ei.value)
        assert "cpu" in msg and "cuda:0" in msg and "test_contract.py" in msg and "all_reduce" in msg
        with pytest.raises(contract.ContractError):
            contract.check_tensor([1.0], "broadcast")
    finally:
        contract._DEV = None


def _bench(args, env, nproc=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), *args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT,
                          env=dict(os.environ, OMP_NUM_THREADS="1", **env))


def _rec(r):
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])


def test_contract_bench_two_ranks_cpu():
    """The nccl branches (device scalars, object collectives, RCCL-halo p2p via
    batch_isend_irecv) run under the contract and give the gloo results."""
    args = ["--gpus", "2", "--device", "cpu", "--size", "64", "--steps", "3", "--warmup", "1", "--rotate", "2",
            "--halo", "rccl", "--warmup-ms", "0"]
    rec = _rec(_bench(args, {"MPX_DIST_CONTRACT": "nccl"}))
    assert rec["n_gpus"] == 2 and rec["verified_bit_exact"] is True and rec["verified_bit_exact_streaming"] is True
    assert rec["rehearsal"] is True


def test_contract_worker_collectives_cpu():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "tests", "contract_worker.py"), "cpu"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="1", MPX_DIST_CONTRACT="nccl"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert r.stdout.count("contract worker ok") == 3


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_contract_bench_gpu(world):
    env = {"MPX_DIST_CONTRACT": "nccl", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    for halo in ("auto", "rccl"):
        rec = _rec(_bench(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--rotate", "2", "--halo", halo,
                           "--no-cpu-baseline", "--warmup-ms", "0"], env, nproc=world))
        assert rec["n_gpus"] == world and rec["verified_bit_exact"] is True
        assert rec["verified_bit_exact_streaming"] is True and rec["rehearsal"] is True


@pytest.mark.gpu
def test_contract_worker_collectives_gpu():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "tests", "contract_worker.py"), "cuda"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, MPX_DIST_CONTRACT="nccl", HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert r.stdout.count("contract worker ok") == 2


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_contract_jacobi_gpu(world):
    cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_jacobi.py"), "--gpus", str(world), "--size", "2048",
           "--iters", "40", "--warmup", "4", "--check-every", "10"]
    for halo in ("peer", "rccl"):
        r = subprocess.run(cmd + ["--halo", halo], capture_output=True, text=True, timeout=600, cwd=ROOT,
                           env=dict(os.environ, MPX_DIST_CONTRACT="nccl", HSA_ENABLE_IPC_MODE_LEGACY="0"))
        rec = _rec(r)
        assert rec["n_gpus"] == world and rec["verified"] is True


@pytest.mark.gpu
def test_contract_scale_rehearsal_gpu(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale.py"), "--gpus", "1,2,4", "--rehearse",
                        "--contract", "--quick", "--only", "conv", "--out", str(tmp_path), "--timeout", "300"],
                       capture_output=True, text=True, timeout=1100, cwd=ROOT,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    runs = json.load(open(tmp_path / "scaling.json"))["runs"]
    ok = [x for x in runs if x["status"] == "ok"]
    assert {x["n"] for x in ok} == {1, 2, 4}
    assert all(x.get("verified") is True for x in ok if x["n"] > 1)
    assert any(x["name"] == "conv/rccl" and x["n"] == 4 for x in ok)  # the RCCL-halo path ran at N = 4


@pytest.mark.gpu
def test_contract_catches_injected_host_tensor_gpu():
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--rotate", "2", "--no-cpu-baseline", "--no-stream",
                "--warmup-ms", "0"], {"MPX_DIST_CONTRACT": "nccl", "MPX_CONTRACT_INJECT": "all_gather_floats",
                                      "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert r.returncode != 0
    assert "ContractError" in r.stderr and "collectives.py" in r.stderr and "all_gather_floats" in r.stderr
