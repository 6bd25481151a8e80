#!/bin/bash
# Native RCCL tier: GPU tests, host step overhead, single-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_native_comm.py -m gpu -x -q -s > gpurun_out/pytest_comm.log 2>&1 || { tail -40 gpurun_out/pytest_comm.log; exit 1; }
grep -E "passed|failed|host cost" gpurun_out/pytest_comm.log
timeout -k 10 300 python tools/step_overhead.py > gpurun_out/step_overhead.log 2>&1 || { tail -30 gpurun_out/step_overhead.log; exit 2; }
grep -v amdgpu.ids gpurun_out/step_overhead.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/bench.log
