#!/bin/bash
# Jacobi wave kernel + vsub auto geometry: tests and bandwidth.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "jacobi or vsub" > gpurun_out/pytest_jv.log 2>&1 || { tail -30 gpurun_out/pytest_jv.log; exit 1; }
tail -2 gpurun_out/pytest_jv.log
timeout -k 10 300 python tools/bench_suite.py --only lab1,jacobi > gpurun_out/suite_jv.log 2>&1 || { cat gpurun_out/suite_jv.log; exit 2; }
grep -v amdgpu.ids gpurun_out/suite_jv.log
