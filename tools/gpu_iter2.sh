#!/bin/bash
# lab3 fp32/MFMA classifier validation + lab1 geometry sweep.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k classify > gpurun_out/pytest_cls.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_cls.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_suite.py --only lab3 > gpurun_out/suite_lab3.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/suite_lab3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/vsub_sweep.py > gpurun_out/vsub_sweep.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/vsub_sweep.log
exit $rc
