#!/bin/bash
# correctness sweep + variant timing + GPU unit tests
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python tools/kcheck.py > gpurun_out/kcheck.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/kcheck.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/kbench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
