#!/bin/bash
# Round-2 GPU pass: flagship bench checks, then the GPU test tier.
set -o pipefail
mkdir -p gpurun_out/r2
bash tools/gpu_r2_bench.sh || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r2/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r2/pytest_gpu.log
exit $rc
