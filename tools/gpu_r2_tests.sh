#!/bin/bash
# The full GPU test tier (headline geometries included), one process.
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r2/pytest_gpu_full.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r2/pytest_gpu_full.log | tail -5
grep -E "FAILED|Error" gpurun_out/r2/pytest_gpu_full.log | head -20
exit $rc
