#!/bin/bash
# First GPU validation: kernels, smoke, bench, kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 4
cat gpurun_out/bench.log
timeout -k 10 300 python bench.py --filter roberts > gpurun_out/bench_roberts.log 2>&1 || exit 5
cat gpurun_out/bench_roberts.log
