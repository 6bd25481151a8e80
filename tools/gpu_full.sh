#!/bin/bash
# Full GPU validation: unit tests, smoke, suite benchmarks, flagship bench.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
timeout -k 10 600 python tools/bench_suite.py > gpurun_out/suite.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 5; }
grep -v amdgpu.ids gpurun_out/bench.log
