#!/bin/bash
# Round-end rehearsal: smoke(), the full GPU test tier, the N=1 flagship bench.
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1 || { cat gpurun_out/r2/smoke.log; exit 1; }
tail -1 gpurun_out/r2/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/pytest_gpu_full.log 2>&1
rc=$?; tail -2 gpurun_out/r2/pytest_gpu_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r2/bench_final.json 2> gpurun_out/r2/bench_final.err || exit $?
cat gpurun_out/r2/bench_final.json
