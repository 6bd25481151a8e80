#!/bin/bash
# lab5 radix sort: GPU tests, timing vs torch.sort, and a kernel trace.
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_lab5_sort.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r2/pytest_sort.log 2>&1
rc=$?; tail -15 gpurun_out/r2/pytest_sort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lab5_bench.py > gpurun_out/r2/lab5_bench.jsonl 2>&1 || exit $?
cat gpurun_out/r2/lab5_bench.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_sort -o run -- python3 tools/lab5_bench.py > gpurun_out/r2/prof_sort.log 2>&1 || exit $?
