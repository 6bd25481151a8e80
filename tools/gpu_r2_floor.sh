#!/bin/bash
# HBM-honest floors and flagship kernel timing: kbench over 6 rotated pairs vs
# one resident pair, bench with a step graph, and a rocprofv3 kernel trace of
# the rotated bench.
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u tools/kbench.py --rotate 6 --rounds 3 > gpurun_out/r2/kbench_rot6.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/kbench.py --rotate 1 --rounds 3 > gpurun_out/r2/kbench_rot1.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --graph 10 --no-cpu-baseline > gpurun_out/r2/bench_graph10.json 2>&1 || exit $?
cat gpurun_out/r2/bench_graph10.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/prof_bench -o run -- python3 bench.py --no-cpu-baseline --no-verify > gpurun_out/r2/prof_bench.log 2>&1 || exit $?
