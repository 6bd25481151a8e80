#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1/conv -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof1/bench_conv.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1/rob -o run -- python3 bench.py --filter roberts --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof1/bench_rob.log 2>&1 || exit 3
find gpurun_out/prof1 -name "*stats*" | head
for f in $(find gpurun_out/prof1 -name "*kernel_stats.csv"); do echo "== $f"; cut -c1-300 $f | head -20; done
