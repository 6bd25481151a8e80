#!/bin/bash
# Kernel timeline of eager vs HIP-graph Jacobi iterations (rocprofv3 kernel trace).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD; O=$R/gpurun_out/graphprof; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in eager graph; do
  flag=""; [ $g = graph ] && flag="--graph"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$g -o run -- python3 $R/tools/bench_jacobi.py --size 2048 --iters 40 --warmup 10 $flag > $O/$g.log 2>&1 || { tail -5 $O/$g.log; exit 1; }
  grep -o '"value": [0-9.]*' $O/$g.log
done
