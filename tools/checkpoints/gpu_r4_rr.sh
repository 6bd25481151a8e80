#!/bin/bash
# Round-4 checkpoint RR (final tree): the one-GPU benchmark suite, every
# workload at its BASELINE size, verified.
set -o pipefail
O=${O:-gpurun_out/r4/rr}
export O
mkdir -p "$O"
bash tools/gpu.sh run suite 600 python tools/bench_suite.py
