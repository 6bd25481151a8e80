#!/bin/bash
# Round-4 checkpoint HH: checkpoint Z again after the clock moved before the closing
# barrier (each rank stops at its own device sync); bench launch and contract tests.
set -o pipefail
O=${O:-gpurun_out/r4/hh}
export O
mkdir -p "$O"
bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n2 300 python bench.py --gpus 2 --steps 20 --warmup 5 &&
MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n4 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu-baseline &&
bash tools/gpu.sh tests tests/test_gpu_bench_launch.py tests/test_contract.py
