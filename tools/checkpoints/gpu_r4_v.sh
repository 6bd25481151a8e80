#!/bin/bash
# Round-4 checkpoint V (final tree): full GPU suite, smoke, the driver's bench
# command, and the 2-rank rehearsal bench.
set -o pipefail
O=${O:-gpurun_out/r4/v}
export O
mkdir -p "$O"
bash tools/gpu.sh tests &&
bash tools/gpu.sh smoke &&
bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
MPX_DIST_BACKEND=gloo bash tools/gpu.sh run bench_n2 300 python bench.py --gpus 2 --steps 20 --warmup 5
