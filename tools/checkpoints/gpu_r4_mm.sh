#!/bin/bash
# Round-4 checkpoint MM: host enqueue time per step (static vs streaming
# phase) beside the step time; the driver's bench command twice.
set -o pipefail
O=${O:-gpurun_out/r4/mm}
export O
mkdir -p "$O"
bash tools/gpu.sh run b1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
bash tools/gpu.sh run b2 300 python bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu-baseline
