#!/bin/bash
# Round-4 checkpoint FF: step_twin test; bench with the two-stream
# cache-resident pass (value_warm_cache) beside the one-stream one.
set -o pipefail
O=${O:-gpurun_out/r4/ff}
export O
mkdir -p "$O"
bash tools/gpu.sh tests tests/test_streams.py &&
bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
bash tools/gpu.sh run bench50 300 python bench.py --gpus 1 --steps 50 --warmup 5
