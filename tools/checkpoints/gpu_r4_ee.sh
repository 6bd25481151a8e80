#!/bin/bash
# Round-4 checkpoint EE: stream-set test and the driver's bench command.
set -o pipefail
O=${O:-gpurun_out/r4/ee}
export O
mkdir -p "$O"
bash tools/gpu.sh tests tests/test_streams.py tests/test_lab5_sort.py -k "streams or variants" &&
bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
