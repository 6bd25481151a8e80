#!/bin/bash
# Round-4 checkpoint TT (final tree, after the sort variant-17 rebuild): the full GPU suite, smoke, and the
# driver's bench command.
set -o pipefail
O=${O:-gpurun_out/r4/tt}
export O
mkdir -p "$O"
bash tools/gpu.sh tests && bash tools/gpu.sh smoke &&
bash tools/gpu.sh run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
