#!/bin/bash
# Round-4 checkpoint VV (final tree): lab3 on three rotated 8192^2 images
# (the lab3_classify.md methodology) for the README's figures, and the
# driver's bench command twice more.
set -o pipefail
O=${O:-gpurun_out/r4/vv}
export O
mkdir -p "$O"
LAB3_NCS=4,16,32 LAB3_PATHS=fast,mfma8,auto bash tools/gpu.sh run lab3 300 python tools/experiments/lab3_ab.py &&
bash tools/gpu.sh run bench1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
bash tools/gpu.sh run bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
