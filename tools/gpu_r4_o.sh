#!/bin/bash
# Round-4 checkpoint O (final tree): smoke, bench, and the per-kernel profile
# (kernel trace + the standard counter passes over tools/prof_all.py).
set -o pipefail
O=${O:-gpurun_out/r4/o}
export O
mkdir -p "$O"
bash tools/gpu.sh smoke &&
bash tools/gpu.sh run bench 300 python bench.py &&
bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py
