#!/bin/bash
# Round-4 checkpoint PP: the timed region's fixed cost, T(K) for K = 0..50.
set -o pipefail
O=${O:-gpurun_out/r4/pp}
export O
mkdir -p "$O"
bash tools/gpu.sh run timed_k 300 python tools/experiments/timed_k.py
