#!/bin/bash
# Round-4 checkpoint LL: is the conv's time data dependent (value_streaming
# trails value by ~6 %; its kernels ran ~6 % longer in trace JJ)?
set -o pipefail
O=${O:-gpurun_out/r4/ll}
export O
mkdir -p "$O"
bash tools/gpu.sh run datadep 300 python tools/experiments/conv_data_dep.py
