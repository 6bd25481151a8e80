#!/bin/bash
# Round-4 checkpoint NN (checkpoint X again, after the clock change): the scaling driver's one-GPU rehearsal (ranks share the
# GPU) at 1 / 2 / 4 ranks over every multi-GPU workload.
set -o pipefail
O=${O:-gpurun_out/r4/nn}
export O
mkdir -p "$O"
bash tools/gpu.sh run scale 1000 python -u tools/scale.py --gpus 1,2,4 --rehearse --out "$O/scaling" --timeout 300
