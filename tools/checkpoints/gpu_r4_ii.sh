#!/bin/bash
# Round-4 checkpoint II: host wait policy A/B (MPX_HIP_WAIT=auto, the HIP
# default, vs spin) on the driver's bench command, alternated twice.
set -o pipefail
O=${O:-gpurun_out/r4/ii}
export O
mkdir -p "$O"
for i in 1 2; do
  MPX_HIP_WAIT=auto bash tools/gpu.sh run auto_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
  MPX_HIP_WAIT=spin bash tools/gpu.sh run spin_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
