#!/bin/bash
# Round-4 checkpoint GG: bench.py with 2 vs 3 compute streams, alternated
# (3 streams were last measured before the process-wide stream pool).
set -o pipefail
O=${O:-gpurun_out/r4/gg}
export O
mkdir -p "$O"
for i in 1 2; do
  bash tools/gpu.sh run s2_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --streams 2 &&
  bash tools/gpu.sh run s3_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --streams 3 || exit 1
done
