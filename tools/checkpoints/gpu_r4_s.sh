#!/bin/bash
# Round-4 checkpoint S: load policy per regime — band mode 3 (NT interior
# loads, default) vs 2 (plain loads) on all three bench numbers (streaming
# from HBM, streaming iterated frames, one cache-resident pair).
set -o pipefail
O=${O:-gpurun_out/r4/s}
export O
mkdir -p "$O"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --gpus 1"
for r in 1 2; do
  bash tools/gpu.sh run m3_$r 200 $B &&
  MPX_CONV_BAND=2 bash tools/gpu.sh run m2_$r 200 $B || exit 1
done
