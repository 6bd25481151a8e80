#!/bin/bash
# Round-4 checkpoint KK: does value_streaming trail value because its phase
# runs after ~50 ms of sustained load and the warm passes? The driver's bench
# command with and without those passes, alternated.
set -o pipefail
O=${O:-gpurun_out/r4/kk}
export O
mkdir -p "$O"
for i in 1 2; do
  bash tools/gpu.sh run full_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
  bash tools/gpu.sh run bare_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --no-warm || exit 1
done
