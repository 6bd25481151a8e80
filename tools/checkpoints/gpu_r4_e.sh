#!/bin/bash
# Round-4 checkpoint E: bench.py over the stream count (2 / 3 / 6) and band
# modes under 2 streams, alternated; lab3 grid sweep with larger grids.
set -o pipefail
O=${O:-gpurun_out/r4/e}
export O
mkdir -p "$O"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-stream"
bash tools/gpu.sh run bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
for r in 1 2; do
  bash tools/gpu.sh run s2_$r 200 $B &&
  bash tools/gpu.sh run s3_$r 200 $B --streams 3 &&
  bash tools/gpu.sh run s6_$r 200 $B --streams 6 &&
  MPX_CONV_BAND=4 bash tools/gpu.sh run s2_band4_$r 200 $B &&
  MPX_CONV_BAND=2 bash tools/gpu.sh run s2_band2_$r 200 $B || exit 1
done &&
LAB3_NCS=2,4,32 LAB3_GRIDS=0,2048,4096,8192,16384 bash tools/gpu.sh run lab3_grid 400 python -u tools/experiments/lab3_grid_sweep.py &&
bash tools/gpu.sh prof bench_trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
