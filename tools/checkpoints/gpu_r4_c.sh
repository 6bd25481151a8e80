#!/bin/bash
# Round-4 checkpoint C: bench.py A/B of the 2-stream alternation and of the
# time-based warm-up (driver command: --steps 20 --warmup 5), alternated
# twice, then a kernel trace of the default bench. Time-bounded steps.
set -o pipefail
O=${O:-gpurun_out/r4/c}
export O
mkdir -p "$O"
B="python bench.py --gpus 1 --steps 20 --warmup 5"
bash tools/gpu.sh run bench_default 300 $B &&
for r in 1 2; do
  bash tools/gpu.sh run ab_s2_w30_$r 200 $B --no-cpu-baseline --no-stream &&
  bash tools/gpu.sh run ab_s1_w30_$r 200 $B --no-cpu-baseline --no-stream --streams 1 &&
  bash tools/gpu.sh run ab_s2_w0_$r 200 $B --no-cpu-baseline --no-stream --warmup-ms 0 &&
  bash tools/gpu.sh run ab_s1_w0_$r 200 $B --no-cpu-baseline --no-stream --streams 1 --warmup-ms 0 || exit 1
done &&
bash tools/gpu.sh prof bench_trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
bash tools/gpu.sh run lab3_grid 400 python -u tools/experiments/lab3_grid_sweep.py
