#!/bin/bash
# Round-4 checkpoint AA: the driver's bench command three times on one box and
# a kernel trace of it (hardware queue of each phase's streams).
set -o pipefail
O=${O:-gpurun_out/r4/aa}
export O
mkdir -p "$O"
for r in 1 2 3; do
  bash tools/gpu.sh run bench_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done &&
bash tools/gpu.sh prof trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline &&
python tools/experiments/trace_db.py "$O/trace" --top 5 > "$O/trace.md" && find "$O" -name "*.db" -size +20M -delete
