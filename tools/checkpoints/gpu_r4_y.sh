#!/bin/bash
# Round-4 checkpoint Y: the streaming phase on the static phase's two streams
# (one process-wide stream set) vs one stream, N = 1, alternated; trace.
set -o pipefail
O=${O:-gpurun_out/r4/y}
export O
mkdir -p "$O"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
  bash tools/gpu.sh run ss1_$r 200 $B --stream-streams 1 &&
  bash tools/gpu.sh run ss2_$r 200 $B --stream-streams 2 || exit 1
done &&
bash tools/gpu.sh prof ss2_trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --stream-streams 2 &&
python tools/experiments/trace_db.py "$O/ss2_trace" --top 5 > "$O/ss2_trace.md" && find "$O" -name "*.db" -size +20M -delete
