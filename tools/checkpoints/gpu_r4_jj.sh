#!/bin/bash
# Round-4 checkpoint JJ: kernel trace of bench.py (N = 1, no sustain / warm
# passes) to compare the static and streaming phases burst by burst.
set -o pipefail
O=${O:-gpurun_out/r4/jj}
export O
mkdir -p "$O"
bash tools/gpu.sh prof bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --sustain-ms 0 --no-warm --no-cpu-baseline &&
python3 tools/experiments/phase_trace.py "$O/bench" > "$O/phases.md" &&
python3 tools/experiments/trace_db.py "$O/bench" > "$O/kernels.md" &&
find "$O/bench" -name "*.db" -delete
