#!/bin/bash
# Round-4 checkpoint QQ: kernel trace of the T(K) probe (queues and per-burst
# overlap of the K-step runs).
set -o pipefail
O=${O:-gpurun_out/r4/qq}
export O
mkdir -p "$O"
bash tools/gpu.sh prof tk -- python3 tools/experiments/timed_k.py &&
python3 tools/experiments/phase_trace.py "$O/tk" --gap 3 > "$O/phases.md"
