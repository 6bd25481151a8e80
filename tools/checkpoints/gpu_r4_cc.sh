#!/bin/bash
# Round-4 checkpoint CC: lean onesweep at 1 block per CU (variant 15) vs 2 (14)
# vs the AUTO reduce-then-scan (12).
set -o pipefail
O=${O:-gpurun_out/r4/cc}
export O
mkdir -p "$O"
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14,15 SORT_PROBE_SMALL=1 bash tools/gpu.sh run sort_os1 300 \
  python -u tools/experiments/sort_probe.py
