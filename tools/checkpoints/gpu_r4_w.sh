#!/bin/bash
# Round-4 checkpoint W: float32's skewed last pass on the peer-mask ranking
# (variant 15) vs the returning add (12, AUTO); the sort GPU suite.
set -o pipefail
O=${O:-gpurun_out/r4/w}
export O
mkdir -p "$O"
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,15 SORT_PROBE_ITERS=9 bash tools/gpu.sh run sort_v15 300 \
  python -u tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=15,12 SORT_PROBE_ITERS=9 SORT_PROBE_SMALL=0 bash tools/gpu.sh run sort_v15b 300 \
  python -u tools/experiments/sort_probe.py &&
bash tools/gpu.sh tests tests/test_lab5_sort.py
