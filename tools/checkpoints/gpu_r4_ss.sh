#!/bin/bash
# Round-4 checkpoint SS: variant 17 (a counter row per half-wave) — the sort
# variant tests, then 12 vs 17 alternated at 2^24 / 2^26 int32 / float32.
set -o pipefail
O=${O:-gpurun_out/r4/ss}
export O
mkdir -p "$O"
bash tools/gpu.sh tests tests/test_lab5_sort.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,17 SORT_PROBE_SMALL=1 \
  bash tools/gpu.sh run probe1 300 python tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=17,12 SORT_PROBE_SMALL=0 \
  bash tools/gpu.sh run probe2 300 python tools/experiments/sort_probe.py
