#!/bin/bash
# Round-4 checkpoint L: lean onesweep look-back window 8 / 16 / 32 vs the PF-2
# lean scatter (AUTO); sort GPU suite.
set -o pipefail
O=${O:-gpurun_out/r4/l}
export O
mkdir -p "$O"
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14,15,16 SORT_PROBE_SMALL=0 bash tools/gpu.sh run sort_lbw 300 \
  python -u tools/experiments/sort_probe.py &&
bash tools/gpu.sh tests tests/test_lab5_sort.py -k "radix_variants"
