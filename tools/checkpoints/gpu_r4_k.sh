#!/bin/bash
# Round-4 checkpoint K: the lean onesweep (variant 14) against the PF-2 lean
# scatters (12 / 13, the new AUTO): times on every stability case, HBM bytes,
# kernel trace; the sort GPU suite.
set -o pipefail
O=${O:-gpurun_out/r4/k}
export O
mkdir -p "$O"
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14,13 bash tools/gpu.sh run sort_os 300 \
  python -u tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=14 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=2 \
  bash tools/gpu.sh prof sort_os_trace -- python3 tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,14 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
  bash tools/gpu.sh pmc sort_os_wr "WRITE_SIZE" -- python3 tools/experiments/sort_probe.py &&
bash tools/gpu.sh tests tests/test_lab5_sort.py
