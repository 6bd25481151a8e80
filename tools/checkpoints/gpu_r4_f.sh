#!/bin/bash
# Round-4 checkpoint F: radix scatter attribution (knock-out probes, times and
# LDS counters) and the returning-add ranking (variant 9) vs production.
set -o pipefail
O=${O:-gpurun_out/r4/f}
export O
mkdir -p "$O"
bash tools/gpu.sh run sort_probe 300 python -u tools/experiments/sort_probe.py &&
SORT_PROBE_ITERS=1 SORT_PROBE_PARTS=knock bash tools/gpu.sh pmc probe_lds \
  "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES" -- python3 tools/experiments/sort_probe.py &&
SORT_PROBE_ITERS=1 SORT_PROBE_PARTS=knock bash tools/gpu.sh prof probe_trace -- python3 tools/experiments/sort_probe.py &&
bash tools/gpu.sh tests tests/test_lab5_sort.py
