#!/bin/bash
# Round-4 checkpoint DD: lean onesweep with a static tile order (variant 16,
# no tile counter) vs the counter form (14) and AUTO (12); its GPU tests.
set -o pipefail
O=${O:-gpurun_out/r4/dd}
export O
mkdir -p "$O"
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=12,16,14 bash tools/gpu.sh run sort_os_static 300 \
  python -u tools/experiments/sort_probe.py &&
bash tools/gpu.sh tests tests/test_lab5_sort.py -k "variants and 16"
