#!/bin/bash
# Round-4 checkpoint Q: fast32 with two trips of loads in flight (OPT 24 / 26)
# against the default (8), alternated twice; classify tests.
set -o pipefail
O=${O:-gpurun_out/r4/q}
export O
mkdir -p "$O"
for r in 1 2; do
  for o in 8 24 26; do
    MPX_CLS_OPT=$o LAB3_NCS=2,4,8,16,32 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run lab3_fast_o${o}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
done &&
bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify"
