#!/bin/bash
# Round-4 checkpoint M: fast32 with interleaved FMA chains (MPX_CLS_OPT=8)
# against the default, alternated twice; mfma8's fp32 re-rank stage on/off;
# the classify env-variant tests.
set -o pipefail
O=${O:-gpurun_out/r4/m}
export O
mkdir -p "$O"
for r in 1 2; do
  for o in 0 8 10; do
    MPX_CLS_OPT=$o LAB3_NCS=2,4,8,16,32 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run lab3_fast_o${o}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
  for f in 1 0; do
    MPX_CLS_MFMA8_FP32=$f LAB3_NCS=16,24,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_fp32_${f}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
done &&
bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "classify"
