#!/bin/bash
# Round-4 checkpoint N: mfma8 windowed fix-ups (now with the fp32 stage) vs
# after-loop, with write bytes; then the full GPU suite.
set -o pipefail
O=${O:-gpurun_out/r4/n}
export O
mkdir -p "$O"
for r in 1 2; do
  for wv in 0 1; do
    MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=16,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_w${wv}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
done &&
for wv in 0 1; do
  MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=32 LAB3_PATHS=mfma8 bash tools/gpu.sh pmc lab3_mfma8_w${wv}_bytes "WRITE_SIZE" \
    -- python3 tools/experiments/lab3_ab.py || exit 1
done &&
bash tools/gpu.sh tests
