#!/bin/bash
# Round-4 checkpoint R: fast32 vs mfma8 over nc (AUTO re-derived with the
# fp32 re-rank stage), two rounds.
set -o pipefail
O=${O:-gpurun_out/r4/r}
export O
mkdir -p "$O"
for r in 1 2; do
  LAB3_NCS=6,8,10,12,13,14,15,16,17,18,19,20,21,22,23,24,28,32 LAB3_PATHS=fast,mfma8 LAB3_TAG=r$r \
    bash tools/gpu.sh run lab3_nc_sweep_r$r 400 python -u tools/experiments/lab3_ab.py || exit 1
done
