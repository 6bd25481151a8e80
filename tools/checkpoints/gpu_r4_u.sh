#!/bin/bash
# Round-4 checkpoint U: fast32 at 4 pixels per thread (5 waves per SIMD) with
# interleaved chains and two trips in flight, small nc, alternated twice.
set -o pipefail
O=${O:-gpurun_out/r4/u}
export O
mkdir -p "$O"
for r in 1 2; do
  LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run nq2_o8_r$r 200 python -u tools/experiments/lab3_ab.py &&
  MPX_CLS_NQ=1 MPX_CLS_OPT=8 LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run nq1_o8_r$r 200 python -u tools/experiments/lab3_ab.py &&
  MPX_CLS_NQ=1 MPX_CLS_OPT=24 LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run nq1_o24_r$r 200 python -u tools/experiments/lab3_ab.py || exit 1
done
