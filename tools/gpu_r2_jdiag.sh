#!/bin/bash
# Diagnose the 2-rank one-GPU peer Jacobi at growing sizes (progress on stderr).
set -o pipefail
mkdir -p gpurun_out/r2
export MPX_DIST_BACKEND=gloo MPX_PEER_SPIN_LIMIT=65536 MPX_DEBUG_PEER=1
for sz in 16384; do
  echo "== size $sz"
  timeout -k 10 60 python -u tools/bench_jacobi.py --gpus 2 --halo peer --size $sz --iters 10 --warmup 4 --progress \
      > gpurun_out/r2/jdiag_$sz.log 2>&1
  rc=$?
  grep -E "jacobi r|peer r|metric|Error|error" gpurun_out/r2/jdiag_$sz.log | tail -20
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
done
