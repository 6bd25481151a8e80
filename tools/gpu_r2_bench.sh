#!/bin/bash
# Round-2 bench checks on one MI355X: the N=1 flagship (rotated, HBM-honest),
# the 2-rank refusal on a one-GPU box, and a 2/4-rank one-GPU rehearsal (gloo
# control plane, peer halos over IPC).
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u bench.py > gpurun_out/r2/bench_n1.json 2> gpurun_out/r2/bench_n1.err || exit $?
cat gpurun_out/r2/bench_n1.json
timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r2/refuse.out 2>&1
rc=$?
echo "refuse rc=$rc"; tail -2 gpurun_out/r2/refuse.out
[ $rc -eq 2 ] || exit 1
for n in 2 4; do
  MPX_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus $n --steps 20 --warmup 5 \
      > gpurun_out/r2/bench_gloo$n.json 2> gpurun_out/r2/bench_gloo$n.err || exit $?
  cat gpurun_out/r2/bench_gloo$n.json
done
