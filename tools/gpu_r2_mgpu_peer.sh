#!/bin/bash
# Native runtime, device-signalled peer Jacobi, ranks sharing one MI355X (one
# stream each, one process): tests, then per-iteration time vs 1 rank at
# 16384^2 and on launch-bound 64-row-per-rank slabs.
set -o pipefail
mkdir -p gpurun_out/r2/mgpu
O=gpurun_out/r2/mgpu
timeout -k 10 300 python -u -m pytest tests/test_cli_programs.py -m gpu -x -q -k "mgpu" --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for n in 1 2 3 4; do
  timeout -k 10 120 bin/mpx_mgpu jacobi --halo peer --shared --gpus $n --iters 400 --warmup 40 > $O/full$n.json 2> $O/full$n.err || { cat $O/full$n.err; exit 3; }
  echo "full $n $(cat $O/full$n.json)"
  for h in peer none; do
    timeout -k 10 120 bin/mpx_mgpu jacobi --halo $h --shared --gpus $n --rows $((64 * n)) --iters 2000 --warmup 100 > $O/small_$h$n.json 2> $O/small_$h$n.err || { cat $O/small_$h$n.err; exit 3; }
    echo "small_$h $n $(cat $O/small_$h$n.json)"
  done
  timeout -k 10 120 bin/mpx_mgpu jacobi --halo none --shared --gpus $n --iters 400 --warmup 40 > $O/full_none$n.json 2> $O/full_none$n.err || { cat $O/full_none$n.err; exit 3; }
  echo "full_none $n $(cat $O/full_none$n.json)"
done
timeout -k 10 120 bin/mpx_mgpu jacobi --gpus 1 --iters 400 --warmup 40 > $O/rccl1.json 2> $O/rccl1.err || exit 4
echo "rccl 1 $(cat $O/rccl1.json)"
