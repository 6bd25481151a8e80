#!/bin/bash
# Device-signalled one-sided Jacobi halos on one MI355X (gloo control plane,
# N ranks share the GPU). Per rank count N in 2/4/8, same box, interleaved:
#   * 16384^2 fp64: peer halos vs the no-exchange ablation vs 1 rank;
#   * small slabs (64 rows x 16384 per rank, launch-bound): peer vs ablation,
#     whose difference is the per-iteration cost of the device-side ordering.
set -o pipefail
mkdir -p gpurun_out/r2/jpeer
O=gpurun_out/r2/jpeer
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 200 python -u tools/bench_jacobi.py "$@" --iters 400 --warmup 40 > $O/$name.json 2>&1 \
      || { tail -20 $O/$name.json; exit 3; }
  echo "$name $(grep metric $O/$name.json)"
}
run n1 
run n1_small --rows 64
for n in 2 4 8; do
  for h in peer none; do
    MPX_DIST_BACKEND=gloo run ${h}$n --gpus $n --halo $h
    MPX_DIST_BACKEND=gloo run ${h}${n}_small --gpus $n --halo $h --rows $((64 * n))
  done
done
