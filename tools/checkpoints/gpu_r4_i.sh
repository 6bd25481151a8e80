#!/bin/bash
# Round-4 checkpoint I: the streaming phase on 1 vs 2 streams (N = 1, both
# phases), the fused streaming halo rehearsed at 2 and 4 ranks on one GPU
# (retained vs N = 1) with a kernel trace of the 2-rank run (one dispatch per
# streaming step), and the radix scatter's HBM bytes for 8192- vs 4096-key tiles.
set -o pipefail
O=${O:-gpurun_out/r4/i}
export O
mkdir -p "$O"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
  bash tools/gpu.sh run n1_s1_$r 200 $B --gpus 1 --streams 1 &&
  bash tools/gpu.sh run n1_s2_$r 200 $B --gpus 1 || exit 1
done &&
MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n2 300 $B --gpus 2 &&
MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n4 300 $B --gpus 4 &&
MPX_DIST_BACKEND=gloo bash tools/gpu.sh prof n2_trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --gpus 2 &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
  bash tools/gpu.sh pmc sort_wr "WRITE_SIZE" -- python3 tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
  bash tools/gpu.sh pmc sort_rd "FETCH_SIZE" -- python3 tools/experiments/sort_probe.py &&
bash tools/gpu.sh jpeer 2 4 && bash tools/gpu.sh mgpu jacobi --halo peer --shared --gpus 2 --size 16384
[ $? -eq 0 ] || exit 1
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,12,10,13 bash tools/gpu.sh run sort_pf2 300 \
  python -u tools/experiments/sort_probe.py
