#!/bin/bash
# Round-4 checkpoint J: streaming-phase stream count at 2 ranks (rehearsal),
# N = 1 default bench (streaming back on one stream), radix 2-deep prefetch
# variants and HBM bytes, Jacobi peer cost with mailboxes.
set -o pipefail
O=${O:-gpurun_out/r4/j}
export O
mkdir -p "$O"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
bash tools/gpu.sh run n1 200 $B --gpus 1 &&
for r in 1 2; do
  MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n2_ss1_$r 300 $B --gpus 2 --stream-streams 1 &&
  MPX_DIST_BACKEND=gloo bash tools/gpu.sh run n2_ss2_$r 300 $B --gpus 2 --stream-streams 2 || exit 1
done &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,12,10,13 bash tools/gpu.sh run sort_pf2 300 \
  python -u tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10,12 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
  bash tools/gpu.sh pmc sort_wr "WRITE_SIZE" -- python3 tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9,10,12 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
  bash tools/gpu.sh pmc sort_rd "FETCH_SIZE" -- python3 tools/experiments/sort_probe.py &&
bash tools/gpu.sh jpeer 2 4 &&
bash tools/gpu.sh mgpu jacobi --halo peer --shared --gpus 2 --size 16384
