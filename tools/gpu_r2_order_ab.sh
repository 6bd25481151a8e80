#!/bin/bash
# Same-box A/B of the conv wave order for every production filter path:
# MPX_CONV_ORDER=1 (strip-minor, all segments down) vs 3 (alternating), rotated.
set -o pipefail
mkdir -p gpurun_out/r2
for r in 1 2; do
  for o in 1 3; do
    MPX_CONV_ORDER=$o timeout -k 10 300 python -u tools/kbench.py --rotate 6 --rounds 5 --only production \
        > gpurun_out/r2/order_$o.jsonl 2>&1 || exit $?
    echo "order $o round $r"; grep us_median gpurun_out/r2/order_$o.jsonl | sed 's/"TBps.*//'
  done
done
