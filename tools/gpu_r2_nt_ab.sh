#!/bin/bash
# NT vs plain output stores of the band kernel, two views on one box:
# bench.py (MPX_CONV_BAND=1 plain, 2 NT) and tools/kbench.py band4 variants.
set -o pipefail
O=gpurun_out/r2/nt_ab; mkdir -p $O
for r in 1 2 3; do
  for b in 1 2; do
    MPX_CONV_BAND=$b timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_b${b}_r${r}.json 2> $O/bench_b${b}_r${r}.err || exit 1
    python -c "import json; d=json.loads(open('$O/bench_b${b}_r${r}.json').read().strip().splitlines()[-1]); print('bench band=$b', d['value'], d['ms_per_step'], d.get('value_warm_cache'))"
  done
done
timeout -k 10 300 python tools/kbench.py --rotate 6 --rounds 7 --only sobel5-sep/band4 > $O/kbench.jsonl 2>&1 || exit 1
grep -h variant $O/kbench.jsonl
