#!/bin/bash
# bench.py A/B, MPX_CONV_BAND=2 (NT stores) vs 3 (+ NT loads of interior rows), 5 alternations.
set -o pipefail
O=gpurun_out/r2/ntload_bench; mkdir -p $O
for r in 1 2 3 4 5; do
  for b in 2 3; do
    MPX_CONV_BAND=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-warm > $O/bench_b${b}_r${r}.json 2> $O/bench_b${b}_r${r}.err || { tail -20 $O/bench_b${b}_r${r}.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_b${b}_r${r}.json').read().strip().splitlines()[-1]); print('bench band=$b', d['value'], d['ms_per_step'], d.get('verified_bit_exact'))"
  done
done
