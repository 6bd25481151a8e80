#!/bin/bash
# Band kernel interior-row NT loads, second pass: kernel variants (apron policy,
# segment length), every production filter through ops.conv and bench.py, each
# A/B'd between MPX_CONV_BAND=2 (NT stores, plain loads) and 3 (+ NT interior loads).
set -o pipefail
O=gpurun_out/r2/ntload_ab2; mkdir -p $O
timeout -k 10 400 python tools/kbench.py --rotate 6 --rounds 9 --only sobel5-sep/band4 > $O/kbench.jsonl 2>&1 || { tail -20 $O/kbench.jsonl; exit 1; }
grep -h "variant\|bit_exact" $O/kbench.jsonl
for r in 1 2; do
  for b in 2 3; do
    MPX_CONV_BAND=$b timeout -k 10 300 python tools/kbench.py --rotate 6 --rounds 5 --only production > $O/prod_b${b}_r${r}.jsonl 2>&1 || { tail -20 $O/prod_b${b}_r${r}.jsonl; exit 1; }
    grep -h "variant\|ERROR" $O/prod_b${b}_r${r}.jsonl | sed "s/^/b$b r$r /"
  done
done
for r in 1 2 3; do
  for b in 2 3; do
    MPX_CONV_BAND=$b timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_b${b}_r${r}.json 2> $O/bench_b${b}_r${r}.err || { tail -20 $O/bench_b${b}_r${r}.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_b${b}_r${r}.json').read().strip().splitlines()[-1]); print('bench band=$b', d['value'], d['ms_per_step'], d.get('value_warm_cache'), d.get('verified_bit_exact'))"
  done
done
