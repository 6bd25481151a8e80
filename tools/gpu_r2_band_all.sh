#!/bin/bash
# Full GPU test suite + production conv timings after routing the dense and
# separable conv launches through the band kernel. Output: gpurun_out/r2/band_all/.
set -o pipefail
O=gpurun_out/r2/band_all
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/kbench.py --rotate 6 --rounds 5 --only production > $O/prod.jsonl 2>&1 || { tail -20 $O/prod.jsonl; exit 1; }
grep -E "ERROR|variant" $O/prod.jsonl
for b in 0 2; do
  MPX_CONV_BAND=$b timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_b$b.json 2> $O/bench_b$b.err || exit 1
  python -c "import json; d=json.loads(open('$O/bench_b$b.json').read().strip().splitlines()[-1]); print('band=$b', d['value'], d['ms_per_step'], d.get('value_warm_cache'), d.get('verified_bit_exact'))"
done
