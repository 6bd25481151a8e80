#!/bin/bash
# Same-box A/B of the sobel5 band kernel (MPX_CONV_BAND=2 default: NT stores,
# 1: plain stores) against the 8-B-lane wave kernel (MPX_CONV_BAND=0): GPU conv tests, then bench.py N=1
# alternated. Output: gpurun_out/r2/band_ab/.
set -o pipefail
O=gpurun_out/r2/band_ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_peer_halo.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for b in 0 1 2; do
    MPX_CONV_BAND=$b timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_b${b}_r${r}.json 2> $O/bench_b${b}_r${r}.err || exit 1
    python -c "import json,sys; d=json.loads(open('$O/bench_b${b}_r${r}.json').read().strip().splitlines()[-1]); print('band=$b', d['value'], d['ms_per_step'], d.get('value_warm_cache'), d.get('verified_bit_exact'))"
  done
done
