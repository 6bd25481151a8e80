#!/bin/bash
# Conv GPU tests (kernels, headline, peer halos) + bench.py N=1 twice.
set -o pipefail
O=gpurun_out/r2/band_check; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_peer_halo.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  python -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('verified_bit_exact'))"
done
