#!/bin/bash
# Very thin harness geometries (<= 2048 threads, <= 256 per block): 16 loads in
# flight per lane (vsub, Roberts thin kernel) vs the 8-deep build (build_ab/libmpx_old.so).
set -o pipefail
O=gpurun_out/r2/thin_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "vsub or roberts" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  MPX_LIB_PATH=$PWD/build_ab/libmpx_old.so timeout -k 10 300 python tools/thin_geom_bench.py > $O/old_$r.jsonl 2>&1 || { tail -20 $O/old_$r.jsonl; exit 1; }
  timeout -k 10 300 python tools/thin_geom_bench.py > $O/new_$r.jsonl 2>&1 || { tail -20 $O/new_$r.jsonl; exit 1; }
done
for f in $O/*.jsonl; do echo "== $f"; cat $f; done
