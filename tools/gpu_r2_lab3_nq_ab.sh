#!/bin/bash
# lab3 fast32: previous source (build_ab/libmpx_old.so, MPX_LIB_PATH) vs the
# current tree with 4 (MPX_CLS_NQ=1) and 8 (MPX_CLS_NQ=2) pixels per thread.
set -o pipefail
O=gpurun_out/r2/lab3nq; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "classif or lab3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MPX_CLS_NQ=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "classif or lab3" > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -1 $O/pytest2.log
for r in 1 2; do
  MPX_LIB_PATH=$PWD/build_ab/libmpx_old.so timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/old_$r.jsonl 2>&1 || exit 1
  MPX_CLS_NQ=1 timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/nq1_$r.jsonl 2>&1 || exit 1
  MPX_CLS_NQ=2 timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/nq2_$r.jsonl 2>&1 || exit 1
done
grep -H '"path": "fast"' $O/*.jsonl | sed 's/.*lab3nq.//' | python3 -c "
import sys, json
for l in sys.stdin:
    f, j = l.split(':', 1)
    r = json.loads(j)
    print(f, r['nc'], r['us'], r['verified'])
"
