#!/bin/bash
# lab3 fast32 with deferred fp64 re-ranking (current tree) vs a libmpx built
# from the previous classify.hip in build_ab/ (MPX_LIB_PATH); lab3 GPU tests first.
set -o pipefail
O=gpurun_out/r2/lab3defer; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "classif or lab3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  MPX_LIB_PATH=$PWD/build_ab/libmpx_old.so timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/old_$r.jsonl 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/new_$r.jsonl 2>&1 || exit 1
done
grep -H '"path": "fast"' $O/*.jsonl | sed 's/.*lab3defer.//' | cut -c1-200
