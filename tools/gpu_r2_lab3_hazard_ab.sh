#!/bin/bash
# lab3 fast32: previous source (build_ab/libmpx_old.so via MPX_LIB_PATH) vs the
# current tree (key tag and top-2 update written so the compiler sees them:
# 17 fewer s_nop hazard pads per 4-class loop trip).
set -o pipefail
O=gpurun_out/r2/lab3hz; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "classif or lab3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  MPX_LIB_PATH=$PWD/build_ab/libmpx_old.so timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/old_$r.jsonl 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/new_$r.jsonl 2>&1 || exit 1
done
grep -H '"path": "fast"' $O/*.jsonl | sed 's/.*lab3hz.//' | python3 -c "
import sys, json
for l in sys.stdin:
    f, j = l.split(':', 1)
    r = json.loads(j)
    print(f, r['nc'], r['us'], r['verified'])
"
