#!/bin/bash
# A/B of the radix sort (current tree) against a libmpx built from the previous
# sort.hip in build_ab/ (MPX_LIB_PATH); sort GPU tests on the current tree first.
set -o pipefail
O=gpurun_out/r2/sortab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lab5_sort.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  MPX_LIB_PATH=$PWD/build_ab/libmpx_old.so timeout -k 10 300 python tools/lab5_bench.py > $O/old_$r.jsonl 2>&1 || exit 1
  timeout -k 10 300 python tools/lab5_bench.py > $O/new_$r.jsonl 2>&1 || exit 1
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r2/sortab/*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            if r.get("n") in (16777216, 67108864) and r.get("dtype") in ("int32", "float32"):
                print(f.split("/")[-1], r["dtype"], r["n"], r["mpx_ms"], r["variants"].get("persistent", r["variants"]))
PY
