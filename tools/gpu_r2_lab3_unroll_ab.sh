#!/bin/bash
# A/B of the lab3 fast32 class loop unrolled by four (current tree) against a
# libmpx built from the previous classify.hip in build_ab/ (MPX_LIB_PATH).
set -o pipefail
O=gpurun_out/r2/lab3ab; mkdir -p $O
for r in 1 2; do
  MPX_LIB_PATH=$PWD/build_ab/libmpx_old.so  # a libmpx built from the previous classify.hip timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/old_$r.jsonl 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_suite.py --only lab3 > $O/new_$r.jsonl 2>&1 || exit 1
done
grep -h '"path": "fast"' $O/*.jsonl | cut -c1-250
