#!/bin/bash
# Alternating-direction conv segments: exactness, then rotated timing A/B.
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "alternating" --timeout 120 \
    --timeout-method thread > gpurun_out/r2/alt_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r2/alt_tests.log; [ $rc -eq 0 ] || exit $rc
for only in "sobel5-sep/wave-const/seg" "copy/strip-v4-d4-seg24" "sobel5/production"; do
  timeout -k 10 300 python -u tools/kbench.py --rotate 6 --rounds 5 --only "$only" > gpurun_out/r2/alt_kb.jsonl 2>&1 || exit $?
  grep -E "us_median|ERROR" gpurun_out/r2/alt_kb.jsonl | grep -v "pf8\|pf12"
done
