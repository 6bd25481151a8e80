#!/bin/bash
# Production conv with alternating segments: kernel tests, peer tests, rotated
# production timings, the flagship bench.
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_peer_halo.py -m gpu -x -q \
    --timeout 280 --timeout-method thread > gpurun_out/r2/alt2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r2/alt2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kbench.py --rotate 6 --rounds 5 --only "production" > gpurun_out/r2/alt2_kb.jsonl 2>&1 || exit $?
grep -E "us_median|ERROR|bit_exact" gpurun_out/r2/alt2_kb.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/r2/alt2_bench.json 2> gpurun_out/r2/alt2_bench.err || exit $?
cat gpurun_out/r2/alt2_bench.json
