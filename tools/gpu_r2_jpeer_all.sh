#!/bin/bash
# Peer-signalled Jacobi: multi-process tests (2/3/4/8 ranks on one GPU), then
# the native one-process rehearsal timings (tools/gpu_r2_mgpu_peer.sh).
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests/test_peer_halo.py -m gpu -x -q --timeout 280 --timeout-method thread \
    > gpurun_out/r2/peer_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2/peer_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r2_mgpu_peer.sh
