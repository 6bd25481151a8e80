#!/bin/bash
# Peer-halo transport on one MI355X: multi-process tests (2-3 ranks share the
# GPU, gloo control plane) + 2- and 4-rank bench rehearsals + the 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_peer_halo.py -x -v --timeout 280 -m gpu > gpurun_out/peer_tests.log 2>&1 || { tail -40 gpurun_out/peer_tests.log; exit 2; }
tail -5 gpurun_out/peer_tests.log
MPX_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench2_rehearsal.log 2>&1 \
    || { tail -30 gpurun_out/bench2_rehearsal.log; exit 3; }
grep metric gpurun_out/bench2_rehearsal.log
# 4 ranks: interior ranks map both neighbours (the N = 8 code path, on one card)
MPX_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/bench4_rehearsal.log 2>&1 \
    || { tail -30 gpurun_out/bench4_rehearsal.log; exit 5; }
grep metric gpurun_out/bench4_rehearsal.log
timeout -k 10 240 python bench.py > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 4; }
grep metric gpurun_out/bench1.log
