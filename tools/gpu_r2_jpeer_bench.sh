#!/bin/bash
# Peer-signalled Jacobi timings after the fence removal: multi-process Python
# path (tools/gpu_r2_jpeer.sh) and the native one-process path with the
# no-exchange ablation (tools/gpu_r2_mgpu_peer.sh).
set -o pipefail
bash tools/gpu_r2_jpeer.sh || exit $?
bash tools/gpu_r2_mgpu_peer.sh || exit $?
