#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py "$@" > gpurun_out/kbench.log 2>&1; rc=$?
cat gpurun_out/kbench.log
exit $rc
