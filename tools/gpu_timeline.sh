#!/bin/bash
# Kernel timeline of the emulated N>1 step (native RCCL self exchange + convs).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
mkdir -p gpurun_out/timeline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/timeline -o run -- python3 $R/tools/step_overhead.py --native-only > $R/gpurun_out/timeline/run.log 2>&1 || { tail -20 $R/gpurun_out/timeline/run.log; exit 1; }
find $R/gpurun_out/timeline -name "*kernel_trace.csv" | head
