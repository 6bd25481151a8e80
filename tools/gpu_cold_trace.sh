#!/bin/bash
# Where does a cold first launch spend its time? HIP runtime log of one cold
# lab2 run, plus cold runs with deferred code-object loading forced off and on
# from the environment.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/cold_trace; mkdir -p $O
B=labs/lab2/src/to_plot_hip_exe
IMG=labs/lab2/metric_calc/small/02.data
run() { printf "32 32 16 16\n%s\n%s\n" "$IMG" "$O/out.data" | timeout -k 5 60 "$@" $B; }
AMD_LOG_LEVEL=4 MPX_TIMING=cold run env > $O/stdout.txt 2> $O/amdlog.txt
for v in 0 1; do for i in 1 2 3; do
  echo "DEFERRED=$v $(HIP_ENABLE_DEFERRED_LOADING=$v MPX_TIMING=cold run env | head -1)"
done; done | tee $O/deferred_ab.txt
wc -l $O/amdlog.txt
