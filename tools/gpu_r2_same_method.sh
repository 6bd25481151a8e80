#!/bin/bash
# Refresh of the same-methodology lab2 number (bench.py vs_reference_same_method):
# run_test.py on the reference's metric_calc/large bucket, cold (one launch per
# process, as published), best published geometry [[32,32],[16,16]] and the
# tuned launch [[0,0],[0,0]]. Output: gpurun_out/r2/same_method/.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
W=$PWD/gpurun_out/r2/same_method/lab2; mkdir -p $W/src
cp labs/lab2/src/to_plot_hip_exe labs/lab2/src/cpu_exe $W/src/
timeout -k 10 600 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe --binary_path_cpu $W/src/cpu_exe \
  --k_times 12 --kernel_sizes '[[[32,32],[16,16]],[[0,0],[0,0]]]' --timing cold --dir_to_data labs/lab2/metric_calc/large \
  --dir_to_data_out $W/data_out --metadata_columns2plot '["filename"]' > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 1; }
grep -E "SUCCESS|FAILED|median|Speedup" $W/run.log | tail -12
rm -rf $W/data_out $W/src
