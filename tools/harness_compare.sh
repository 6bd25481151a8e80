#!/bin/bash
# Same-methodology comparison with BASELINE.md: the reference harness on the
# reference's own inputs and published launch geometries, cold (one launch per
# process, as published) and warm. CSVs land in gpurun_out/harness_cmp/.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
# usage: harness_compare.sh [lab2] [lab2xl] [lab1] [literal] [lazy]
#   (default: lab2 lab2xl lab1)
#   literal: lab2 [[16,16],[1024,1024]] with MPX_GEOM_LITERAL=1 (every
#   workgroup of the published grid launched, empty ones included), cold,
#   warm and cold-lazy, every bucket
#   lazy: --timing cold-lazy (no code-object preload, no first dispatch before
#   the timer: HIP's lazy module load lands in the timed span), every lab2
#   bucket and lab1 n = 10^6
#   lab2xl: the BASELINE shape through the same harness — one synthetic 4096^2
#   random RGBA8 image (--synthetic 4096x4096, seeded), no other input
WHICH="${*:-lab2 lab2xl lab1}"
O=$PWD/gpurun_out/harness_cmp
mkdir -p $O
GEOMS2='[[[16,16],[1024,1024]],[[16,16],[32,32]],[[2,2],[16,16]],[[32,32],[16,16]],[[32,32],[64,64]],[[0,0],[0,0]]]'
for bucket in $([[ " $WHICH " == *" lab2 "* ]] && echo small medium large); do
  for timing in cold warm; do
    W=$O/lab2_${bucket}_${timing}/lab2; mkdir -p $W/src
    cp labs/lab2/src/to_plot_hip_exe labs/lab2/src/cpu_exe $W/src/
    timeout -k 10 600 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe --binary_path_cpu $W/src/cpu_exe \
      --k_times 12 --kernel_sizes "$GEOMS2" --timing $timing --dir_to_data labs/lab2/metric_calc/$bucket --dir_to_data_out $W/data_out \
      --metadata_columns2plot '["filename"]' > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 1; }
    grep -E "SUCCESS|FAILED|Speedup" $W/run.log | head -5
    rm -rf $W/data_out $W/src/*.png
  done
done
for bucket in $([[ " $WHICH " == *" lab2xl "* ]] && echo xl4096); do
  mkdir -p $O/empty_inputs
  for timing in cold warm; do
    W=$O/lab2_${bucket}_${timing}/lab2; mkdir -p $W/src
    cp labs/lab2/src/to_plot_hip_exe labs/lab2/src/cpu_exe $W/src/
    timeout -k 10 900 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe --binary_path_cpu $W/src/cpu_exe \
      --k_times 6 --kernel_sizes "$GEOMS2" --timing $timing --dir_to_data $O/empty_inputs --synthetic 4096x4096 \
      --dir_to_data_out $W/data_out --metadata_columns2plot '["filename"]' > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 1; }
    grep -E "SUCCESS|FAILED|Speedup" $W/run.log | head -5
    rm -rf $W/data_out $W/src/*.png
  done
done
for bucket in $([[ " $WHICH " == *" literal "* ]] && echo small medium large); do
  for timing in cold warm cold-lazy; do
    W=$O/lab2_${bucket}_${timing}_literal/lab2; mkdir -p $W/src
    cp labs/lab2/src/to_plot_hip_exe labs/lab2/src/cpu_exe $W/src/
    MPX_GEOM_LITERAL=1 timeout -k 10 600 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe \
      --binary_path_cpu $W/src/cpu_exe --k_times 12 --kernel_sizes '[[[16,16],[1024,1024]]]' --timing $timing \
      --dir_to_data labs/lab2/metric_calc/$bucket --dir_to_data_out $W/data_out \
      --metadata_columns2plot '["filename"]' > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 1; }
    grep -E "SUCCESS|FAILED|Speedup" $W/run.log | head -5
    rm -rf $W/data_out $W/src/*.png
  done
done
for bucket in $([[ " $WHICH " == *" lazy "* ]] && echo small medium large); do
  W=$O/lab2_${bucket}_cold-lazy/lab2; mkdir -p $W/src
  cp labs/lab2/src/to_plot_hip_exe labs/lab2/src/cpu_exe $W/src/
  timeout -k 10 600 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe --binary_path_cpu $W/src/cpu_exe \
    --k_times 12 --kernel_sizes "$GEOMS2" --timing cold-lazy --dir_to_data labs/lab2/metric_calc/$bucket \
    --dir_to_data_out $W/data_out --metadata_columns2plot '["filename"]' > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 1; }
  grep -E "SUCCESS|FAILED|Speedup" $W/run.log | head -5
  rm -rf $W/data_out $W/src/*.png
done
GEOMS1='[[1,32],[4,64],[32,128],[512,512],[1024,1024],[-1,-1]]'
for n in $([[ " $WHICH " == *" lazy "* ]] && echo 1000000); do
  W=$O/lab1_${n}_cold-lazy/lab1; mkdir -p $W/src
  cp labs/lab1/src/to_plot_hip_exe labs/lab1/src/cpu_exe $W/src/
  timeout -k 10 900 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe --binary_path_cpu $W/src/cpu_exe \
    --k_times 10 --kernel_sizes "$GEOMS1" --timing cold-lazy --min_vector_size $n --max_vector_size $n \
    > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 2; }
  grep -E "SUCCESS|FAILED|Speedup" $W/run.log | head -5
done
for n in $([[ " $WHICH " == *" lab1 "* ]] && echo 1000 10000 1000000); do
  for timing in cold warm; do
    W=$O/lab1_${n}_${timing}/lab1; mkdir -p $W/src
    cp labs/lab1/src/to_plot_hip_exe labs/lab1/src/cpu_exe $W/src/
    timeout -k 10 900 python run_test.py --binary_path_cuda $W/src/to_plot_hip_exe --binary_path_cpu $W/src/cpu_exe \
      --k_times 10 --kernel_sizes "$GEOMS1" --timing $timing --min_vector_size $n --max_vector_size $n \
      > $W/run.log 2>&1 || { tail -20 $W/run.log; exit 2; }
    grep -E "SUCCESS|FAILED|Speedup" $W/run.log | head -5
  done
done
echo done
