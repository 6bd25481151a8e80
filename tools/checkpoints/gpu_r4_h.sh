#!/bin/bash
# Round-4 checkpoint H: bench.py (streaming phase now on 2 streams) and the
# stream count A/B; mfma8 windowed fix-ups with a single chunk body; lab5 with
# the new AUTO (returning-add ranking); kernel trace of the bench; GPU tests.
set -o pipefail
O=${O:-gpurun_out/r4/h}
export O
mkdir -p "$O"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-stream"
bash tools/gpu.sh run bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
for r in 1 2; do
  bash tools/gpu.sh run s1_$r 200 $B --streams 1 &&
  bash tools/gpu.sh run s2_$r 200 $B &&
  bash tools/gpu.sh run s3_$r 200 $B --streams 3 || exit 1
  for wv in 0 1; do
    MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=8,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_w${wv}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
done &&
LAB5_DTYPES=int32,float32 LAB5_LOGN=20,24,26 LAB5_VARIANTS=7,9,10 bash tools/gpu.sh run lab5 300 \
  python -u tools/experiments/lab5_bench.py &&
bash tools/gpu.sh prof bench_trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
bash tools/gpu.sh tests tests/test_lab5_sort.py tests/test_gpu_kernels.py -k "sort or radix or classify"
