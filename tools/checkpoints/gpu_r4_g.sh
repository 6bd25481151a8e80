#!/bin/bash
# Round-4 checkpoint G: sort ranking variants (7 production, 9 returning-add,
# 10 = 9 on 4096-key tiles, 11 = 9 at 3 blocks/CU) timed, traced and counted;
# lab3 fast32 memory-policy variants and the mfma8 windowed fix-ups A/B'd,
# mfma8 write bytes; the lab3 / lab5 GPU suites on the new kernels.
set -o pipefail
O=${O:-gpurun_out/r4/g}
export O
mkdir -p "$O"
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=7,8,9,10,11 bash tools/gpu.sh run sort_variants 300 \
  python -u tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=9 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=2 \
  bash tools/gpu.sh prof sort_v9_trace -- python3 tools/experiments/sort_probe.py &&
SORT_PROBE_PARTS=variants SORT_PROBE_VARIANTS=7,9 SORT_PROBE_LOGN=26 SORT_PROBE_SMALL=0 SORT_PROBE_ITERS=1 \
  bash tools/gpu.sh pmc sort_v79_lds "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES" \
  -- python3 tools/experiments/sort_probe.py &&
for r in 1 2; do
  for o in 0 1 2 3 4 7; do
    MPX_CLS_OPT=$o LAB3_NCS=2,4,8 LAB3_PATHS=fast LAB3_TAG=r$r bash tools/gpu.sh run lab3_fast_o${o}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
  for wv in 0 1; do
    MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=8,32 LAB3_PATHS=mfma8 LAB3_TAG=r$r bash tools/gpu.sh run lab3_mfma8_w${wv}_r$r 200 \
      python -u tools/experiments/lab3_ab.py || exit 1
  done
done &&
for wv in 0 1; do
  MPX_CLS_MFMA8_WIN=$wv LAB3_NCS=32 LAB3_PATHS=mfma8 bash tools/gpu.sh pmc lab3_mfma8_w${wv}_bytes "WRITE_SIZE" \
    -- python3 tools/experiments/lab3_ab.py || exit 1
done &&
bash tools/gpu.sh tests tests/test_lab5_sort.py tests/test_classify_i8.py tests/test_gpu_kernels.py tests/test_gpu_headline.py
