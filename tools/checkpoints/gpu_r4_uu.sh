#!/bin/bash
# Round-4 checkpoint UU (final tree, checkpoint O again after the last native rebuild): smoke, bench, and the per-kernel profile
# (kernel trace + the standard counter passes over tools/prof_all.py),
# summarised on the box (the rocpd databases exceed gpurun's 64 MiB return).
set -o pipefail
O=${O:-gpurun_out/r4/uu}
export O
mkdir -p "$O"
bash tools/gpu.sh smoke &&
bash tools/gpu.sh run bench 300 python bench.py &&
bash tools/gpu.sh profile kfinal -- python3 tools/prof_all.py &&
python tools/experiments/kprof_table.py "$O" > "$O/kernels_table.md" &&
python tools/experiments/kprof_table.py "$O" --grep "<" > /dev/null &&
python tools/pmc_median.py "$O"/kfinal.pmc* > "$O/medians.md" &&
python tools/experiments/trace_db.py "$O/kfinal" --top 40 > "$O/trace.md" &&
du -sh "$O" && find "$O" -name "*.db" -delete && du -sh "$O"
