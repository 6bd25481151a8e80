#!/bin/bash
# Round-4 checkpoint D: the vertical-halo-sharing band kernel (conv_band16v)
# against production and the copy floors, its GPU test, then checkpoint C
# (bench A/B of streams / warm-up, kernel trace, lab3 grid sweep).
set -o pipefail
O=${O:-gpurun_out/r4/d}
export O
mkdir -p "$O"
bash tools/gpu.sh run kbench_vs 300 python -u tools/kbench.py --rotate 6 --rounds 7 --iters 20 \
    --only "band16v,sobel5/production,gauss5/production,band4/seg0/w34000,copy/band-seg16-f106,copy/band-seg16-f74,copy/linear" &&
bash tools/gpu.sh tests tests/test_gpu_kernels.py -k "vertical_share or strip_edges or fast_sqrt" &&
cp "$O/pytest.log" "$O/pytest_vs.log" &&
O=gpurun_out/r4/c bash tools/gpu_r4_c.sh
