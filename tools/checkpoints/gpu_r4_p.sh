#!/bin/bash
# Round-4 checkpoint P: copy floors and conv schedules with launches
# overlapped on 2 streams (the bench's regime) vs one stream.
set -o pipefail
O=${O:-gpurun_out/r4/p}
export O
mkdir -p "$O"
V="copy/linear,copy/band-seg16-f106,copy/band-seg16-f74,copy/band-seg16-f10,copy/burst-r16-t512-f7,copy/burst-r8-t256-f4,copy/burst-r16-t1024-f15,sobel5/production,copy/torch"
bash tools/gpu.sh run kb_s2 300 python -u tools/kbench.py --rotate 6 --streams 2 --rounds 5 --only "$V" &&
bash tools/gpu.sh run kb_s1 300 python -u tools/kbench.py --rotate 6 --streams 1 --rounds 5 --only "$V" &&
bash tools/gpu.sh run kb_s3 300 python -u tools/kbench.py --rotate 6 --streams 3 --rounds 5 --only "$V"
