#!/bin/bash
# Round-4 checkpoint BB (final tree): the full GPU suite and smoke.
set -o pipefail
O=${O:-gpurun_out/r4/bb}
export O
mkdir -p "$O"
bash tools/gpu.sh tests && bash tools/gpu.sh smoke
