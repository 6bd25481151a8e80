#!/bin/bash
# Round-4 checkpoint B: more copy probes (band copies with NT loads, burst
# tiles with a one-workgroup-per-CU residency cap), then the peer / contract /
# oracle GPU tests. Each step time-bounded, chained with &&.
set -o pipefail
O=${O:-gpurun_out/r4/b}
export O
mkdir -p "$O"
bash tools/gpu.sh run kbench_copy2 300 python -u tools/kbench.py --only copy/ --rotate 6 --rounds 5 --iters 20 &&
bash tools/gpu.sh tests tests/test_peer_halo.py &&
cp "$O/pytest.log" "$O/pytest_peer.log" &&
bash tools/gpu.sh tests tests/test_contract.py &&
cp "$O/pytest.log" "$O/pytest_contract.log" &&
bash tools/gpu.sh tests tests/test_gpu_headline.py tests/test_gpu_kernels.py -k "oracle or fast_sqrt"
