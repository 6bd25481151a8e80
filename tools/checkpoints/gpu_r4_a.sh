#!/bin/bash
# Round-4 checkpoint A on one MI355X: burst-tile copy probes,
# then the mailbox / fused-streaming peer tests, the nccl-contract tests and
# the headline torch oracles. Each step time-bounded, chained with &&.
set -o pipefail
O=${O:-gpurun_out/r4/a}
export O
mkdir -p "$O"
bash tools/gpu.sh run kbench_copy 300 python -u tools/kbench.py --only copy/ --rotate 6 --rounds 5 --iters 20 &&
bash tools/gpu.sh tests tests/test_peer_halo.py -k "stream or beyond or jacobi_peer_signalled_equals" &&
cp "$O/pytest.log" "$O/pytest_peer.log" &&
bash tools/gpu.sh tests tests/test_contract.py &&
cp "$O/pytest.log" "$O/pytest_contract.log" &&
bash tools/gpu.sh tests tests/test_gpu_headline.py tests/test_gpu_kernels.py -k "oracle or fast_sqrt"
