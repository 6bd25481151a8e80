#!/bin/bash
# Band kernel with one batched apron load per walk (OPT bit 3) vs production.
set -o pipefail
O=gpurun_out/r2/apron_batch; mkdir -p $O
timeout -k 10 400 python tools/kbench.py --rotate 6 --rounds 11 --only band4/seg > $O/kbench.jsonl 2>&1 || { tail -20 $O/kbench.jsonl; exit 1; }
grep -h "variant\|bit_exact" $O/kbench.jsonl
