#!/bin/bash
# Band kernel row-load cache policy A/B (rotated): NT stores (production, w2000)
# vs NT stores + NT loads of interior rows (w34000) or of every row (w66000).
set -o pipefail
O=gpurun_out/r2/ntload_ab; mkdir -p $O
timeout -k 10 400 python tools/kbench.py --rotate 6 --rounds 9 --only sobel5-sep/band4 > $O/kbench.jsonl 2>&1 || { tail -20 $O/kbench.jsonl; exit 1; }
grep -h "variant\|bit_exact" $O/kbench.jsonl
