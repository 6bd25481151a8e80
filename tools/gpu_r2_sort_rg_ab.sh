#!/bin/bash
# Radix scatter ranking batch (MPX_SORT_RG slices per batch) A/B: production
# libmpx (4) vs build_ab/libmpx_rg{2,8}.so, alternated twice.
set -o pipefail
O=gpurun_out/r2/sort_rg; mkdir -p $O
for r in 1 2; do
  for v in base rg2 rg8; do
    if [ $v = base ]; then L=""; else L=$PWD/build_ab/libmpx_$v.so; fi
    MPX_LIB_PATH=$L timeout -k 10 300 python tools/lab5_bench.py > $O/${v}_$r.jsonl 2>&1 || { tail -20 $O/${v}_$r.jsonl; exit 1; }
  done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r2/sort_rg/*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            if r.get("n") in (16777216, 67108864) and r.get("dtype") in ("int32", "float32"):
                print(f.split("/")[-1], r["dtype"], r["n"], r["mpx_ms"], r["verified_vs_torch"], r["torch_sort_ms"])
PY
