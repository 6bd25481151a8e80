#!/bin/bash
# Wave kernel (MPX_CONV_BAND=0) vs band kernel (default) for every named
# filter, rotated 4096^2, two alternations. Output: gpurun_out/r2/filters/.
set -o pipefail
O=gpurun_out/r2/filters
mkdir -p $O; rm -f $O/ab.jsonl
for r in 1 2; do
  for b in 0 2; do
    MPX_CONV_BAND=$b timeout -k 10 200 python tools/conv_filters_bench.py >> $O/ab.jsonl 2> $O/err_$b_$r.log || exit 1
  done
done
python - <<'PY'
import collections, json
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/r2/filters/ab.jsonl"):
    r = json.loads(l)
    d[r["filter"]][r["band_mode"]].append(r["us_median"])
for f, v in d.items():
    print(f, "wave", v["0"], "band", v["2"])
PY
