#!/usr/bin/env python3
"""Summarise gpurun_out/harness_cmp (tools/harness_compare.sh) as markdown:
median kernel ms per (bucket/n, timing, geometry), next to BASELINE.md."""
import glob
import json
import os
import sys

import pandas as pd

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/harness_cmp"
rows = []
for d in sorted(glob.glob(os.path.join(root, "*", "lab*"))):
    tag = os.path.basename(os.path.dirname(d))
    lab, size, timing = tag.split("_")
    for f in glob.glob(os.path.join(d, "src", "stats_*.csv")):
        df = pd.read_csv(f)
        dev = "CPU (-O0, 1 thread)" if os.path.basename(f).startswith("stats_cpu_") else "MI355X"
        for ks, g in df.groupby(df["kernel_size"].astype(str)):
            rows.append({"lab": lab, "size": size, "timing": timing, "device": dev, "geometry": ks,
                         "median_ms": g["time_kernel_exe_ms"].median(), "runs": len(g)})
out = pd.DataFrame(rows)
for (lab, size), g in out.groupby(["lab", "size"], sort=False):
    print(f"\n### {lab} {size}\n")
    piv = g.pivot_table(index=["device", "geometry"], columns="timing", values="median_ms", aggfunc="first")
    print(piv.round(5).to_markdown())
