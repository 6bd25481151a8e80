#!/usr/bin/env python3
"""Median of every PMC counter per kernel over all its dispatches, merged over
several rocprofv3 --pmc output directories (one counter group per pass):
CSV output (*counter_collection.csv) or the rocpd SQLite database
(*_results.db, the rocprofv3 default on this stack).

  pmc_median.py <dir> [<dir> ...]   -> markdown table: kernel x counter
"""
import csv
import glob
import os
import sqlite3
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("mpx::(anonymous namespace)::", "").replace("mpx::edge::", "").replace("void ", "")
    name = name.split("(")[0]
    return name[:60]


def main(dirs) -> None:
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)  # (dispatch, kernel, counter) -> summed over dimensions
            for r in csv.DictReader(open(f)):
                per[(r["Dispatch_Id"], short(r["Kernel_Name"]), r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, k, c), v in per.items():
                vals[k][c].append(v)
        for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            per = defaultdict(float)
            con = sqlite3.connect(f)
            for disp, kname, cname, v in con.execute(
                    "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
                per[(disp, short(kname), cname)] += float(v)
            for (_, k, c), v in per.items():
                vals[k][c].append(v)
    counters = sorted({c for k in vals for c in vals[k]})
    print("| kernel | " + " | ".join(counters) + " |")
    print("|---" * (len(counters) + 1) + "|")
    for k in sorted(vals):
        cells = []
        for c in counters:
            v = vals[k].get(c)
            cells.append(f"{statistics.median(v):,.0f}" if v else "")
        print(f"| `{k}` | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
