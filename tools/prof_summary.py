#!/usr/bin/env python3
"""Summarise rocprofv3 output into markdown for profiles/.

  prof_summary.py trace <dir>      kernel-trace stats (rocpd *.db or *_kernel_stats.csv)
  prof_summary.py pmc <dir> [...]  PMC counters per kernel (run_counter_collection.csv),
                                   summed over the dispatches of the LAST call of each kernel

Output is a markdown table on stdout.
"""

import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name: str, n: int = 70) -> str:
    name = name.replace("mpx::(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0] if "(" in name else name
    return name[:n]


def trace(d: str) -> None:
    rows = []
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if dbs:
        c = sqlite3.connect(dbs[0])
        for name, dur in c.execute("select name, duration from kernels"):
            rows.append((name, dur / 1e3))
    else:
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                rows.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    if not rows:
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        print("| kernel | calls | avg us | min us | max us | % |\n|---|---|---|---|---|---|")
        for f in stats:
            for r in csv.DictReader(open(f)):
                print(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                      f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
        return
    agg = defaultdict(list)
    for n, us in rows:
        agg[n].append(us)
    tot = sum(us for _, us in rows)
    print("| kernel | calls | avg us | min us | max us | % |\n|---|---|---|---|---|---|")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {short(n)} | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} | "
              f"{100 * sum(v) / tot:.1f} |")


def pmc(dirs) -> None:
    # counter -> kernel -> value of the last dispatch
    vals = defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            last = {}
            for r in csv.DictReader(open(f)):
                key = (r["Kernel_Name"], r["Counter_Name"])
                did = int(r["Dispatch_Id"])
                if key not in last or did >= last[key][0]:
                    prev = last.get(key)
                    v = float(r["Counter_Value"])
                    if prev and prev[0] == did:
                        v += prev[1]
                    last[key] = (did, v)
            for (k, c), (_, v) in last.items():
                vals[c][k] = v
    kernels = sorted({k for m in vals.values() for k in m})
    counters = sorted(vals)
    print("| counter | " + " | ".join(short(k, 40) for k in kernels) + " |")
    print("|---|" + "---|" * len(kernels))
    for c in counters:
        print(f"| {c} | " + " | ".join(f"{vals[c].get(k, float('nan')):.4g}" for k in kernels) + " |")
    # derived ratios when available
    def get(c, k):
        return vals.get(c, {}).get(k)
    lines = []
    for k in kernels:
        wc, wi, ai = get("SQ_WAVE_CYCLES", k), get("SQ_WAIT_INST_ANY", k), get("SQ_ACTIVE_INST_ANY", k)
        if wc:
            parts = []
            if wi is not None:
                parts.append(f"wait-inst {100 * wi / wc:.0f}%")
            if ai is not None:
                parts.append(f"active-inst {100 * ai / wc:.0f}%")
            lines.append(f"* {short(k, 50)}: " + ", ".join(parts) + " of wave-cycles")
    if lines:
        print()
        print("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) < 3 or sys.argv[1] not in ("trace", "pmc"):
        print(__doc__)
        sys.exit(2)
    if sys.argv[1] == "trace":
        trace(sys.argv[2])
    else:
        pmc(sys.argv[2:])
