#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 rocpd database (kernel trace).

  python tools/experiments/trace_db.py <dir-or-db> [--top N] [--grep SUBSTR]

Groups dispatches by (kernel name, grid x) and prints calls, median, min and
total microseconds, sorted by total time.
"""
import argparse
import collections
import glob
import os
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--top", type=int, default=25)
    p.add_argument("--grep", default="")
    a = p.parse_args()
    db = a.path if a.path.endswith(".db") else glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    agg = collections.defaultdict(list)
    for name, dur, gx in c.execute("select name, duration, grid_x from kernels order by start"):
        short = name.replace("mpx::(anonymous namespace)::", "").split("(")[0]
        if a.grep in short:
            agg[(short[-70:], gx)].append(dur / 1e3)
    print("| kernel | grid x | calls | median us | min us | total us |\n|---|---|---|---|---|---|")
    for (k, gx), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        s = sorted(v)
        print(f"| `{k}` | {gx} | {len(v)} | {s[len(s) // 2]:.2f} | {s[0]:.2f} | {sum(v):.1f} |")


if __name__ == "__main__":
    main()
