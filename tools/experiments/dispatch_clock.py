#!/usr/bin/env python3
"""Per-dispatch effective shader clock from a rocprofv3 ``--pmc GRBM_GUI_ACTIVE``
results database (ROCm 7.2 sqlite): clock = GRBM_GUI_ACTIVE cycles (rocprofv3
reports them summed over the 8 XCDs: --xcds) / 8 / dispatch duration. Lists
each dispatch of the kernels matching ``--grep`` in start order with its time
since the first one, so a clock trajectory under sustained load can be put
next to the step times (VERDICT r4 Next #2; the 200 Hz SMU metrics of
utils/clocks.py average over milliseconds, this is per kernel).

  python tools/experiments/dispatch_clock.py DB [--grep conv_band4] [--bins 0,10,20,50,100,500,1000,3000]
"""
import argparse
import re
import sqlite3
import statistics
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name)
    return re.sub(r"<.*$", "", name).split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grep", default="")
    ap.add_argument("--bins", default="0,10,20,50,100,200,500,1000,2000,5000")
    ap.add_argument("--csv", default="")
    ap.add_argument("--xcds", type=int, default=8, help="GRBM_GUI_ACTIVE comes summed over this many XCD instances")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select dispatch_id, kernel_name, value, start, end from counters_collection "
                      "where counter_name = 'GRBM_GUI_ACTIVE'").fetchall()
    per = defaultdict(lambda: [0.0, 0, None, None, None])
    for did, kn, v, st, en in rows:
        p = per[did]
        p[0] += v
        p[1] += 1
        p[2], p[3], p[4] = short(kn), st, en
    ds = sorted((p[3], p[4], p[2], p[0] / a.xcds) for p in per.values() if a.grep in p[2])
    if not ds:
        print("no dispatches")
        return
    t00 = ds[0][0]
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("t_ms,kernel,us,ghz\n")
            for st, en, kn, cyc in ds:
                f.write(f"{(st - t00) / 1e6:.4f},{kn},{(en - st) / 1e3:.3f},{cyc / (en - st):.4f}\n")
    # bins by time since each kernel's own first dispatch after an idle gap (> 200 ms)
    bins = [float(x) for x in a.bins.split(",")]
    runs, cur, last_end = [], [], None
    for d in ds:
        if last_end is not None and d[0] - last_end > 200e6:
            runs.append(cur)
            cur = []
        cur.append(d)
        last_end = d[1]
    runs.append(cur)
    print("| run | kernel | dispatches | " + " | ".join(f"{int(lo)}-{int(hi)} ms µs (GHz)" for lo, hi in
                                                      zip(bins[:-1], bins[1:])) + " |")
    print("|---|---|---|" + "---|" * (len(bins) - 1))
    for i, r in enumerate(runs):
        t0 = r[0][0]
        kn = r[0][2]
        cells = []
        for lo, hi in zip(bins[:-1], bins[1:]):
            sel = [d for d in r if lo <= (d[0] - t0) / 1e6 < hi]
            if not sel:
                cells.append("–")
                continue
            us = statistics.median((d[1] - d[0]) / 1e3 for d in sel)
            ghz = statistics.median(d[3] / (d[1] - d[0]) for d in sel)
            cells.append(f"{us:.2f} ({ghz:.2f})")
        print(f"| {i} | {kn} | {len(r)} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
