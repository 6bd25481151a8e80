#!/usr/bin/env python3
"""Bursts of one kernel family in a rocprofv3 kernel trace (rocpd sqlite):
dispatches whose name contains --grep, in start order, split wherever the GPU
sat idle for more than --gap us. Per burst: dispatches, wall time from the
first start to the last end, wall per dispatch, median / min duration, the
hardware queues used and the busy fraction (union of the dispatch intervals
over the wall). Used to compare the bench's static and streaming phases.

  python tools/experiments/phase_trace.py <dir-or-db> [--grep conv_band] [--gap 200]
"""
import argparse
import glob
import os
import sqlite3
import statistics


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--grep", default="conv_band")
    p.add_argument("--gap", type=float, default=200.0)
    a = p.parse_args()
    dbs = [a.path] if a.path.endswith(".db") else glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True)
    for db in dbs:
        c = sqlite3.connect(db)
        rows = [r for r in c.execute("select name, start, end, queue_id from kernels order by start")
                if a.grep in r[0]]
        if not rows:
            continue
        print(f"### {os.path.basename(db)}\n")
        print("| burst | dispatches | wall us | wall / dispatch us | median dur us | min dur us | queues | busy |")
        print("|---|---|---|---|---|---|---|---|")
        bursts, cur, last_end = [], [], None
        for r in rows:
            if cur and (r[1] - last_end) / 1e3 > a.gap:
                bursts.append(cur)
                cur = []
            cur.append(r)
            last_end = r[2] if last_end is None or not cur[:-1] else max(last_end, r[2])
        bursts.append(cur)
        for i, b in enumerate(bursts):
            t0, t1 = b[0][1], max(r[2] for r in b)
            d = [(r[2] - r[1]) / 1e3 for r in b]
            busy, s, e = 0, None, None
            for r in sorted(b, key=lambda r: r[1]):
                if s is None or r[1] > e:
                    busy += 0 if s is None else e - s
                    s, e = r[1], r[2]
                else:
                    e = max(e, r[2])
            busy += e - s
            wall = (t1 - t0) / 1e3
            print(f"| {i} | {len(b)} | {wall:.1f} | {wall / len(b):.2f} | {statistics.median(d):.2f} | {min(d):.2f} | "
                  f"{sorted({r[3] for r in b})} | {busy / 1e3 / wall:.2f} |")
        print()


if __name__ == "__main__":
    main()
