#!/usr/bin/env python3
"""Per-kernel counter table from a rocprofv3 --pmc results .db (ROCm 7.2 writes
sqlite): value summed over a dispatch's components, median over dispatches of
the same kernel. `--grep` narrows to kernel names containing a substring;
`--short` trims template arguments after the first '<' except the ones listed."""
import argparse
import re
import sqlite3
import statistics
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grep", default="")
    args = ap.parse_args()
    db = sqlite3.connect(args.db)
    rows = db.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for did, kn, cn, v in rows:
        if args.grep and args.grep not in kn:
            continue
        per[did][cn] += v
        names[did] = short(kn)
    agg = defaultdict(lambda: defaultdict(list))
    counters = set()
    for did, cs in per.items():
        for cn, v in cs.items():
            agg[names[did]][cn].append(v)
            counters.add(cn)
    counters = sorted(counters)
    print("| kernel | dispatches | " + " | ".join(counters) + " |")
    print("|---|---|" + "---|" * len(counters))
    for kn, cs in agg.items():
        n = max(len(v) for v in cs.values())
        vals = [statistics.median(cs[c]) if c in cs else float("nan") for c in counters]
        print(f"| {kn} | {n} | " + " | ".join(f"{v / 1e6:.2f}M" for v in vals) + " |")


if __name__ == "__main__":
    main()
