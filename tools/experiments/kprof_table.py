#!/usr/bin/env python3
"""Production-kernel table for profiles/kernels_rN.md from one `tools/gpu.sh
profile NAME -- python3 tools/prof_all.py` run: the kernel-trace database
(durations) and the counter passes' databases (NAME.pmc*), every rocprofv3
sqlite file under the given directory. Per kernel name (template arguments
kept): median / min µs over its dispatches, and the median of each counter
over the dispatches of every pass that collected it (per-dispatch values
summed over the counter's instances). Read bytes are TCC_EA0_RDREQ_sum x 128
and write bytes TCC_EA0_WRREQ_sum x 64 (profiles/README.md, "Counter caveat").

  python tools/experiments/kprof_table.py gpurun_out/r4/o [--grep mpx::]
"""
import argparse
import glob
import os
import re
import sqlite3
import statistics
from collections import defaultdict

COLS = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_MFMA")


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "").replace("mpx::", "")
    return re.sub(r"\(.*$", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    dur = defaultdict(list)
    ctr = defaultdict(lambda: defaultdict(list))
    for db in glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        tabs = {r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")}
        if "counters_collection" in tabs:
            per = defaultdict(lambda: defaultdict(float))
            names = {}
            for did, kn, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
                per[did][cn] += v
                names[did] = short(kn)
            for did, cs in per.items():
                for cn, v in cs.items():
                    ctr[names[did]][cn].append(v)
        if "kernels" in tabs:
            for kn, d in c.execute("select name, duration from kernels"):
                dur[short(kn)].append(d / 1e3)
    rows = []
    for k, ds in dur.items():
        if a.grep and a.grep not in k:
            continue
        cs = ctr.get(k, {})
        med = lambda n: statistics.median(cs[n]) if n in cs else None  # noqa: E731
        rd = med("TCC_EA0_RDREQ_sum")
        wr = med("TCC_EA0_WRREQ_sum")
        rows.append((k, statistics.median(ds), min(ds), len(ds), None if rd is None else rd * 128 / 2**20,
                     None if wr is None else wr * 64 / 2**20, [med(n) for n in COLS]))
    rows.sort(key=lambda r: r[0])
    f = lambda v, d=1: "—" if v is None else f"{v:,.{d}f}"  # noqa: E731
    print("| kernel | dispatches | median µs | min µs | read MiB (EA RDREQ×128) | write MiB (EA WRREQ×64) | VALU insts | "
          "LDS insts | LDS conflict cycles | MFMA insts |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for k, md, mn, n, rd, wr, cs in rows:
        print(f"| `{k}` | {n} | {md:.1f} | {mn:.1f} | {f(rd)} | {f(wr)} | "
              + " | ".join("—" if v is None else f"{v / 1e6:.2f}M" for v in cs) + " |")


if __name__ == "__main__":
    main()
