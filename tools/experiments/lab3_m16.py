#!/usr/bin/env python3
"""lab3 mfma16 A/B at 8192^2 (round 6): three rotated images, one JSON line
per (nc, path, grid); classes checked against the exact DIRECT path once per
(nc, path). LAB3_NCS / LAB3_PATHS / LAB3_GRIDS (0 = the library's default
grid) / LAB3_TAG select and label a run. With LAB3_PROF=1 each (nc, path)
runs 3 times on one image and nothing is timed (rocprofv3 driver)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402


def time_us(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    ts.sort()
    return ts[2], ts[0]


def main():
    dev = torch.device("cuda:0")
    size = 8192
    prof = os.environ.get("LAB3_PROF", "0") == "1"
    imgs = [torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev) for _ in range(1 if prof else 3)]
    host = imgs[0].cpu()
    ncs = [int(v) for v in os.environ.get("LAB3_NCS", "4,16,32").split(",")]
    paths = os.environ.get("LAB3_PATHS", "mfma16").split(",")
    grids = [int(v) for v in os.environ.get("LAB3_GRIDS", "0").split(",")]
    tag = os.environ.get("LAB3_TAG", "")
    for nc in ncs:
        mu, inv = ops.class_stats(host, class_points_for(size, size, nc, 64, seed=nc))
        if prof:
            for path in paths:
                for _ in range(3):
                    ops.classify_(imgs[0], mu, inv, path=path)
            torch.cuda.synchronize()
            continue
        ref = imgs[0].clone()
        ops.classify_(ref, mu, inv, path="direct")
        for path in paths:
            amb = torch.zeros(1, dtype=torch.int32, device=dev)
            work = imgs[0].clone()
            ops.classify_(work, mu, inv, path=path, ambiguous=amb)
            ok = torch.equal(work, ref)
            for g in grids:
                cyc = [0]

                def run(g=g):
                    ops.classify_(imgs[cyc[0] % 3], mu, inv, path=path, grid=g)
                    cyc[0] += 1
                med, mn = time_us(run)
                print(json.dumps({"tag": tag, "nc": nc, "path": path, "ran": ops.classify_plan(mu, inv, path)[0], "grid": g, "us": round(med, 1),
                                  "us_min": round(mn, 1), "same_as_direct": ok,
                                  "undecided": int(amb.item())}),
                      flush=True)


if __name__ == "__main__":
    main()
