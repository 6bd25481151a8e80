#!/usr/bin/env python3
"""lab3 launch-grid sweep: fast32 / mfma8 at 8192^2 over
the number of workgroups (a grid-stride kernel whose default grid of
CUs x 8 blocks may leave a partial second round), every result checked
against the default launch. One JSON line per (nc, path, grid)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402


def time_us(fn, iters=10, warmup=2):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    return sorted(ts)[1]


def main():
    dev = torch.device("cuda:0")
    size = 8192
    # three images cycled: 768 MiB working set, beyond the 256 MB MALL (HBM-honest)
    imgs = [torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev) for _ in range(3)]
    host = imgs[0].cpu()
    ncs = [int(v) for v in os.environ.get("LAB3_NCS", "2,4,8,32").split(",")]
    grids = [int(g) for g in os.environ.get("LAB3_GRIDS", "0,256,512,768,1024,1280,1536,2048,4096,8192,16384").split(",")]
    for nc in ncs:
        pts = class_points_for(size, size, nc, 64, seed=nc)
        mu, inv = ops.class_stats(host, pts)
        for path in ("fast", "mfma8"):
            ref = imgs[0].clone()
            ops.classify_(ref, mu, inv, path=path)
            for g in grids:
                work = imgs[0].clone()
                ops.classify_(work, mu, inv, path=path, grid=g)
                ok = torch.equal(work, ref)
                cyc = [0]

                def run():
                    ops.classify_(imgs[cyc[0] % 3], mu, inv, path=path, grid=g)
                    cyc[0] += 1
                us = time_us(run)
                print(json.dumps({"nc": nc, "path": path, "grid": g, "us": round(us, 1), "same": ok}), flush=True)


if __name__ == "__main__":
    main()
