#!/usr/bin/env python3
"""Where the fixed cost of bench.py's timed region goes: T(K) = host time of
(sync; K rotated static steps on the 2-stream pair; sync) for K = 0..50, the
bench's detectors and streams, median of 9 repeats. K = 0 is the bare sync;
the slope is the steady per-step cost, the intercept the fill / drain / launch
/ wake-up cost the driver's K = 20 pays once. Also: the first step alone
(K = 1) split into enqueue and completion."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import parallel  # noqa: E402
from cuda_mpi_openmp_amd.models.edge import SlabEdgeDetector  # noqa: E402
from cuda_mpi_openmp_amd.utils.streams import compute_streams  # noqa: E402


def main():
    ctx = parallel.init(device="cuda")
    dev = ctx.device
    dets = []
    for r in range(6):
        d = SlabEdgeDetector(ctx, 4096, 4096, "sobel5")
        d.fill_random(seed=1234 + 7919 * r)
        dets.append(d)
    streams = compute_streams(dev, 2)
    hs = [s.cuda_stream for s in streams]
    main_s = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(main_s)
    cyc = [0]

    def step():
        i = cyc[0] % 6
        dets[i].step(hs[i % 2])
        cyc[0] += 1
    for _ in range(12):
        step()
    torch.cuda.synchronize(dev)
    res = {}
    for k in (0, 1, 2, 4, 8, 20, 50):
        ts, enq = [], []
        for _ in range(9):
            cyc[0] = 0
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(k):
                step()
            t1 = time.perf_counter()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            ts.append((t2 - t0) * 1e6)
            enq.append((t1 - t0) * 1e6)
        res[k] = statistics.median(ts)
        print(json.dumps({"K": k, "us": round(res[k], 1), "us_min": round(min(ts), 1),
                          "enqueue_us": round(statistics.median(enq), 1)}), flush=True)
    slope = (res[50] - res[20]) / 30
    print(json.dumps({"slope_us_per_step": round(slope, 2), "intercept_us": round(res[20] - 20 * slope, 1),
                      "bare_sync_us": round(res[0], 1)}), flush=True)


if __name__ == "__main__":
    main()
