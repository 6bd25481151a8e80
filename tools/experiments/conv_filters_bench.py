#!/usr/bin/env python3
"""Rotated (HBM-honest) kernel time of every named lab2 filter through
ops.conv: 6 independent 4096^2 input/output pairs, median of 5 rounds of 20
event-timed launches. Run twice with MPX_CONV_BAND=0 / 2 for the wave-vs-band
A/B (tools/gpu_r2_conv_filters_ab.sh). One JSON line per filter."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402

FILTERS = ["roberts", "sobel3", "prewitt3", "scharr3", "laplace3", "box3", "sharpen3", "sobel5", "gauss5", "log5",
           "sobel5_dense", "gauss5_dense"]


def main():
    n, R, iters = 4096, 6, 20
    dev = torch.device("cuda:0")
    pairs = [(torch.randint(0, 256, (n, n, 4), dtype=torch.uint8, device=dev),
              torch.empty((n, n, 4), dtype=torch.uint8, device=dev)) for _ in range(R)]
    filt = {f: ops.get_filter(f) for f in FILTERS}
    res = {f: [] for f in FILTERS}
    for _ in range(5):
        for name, f in filt.items():
            for k in range(R):
                ops.conv(pairs[k][0], f, pairs[k][1])
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for k in range(iters):
                a, b = pairs[k % R]
                ops.conv(a, f, b)
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) * 1e3 / iters)
    band = os.environ.get("MPX_CONV_BAND", "2")
    for name in FILTERS:
        med = statistics.median(res[name])
        print(json.dumps({"filter": name, "band_mode": band, "us_median": round(med, 2),
                          "gpix_s": round(n * n / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
