#!/usr/bin/env python3
"""Row-pitch probe for the lab2 band kernel (HBM channel spread).

The band kernel's waves sit on row bands 16 rows apart, so with a 16 KiB row
pitch their concurrent row addresses are 256 KiB apart and share their low
address bits. This times the production sobel5 launch (``mpx_conv``) over
rotated 4096^2 pairs whose rows are padded to ``pitch = 4096 + pad`` pixels,
to see whether breaking that alignment spreads the traffic over more HBM
channels. Outputs are checked against the contiguous launch.

  python tools/experiments/pitch_probe.py [--pads 0,16,32,64,128,256] [--rotate 6] [--rounds 7]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--pads", default="0,16,32,64,128,256")
    p.add_argument("--rotate", type=int, default=6)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--filter", default="sobel5")
    args = p.parse_args()
    L = _native.lib()
    dev = torch.device("cuda:0")
    n = args.size
    f = ops.get_filter(args.filter)
    wx, wy = f.c_taps()
    pads = [int(x) for x in args.pads.split(",")]
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randint(0, 256, (n, n, 4), dtype=torch.uint8, device=dev, generator=g)
    ref = ops.conv(base, f)
    sets = {}
    for pad in pads:
        pitch = n + pad
        pairs = []
        for _ in range(args.rotate):
            a = torch.empty((n, pitch, 4), dtype=torch.uint8, device=dev)
            a[:, :n] = base
            pairs.append((a, torch.zeros_like(a)))
        sets[pad] = (pitch, pairs)

    def launch(pad, k):
        pitch, pairs = sets[pad]
        a, o = pairs[k % len(pairs)]
        _native.check(L.mpx_conv(a.data_ptr(), o.data_ptr(), n, pitch, 0, n, 0, n - 1, f.k, f.anchor, f.mode,
                                 wx, wy, _native.stream_of(a)))

    for pad in pads:
        launch(pad, 0)
        torch.cuda.synchronize()
        ok = torch.equal(sets[pad][1][0][1][:, :n], ref)  # (pitch, pairs)[1][pair 0][output]
        print(json.dumps({"pad": pad, "bit_exact": bool(ok)}), flush=True)
    times = {pad: [] for pad in pads}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.rounds):
        for pad in pads:
            launch(pad, 0)
            torch.cuda.synchronize()
            s.record()
            for k in range(args.iters):
                launch(pad, k + 1)
            e.record()
            e.synchronize()
            times[pad].append(s.elapsed_time(e) * 1e3 / args.iters)
    for pad in pads:
        ts = times[pad]
        med = statistics.median(ts)
        print(json.dumps({"filter": args.filter, "pad_px": pad, "pitch_bytes": (n + pad) * 4, "us_median": round(med, 2),
                          "us_min": round(min(ts), 2), "Gpix_s": round(n * n / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
