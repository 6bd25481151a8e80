#!/usr/bin/env python3
"""Warm kernel time of the harness's thin launch geometries (lab1 [grid, block]
at n = 10^6 fp64, lab2 Roberts [[bx, by], [gx, gy]] on a 1266x709 image), each
checked against the CPU reference. One JSON line per configuration."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402


def t_us(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda:0")
    a = torch.rand(10**6, dtype=torch.float64, device=dev)
    b = torch.rand(10**6, dtype=torch.float64, device=dev)
    c = torch.empty_like(a)
    for g in ((1, 32), (4, 64), (32, 128), (512, 512), (1024, 1024), (0, 0)):
        us = t_us(lambda g=g: ops.vsub(a, b, c, grid=g[0], block=g[1]))
        ok = torch.equal(c, a - b)
        print(json.dumps({"lab": 1, "n": 10**6, "geometry": list(g), "us": round(us, 2), "verified": ok}), flush=True)
    for hw in ((709, 1266), (640, 1024)):
        lab2(dev, hw)


def lab2(dev, hw):
    img = torch.randint(0, 256, (*hw, 4), dtype=torch.uint8)
    ref = ops.roberts(img)
    d = img.to(dev)
    o = torch.empty_like(d)
    for geo in (((2, 2), (16, 16)), ((16, 16), (32, 32)), ((32, 32), (16, 16)), ((32, 32), (64, 64)),
                ((16, 16), (1024, 1024)), None):
        us = t_us(lambda geo=geo: ops.roberts(d, o, geometry=geo))
        ok = torch.equal(o.cpu(), ref)
        print(json.dumps({"lab": 2, "hw": list(hw), "geometry": geo, "us": round(us, 2), "verified": ok}), flush=True)


if __name__ == "__main__":
    main()
