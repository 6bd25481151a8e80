"""Compile-time vs runtime taps for the named filters (lab2, 4096^2).

Each named filter runs twice: by name (edgel::launch_named / launch_sep match
its taps and pick the compile-time tap class: zero taps dropped, +-1 folded)
and as a custom filter whose zero taps are -0.0 (same operator, but the bit
patterns no longer match, so the runtime-tap kernel runs). Both outputs are
checked against the native CPU reference.
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from cuda_mpi_openmp_amd import ops  # noqa: E402


def gpu_time_us(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def negzero(t):
    return tuple(-0.0 if v == 0.0 else v for v in t)


def main():
    dev = torch.device("cuda:0")
    size = 4096
    img = torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev)
    host = img.cpu()
    out = torch.empty_like(img)
    for name in ("roberts", "sobel3", "prewitt3", "scharr3", "laplace3", "sharpen3", "sobel5_dense", "log5", "sobel5", "gauss5"):
        f = ops.get_filter(name)
        rt = ops.Filter(name + "_rt", f.k, f.anchor, f.mode, negzero(f.wx), negzero(f.wy))
        ref = ops.conv(host, f)
        row = {"filter": name, "hw": [size, size]}
        for tag, filt in (("const", f), ("runtime", rt)):
            us = gpu_time_us(lambda: ops.conv(img, filt, out))
            row[tag + "_us"] = round(us, 2)
            row[tag + "_verified"] = bool(torch.equal(out.cpu(), ref))
        row["speedup"] = round(row["runtime_us"] / row["const_us"], 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
