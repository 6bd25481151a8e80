#!/usr/bin/env python3
"""lab3 variant A/B at 8192^2: the kernels read their
variant from the environment once per process (MPX_CLS_OPT = fast32 memory
policy / layout bits, MPX_CLS_MFMA8_WIN = windowed fix-ups), so the calling
script runs this once per setting, alternating. Three rotated images (768 MiB,
beyond the MALL); every result equal to the exact DIRECT path's. One JSON line
per (nc, path); LAB3_NCS / LAB3_PATHS / LAB3_TAG narrow and label a run."""

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
    imgs = [torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev) for _ in range(3)]
    host = imgs[0].cpu()
    ncs = [int(v) for v in os.environ.get("LAB3_NCS", "2,4,8,32").split(",")]
    paths = os.environ.get("LAB3_PATHS", "fast,mfma8").split(",")
    tag = os.environ.get("LAB3_TAG", "")
    if os.environ.get("LAB3_FLOOR", "0") == "1":
        # the in-place read-modify-write floor of the same bytes: the tune
        # library's linear 16-B copy with source == destination (d = 0 plain,
        # 1 non-temporal), same rotation, same timing
        from cuda_mpi_openmp_amd import _native
        T = _native.tune_lib()
        for d in (0, 1):
            cyc = [0]

            def run_copy(d=d):
                x = imgs[cyc[0] % 3]
                _native.check(T.mpx_strip_copy_probe(x.data_ptr(), x.data_ptr(), size, size, 0, d, 0,
                                                     _native.stream_of(x)))
                cyc[0] += 1
            med, mn = time_us(run_copy)
            print(json.dumps({"tag": tag, "path": f"inplace_copy_d{d}", "us": round(med, 1), "us_min": round(mn, 1),
                              "tbps": round(2 * size * size * 4 / (med * 1e-6) / 1e12, 2)}), flush=True)
    for nc in ncs:
        pts = class_points_for(size, size, nc, 64, seed=nc)
        mu, inv = ops.class_stats(host, pts)
        ref = imgs[0].clone()
        ops.classify_(ref, mu, inv, path="direct")
        for path in paths:
            work = imgs[0].clone()
            ops.classify_(work, mu, inv, path=path)
            ok = torch.equal(work, ref)
            cyc = [0]

            def run():
                ops.classify_(imgs[cyc[0] % 3], mu, inv, path=path)
                cyc[0] += 1
            med, mn = time_us(run)
            print(json.dumps({"tag": tag, "nc": nc, "path": path, "us": round(med, 1), "us_min": round(mn, 1),
                              "same_as_direct": ok, "opt": os.environ.get("MPX_CLS_OPT", "0"),
                              "win": os.environ.get("MPX_CLS_MFMA8_WIN", "0")}), flush=True)


if __name__ == "__main__":
    main()
