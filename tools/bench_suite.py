#!/usr/bin/env python3
"""Single-GPU benchmark of every workload at the BASELINE.json configurations,
each checked against its CPU reference, with the OpenMP CPU time for the
GPU/CPU speedup. Prints one JSON line per measurement.

  lab1  vsub fp32 N = 2^26 and fp64 N = 2^25        (HBM streaming)
  lab2  sobel5 / roberts / sobel3 on 4096^2 RGBA8    (see bench.py for the flagship)
  lab3  Mahalanobis classifier 8192^2, nc = 4/16/32, direct vs fp64-MFMA path
  lab5  sort 2^26 keys: int32 / float32 radix, uint8 counting sort, vs torch.sort
  jacobi 2-D 5-point sweep, 16384^2 fp64 and fp32 (one GPU's share of the
         8-GPU north-star grid is 2048 x 16384; the full grid is timed here)
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402


def gpu_time_us(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    return float(np.median(ts))


def cpu_time_ms(fn, reps=1):
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    return best


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_lab1(dev):
    for dtype, n in ((torch.float32, 1 << 26), (torch.float64, 1 << 25)):
        a = torch.rand(n, dtype=dtype, device=dev)
        b = torch.rand(n, dtype=dtype, device=dev)
        c = torch.empty_like(a)
        us = gpu_time_us(lambda: ops.vsub(a, b, c))
        ok = torch.equal(c, a - b)
        ac, bc = a.cpu(), b.cpu()
        cc = torch.empty_like(ac)
        cpu = cpu_time_ms(lambda: ops.vsub(ac, bc, cc), reps=2)
        byts = 3 * n * a.element_size()
        emit(workload="lab1_vsub", dtype=str(dtype).split(".")[-1], n=n, us=round(us, 2),
             TBps=round(byts / us / 1e6, 3), cpu_omp_ms=round(cpu, 3), speedup_vs_cpu=round(cpu * 1e3 / us, 1),
             verified=ok)
        # reference launch geometry [512, 512] for comparison
        us_ref = gpu_time_us(lambda: ops.vsub(a, b, c, grid=512, block=512))
        emit(workload="lab1_vsub", dtype=str(dtype).split(".")[-1], n=n, geometry=[512, 512], us=round(us_ref, 2),
             TBps=round(byts / us_ref / 1e6, 3))
        del a, b, c


def bench_lab2(dev, size=4096):
    img = torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev)
    out = torch.empty_like(img)
    host = img.cpu()
    for f in ("sobel5", "sobel5_dense", "roberts", "sobel3", "gauss5", "gauss5_dense"):
        us = gpu_time_us(lambda: ops.conv(img, f, out))
        ok = torch.equal(out.cpu(), ops.conv(host, f))
        cpu = cpu_time_ms(lambda: ops.conv(host, f))
        emit(workload="lab2_conv", filter=f, hw=[size, size], us=round(us, 2),
             gpix_s=round(size * size / us / 1e3, 1), TBps=round(2 * img.numel() / us / 1e6, 3),
             cpu_omp_ms=round(cpu, 3), speedup_vs_cpu=round(cpu * 1e3 / us, 1), verified=ok)


def bench_lab3(dev, size=8192):
    img = torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev)
    host = img.cpu()
    # LAB3_NCS / LAB3_PATHS narrow a sweep (e.g. the AUTO threshold: LAB3_NCS=8,12,16,20,24 LAB3_PATHS=fast,mfma8)
    ncs = [int(v) for v in os.environ.get("LAB3_NCS", "4,16,32").split(",")]
    paths = os.environ.get("LAB3_PATHS", "direct,fast,mfma,mfma64,mfma8,auto").split(",")
    for nc in ncs:
        pts = class_points_for(size, size, nc, 64, seed=nc)
        mu, inv = ops.class_stats(host, pts)
        ref = host.clone()
        cpu = cpu_time_ms(lambda: ops.classify_(ref, mu, inv))
        for path in paths:
            work = img.clone()
            amb = torch.zeros(1, dtype=torch.int32, device=dev)
            ops.classify_(work, mu, inv, path=path, ambiguous=amb)
            ok = torch.equal(work.cpu(), ref)
            us = gpu_time_us(lambda: ops.classify_(work, mu, inv, path=path), iters=5, warmup=1)
            emit(workload="lab3_classify", path=path, ran=ops.classify_plan(mu, inv, path)[0], nc=nc,
                 hw=[size, size], us=round(us, 1), gpix_s=round(size * size / us / 1e3, 2),
                 cpu_omp_ms=round(cpu, 2), speedup_vs_cpu=round(cpu * 1e3 / us, 1), verified=ok,
                 fallback_pixels=int(amb.item()))
            del work


def bench_jacobi(dev, n=16384):
    for dtype in (torch.float64, torch.float32):
        u = torch.rand((n + 2, n), dtype=dtype, device=dev)
        un = torch.empty_like(u)
        res = torch.zeros(1, dtype=dtype, device=dev)
        us = gpu_time_us(lambda: ops.jacobi_sweep(u, un, 1, n + 1, res), iters=10)
        byts = 2 * n * n * u.element_size()
        ok = None
        if dtype == torch.float64:
            m = 2048  # CPU check on a slice
            uc = u[: m + 2].cpu().contiguous()
            unc = torch.zeros_like(uc)
            ops.jacobi_sweep(uc, unc, 1, m + 1)
            ok = torch.equal(un[1:m + 1].cpu(), unc[1:m + 1])
            cpu = cpu_time_ms(lambda: ops.jacobi_sweep(uc, unc, 1, m + 1)) * (n / m)
        emit(workload="jacobi_sweep", dtype=str(dtype).split(".")[-1], grid=[n, n], us=round(us, 1),
             TBps=round(byts / us / 1e6, 3), gpts_s=round(n * n / us / 1e3, 1), verified=ok,
             **({"cpu_omp_ms_est": round(cpu, 1), "speedup_vs_cpu": round(cpu * 1e3 / us, 1)} if ok is not None else {}))
        del u, un


def bench_lab5(dev):
    """lab5 sort at 2^26 keys: int32 / float32 (LSD radix) and uint8 (counting
    sort) vs torch.sort on the same data; each timed sort starts from the same
    unsorted copy (the copy is outside the events), median of 10."""
    n = 1 << 26
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    srcs = {torch.int32: torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev, generator=g),
            torch.float32: torch.randn(n, device=dev, generator=g),
            torch.uint8: torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)}
    for dt, x0 in srcs.items():
        x = torch.empty_like(x0)

        def timed(fn):
            ts = []
            for it in range(12):
                x.copy_(x0)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                e.synchronize()
                if it >= 2:
                    ts.append(s.elapsed_time(e) * 1e3)
            return float(np.median(ts))
        us = timed(lambda: ops.sort_(x))
        ok = bool(torch.equal(x, torch.sort(x0).values))
        ref = timed(lambda: torch.sort(x))
        emit(workload="lab5_sort", dtype=str(dt).replace("torch.", ""), n=n, us=round(us, 1),
             Gkeys_s=round(n / us / 1e3, 1), torch_sort_us=round(ref, 1), vs_torch_sort=round(ref / us, 2),
             equal_to_torch_sort=ok)
        del x


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default="lab1,lab2,lab3,lab5,jacobi")
    a = p.parse_args()
    dev = torch.device("cuda:0")
    which = a.only.split(",")
    if "lab1" in which:
        bench_lab1(dev)
    if "lab2" in which:
        bench_lab2(dev)
    if "lab3" in which:
        bench_lab3(dev)
    if "lab5" in which:
        bench_lab5(dev)
    if "jacobi" in which:
        bench_jacobi(dev)


if __name__ == "__main__":
    main()
