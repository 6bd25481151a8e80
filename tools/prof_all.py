#!/usr/bin/env python3
"""Profiling driver: every workload's production kernels at the BASELINE sizes,
a few times each after warm-up (run under rocprofv3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402

REPS = 3


def main():
    which = sys.argv[1].split(",") if len(sys.argv) > 1 else ["lab1", "lab2", "lab3", "jacobi"]
    dev = torch.device("cuda:0")
    if "lab2" in which:
        img = torch.randint(0, 256, (4096, 4096, 4), dtype=torch.uint8, device=dev)
        out = torch.empty_like(img)
        for f in ("sobel5", "sobel5_dense", "gauss5", "roberts", "sobel3"):
            for _ in range(REPS + 1):
                ops.conv(img, f, out)
    if "lab1" in which:
        a = torch.rand(1 << 26, device=dev)
        b = torch.rand(1 << 26, device=dev)
        c = torch.empty_like(a)
        for _ in range(REPS + 1):
            ops.vsub(a, b, c)
        del a, b, c
    if "lab3" in which:
        img = torch.randint(0, 256, (8192, 8192, 4), dtype=torch.uint8, device=dev)
        mu, inv = ops.class_stats(img.cpu(), class_points_for(8192, 8192, 16, 64, seed=16))
        for path in ("direct", "fast", "mfma", "mfma64"):
            for _ in range(REPS):
                ops.classify_(img, mu, inv, path=path)
        del img
    if "jacobi" in which:
        n = 16384
        u = torch.rand((n + 2, n), dtype=torch.float64, device=dev)
        un = torch.empty_like(u)
        res = torch.zeros(1, dtype=torch.float64, device=dev)
        for _ in range(REPS + 1):
            ops.jacobi_sweep(u, un, 1, n + 1, res)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
