#!/usr/bin/env python3
"""Profiling driver: every workload's production kernels at the BASELINE sizes,
a few times each after warm-up (run under rocprofv3). lab2 cycles 6
independent 4096^2 input/output pairs (768 MiB, 3x the MALL) so the counters
describe HBM streaming, as bench.py does."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402

REPS = 3


def main():
    which = sys.argv[1].split(",") if len(sys.argv) > 1 else ["lab1", "lab2", "lab3", "jacobi", "lab5"]
    dev = torch.device("cuda:0")
    if "lab2" in which:
        pairs = [(torch.randint(0, 256, (4096, 4096, 4), dtype=torch.uint8, device=dev),
                  torch.empty((4096, 4096, 4), dtype=torch.uint8, device=dev)) for _ in range(6)]
        for f in ("sobel5", "sobel5_dense", "gauss5", "roberts", "sobel3"):
            for k in range(REPS + 6):
                img, out = pairs[k % 6]
                ops.conv(img, f, out)
        # the LDS-tiled variant (conv_band16v_kernel: vertical halo rows shared
        # through LDS; band mode 4, not the default) for its LDS counters
        from cuda_mpi_openmp_amd import _native
        L = _native.lib()
        prev = L.mpx_conv_set_band_mode(4)
        for k in range(REPS + 6):
            img, out = pairs[k % 6]
            ops.conv(img, "sobel5", out)
        torch.cuda.synchronize()
        L.mpx_conv_set_band_mode(prev)
        del pairs
    if "lab1" in which:
        a = torch.rand(1 << 26, device=dev)
        b = torch.rand(1 << 26, device=dev)
        c = torch.empty_like(a)
        for _ in range(REPS + 1):
            ops.vsub(a, b, c)
        del a, b, c
    if "lab3" in which:
        img = torch.randint(0, 256, (8192, 8192, 4), dtype=torch.uint8, device=dev)
        for nc, paths in ((4, ("fast", "mfma8", "mfma16")), (16, ("direct", "fast", "mfma8", "mfma16")),
                          (32, ("fast", "mfma8", "mfma16"))):
            mu, inv = ops.class_stats(img.cpu(), class_points_for(8192, 8192, nc, 64, seed=nc))
            for path in paths:
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
    if "lab5" in which:
        for dt in (torch.int32, torch.float32):
            src = (torch.randint(-2**31, 2**31 - 1, (1 << 26,), dtype=torch.int32, device=dev) if dt == torch.int32
                   else torch.randn(1 << 26, device=dev))
            x = torch.empty_like(src)
            for _ in range(REPS + 1):
                x.copy_(src)
                ops.sort_(x)
        del src, x
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
