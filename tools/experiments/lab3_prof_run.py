"""Profiling driver: each lab3 path once at nc=32 on 8192^2 (after warm-up)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402

dev = torch.device("cuda:0")
size, nc = 8192, int(sys.argv[1]) if len(sys.argv) > 1 else 32
img = torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev)
mu, inv = ops.class_stats(img.cpu(), class_points_for(size, size, nc, 64, seed=nc))
for path in ("direct", "fast", "mfma", "mfma64", "mfma8"):
    for _ in range(2):
        ops.classify_(img, mu, inv, path=path)
torch.cuda.synchronize()
