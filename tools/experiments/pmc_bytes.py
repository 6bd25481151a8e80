#!/usr/bin/env python3
"""Kernels with known HBM traffic, for reconciling the L2->memory request
counters with bytes (run under rocprofv3 --pmc, one pass per
counter group):

  * vsub fp32, 2^26 elements: reads 512 MiB, writes 256 MiB (streaming, no reuse);
  * copy of 768 MiB (torch) for a second calibration point;
  * the bench's sobel5 4096^2 conv over 6 rotated slab pairs (64 MiB read +
    64 MiB written per dispatch; the halo rows a neighbouring segment also
    reads are the only possible re-fetch).

Each kernel runs REPS times after a warm-up; tools/pmc_median.py takes
the per-kernel medians; profiles/lab2_conv.md turns them into bytes.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402

REPS = 3
dev = torch.device("cuda:0")
n = 1 << 26
a = torch.rand(n, device=dev)
b = torch.rand(n, device=dev)
c = torch.empty_like(a)
src = torch.empty(3 * n, dtype=torch.float32, device=dev)
dst = torch.empty_like(src)
imgs = [torch.randint(0, 256, (4096, 4096, 4), dtype=torch.uint8, device=dev) for _ in range(6)]
outs = [torch.empty_like(x) for x in imgs]
for _ in range(2):  # warm-up: code objects, first touch
    ops.vsub(a, b, c)
    dst.copy_(src)
    for x, o in zip(imgs, outs):
        ops.conv(x, "sobel5", o)
torch.cuda.synchronize()
for _ in range(REPS):
    ops.vsub(a, b, c)
    torch.cuda.synchronize()
    dst.copy_(src)
    torch.cuda.synchronize()
    for x, o in zip(imgs, outs):
        ops.conv(x, "sobel5", o)
    torch.cuda.synchronize()
print("pmc_bytes done")
