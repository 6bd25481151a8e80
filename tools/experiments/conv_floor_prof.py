#!/usr/bin/env python3
"""Rotated (HBM-honest) conv vs copy floors for PMC profiling: 6 independent
4096^2 RGBA8 input/output pairs (768 MiB, 3x the MALL), 30 launches each of
the production sobel5 conv (band kernel), the previous 8-B-lane wave kernel,
torch's copy, the 16-B strip-copy probe and the row-band copy probe.
Run under rocprofv3 --pmc (tools/gpu_r2_conv_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402

n, R, iters = 4096, 6, 30
dev = torch.device("cuda:0")
pairs = [(torch.randint(0, 256, (n, n, 4), dtype=torch.uint8, device=dev),
          torch.empty((n, n, 4), dtype=torch.uint8, device=dev)) for _ in range(R)]
L = _native.lib()
T = _native.tune_lib()  # variants / probes live in libmpx_tune.so
f = ops.get_filter("sobel5")
for k in range(iters):
    a, b = pairs[k % R]
    ops.conv(a, f, b)
torch.cuda.synchronize()
for k in range(iters):
    a, b = pairs[k % R]
    b.copy_(a)
torch.cuda.synchronize()
for k in range(iters):
    a, b = pairs[k % R]
    _native.check(T.mpx_strip_copy_probe(a.data_ptr(), b.data_ptr(), n, n, 4, 4, 24, 0))
torch.cuda.synchronize()
wx, wy = f.c_taps()
for k in range(iters):  # the 8-B-lane wave kernel, alternating segments (previous production)
    a, b = pairs[k % R]
    _native.check(T.mpx_conv_variant(a.data_ptr(), b.data_ptr(), n, n, 5, 3, 0, 2000, 1, wx, wy, 0))
torch.cuda.synchronize()
for k in range(iters):  # row-band copy, 16-row bands, alternating
    a, b = pairs[k % R]
    _native.check(T.mpx_strip_copy_probe(a.data_ptr(), b.data_ptr(), n, n, 8, 2, 16, 0))
torch.cuda.synchronize()
print("done")
