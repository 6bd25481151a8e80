#!/usr/bin/env python3
"""lab5 uint8 counting sort at 2^26 keys, 8 sorts (run under rocprofv3 --kernel-trace --stats)."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops
dev = torch.device("cuda:0")
src = torch.randint(0, 256, (1 << 26,), dtype=torch.uint8, device=dev)
x = torch.empty_like(src)
for _ in range(8):
    x.copy_(src)
    ops.sort_(x)
torch.cuda.synchronize()
print("ok")
