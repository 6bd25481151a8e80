"""cuda_mpi_openmp_amd — an MI355X-native (gfx950 / CDNA4) heterogeneous
numerical-kernel suite with the capabilities of the KoryakovDmitry/cuda-mpi-openmp
coursework framework (the distribution name keeps the upstream's hyphens; the
import name uses underscores because hyphens are not valid Python identifiers).

Layers
  native/            libmpx: hand-written HIP kernels, OpenMP CPU references,
                     RCCL multi-GPU tools, lab CLIs (C/C++)
  ops/               torch-tensor entry points into libmpx (+ plain-torch oracles)
  models/            the workloads: lab1 vector op, lab2 edge/conv, lab3 classifier,
                     2-D Jacobi — single- and multi-GPU
  parallel/          one process per GPU over torch.distributed (RCCL/xGMI):
                     slab decomposition, halo exchange, collectives
  harness/           drop-in run_test.py / tester.py compatible benchmark harness
  utils/             image codec, timing, statistics
"""

__version__ = "0.1.0"

from . import ops  # noqa: E402,F401
