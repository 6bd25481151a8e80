#!/usr/bin/env python3
"""Weak-scaling benchmark of the embarrassingly parallel labs over N GPUs:
lab1 vector subtraction and lab3 Mahalanobis classification, one process per
GPU ("lab1, lab2 and lab3 across 1/2/4/8 GPUs"; lab2 is
bench.py, the Jacobi stencil tools/bench_jacobi.py).

  python tools/bench_workloads.py --workload vsub|classify [--gpus N] [--steps K] [--warmup W]

* vsub: every rank owns 2^26 fp32 elements (768 MiB of traffic per step),
  c = a - b, checked exactly on the device after the timed region.
* classify: every rank owns an 8192 x 8192 RGBA8 slab of one global image;
  16 classes from 64 random points each; class statistics all-gathered so
  every rank holds the reference's fp64 statistics; a 64-row band of every
  rank's classes is compared with the OpenMP CPU reference.

Prints one JSON line on rank 0 (whole-job throughput over the job span
max(t_end) - min(t_start) on the node's shared monotonic clock).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import ops, parallel  # noqa: E402
from cuda_mpi_openmp_amd.parallel.timing import aligned_start, clock_ns, gather_span, start_delay  # noqa: E402
from cuda_mpi_openmp_amd.models import ShardedVectorSub, SlabPixelClassifier  # noqa: E402
from cuda_mpi_openmp_amd.models.classifier import class_points_for  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["vsub", "classify"], required=True)
    p.add_argument("--gpus", type=int, default=None)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--elems", type=int, default=1 << 26, help="vsub elements per rank")
    p.add_argument("--size", type=int, default=8192, help="classify slab side per rank")
    p.add_argument("--classes", type=int, default=16)
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    a = p.parse_args()
    from cuda_mpi_openmp_amd.parallel import launch

    if a.gpus is not None:
        rc = launch.relaunch_if_needed(os.path.abspath(__file__), sys.argv[1:], a.gpus, a.device)
        if rc is not None:
            return rc
    ctx = parallel.init(device=a.device)
    if a.gpus is not None:
        launch.check_world(a.gpus, ctx.world)
    n_ranks = ctx.world
    sync = (lambda: torch.cuda.synchronize(ctx.device)) if ctx.device.type == "cuda" else (lambda: None)

    if a.workload == "vsub":
        m = ShardedVectorSub(ctx, a.elems * n_ranks, dtype=torch.float32)
        m.fill_random(seed=3)
        step = m.step
        bytes_per_step = 3 * 4 * m.slab.rows
    else:
        h = a.size * n_ranks
        clf = SlabPixelClassifier(ctx, h, a.size, path="auto")
        g = torch.Generator(device="cpu").manual_seed(11 + ctx.rank)
        clf.img.copy_(torch.randint(0, 256, clf.img.shape, dtype=torch.uint8, generator=g))
        clf.fit(class_points_for(h, a.size, a.classes, 64, seed=5))
        orig = clf.img.clone()
        step = clf.classify

    for _ in range(a.warmup):
        step()
    sync()
    ctx.barrier()
    aligned_start(ctx)  # every rank leaves at one agreed instant of the shared clock
    start_delay(ctx.rank)  # MPX_BENCH_START_DELAY test hook
    t0 = clock_ns()
    for _ in range(a.steps):
        step()
    sync()
    t1 = clock_ns()  # this rank's end; the job span is max(t1) - min(t0) (bench.py timed())
    ctx.barrier()
    span = gather_span(t0, t1, ctx)
    el = span.job_s

    if a.workload == "vsub":
        ok = bool(torch.equal(m.c, m.a - m.b))
        value, unit = n_ranks * bytes_per_step * a.steps / el / 1e12, "TB/s"
        extra = {"n_per_gpu": m.slab.rows, "dtype": "fp32"}
    else:
        band = slice(0, min(64, clf.slab.rows))
        ref = orig[band].cpu().clone()
        ops.classify_(ref, clf.mu, clf.inv)
        ok = bool(torch.equal(clf.img[band].cpu(), ref))
        value, unit = n_ranks * a.size * a.size * a.steps / el / 1e9, "Gpixel/s"
        extra = {"slab": [a.size, a.size], "classes": a.classes, "path": "auto"}
    ok = parallel.max_over_ranks(0.0 if ok else 1.0, ctx) == 0.0
    if ctx.rank == 0:
        print(json.dumps({"workload": a.workload, "n_gpus": n_ranks, "steps": a.steps, "warmup": a.warmup,
                          "value": float(f"{value:.6g}"), "unit": unit, "ms_per_step": round(el * 1e3 / a.steps, 5),
                          **span.fields(a.steps), "scaling": "weak",
                          "verified": ok, **extra}), flush=True)
    parallel.shutdown()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
