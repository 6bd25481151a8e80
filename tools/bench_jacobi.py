#!/usr/bin/env python3
"""BASELINE north star 5: 2-D Jacobi on a 16384^2 fp64 grid, row-slab
decomposed over N GPUs (strong scaling), halos over RCCL (native tier when
available), residual all-reduce every --check-every iterations.

  python tools/bench_jacobi.py [--size 16384] [--iters 100] [--warmup 10]
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_jacobi.py
  python tools/bench_jacobi.py --gpus 8      (launches the 8 ranks itself)

Prints one JSON line on rank 0 (max time over ranks).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import parallel  # noqa: E402
from cuda_mpi_openmp_amd.models import SlabJacobi  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=16384)
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--check-every", type=int, default=10)
    p.add_argument("--fp32", action="store_true")
    p.add_argument("--overlap", choices=["auto", "on", "off"], default="auto")
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    p.add_argument("--graph", action="store_true", help="replay HIP graphs of whole residual cycles")
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks to run (self-launched when no torchrun environment); default WORLD_SIZE or 1")
    a = p.parse_args()
    from cuda_mpi_openmp_amd.parallel import launch

    if a.gpus is not None:
        rc = launch.relaunch_if_needed(os.path.abspath(__file__), sys.argv[1:], a.gpus, a.device)
        if rc is not None:
            return rc
    ctx = parallel.init(device=a.device)
    if a.gpus is not None:
        launch.check_world(a.gpus, ctx.world)
    dt = torch.float32 if a.fp32 else torch.float64
    sol = SlabJacobi(ctx, a.size, a.size, dtype=dt, check_every=a.check_every,
                     overlap={"auto": "auto", "on": True, "off": False}[a.overlap])
    sol.set_boundary(top=1.0)
    sol.fill(seed=0)
    sync = (lambda: torch.cuda.synchronize(ctx.device)) if ctx.device.type == "cuda" else (lambda: None)
    sol.run(a.warmup, graph=a.graph)
    sync()
    ctx.barrier()
    t0 = time.perf_counter()
    sol.run(a.iters, graph=a.graph)
    sync()
    ctx.barrier()
    el = parallel.max_over_ranks(time.perf_counter() - t0, ctx)
    if ctx.rank == 0:
        ms = el * 1e3 / a.iters
        es = 4 if a.fp32 else 8
        print(json.dumps({
            "metric": "2-D Jacobi iteration time, 16384^2 grid domain-decomposed over N MI355X",
            "value": round(ms, 5), "unit": "ms/iteration", "higher_is_better": False, "scaling": "strong",
            "n_gpus": ctx.world, "iters": a.iters, "warmup": a.warmup, "grid": [a.size, a.size],
            "dtype": "fp32" if a.fp32 else "fp64", "check_every": a.check_every,
            "gpoints_per_s": round(a.size * a.size / (ms * 1e-3) / 1e9, 3),
            "TBps_aggregate": round(2 * a.size * a.size * es / (ms * 1e-3) / 1e12, 3),
            "residual": sol.last_residual,
            "transport": ("native-rccl" if ctx.native is not None else "torch.distributed") if ctx.world > 1 else None,
            "halo": ("overlap" if sol.overlap else "inorder") if ctx.world > 1 else None,
            "hip_graph": bool(a.graph and ctx.device.type == "cuda")}), flush=True)
    parallel.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
