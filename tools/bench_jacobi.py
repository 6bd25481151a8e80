#!/usr/bin/env python3
"""BASELINE north star 5: 2-D Jacobi on a 16384^2 fp64 grid, row-slab
decomposed over N GPUs (strong scaling), residual all-reduce every
--check-every iterations. Halos (--halo): one-sided device-signalled xGMI
reads of the neighbours' buffers (peer, default when the IPC links map) or
RCCL send/recv (native tier when available).

One-GPU rehearsal of N ranks (peer halos, gloo control plane):
  MPX_DIST_BACKEND=gloo python tools/bench_jacobi.py --gpus 4

  python tools/bench_jacobi.py [--size 16384] [--iters 100] [--warmup 10]
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_jacobi.py
  python tools/bench_jacobi.py --gpus 8      (launches the 8 ranks itself)

Prints one JSON line on rank 0 (max time over ranks). With N > 1 ranks the
final field is gathered and compared bit for bit with ONE device running the
same warmup + iters iterations from the same initial field ("verified",
VERDICT r2 #3); a mismatch exits 3.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd.parallel.timing import aligned_start, clock_ns, gather_span, start_delay  # noqa: E402
from cuda_mpi_openmp_amd import parallel  # noqa: E402
from cuda_mpi_openmp_amd.models import SlabJacobi  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=16384)
    p.add_argument("--rows", type=int, default=None, help="global rows (default --size: a square grid)")
    p.add_argument("--iters", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--check-every", type=int, default=10)
    p.add_argument("--fp32", action="store_true")
    p.add_argument("--overlap", choices=["auto", "on", "off"], default="auto")
    p.add_argument("--halo", choices=["auto", "peer", "rccl", "none"], default="auto",
                   help="none = ablation without any halo exchange (wrong answer; isolates the exchange cost)")
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    p.add_argument("--graph", action="store_true", help="replay HIP graphs of whole residual cycles")
    p.add_argument("--progress", action="store_true", help="per-phase and per-check timing on stderr")
    p.add_argument("--no-verify", action="store_true", help="skip the N-rank == one-device comparison")
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
    rows = a.rows or a.size
    sol = SlabJacobi(ctx, rows, a.size, dtype=dt, check_every=a.check_every,
                     overlap={"auto": "auto", "on": True, "off": False}[a.overlap], halo=a.halo)
    def say(msg):
        if a.progress:
            print(f"[jacobi r{ctx.rank} {time.perf_counter() - t_start:8.3f}s] {msg}", file=sys.stderr, flush=True)

    t_start = time.perf_counter()
    say(f"solver ready, transport {sol.transport}")
    sol.set_boundary(top=1.0)
    sol.fill(seed=0)
    say("filled")
    sync = (lambda: torch.cuda.synchronize(ctx.device)) if ctx.device.type == "cuda" else (lambda: None)
    if a.progress:
        for k in range(a.warmup):
            r = sol.step()
            sync()
            say(f"warmup step {k} residual {r}")
    else:
        sol.run(a.warmup, graph=a.graph)
    sync()
    ctx.barrier()
    aligned_start(ctx)  # every rank leaves at one agreed instant of the shared clock
    start_delay(ctx.rank)  # MPX_BENCH_START_DELAY test hook
    t0 = clock_ns()
    sol.run(a.iters, graph=a.graph)
    sync()
    t1 = clock_ns()  # this rank's end; the job span is max(t1) - min(t0) (bench.py timed())
    ctx.barrier()
    sol.check_peer()
    span = gather_span(t0, t1, ctx)  # collective: every rank
    el = span.job_s
    verified = None
    if ctx.world > 1 and not a.no_verify and a.halo != "none":  # the ablation is wrong by design
        got = sol.gather()
        if ctx.rank == 0:
            verified = one_device_equal(got, sol, rows, a, dt, ctx)
        verified = parallel.broadcast_object(verified, ctx)
    if ctx.rank == 0:
        ms = el * 1e3 / a.iters
        es = 4 if a.fp32 else 8
        print(json.dumps({
            "metric": "2-D Jacobi iteration time, 16384^2 grid domain-decomposed over N MI355X",
            "value": round(ms, 5), "unit": "ms/iteration", "higher_is_better": False, "scaling": "strong",
            "n_gpus": ctx.world, "iters": a.iters, "warmup": a.warmup, "grid": [rows, a.size],
            "dtype": "fp32" if a.fp32 else "fp64", "check_every": a.check_every,
            "gpoints_per_s": round(rows * a.size / (ms * 1e-3) / 1e9, 3),
            "TBps_aggregate": round(2 * rows * a.size * es / (ms * 1e-3) / 1e12, 3),
            "residual": sol.last_residual,
            "transport": sol.transport,
            "halo": ("one-launch" if sol.peer is not None else "overlap" if sol.overlap else "inorder")
            if ctx.world > 1 else None,
            **span.fields(a.iters),
            "hip_graph": bool(a.graph and ctx.device.type == "cuda"),
            "peer_probe": ("ok" if sol.peer is not None else "fallback")
            if ctx.world > 1 and a.halo in ("auto", "peer") and ctx.device.type == "cuda" else None,
            "verified": verified,
            "verified_what": "gathered N-rank field == one-device run of the same iterations (bit-exact)"
            if verified is not None else None}), flush=True)
    sol.close()
    parallel.shutdown()
    return 3 if verified is False else 0


def one_device_equal(got, sol, rows, a, dt, ctx) -> bool:
    """Rank 0: rebuild every rank's initial field (SlabJacobi.fill(seed=0) draws
    rank r's rows from seed 7919 * r), run warmup + iters iterations on this
    device alone, compare with the gathered N-rank field."""
    from cuda_mpi_openmp_amd.parallel.slab import Slab

    ref = SlabJacobi(parallel.DistContext(device=ctx.device), rows, a.size, dtype=dt, check_every=a.check_every)
    ref.set_boundary(top=1.0)
    parts = []
    for r in range(ctx.world):
        sr = Slab(rows, ctx.world, r, 1, 1)
        g = torch.Generator(device="cpu").manual_seed(0 + 7919 * r)
        parts.append(torch.rand((sr.rows, a.size - 2), generator=g, dtype=torch.float64))
    ref.u[1:1 + rows, 1:-1] = torch.cat(parts).to(ref.u.device).to(dt)
    ref.un.copy_(ref.u)
    ref.run(a.warmup + a.iters)
    same = bool(torch.equal(got.to(ref.u.device), ref.owned))
    del ref
    return same


if __name__ == "__main__":
    sys.exit(main())
