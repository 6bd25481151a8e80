#!/usr/bin/env python3
"""Scaling driver: 1/2/4/8-GPU curves of every multi-GPU workload, one command.

  python tools/scale.py [--gpus 1,2,4,8] [--out scaling] [--rehearse] [--device cpu] [--quick]

For each N it runs, each as its own launched job (one process per GPU, the
same commands a user would type):

  * conv (weak scaling, the flagship): ``bench.py --gpus N`` with one-sided
    peer halos and with RCCL halos — every rank owns a 4096^2 slab;
  * conv/strong: ``bench.py --gpus N --layout strong`` — one 4096^2 frame
    split into N row slabs (strong scaling, t_1 / (N t_N));
  * Jacobi 16384^2 fp64 (strong scaling): ``tools/bench_jacobi.py --gpus N``
    with device-signalled peer halos and with RCCL halos;
  * the native one-process runtime: ``bin/mpx_mgpu conv|jacobi --gpus N``;
  * lab1 vector subtraction and lab3 classification (weak scaling, 2^26 fp32
    elements / one 8192^2 slab per rank): ``tools/bench_workloads.py``.

and writes ``<out>/scaling.json`` (one record per run: N, value, ms/step,
efficiency vs N = 1, transport, world size the job saw), ``scaling.csv`` and
``scaling.png`` (weak-scaling throughput and strong-scaling speedup against
the ideal lines). Efficiency: weak = value_N / (N * value_1); strong =
t_1 / (N * t_N); every rate comes from the job span max(t_end) - min(t_start)
(parallel/timing.py), and ``efficiency_max_rank`` shows the same ratio on the
slowest rank's own span. ``conv/driver`` is the round-end driver's exact
``bench.py --gpus N --steps K --warmup W``, so its N = 1 point equals BENCH. Runs that cannot execute here (fewer devices than N, RCCL
with several ranks on one GPU) are recorded as skipped with the reason.

``--rehearse``: several ranks share the GPUs (gloo control plane, peer halos
only; the native runtime in ``--shared`` mode up to 4 ranks) — the N = 8
code paths on a one-GPU box. ``--device cpu``: gloo on the CPU with small
problems (CI dry run). The reference has no multi-GPU code and no scaling
plot (its only plot: /root/reference/tester.py:325-407, the per-run median
bar chart); SURVEY §5 and §7.2 step 7 ask for this one.
"""

from __future__ import annotations

import argparse
import csv
import json
import os
import subprocess
import sys
import time
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def visible_gpus() -> int:
    try:
        import torch

        return int(torch.cuda.device_count())  # counts devices without creating a HIP context
    except Exception:  # noqa: BLE001
        return 0


def last_json(text: str) -> Optional[dict]:
    for line in reversed(text.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                continue
    return None


def run_job(cmd: List[str], env: Dict[str, str], timeout: float, log) -> dict:
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"status": "timeout", "wall_s": round(time.perf_counter() - t0, 1)}
    log.write(f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr[-4000:]}\n")
    log.flush()
    rec = last_json(r.stdout)
    if r.returncode != 0 or rec is None:
        return {"status": f"failed rc={r.returncode}", "stderr_tail": r.stderr[-800:],
                "wall_s": round(time.perf_counter() - t0, 1)}
    return {"status": "ok", "record": rec, "wall_s": round(time.perf_counter() - t0, 1)}


def plan(n: int, a, ndev: int) -> List[dict]:
    """The jobs of one rank count: name, kind (weak/strong), command, skip reason."""
    py = sys.executable
    cpu = a.device == "cpu"
    shared = a.rehearse or cpu
    conv_sz = ["--size", "128", "--steps", "3", "--warmup", "1", "--rotate", "2"] if cpu else (
        ["--steps", "20", "--warmup", "5"] if a.quick else ["--steps", "50", "--warmup", "10"])
    jac_sz = ["--size", "256", "--iters", "10", "--warmup", "2"] if cpu else (
        ["--iters", "50", "--warmup", "10"] if a.quick else ["--iters", "200", "--warmup", "20"])
    dev = ["--device", "cpu"] if cpu else []
    jobs = []
    lacks = None if shared or n <= ndev else f"needs {n} GPUs, {ndev} visible"
    # the driver's own command (BENCH at N = 1, SCALE at every N): bench.py with
    # exactly --gpus N --steps K --warmup W, so this curve's N = 1 point is the
    # BENCH number (VERDICT r4 Next #1)
    drv = [py, "bench.py", "--gpus", str(n), "--steps", str(a.driver_steps), "--warmup", str(a.driver_warmup)]
    if not cpu:
        assert drv[1:] == driver_command(n, a.driver_steps, a.driver_warmup), drv
    jobs.append({"name": "conv/driver", "kind": "weak", "skip": lacks,
                 "cmd": drv + (dev + ["--size", "128", "--rotate", "2"] if cpu else [])})
    # strong scaling of the flagship (VERDICT r5 Next #2): ONE 4096^2 frame split
    # into N row slabs (512 rows per rank at N = 8), the driver's K / W, halos
    # by the default transport; efficiency t_1 / (N t_N)
    jobs.append({"name": "conv/strong", "kind": "strong", "skip": lacks,
                 "cmd": [py, "bench.py", "--gpus", str(n), "--layout", "strong", "--steps", str(a.driver_steps),
                         "--warmup", str(a.driver_warmup), "--no-cpu-baseline"]
                 + (dev + ["--size", "128", "--rotate", "2"] if cpu else [])})
    for halo in ("peer", "rccl"):
        skip = lacks
        if n > 1 and halo == "rccl" and a.rehearse and not cpu and not a.contract:
            skip = "RCCL refuses several ranks on one GPU (rehearsal uses peer halos)"
        if n == 1 and halo == "rccl":
            skip = "single rank: no halo transport"
        if cpu and halo == "peer" and n > 1:  # (also under --contract)
            skip = "peer halos need GPUs (IPC); the CPU run uses gloo send/recv"
        jobs.append({"name": f"conv/{halo}", "kind": "weak", "skip": skip,
                     "cmd": [py, "bench.py", "--gpus", str(n), "--halo", halo, "--no-cpu-baseline", *dev, *conv_sz]})
        jobs.append({"name": f"jacobi/{halo}", "kind": "strong",
                     "skip": skip,
                     "cmd": [py, "tools/bench_jacobi.py", "--gpus", str(n), "--halo", halo, *dev, *jac_sz]})
    for wl in ("vsub", "classify"):
        sz = (["--elems", "65536"] if wl == "vsub" else ["--size", "96"]) if cpu else []
        st = ["--steps", "3", "--warmup", "1"] if cpu else (
            ["--steps", "20", "--warmup", "3"] if a.quick else ["--steps", "100", "--warmup", "10"])
        jobs.append({"name": f"lab{1 if wl == 'vsub' else 3}/{wl}", "kind": "weak", "skip": lacks,
                     "cmd": [py, "tools/bench_workloads.py", "--workload", wl, "--gpus", str(n), *dev, *sz, *st]})
    mg = os.path.join(ROOT, "bin", "mpx_mgpu")
    if cpu:
        jobs.append({"name": "mgpu/conv", "kind": "weak", "skip": "native runtime needs GPUs", "cmd": []})
        jobs.append({"name": "mgpu/jacobi-peer", "kind": "strong", "skip": "native runtime needs GPUs", "cmd": []})
    else:
        steps = ["--steps", "20", "--warmup", "5"] if a.quick else ["--steps", "50", "--warmup", "10"]
        jobs.append({"name": "mgpu/conv", "kind": "weak",
                     "skip": (f"needs {n} GPUs, {ndev} visible (RCCL: one rank per GPU)" if n > ndev else None),
                     "cmd": [mg, "conv", "--gpus", str(n), *steps]})
        sh = n > ndev
        jobs.append({"name": "mgpu/jacobi-peer", "kind": "strong",
                     "skip": ("the one-process rehearsal shares at most 4 ranks per GPU" if sh and n > 4 * ndev
                              else None),
                     "cmd": [mg, "jacobi", "--halo", "peer", *(["--shared"] if sh else []), "--gpus", str(n),
                             "--iters", steps[1], "--warmup", steps[3]]})
    return jobs


def driver_command(n: int, steps: int, warmup: int) -> List[str]:
    """The round-end driver's bench invocation (task contract), argv after the interpreter."""
    return ["bench.py", "--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup)]


def value_of(rec: dict) -> Optional[float]:
    for k in ("value",):
        if k in rec:
            return float(rec[k])
    return None


def ms_of(rec: dict) -> Optional[float]:
    for k in ("ms_per_step", "ms_per_iter"):
        if k in rec:
            return float(rec[k])
    if rec.get("unit") == "ms/iteration":
        return float(rec["value"])
    return None


def efficiencies(rows: List[dict], rehearse: bool = False) -> None:
    """Scaling efficiency vs N = 1. In a rehearsal all ranks share the same
    GPUs, so the meaningful number is ``retained``: the fraction of the
    single-rank throughput the N-rank decomposition keeps on that hardware
    (1.0 = the halos and the ordering cost nothing)."""
    base: Dict[str, dict] = {}
    for r in rows:
        if r["n"] == 1 and r["status"] == "ok":
            base[r["name"]] = r
    for r in rows:
        b = base.get(r["name"]) or base.get(r["name"].replace("/rccl", "/peer"))
        r["efficiency"] = None
        if r["status"] != "ok" or b is None:
            continue
        if r is b:  # the baseline itself, whatever its rounding
            r["efficiency"] = 1.0
            if r["kind"] == "strong":
                r["speedup"] = 1.0
            if rehearse:
                r["retained"] = 1.0
            continue
        if r["kind"] == "weak" and r.get("value") is not None and b.get("value"):
            r["efficiency"] = round(r["value"] / (r["n"] * b["value"]), 4)
            if r.get("value_max_rank") and b.get("value_max_rank"):
                # the round-4 accounting (slowest rank's own span): shows what start skew costs
                r["efficiency_max_rank"] = round(r["value_max_rank"] / (r["n"] * b["value_max_rank"]), 4)
            if rehearse:
                r["retained"] = round(r["value"] / b["value"], 4)
        elif r["kind"] == "strong" and r.get("ms") is not None and b.get("ms"):
            r["efficiency"] = round(b["ms"] / (r["n"] * r["ms"]), 4)
            r["speedup"] = round(b["ms"] / r["ms"], 3)
            if rehearse:
                r["retained"] = r["speedup"]


def plot(rows: List[dict], path: str, title: str) -> Optional[str]:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cuda_mpi_openmp_amd.utils.plots import scaling_figure

    return scaling_figure(rows, path, title)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", default="1,2,4,8")
    p.add_argument("--out", default="scaling")
    p.add_argument("--device", choices=["auto", "cpu"], default="auto")
    p.add_argument("--rehearse", action="store_true", help="ranks share the visible GPUs (gloo control plane)")
    p.add_argument("--contract", action="store_true",
                   help="with --rehearse: run the ranks through the framework's RCCL code paths under the nccl "
                        "device contract (MPX_DIST_CONTRACT=nccl, parallel/contract.py) instead of plain gloo")
    p.add_argument("--quick", action="store_true", help="fewer steps per run")
    p.add_argument("--only", default="", help="run only jobs whose name contains this string")
    p.add_argument("--timeout", type=float, default=600.0, help="seconds per job")
    p.add_argument("--driver-steps", type=int, default=20, help="K of the driver's bench command (conv/driver)")
    p.add_argument("--driver-warmup", type=int, default=5, help="W of the driver's bench command (conv/driver)")
    a = p.parse_args(argv)
    ns = [int(x) for x in a.gpus.split(",") if x.strip()]
    out = a.out if os.path.isabs(a.out) else os.path.join(ROOT, a.out)
    os.makedirs(out, exist_ok=True)
    ndev = 0 if a.device == "cpu" else visible_gpus()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if a.contract:
        env["MPX_DIST_CONTRACT"] = "nccl"
        env.pop("MPX_DIST_BACKEND", None)
    elif a.device == "cpu" or a.rehearse:
        env["MPX_DIST_BACKEND"] = "gloo"
    rows: List[dict] = []
    with open(os.path.join(out, "scaling.log"), "w") as log:
        for n in ns:
            for job in plan(n, a, ndev):
                if a.only and a.only not in job["name"]:
                    continue
                row = {"name": job["name"], "kind": job["kind"], "n": n, "cmd": " ".join(job["cmd"])}
                if job["skip"]:
                    row["status"] = "skipped"
                    row["reason"] = job["skip"]
                else:
                    res = run_job(job["cmd"], env, a.timeout, log)
                    row["status"] = res["status"]
                    row["wall_s"] = res["wall_s"]
                    if res["status"] == "ok":
                        rec = res["record"]
                        row["value"] = value_of(rec)
                        row["unit"] = rec.get("unit")
                        row["ms"] = ms_of(rec)
                        row["n_reported"] = rec.get("n_gpus")
                        row["transport"] = (rec.get("config") or {}).get("transport") or rec.get("transport") or \
                            rec.get("halo")
                        row["world_size_seen"] = rec.get("world_size_seen")
                        row["verified"] = rec.get("verified_bit_exact", rec.get("verified"))
                        row["job_span_ms"] = rec.get("job_span_ms")
                        row["max_rank_span_ms"] = rec.get("max_rank_span_ms")
                        row["start_skew_ms"] = rec.get("start_skew_ms")
                        if row["value"] and rec.get("job_span_ms") and rec.get("max_rank_span_ms") \
                                and row["kind"] == "weak":
                            row["value_max_rank"] = row["value"] * rec["job_span_ms"] / rec["max_rank_span_ms"]
                    else:
                        row["stderr_tail"] = res.get("stderr_tail")
                rows.append(row)
                # bench.py's streaming conv (each step convolves the previous
                # output: halos with a real inter-rank dependency) as its own curve
                rec = res["record"] if not job["skip"] and res["status"] == "ok" else {}
                if job["name"].startswith("conv/") and (job["skip"] or rec.get("value_streaming") is not None):
                    srow = {"name": job["name"].replace("conv/", "conv-stream/"), "kind": job["kind"], "n": n,
                            "cmd": row["cmd"], "status": row["status"]}
                    if job["skip"]:
                        srow["reason"] = job["skip"]
                    else:
                        srow.update(value=float(rec["value_streaming"]), unit=rec.get("unit"),
                                    ms=rec.get("ms_per_step_streaming"), n_reported=rec.get("n_gpus"),
                                    transport=rec.get("transport_streaming"),
                                    world_size_seen=rec.get("world_size_seen"),
                                    verified=rec.get("verified_bit_exact_streaming"), wall_s=row.get("wall_s"))
                    rows.append(srow)
                for r in rows[-2:] if rows[-1] is not row else [row]:
                    print(json.dumps({k: r.get(k) for k in ("name", "n", "status", "value", "unit", "ms", "transport",
                                                             "reason")}), flush=True)
    efficiencies(rows, a.rehearse)
    meta = {"devices_visible": ndev, "device": a.device, "rehearse": a.rehearse, "gpus": ns,
            "host": os.uname().nodename, "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    with open(os.path.join(out, "scaling.json"), "w") as f:
        json.dump({"meta": meta, "runs": rows}, f, indent=1)
    cols = ["name", "kind", "n", "status", "value", "unit", "ms", "efficiency", "efficiency_max_rank", "speedup",
            "retained", "job_span_ms", "max_rank_span_ms", "start_skew_ms", "transport", "verified", "reason"]
    with open(os.path.join(out, "scaling.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols, extrasaction="ignore")
        w.writeheader()
        for r in rows:
            w.writerow(r)
    title = f"mpx scaling ({'CPU/gloo dry run' if a.device == 'cpu' else 'rehearsal: ranks share GPUs' if a.rehearse else 'one rank per MI355X'})"
    png = plot(rows, os.path.join(out, "scaling.png"), title)
    print(json.dumps({"scaling_json": os.path.join(out, "scaling.json"), "plot": png,
                      "ok": sum(r["status"] == "ok" for r in rows), "skipped": sum(r["status"] == "skipped" for r in rows),
                      "failed": sum(r["status"] not in ("ok", "skipped") for r in rows)}), flush=True)
    return 0 if all(r["status"] in ("ok", "skipped") for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
