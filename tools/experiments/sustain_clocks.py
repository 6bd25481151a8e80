#!/usr/bin/env python3
"""Attribute the sustained-load slowdown (VERDICT r4 Next #2): the bench's
burst / sustain protocol on the flagship conv AND on controls, with the board's
clocks, power and temperature sampled at ~200 Hz beside every phase.

  python tools/experiments/sustain_clocks.py [--sustain-ms 2000] [--rounds 2] [--out DIR]

Workloads (each on 6 rotated 128 MiB in/out pairs, steps alternating over two
HIP streams — bench.py's regime; 64 MiB read + 64 MiB written per step except
vsub, 64 + 64 read + 64 written):

* ``copy``    linear non-temporal 16-B copy (libmpx_tune.so probe): no ALU work;
* ``vsub``    lab1 fp32 c = a - b (libmpx);
* ``roberts`` Roberts cross 4096^2 (the bench's SlabEdgeDetector, N = 1);
* ``sobel5``  the headline 5x5 (the same detector the bench times).

Protocol per workload, after --idle-ms with the GPU idle: W = 5 warm-up
steps, a burst of K = 20 steps (bench ``value``), then continuous chunks of
50 steps for --sustain-ms (each chunk host-timed between device syncs on the
node's monotonic clock, the sampler's clock), then K = 20 again (bench
``value_sustained``). The chunks are binned by time under load; each bin's
rate is also given as a fraction of the workload's burst rate, so a board
property (every workload loses the same fraction) and a kernel property (only
the VALU-heavy ones lose) tell themselves apart. Workload order alternates
between rounds.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from cuda_mpi_openmp_amd import _native, ops, parallel  # noqa: E402
from cuda_mpi_openmp_amd.utils.clocks import ClockSampler, key_fields  # noqa: E402

BINS_MS = (0, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000, 1e9)


def clock_ns() -> int:
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def make_workload(name: str, dev, size: int, rotate: int, streams):
    """(step function cycling the rotated pairs over the streams, pixels-or-elements per step, bytes per step)."""
    cyc = [0]
    if name in ("roberts", "sobel5"):
        from cuda_mpi_openmp_amd.models.edge import SlabEdgeDetector

        ctx = parallel.DistContext(device=dev)
        dets = []
        for r in range(rotate):
            d = SlabEdgeDetector(ctx, size, size, name)
            d.fill_random(seed=1234 + 7919 * r)
            dets.append(d)
        handles = [s.cuda_stream for s in streams]

        def step():
            i = cyc[0] % rotate
            dets[i].step(handles[i % len(handles)])
            cyc[0] += 1
        return step, size * size, 8 * size * size, dets
    if name == "copy":
        T = _native.tune_lib()
        pairs = [(torch.randint(0, 256, (size, size, 4), dtype=torch.uint8, device=dev),
                  torch.empty((size, size, 4), dtype=torch.uint8, device=dev)) for _ in range(rotate)]

        def step():
            i = cyc[0] % rotate
            a, b = pairs[i]
            _native.check(T.mpx_strip_copy_probe(a.data_ptr(), b.data_ptr(), size, size, 0, 1, 0,
                                                  streams[i % len(streams)].cuda_stream))
            cyc[0] += 1
        return step, size * size, 8 * size * size, pairs
    if name == "vsub":
        n = size * size
        trip = [(torch.rand(n, device=dev), torch.rand(n, device=dev), torch.empty(n, device=dev))
                for _ in range(rotate)]

        def step():
            i = cyc[0] % rotate
            a, b, c = trip[i]
            with torch.cuda.stream(streams[i % len(streams)]):
                ops.vsub(a, b, c)
            cyc[0] += 1
        return step, n, 12 * n, trip
    raise SystemExit(f"unknown workload {name}")


def run_one(name, args, dev, streams, cs):
    step, units, nbytes, keep = make_workload(name, dev, args.size, args.rotate, streams)
    for s in streams:
        s.wait_stream(torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    time.sleep(args.idle_ms / 1e3)  # the board settles idle between workloads

    def k_steps(k):
        for _ in range(k):
            step()
        torch.cuda.synchronize(dev)

    k_steps(args.warmup)
    t0 = clock_ns()
    k_steps(args.steps)
    t1 = clock_ns()
    burst = {"t0": t0, "t1": t1, "us_per_step": (t1 - t0) / 1e3 / args.steps}
    chunks = []
    start = clock_ns()
    while (clock_ns() - start) / 1e6 < args.sustain_ms:
        a = clock_ns()
        k_steps(args.chunk)
        b = clock_ns()
        chunks.append((a, b))
    t0 = clock_ns()
    k_steps(args.steps)
    t1 = clock_ns()
    after = {"t0": t0, "t1": t1, "us_per_step": (t1 - t0) / 1e3 / args.steps}
    del keep
    rec = {"workload": name, "bytes_per_step": nbytes, "units_per_step": units,
           "burst_us": round(burst["us_per_step"], 3), "after_us": round(after["us_per_step"], 3),
           "burst_clocks": key_fields(cs.summary(burst["t0"], burst["t1"], pad_ns=3_000_000)) if cs else None,
           "after_clocks": key_fields(cs.summary(after["t0"], after["t1"], pad_ns=3_000_000)) if cs else None,
           "bins": []}
    for lo, hi in zip(BINS_MS[:-1], BINS_MS[1:]):
        sel = [(a, b) for a, b in chunks if lo <= (a - start) / 1e6 < hi]
        if not sel:
            continue
        us = [(b - a) / 1e3 / args.chunk for a, b in sel]
        med = statistics.median(us)
        row = {"ms": [lo, hi if hi < 1e8 else None], "chunks": len(sel), "us_per_step": round(med, 3),
               "retained": round(burst["us_per_step"] / med, 4),
               "TBps": round(nbytes / (med * 1e-6) / 1e12, 3)}
        if cs:
            row["clocks"] = key_fields(cs.summary(sel[0][0], sel[-1][1]))
        rec["bins"].append(row)
    rec["burst_TBps"] = round(nbytes / (burst["us_per_step"] * 1e-6) / 1e12, 3)
    rec["after_TBps"] = round(nbytes / (after["us_per_step"] * 1e-6) / 1e12, 3)
    rec["after_retained"] = round(burst["us_per_step"] / after["us_per_step"], 4)
    return rec


def render(path: str) -> str:
    """Markdown tables of a sustain_clocks.json: per workload and round, the
    burst / steady / after-load step times and the board state in each phase."""
    d = json.load(open(path))
    out = ["| workload | round | burst µs (clock MHz) | 0-10 ms | 10-20 ms | 20-50 ms | 50-100 ms | 0.5-1 s | 1-2 s "
           "(MHz, W) | K=20 after 2 s µs | after / burst |", "|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in d["runs"]:
        bins = {tuple(b["ms"]): b for b in r["bins"]}

        def cell(lo, hi, clocks=False):
            b = bins.get((lo, hi))
            if not b:
                return "–"
            c = b.get("clocks") or {}
            extra = f" ({c.get('gfxclk_mhz', 0):.0f}, {c.get('power_w', 0):.0f})" if clocks else ""
            return f"{b['us_per_step']:.2f}{extra}"
        bc = r.get("burst_clocks") or {}
        out.append(f"| {r['workload']} | {r['round']} | {r['burst_us']:.2f} ({bc.get('gfxclk_mhz', 0):.0f}) | "
                   f"{cell(0, 10)} | {cell(10, 20)} | {cell(20, 50)} | {cell(50, 100)} | {cell(500, 1000)} | "
                   f"{cell(1000, 2000, True)} | {r['after_us']:.2f} | {r['after_retained']:.3f} |")
    m = d["meta"]
    out.append("")
    out.append(f"Sampler: {m['sampler']} at {m['sampler_hz']:.0f} Hz ({m['samples']} samples, "
               f"{m['read_us_med']:.0f} µs per read); chunks of {m['args']['chunk']} steps; "
               f"{m['args']['idle_ms']:.0f} ms idle before each workload.")
    return "\n".join(out)


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--render":
        print(render(sys.argv[2]))
        return
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--workloads", default="copy,vsub,roberts,sobel5")
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--rotate", type=int, default=6)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--chunk", type=int, default=50)
    p.add_argument("--sustain-ms", type=float, default=2000.0)
    p.add_argument("--idle-ms", type=float, default=1500.0)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--hz", type=float, default=200.0)
    p.add_argument("--out", default="gpurun_out/sustain")
    a = p.parse_args()
    os.makedirs(a.out, exist_ok=True)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from cuda_mpi_openmp_amd.utils.streams import compute_streams

    streams = compute_streams(dev, 2)
    cs = ClockSampler(hz=a.hz).start()
    print(json.dumps({"sampler": cs.source, "error": cs.error}), flush=True)
    names = [w for w in a.workloads.split(",") if w]
    recs = []
    for r in range(a.rounds):
        order = names if r % 2 == 0 else list(reversed(names))
        for nm in order:
            rec = run_one(nm, a, dev, streams, cs if cs.source else None)
            rec["round"] = r
            recs.append(rec)
            print(json.dumps({k: rec[k] for k in ("workload", "round", "burst_us", "after_us", "after_retained",
                                                  "burst_TBps", "after_TBps")}), flush=True)
            torch.cuda.empty_cache()
    cs.stop()
    meta = {"sampler": cs.source, "sampler_error": cs.error, "sampler_hz": cs.rate_hz(),
            "read_us_med": statistics.median(cs.read_us) if cs.read_us else None, "samples": len(cs.samples),
            "device": torch.cuda.get_device_name(dev), "args": vars(a)}
    with open(os.path.join(a.out, "sustain_clocks.json"), "w") as f:
        json.dump({"meta": meta, "runs": recs}, f, indent=1)
    # the raw trace (time from the first sample, the key fields)
    if cs.samples:
        t00 = cs.samples[0][0]
        with open(os.path.join(a.out, "clock_trace.csv"), "w") as f:
            keys = sorted({k for _, m in cs.samples for k in m})
            f.write("t_ms," + ",".join(keys) + "\n")
            for t, m in cs.samples:
                f.write(f"{(t - t00) / 1e6:.3f}," + ",".join(f"{m[k]:.6g}" if k in m else "" for k in keys) + "\n")
    with open(os.path.join(a.out, "sustain_clocks.md"), "w") as f:
        f.write(render(os.path.join(a.out, "sustain_clocks.json")) + "\n")
    print(json.dumps({"meta": meta}), flush=True)


if __name__ == "__main__":
    main()
