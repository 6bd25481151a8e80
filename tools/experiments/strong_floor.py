#!/usr/bin/env python3
"""Per-rank floor of the strong-scaling conv job (VERDICT r5 Next #2): one
rank's share of a 4096^2 sobel5 frame at 4096 / 2048 / 1024 / 512 rows
(N = 1 / 2 / 4 / 8), on one GPU, 6 rotated slabs, two HIP streams as in
bench.py. Three forms per slab height:

* ``edge``: the slab alone, clamp-to-edge at its top and bottom (no halo);
* ``halo``: the same rows with 2 + 2 resident halo rows read from the slab
  buffer (what a rank computes once its halo rows have arrived);
* ``split``: the frame's whole 4096 rows cut into 4096 / rows launches back to
  back on one rank (the total launch count of the strong job, one GPU).

One JSON line per (rows, form): µs per step (median of 5 windows of K steps)
and the rate over the slab's own pixels."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.ops.edge import ConvLauncher  # noqa: E402
from cuda_mpi_openmp_amd.ops.filters import get_filter  # noqa: E402

W = 4096
ROT = 6
K = int(os.environ.get("SF_STEPS", "200"))


def timed(launches, streams):
    s0 = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(2 * len(launches)):  # warm-up
        launches[i % len(launches)](streams[i % 2].cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record(s0)
        for st in streams:
            st.wait_stream(s0)
        for i in range(K):
            launches[i % len(launches)](streams[i % 2].cuda_stream)
        for st in streams:
            s0.wait_stream(st)
        ev[1].record(s0)
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / K)
    return statistics.median(ts), min(ts)


def main():
    dev = torch.device("cuda:0")
    f = get_filter("sobel5")
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for rows in (4096, 2048, 1024, 512):
        srcs = [torch.randint(0, 256, (rows + 4, W, 4), dtype=torch.uint8, device=dev) for _ in range(ROT)]
        outs = [torch.empty((rows, W, 4), dtype=torch.uint8, device=dev) for _ in range(ROT)]
        forms = {
            "edge": [ConvLauncher(s, o, f, src_row0=2, out_row0=0, oy0=0, oy1=rows, y_lo=0, y_hi=rows - 1)
                     for s, o in zip(srcs, outs)],
            "halo": [ConvLauncher(s, o, f, src_row0=2, out_row0=0, oy0=0, oy1=rows, y_lo=-2, y_hi=rows + 1)
                     for s, o in zip(srcs, outs)],
        }
        for name, ls in forms.items():
            med, mn = timed(ls, streams)
            print(json.dumps({"rows": rows, "form": name, "us_per_step": round(med, 2), "us_min": round(mn, 2),
                              "gpix_s": round(rows * W / med / 1e3, 1)}), flush=True)
        del srcs, outs, forms
        torch.cuda.empty_cache()
    # the strong job's whole frame as 4096 / rows launches on one GPU
    frames = [torch.randint(0, 256, (W, W, 4), dtype=torch.uint8, device=dev) for _ in range(ROT)]
    fouts = [torch.empty_like(x) for x in frames]
    for rows in (4096, 2048, 1024, 512):
        parts = W // rows
        ls = []
        for s, o in zip(frames, fouts):
            ls.append([ConvLauncher(s, o, f, src_row0=0, out_row0=0, oy0=p * rows, oy1=(p + 1) * rows, y_lo=0,
                                    y_hi=W - 1) for p in range(parts)])

        def frame(stream, ls=ls, c=[0]):
            for launch in ls[c[0] % ROT]:
                launch(stream)
            c[0] += 1
        med, mn = timed([frame], streams)
        print(json.dumps({"rows": rows, "form": "split", "launches_per_frame": parts, "us_per_frame": round(med, 2),
                          "us_min": round(mn, 2), "gpix_s": round(W * W / med / 1e3, 1)}), flush=True)
    ops  # noqa: B018 (import kept: loads the library)


if __name__ == "__main__":
    main()
