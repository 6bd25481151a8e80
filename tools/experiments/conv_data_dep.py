#!/usr/bin/env python3
"""Is the production sobel5 conv's time data dependent? The bench's static
phase convolves uniform random frames; its streaming phase convolves frames
the filter itself produced (iterated: gray, mostly 0 / 255 with edges). Same
launches, same 2-stream / 6-pair rotation (ConvLauncher on the compute stream
pair), different inputs: random, iterated 1 / 2 / 8 times, constant, and
random gray, then three buffer layouts (static, ping-pong). Median of 5 rounds of 200 frames, event-timed, us per frame.
One JSON line per input kind."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.ops.filters import get_filter  # noqa: E402
from cuda_mpi_openmp_amd.utils.streams import compute_streams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    streams = compute_streams(dev, 2)
    n, pairs, frames = 4096, 6, 200
    f = get_filter("sobel5")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    rnd = [torch.randint(0, 256, (n, n, 4), dtype=torch.uint8, device=dev, generator=g) for _ in range(pairs)]

    def iterate(imgs, k):
        out = []
        for im in imgs:
            x = im.clone()
            for _ in range(k):
                x = ops.conv(x, f)
            out.append(x)
        return out

    gray = []
    for im in rnd:
        x = im.clone()
        x[..., 1] = x[..., 0]
        x[..., 2] = x[..., 0]
        gray.append(x)
    kinds = {"random_first": rnd, "random": rnd, "iter1": iterate(rnd, 1), "iter2": iterate(rnd, 2), "iter8": iterate(rnd, 8),
             "const128": [torch.full_like(rnd[0], 128) for _ in range(pairs)], "random_gray": gray}
    outs = [torch.empty_like(rnd[0]) for _ in range(pairs)]
    main_s = torch.cuda.current_stream(dev)
    for name, imgs in kinds.items():
        fr = {}
        for im in imgs:
            v = (im[..., :3].int()).flatten()
            fr["sat"] = fr.get("sat", 0) + int(((v == 0) | (v == 255)).sum())
        launches = [ops.ConvLauncher(imgs[i], outs[i], f, src_row0=0, out_row0=0, oy0=0, oy1=n, y_lo=0, y_hi=n - 1)
                    for i in range(pairs)]
        hs = [s.cuda_stream for s in streams]
        ts = []
        for rnd_i in range(6):
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for s in streams:
                s.wait_stream(main_s)
            for k in range(frames):
                launches[k % pairs](hs[k % 2])
            for s in streams:
                main_s.wait_stream(s)
            e1.record(main_s)
            e1.synchronize()
            if rnd_i:
                ts.append(e0.elapsed_time(e1) * 1e3 / frames)
        ts.sort()
        print(json.dumps({"input": name, "us_per_frame": round(ts[len(ts) // 2], 2), "min": round(ts[0], 2),
                          "saturated_channel_frac": round(fr["sat"] / (pairs * n * n * 3), 3)}), flush=True)

    # layouts: the static phase reads halo-padded buffers into separate
    # outputs; the streaming phase ping-pongs between two halo-padded buffers
    # per sequence (writes land where the previous step of the sequence read)
    pad = [torch.empty((n + 4, n, 4), dtype=torch.uint8, device=dev) for _ in range(2 * pairs)]
    for i in range(pairs):
        pad[2 * i][2:2 + n].copy_(rnd[i])
        pad[2 * i + 1][2:2 + n].copy_(rnd[i])
    mk = lambda src, out, orow: ops.ConvLauncher(src, out, f, src_row0=2, out_row0=orow, oy0=0, oy1=n,  # noqa: E731
                                                 y_lo=0, y_hi=n - 1)
    # the same buffers' images at shifted bases: the output slab of a
    # ping-pong step starts `sk` rows (16 KiB each) further from its
    # allocation's alignment than the input slab does
    skew = {}
    for sk in (1, 2, 4):
        bs = [torch.empty((n + 4 + sk, n, 4), dtype=torch.uint8, device=dev) for _ in range(pairs)]
        for i in range(pairs):
            bs[i][sk + 2:sk + 2 + n].copy_(rnd[i])
        skew[sk] = [b[sk:] for b in bs]
    aligned_out = [torch.empty((n + 4, n, 4), dtype=torch.uint8, device=dev) for _ in range(pairs)]
    layouts = {
        "static_padded_src": [[mk(pad[2 * i], outs[i], 0)] for i in range(pairs)],
        "static_out_at_row2": [[mk(pad[2 * i], aligned_out[i], 2)] for i in range(pairs)],
        "pingpong_skew1": [[mk(pad[2 * i], skew[1][i], 2), mk(skew[1][i], pad[2 * i], 2)] for i in range(pairs)],
        "pingpong_skew2": [[mk(pad[2 * i], skew[2][i], 2), mk(skew[2][i], pad[2 * i], 2)] for i in range(pairs)],
        "pingpong_skew4": [[mk(pad[2 * i], skew[4][i], 2), mk(skew[4][i], pad[2 * i], 2)] for i in range(pairs)],
        "pingpong": [[mk(pad[2 * i], pad[2 * i + 1], 2), mk(pad[2 * i + 1], pad[2 * i], 2)] for i in range(pairs)],
        "pingpong_one_way": [[mk(pad[2 * i], pad[2 * i + 1], 2)] for i in range(pairs)],
    }
    hs = [s.cuda_stream for s in streams]
    for name, ls in layouts.items():
        ts = []
        for rnd_i in range(6):
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for s in streams:
                s.wait_stream(main_s)
            for k in range(frames):
                seq = ls[k % pairs]
                seq[(k // pairs) % len(seq)](hs[k % 2])
            for s in streams:
                main_s.wait_stream(s)
            e1.record(main_s)
            e1.synchronize()
            if rnd_i:
                ts.append(e0.elapsed_time(e1) * 1e3 / frames)
        ts.sort()
        print(json.dumps({"layout": name, "us_per_frame": round(ts[len(ts) // 2], 2), "min": round(ts[0], 2)}),
              flush=True)


if __name__ == "__main__":
    main()
