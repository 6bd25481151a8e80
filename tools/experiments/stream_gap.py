#!/usr/bin/env python3
"""Why does bench.py's ``value_streaming`` trail ``value``? (VERDICT r4 Next #5)

One process, the bench's regime (4096^2 sobel5, 6 slabs on the 2 compute
streams, K = 20 steps between device syncs, W = 6 warm-up steps), every mode
timed in interleaved rounds so clock drift and allocation order cancel:

* ``static``      each slab: halo-padded random input -> separate output
                  (bench ``value``);
* ``static_iter`` the same launches on input frames the filter produced
                  (8 iterations of it), so only the data differs;
* ``pingpong``    each slab's frame k reads buffer k % 2 and writes buffer
                  (k + 1) % 2 at the halo offset (bench ``value_streaming``);
* ``triple``      the same with three buffers: frame k writes the buffer
                  frame k - 2 read, never the one frame k - 1 read;
* ``pingpong_rand`` ping-pong whose buffers are re-filled with random data
                  before each round (layout of the streaming phase, data of
                  the static one);
* ``static_outpad`` static, but the output rows written at the halo offset of
                  a padded buffer (the input's row alignment, as in ping-pong);
* ``pingpong_skewS`` ping-pong whose second buffer starts S rows (S x 16 KiB)
                  later in its allocation than the first;
* ``static_plain`` / ``pingpong_plain``: those layouts with plain loads of
                  every row instead of the default non-temporal interior loads;
* ``static_m1`` / ``pingpong_m1``: band mode 1 — plain output stores too.

GAP_MODES (comma list) picks the modes; GAP_ROUNDS the rounds.

Prints one JSON line per (round, mode) and a summary (median µs per step).
"""

import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402
from cuda_mpi_openmp_amd.ops.filters import get_filter  # noqa: E402
from cuda_mpi_openmp_amd.utils.streams import compute_streams  # noqa: E402

N, ROT, K, W = 4096, 6, 20, 6
HALO = 2


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    f = get_filter("sobel5")
    streams = compute_streams(dev, 2)
    hs = [s.cuda_stream for s in streams]
    g = torch.Generator(device=dev)
    g.manual_seed(7)

    def padded():
        return torch.empty((N + 2 * HALO, N, 4), dtype=torch.uint8, device=dev)

    def launcher(src, dst, dst_row0):
        return ops.ConvLauncher(src, dst, f, src_row0=HALO, out_row0=dst_row0, oy0=0, oy1=N, y_lo=0, y_hi=N - 1)

    rand_in = [padded() for _ in range(ROT)]
    for b in rand_in:
        b[HALO:HALO + N].copy_(torch.randint(0, 256, (N, N, 4), dtype=torch.uint8, device=dev, generator=g))
    outs = [torch.empty((N, N, 4), dtype=torch.uint8, device=dev) for _ in range(ROT)]
    iter_in = [padded() for _ in range(ROT)]
    for i in range(ROT):  # 8 iterations of the filter from the random frame
        a, b = rand_in[i].clone(), padded()
        for _ in range(8):
            launcher(a, b, HALO)(None)
            a, b = b, a
        iter_in[i].copy_(a)
    pp = [[padded(), padded()] for _ in range(ROT)]
    tr = [[padded(), padded(), padded()] for _ in range(ROT)]
    ppr = [[padded(), padded()] for _ in range(ROT)]
    for i in range(ROT):
        for b in pp[i] + tr[i] + ppr[i]:
            b.copy_(rand_in[i])
    outpad = [padded() for _ in range(ROT)]
    skews = (1, 2, 3, 4, 8)
    skewed = {}
    for S in skews:
        bb = []
        for i in range(ROT):
            a = padded()
            big = torch.empty((N + 2 * HALO + S, N, 4), dtype=torch.uint8, device=dev)
            b = big[S:]
            a.copy_(rand_in[i])
            b.copy_(rand_in[i])
            bb.append([a, b])
        skewed[S] = bb
    torch.cuda.synchronize()

    L = {
        "static": [[launcher(rand_in[i], outs[i], 0)] for i in range(ROT)],
        "static_iter": [[launcher(iter_in[i], outs[i], 0)] for i in range(ROT)],
        "pingpong": [[launcher(pp[i][a], pp[i][1 - a], HALO) for a in range(2)] for i in range(ROT)],
        "triple": [[launcher(tr[i][a], tr[i][(a + 1) % 3], HALO) for a in range(3)] for i in range(ROT)],
        "pingpong_rand": [[launcher(ppr[i][a], ppr[i][1 - a], HALO) for a in range(2)] for i in range(ROT)],
        "static_outpad": [[launcher(rand_in[i], outpad[i], HALO)] for i in range(ROT)],
    }
    # the same layouts with plain loads of every row (the resident-input policy,
    # OPT 2) instead of non-temporal loads of the rows no neighbour re-reads
    pl = {"static_plain": [[launcher(rand_in[i], outs[i], 0)] for i in range(ROT)],
          "pingpong_plain": [[launcher(pp[i][a], pp[i][1 - a], HALO) for a in range(2)] for i in range(ROT)]}
    for ls in pl.values():
        for row in ls:
            for ln in row:
                ln.resident = True
    L.update(pl)
    # band mode 1 (plain output stores and plain loads; mpx_conv_set_band_mode):
    # the same launchers, the mode switched around their runs
    L["static_m1"] = L["static"]
    L["pingpong_m1"] = [[launcher(pp[i][a], pp[i][1 - a], HALO) for a in range(2)] for i in range(ROT)]
    from cuda_mpi_openmp_amd import _native
    NL = _native.lib()
    for S in skews:
        L[f"pingpong_skew{S}"] = [[launcher(skewed[S][i][a], skewed[S][i][1 - a], HALO) for a in range(2)]
                                  for i in range(ROT)]
    mod = 1 << 21  # where each buffer starts within a 2 MiB frame (the row offset a launch adds comes on top)
    print(json.dumps({"base_mod_2MiB_KiB": {
        "static_in": rand_in[0].data_ptr() % mod // 1024, "static_out": outs[0].data_ptr() % mod // 1024,
        "pingpong": [b.data_ptr() % mod // 1024 for b in pp[0]],
        **{f"skew{S}": [b.data_ptr() % mod // 1024 for b in skewed[S][0]] for S in skews}}}), flush=True)
    want = [m for m in os.environ.get("GAP_MODES", "").split(",") if m]
    if want:
        L = {m: L[m] for m in want}
    k = {m: [0] * ROT for m in L}

    def run(mode, nsteps):
        for s in range(nsteps):
            i = s % ROT
            ls = L[mode][i]
            ls[k[mode][i] % len(ls)](hs[i % 2])
            k[mode][i] += 1

    res = {m: [] for m in L}
    main_stream = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(main_stream)
    for rnd in range(int(os.environ.get("GAP_ROUNDS", "12"))):
        order = list(L) if rnd % 2 == 0 else list(reversed(list(L)))
        for mode in order:
            if mode == "pingpong_rand":
                for i in range(ROT):
                    for b in ppr[i]:
                        b.copy_(rand_in[i])
                torch.cuda.synchronize()
            prev = NL.mpx_conv_set_band_mode(1) if mode.endswith("_m1") else None
            run(mode, W)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(mode, K)
            torch.cuda.synchronize()
            if prev is not None:
                NL.mpx_conv_set_band_mode(prev)
            us = (time.perf_counter() - t0) * 1e6 / K
            res[mode].append(us)
            print(json.dumps({"round": rnd, "mode": mode, "us_per_step": round(us, 3)}), flush=True)
            time.sleep(0.05)
    summ = {m: {"median_us": round(statistics.median(v), 3), "min_us": round(min(v), 3),
                "gpixel_s": round(N * N / (statistics.median(v) * 1e-6) / 1e9, 1)} for m, v in res.items()}
    print(json.dumps({"summary": summ}), flush=True)


if __name__ == "__main__":
    main()
