#!/usr/bin/env python3
"""Kernel tuning harness: times lab2 conv kernel variants in ONE process with
interleaved rounds (cdna_hip_programming.md §5.4 rule 24) on random 4096^2
RGBA8 data, and checks every variant bit-exact against the production kernel.

  python tools/kbench.py [--size 4096] [--rounds 5] [--iters 20] [--rotate R]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402


STREAMS = []  # --streams S > 1: launch i goes to STREAMS[i % S] (independent pairs overlap, as in bench.py)


def S():  # the stream handle a variant launches on (the current torch stream)
    return torch.cuda.current_stream().cuda_stream


def time_launch(fn, iters, cyc):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    if STREAMS:
        main = torch.cuda.current_stream()
        for st in STREAMS:
            st.wait_stream(main)
        for i in range(iters):
            cyc[0] += 1
            with torch.cuda.stream(STREAMS[i % len(STREAMS)]):
                fn()
        for st in STREAMS:
            main.wait_stream(st)
    else:
        for _ in range(iters):
            cyc[0] += 1
            fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rotate", type=int, default=1, help="input/output pairs cycled per launch (>= 3 at 4096^2 "
                                                          "defeats the MALL)")
    p.add_argument("--only", default="", help="run only the variants whose name contains this string")
    p.add_argument("--streams", type=int, default=1, help="alternate launches over this many HIP streams "
                                                          "(needs --rotate divisible by it: no pair is shared)")
    args = p.parse_args()
    if args.streams > 1:
        if args.rotate % args.streams:
            raise SystemExit("--rotate must be a multiple of --streams")
        STREAMS.extend(torch.cuda.Stream() for _ in range(args.streams))
    L = _native.lib()
    T = _native.tune_lib()  # variants / probes live in libmpx_tune.so
    dev = torch.device("cuda:0")
    n = args.size
    # --rotate R: R independent (input, output) pairs cycled launch by launch,
    # so the working set (R x 128 MiB at 4096^2) exceeds the 256 MB MALL and
    # every launch streams from HBM (cache-assisted floors)
    pairs = []
    for r in range(max(1, args.rotate)):
        a = torch.randint(0, 256, (n, n, 4), dtype=torch.uint8, device=dev)
        pairs.append((a, torch.empty_like(a)))
    img, out = pairs[0]
    cyc = [0]

    def I():  # noqa: E743
        return pairs[cyc[0] % len(pairs)][0]

    def O():  # noqa: E743
        return pairs[cyc[0] % len(pairs)][1]
    bytes_moved = 2 * img.numel()

    # exhaustive fast-sqrt equivalence check
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    _native.check(T.mpx_selftest_fast_sqrt(bad.data_ptr(), 0, 0))
    torch.cuda.synchronize()
    print(json.dumps({"fast_sqrt_selftest_mismatches": int(bad.item())}), flush=True)

    variants = {}
    for fname, k in (("sobel5_dense", 5), ("roberts", 2)):
        f = ops.get_filter(fname)
        wx, wy = f.c_taps()
        ref = ops.conv(img, f)

        def mk(kind, p1, p2, fast, wx=wx, wy=wy, k=k):
            return lambda: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, k, kind, p1, p2, fast,
                                                            wx, wy, S()))

        for seg in (8, 16, 32, 64):
            variants[f"{fname}/wave-rt/seg{seg}"] = (mk(1, seg, 0, 1), ref)
            variants[f"{fname}/wave-const/seg{seg}"] = (mk(2, seg, 0, 1), ref)
        variants[f"{fname}/lds-stream/rpt4"] = (mk(0, 4, 0, 1), ref)
        for seg, p2 in ((0, 0), (0, 2000), (8, 2000), (16, 2000), (0, 2008), (32, 2000)):
            variants[f"{fname}/band/seg{seg}/p{p2}"] = (mk(9, seg, p2, 1), ref)
        variants[f"{fname}/production"] = ((lambda f=f: ops.conv(I(), f, O())), ref)
        variants[f"{fname}/direct"] = ((lambda f=f: ops.conv(I(), f, O(), direct=True)), ref)
    fs5 = ops.get_filter("sobel5")
    swx, swy = fs5.c_taps()
    sref = ops.conv(img, fs5)
    for seg in (0, 16, 32, 48):  # alternating segment direction (production MAG2 order candidate)
        variants[f"sobel5-sep/wave-const/seg{seg}/alt"] = (
            (lambda seg=seg: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 3, seg, 2000, 1,
                                                              swx, swy, S()))), sref)
    for seg in (0, 8, 20, 24):
        for kind, nm in ((3, "const"), (4, "rt")):
            variants[f"sobel5-sep/wave-{nm}/seg{seg}"] = (
                (lambda kind=kind, seg=seg: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5,
                                                                             kind, seg, 0, 1, swx, swy, S()))), sref)
        variants[f"sobel5-sep/wave-const/seg{seg}/strip-major"] = (
            (lambda seg=seg: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 3, seg, 1000, 1,
                                                              swx, swy, S()))), sref)
    for seg, per in ((0, 0), (0, 2000), (24, 2000), (0, 18000), (0, 34000), (0, 66000), (0, 162000),
                     (20, 34000), (24, 34000), (12, 34000),
                     (0, 10000), (0, 10005), (0, 11005), (24, 10000), (0, 514000), (0, 514005)):
        # 18000: no apron loads — a cost probe whose strip edges are wrong (no reference check)
        variants[f"sobel5-sep/band4/seg{seg}/w{per}"] = (
            (lambda seg=seg, per=per: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 8, seg,
                                                                       per, 1, swx, swy, S()))), None if per == 18000 else sref)
    variants["sobel5-sep/band16v"] = (  # vertical halo sharing through LDS (conv_band16v_kernel)
        (lambda: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 10, 0, 0, 1, swx, swy, S()))),
        sref)
    rf = ops.get_filter("roberts")
    rwx, rwy = rf.c_taps()
    rref = ops.conv(img, rf)
    variants["sobel5-sep/stores-nt"] = (
        (lambda: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 6, 0, 3, 1, swx, swy, S()))),
        sref)
    for p2, nm in ((0, "buffer"), (1, "global"), (2, "global-nt")):  # row-load A/B
        variants[f"sobel5-sep/loads-{nm}"] = (
            (lambda p2=p2: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 6, 0, p2, 1,
                                                            swx, swy, S()))), sref)
        variants[f"roberts/loads-{nm}"] = (
            (lambda p2=p2: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 2, 7, 0, p2, 1,
                                                            rwx, rwy, S()))), rref)
    for pf in (4, 8, 12):  # prefetch ring depth (D = 5 / 10 / 15 rows)
        for seg in (0, 16, 24, 32, 40):
            variants[f"sobel5-sep/wave-const/seg{seg}/pf{pf}"] = (
                (lambda seg=seg, pf=pf: _native.check(T.mpx_conv_variant(I().data_ptr(), O().data_ptr(), n, n, 5, 3, seg,
                                                                         pf, 1, swx, swy, S()))), sref)
    for fname in ("sobel5", "gauss5"):  # separable production path (row-sum ring)
        f = ops.get_filter(fname)
        variants[f"{fname}/production"] = ((lambda f=f: ops.conv(I(), f, O())), ops.conv(img, f))
        variants[f"{fname}/direct"] = ((lambda f=f: ops.conv(I(), f, O(), direct=True)), ops.conv(img, f))
    variants["copy/torch"] = ((lambda: O().copy_(I())), img)
    for v, d, seg in ((2, 4, 8), (2, 4, 24), (2, 8, 24), (4, 4, 8), (4, 4, 24), (4, 8, 24), (4, 2, 24), (4, 4, 48)):
        variants[f"copy/strip-v{v}-d{d}-seg{seg}"] = (
            (lambda v=v, d=d, seg=seg: _native.check(T.mpx_strip_copy_probe(I().data_ptr(), O().data_ptr(), n, n, v, d,
                                                                            seg, S()))), img)
    for v, d, seg in ((2, 104, 8), (2, 104, 24), (4, 104, 8), (4, 104, 24), (4, 104, 64)):  # 16 waves per block
        variants[f"copy/strip-v{v}-d{d - 100}-seg{seg}-wpb16"] = (
            (lambda v=v, d=d, seg=seg: _native.check(T.mpx_strip_copy_probe(I().data_ptr(), O().data_ptr(), n, n, v, d,
                                                                            seg, S()))), img)
    for d, nm in ((0, "plain"), (1, "nt")):  # linear 16-B-per-thread copy: the HBM floor of these bytes
        variants[f"copy/linear-{nm}"] = (
            (lambda d=d: _native.check(T.mpx_strip_copy_probe(I().data_ptr(), O().data_ptr(), n, n, 0, d, 0, S()))), img)
    for seg, fl in [(sg, f) for sg in (4, 8, 12, 16, 20) for f in (2, 3, 10, 18, 26, 74)] + [
            (16, 0), (16, 4), (16, 34), (16, 42), (32, 10), (32, 42), (16, 72), (16, 106), (32, 74)]:
        if True:  # row bands, 16-B vector per thread (ref None: XOR of rows, no reference)
            variants[f"copy/band-seg{seg}-f{fl}"] = (
                (lambda fl=fl, seg=seg: _native.check(T.mpx_strip_copy_probe(I().data_ptr(), O().data_ptr(), n, n, 8,
                                                                              fl, seg, S()))), None)
    # burst tiles: R output rows per tile, all R + 4 row
    # loads of a lane issued at once, many rounds of tiles; f = flag bits
    # (1 xcd_remap, 2 NT loads, 4 NT stores), t = threads per workgroup
    for R in (2, 4, 8, 12, 16, 24):
        for tcode in (0, 1, 2):
            for fl in (0, 1, 4, 5, 6, 7, 13, 15):
                if tcode == 1 and fl not in (5, 7):
                    continue
                if fl >= 8 and (tcode != 2 or R < 8):  # residency cap: 1024-thread tiles, R >= 8
                    continue
                d = fl | (tcode << 4)
                variants[f"copy/burst-r{R}-t{256 << tcode}-f{fl}"] = (
                    (lambda d=d, R=R: _native.check(T.mpx_strip_copy_probe(I().data_ptr(), O().data_ptr(), n, n, 16,
                                                                            d, R, S()))), None)
    rob_ref = ops.roberts(img)
    for geom in (((32, 32), (16, 16)), ((64, 4), (64, 64)), ((16, 16), (1024, 1024))):
        variants[f"roberts/geom{geom}"] = ((lambda g=geom: ops.roberts(I(), O(), geometry=g)), rob_ref)

    if args.only:  # comma-separated substrings: a variant runs when its name contains any of them
        keys = [k for k in args.only.split(",") if k]
        variants = {k: v for k, v in variants.items() if any(s in k for s in keys)}
    # correctness first
    cpu_img = img.cpu()
    for fname in ("sobel5_dense", "roberts"):
        cpu = ops.conv(cpu_img, fname)
        print(json.dumps({"production_vs_cpu": fname, "bit_exact": bool(torch.equal(ops.conv(img, fname).cpu(), cpu))}),
              flush=True)
    for name, (fn, ref) in variants.items():
        cyc[0] = 0
        out.zero_()
        fn()
        torch.cuda.synchronize()
        ok = ref is None or torch.equal(out, ref)
        if not ok:
            print(json.dumps({"variant": name, "ERROR": "mismatch vs production"}), flush=True)
    times = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, (fn, _) in variants.items():
            times[name].append(time_launch(fn, args.iters, cyc))
    for name, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"variant": name, "us_median": round(med, 2), "us_min": round(min(ts), 2),
                          "TBps": round(bytes_moved / med / 1e6, 3), "Gpix_s": round(n * n / med / 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
