#!/usr/bin/env python3
"""Band-kernel segment rows for short slabs (the strong-scaling job's 512 /
1024 / 2048 rows per rank of a 4096-wide frame): sobel5 separable on
conv_band4_kernel with the production OPT (34: NT stores, NT interior loads)
through libmpx_tune's mpx_conv_variant (kind 8, p1 = segment rows, 0 = the
production auto rule: one resident round, at least 8 rows), against the
production ops path. 6 rotated slabs, two HIP streams as in bench.py; every
variant's output checked against the production one. One JSON line per
(rows, variant): µs per launch, median of 5 windows."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402

W, ROT, K = 4096, 6, 200


def timed(fn, streams):
    s0 = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(2 * ROT):
        fn(i, streams[i % 2])
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record(s0)
        for st in streams:
            st.wait_stream(s0)
        for i in range(K):
            fn(i, streams[i % 2])
        for st in streams:
            s0.wait_stream(st)
        ev[1].record(s0)
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / K)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda:0")
    T = _native.tune_lib()
    f = ops.get_filter("sobel5")
    wx, wy = f.c_taps()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for rows in (512, 1024, 2048):
        ins = [torch.randint(0, 256, (rows, W, 4), dtype=torch.uint8, device=dev) for _ in range(ROT)]
        outs = [torch.empty_like(x) for x in ins]
        refs = [ops.conv(x, f) for x in ins]

        def prod(i, st):
            with torch.cuda.stream(st):
                ops.conv(ins[i % ROT], f, out=outs[i % ROT])
        print(json.dumps({"rows": rows, "variant": "production", "us": round(timed(prod, streams), 2)}), flush=True)
        for seg in (0, 2, 3, 4, 5, 6, 8, 12, 16):
            for per in (0, 8):
                def var(i, st, seg=seg, per=per):
                    _native.check(T.mpx_conv_variant(ins[i % ROT].data_ptr(), outs[i % ROT].data_ptr(), W, rows, 5, 8,
                                                     seg, 34000 + per, 1, wx, wy, st.cuda_stream))
                for o in outs:
                    o.zero_()
                var(0, streams[0])
                torch.cuda.synchronize()
                ok = torch.equal(outs[0], refs[0])
                print(json.dumps({"rows": rows, "variant": f"band4/seg{seg}/per{per}", "us": round(timed(var, streams), 2),
                                  "same_as_production": ok}), flush=True)
        del ins, outs, refs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
