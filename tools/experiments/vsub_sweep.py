#!/usr/bin/env python3
"""lab1 launch-geometry sweep: GB/s of c = a - b for [grid, block] pairs at the
BASELINE size (fp32 2^26, fp64 2^25), plus torch's own sub/copy as a bandwidth
reference. One JSON line per point."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402


def time_us(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def main():
    dev = torch.device("cuda:0")
    for dtype, n in ((torch.float32, 1 << 26), (torch.float64, 1 << 25)):
        a = torch.rand(n, dtype=dtype, device=dev)
        b = torch.rand(n, dtype=dtype, device=dev)
        c = torch.empty_like(a)
        byts = 3 * n * a.element_size()
        name = str(dtype).split(".")[-1]
        for tag, fn in (("torch_sub", lambda: torch.sub(a, b, out=c)), ("torch_copy", lambda: c.copy_(a))):
            us = time_us(fn)
            nb = byts if tag == "torch_sub" else 2 * n * a.element_size()
            print(json.dumps({"dtype": name, "what": tag, "us": round(us, 1), "TBps": round(nb / us / 1e6, 3)}))
        L = _native.tune_lib()  # the variants live in libmpx_tune.so
        fp64 = int(dtype == torch.float64)
        for kind, what in ((0, "1vec"), (1, "2vec"), (2, "1vec_ntload"), (3, "2vec_ntload")):
            for block in (256, 1024):
                us = time_us(lambda: _native.check(L.mpx_vsub_variant(a.data_ptr(), b.data_ptr(), c.data_ptr(), n, fp64,
                                                                      kind, block, 0)))
                ok = torch.equal(c, a - b)
                print(json.dumps({"dtype": name, "variant": what, "block": block, "us": round(us, 1),
                                  "TBps": round(byts / us / 1e6, 3), "ok": ok}), flush=True)
        if os.environ.get("VSUB_VARIANTS_ONLY"):
            continue
        for grid in (0, 256, 512, 1024, 2048, 4096, 8192, 16384):
            for block in (256, 512, 1024):
                if grid == 0 and block != 256:
                    continue
                us = time_us(lambda: ops.vsub(a, b, c, grid=grid, block=block))
                print(json.dumps({"dtype": name, "grid": grid, "block": block, "us": round(us, 1),
                                  "TBps": round(byts / us / 1e6, 3)}), flush=True)
        del a, b, c


if __name__ == "__main__":
    main()
