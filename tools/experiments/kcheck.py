#!/usr/bin/env python3
"""Large-image correctness sweep of the lab2 kernels against the CPU reference
(sizes that force multi-tile chunks, partial strips and partial tiles)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402


def main():
    L = _native.lib()
    T = _native.tune_lib()  # variants / probes live in libmpx_tune.so
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for (h, w) in ((4096, 4096), (4100, 1024), (2047, 1028), (999, 4096), (517, 333), (3, 1001)):
        img = torch.randint(0, 256, (h, w, 4), dtype=torch.uint8)
        d = img.to(dev)
        for fname in ("roberts", "sobel5_dense", "sobel5"):
            f = ops.get_filter(fname)
            cpu = ops.conv(img, f)
            res = {"hw": [h, w], "filter": fname}
            res["production"] = torch.equal(ops.conv(d, f).cpu(), cpu)
            if w % 4 == 0 and not f.separable:
                wx, wy = f.c_taps()
                for rpt in (4, 8, 16):
                    for chunk in (1, 2, 3, 8):
                        o = torch.empty_like(d)
                        _native.check(T.mpx_conv_variant(d.data_ptr(), o.data_ptr(), w, h, f.k, 0, rpt, chunk, 1, wx, wy,
                                                         0))
                        res[f"rpt{rpt}c{chunk}"] = torch.equal(o.cpu(), cpu)
                for seg in (1, 7, 32, 100):
                    o = torch.empty_like(d)
                    _native.check(T.mpx_conv_variant(d.data_ptr(), o.data_ptr(), w, h, f.k, 1, seg, 0, 1, wx, wy, 0))
                    res[f"wave{seg}"] = torch.equal(o.cpu(), cpu)
            if fname == "roberts":
                for g in (((32, 32), (16, 16)), ((64, 4), (64, 64)), ((16, 16), (1024, 1024))):
                    res[f"geom{g}"] = torch.equal(ops.roberts(d, geometry=g).cpu(), cpu)
                res["cpu_roberts_eq_conv"] = torch.equal(ops.roberts(img), cpu)
            bad = [k for k, v in res.items() if v is False]
            res["all_ok"] = not bad
            print(json.dumps(res if bad else {"hw": [h, w], "filter": fname, "all_ok": True}), flush=True)


if __name__ == "__main__":
    main()
