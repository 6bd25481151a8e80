#!/usr/bin/env python3
"""Jacobi sweep variants (rows per wave, nontemporal stores) at 16384^2, timed
in one process with interleaved rounds; each checked against the production
sweep bit for bit."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native, ops  # noqa: E402


def main():
    L = _native.tune_lib()  # the variants live in libmpx_tune.so
    dev = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    for dt in (torch.float64, torch.float32):
        u = torch.rand((n + 2, n), dtype=dt, device=dev)
        un = torch.empty_like(u)
        ref = torch.empty_like(u)
        ops.jacobi_sweep(u, ref, 1, n + 1)
        res_t = torch.zeros(1, dtype=dt, device=dev)
        var = {"production": lambda: ops.jacobi_sweep(u, un, 1, n + 1),
               "production+residual": lambda: (res_t.zero_(), ops.jacobi_sweep(u, un, 1, n + 1, res_t))}
        Rs = [int(x) for x in os.environ.get("JBENCH_R", "3,4,5,8,10,16,64").split(",")]
        auxs = [int(x) for x in os.environ.get("JBENCH_AUX", "2,10").split(",")]
        for R in Rs:
            for aux in auxs:  # 18: alternating walk directions
                var[f"R{R}/aux{aux}"] = (lambda R=R, aux=aux: _native.check(L.mpx_jacobi_variant(
                    u.data_ptr(), un.data_ptr(), n, n, 1, n + 1, None, int(dt == torch.float64), R, aux, 0)))
                if os.environ.get("JBENCH_RESID"):
                    var[f"R{R}/aux{aux}+residual"] = (lambda R=R, aux=aux: (res_t.zero_(), _native.check(
                        L.mpx_jacobi_variant(u.data_ptr(), un.data_ptr(), n, n, 1, n + 1, res_t.data_ptr(),
                                             int(dt == torch.float64), R, aux, 0))))
        res = {k: [] for k in var}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for name, fn in var.items():
            un.zero_()
            fn()
            torch.cuda.synchronize()
            assert torch.equal(un[1:n + 1, 1:-1], ref[1:n + 1, 1:-1]), name
        for _ in range(5):
            for name, fn in var.items():
                fn()
                s.record()
                for _ in range(5):
                    fn()
                e.record()
                e.synchronize()
                res[name].append(s.elapsed_time(e) * 1e3 / 5)
        byts = 2 * n * n * u.element_size()
        for name, ts in res.items():
            us = statistics.median(ts)
            print(json.dumps({"dtype": str(dt).split(".")[-1], "variant": name, "us": round(us, 1),
                              "TBps": round(byts / us / 1e6, 3)}), flush=True)
        del u, un, ref


if __name__ == "__main__":
    main()
