"""lab5 sort timing on one GPU: mpx_sort (bitonic / counting sort) vs
torch.sort (rocPRIM radix sort) vs the C reference (qsort), uniform random
arrays. One JSON line per (dtype, n)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mpi_openmp_amd import ops  # noqa: E402


def gpu_ms(fn, src, iters=5):
    work = src.clone()
    fn(work)  # warm-up (module load)
    ts = []
    for _ in range(iters):
        work.copy_(src)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(work)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2], work


def main():
    dev = torch.device("cuda:0")
    for dt in (torch.int32, torch.float32, torch.uint8):
        for lg in (16, 20, 24, 26):
            n = 1 << lg
            if dt == torch.uint8:
                src = torch.randint(0, 256, (n,), dtype=dt, device=dev)
            elif dt == torch.int32:
                src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=dt, device=dev)
            else:
                src = torch.randn(n, device=dev)
            ms, out = gpu_ms(ops.sort_, src)
            tms, ref = gpu_ms(lambda x: x.copy_(torch.sort(x).values), src)
            ok = torch.equal(out, ref)
            rec = {"workload": "lab5_sort", "dtype": str(dt).split(".")[-1], "n": n, "mpx_ms": round(ms, 3),
                   "torch_sort_ms": round(tms, 3), "mkeys_s": round(n / ms / 1e3, 1), "verified_vs_torch": ok}
            if lg <= 24:
                host = src.cpu()
                t0 = time.perf_counter()
                ops.sort_(host)
                rec["cpu_qsort_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
                rec["speedup_vs_cpu"] = round(rec["cpu_qsort_ms"] / ms, 1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
