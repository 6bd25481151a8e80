"""lab5 sort timing on one GPU: mpx sort_ (radix / counting sort; scratch from
torch's caching allocator) vs torch.sort (rocPRIM radix sort, into a
preallocated ``out=(values, indices)`` pair — torch has no keys-only sort, so
its time includes producing int64 indices) vs the C reference (qsort, serial;
OpenMP merge sort in the cpu_omp build), uniform random arrays. Every timed
launch sorts the original data (restored outside the events). One JSON line
per (dtype, n)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import ops  # noqa: E402


def gpu_ms(fn, src, iters=int(os.environ.get("LAB5_ITERS", "5"))):
    work = src.clone()
    for _ in range(3):  # warm-up: module load, allocator, clocks (the first path timed ran ~4% slow otherwise)
        work.copy_(src)
        fn(work)
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


def variant_sort(x, variant):
    from cuda_mpi_openmp_amd import _native
    from cuda_mpi_openmp_amd.ops.sort import DTYPES

    L = _native.lib()
    dt = DTYPES[x.dtype]
    nb = int(L.mpx_sort_workspace_bytes(x.numel(), dt))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
    _native.check(_native.tune_lib().mpx_sort_variant(x.data_ptr(), x.numel(), dt, ws.data_ptr(), nb, variant, _native.stream_of(x)))


def main():
    dev = torch.device("cuda:0")
    # LAB5_DTYPES=int32,float32 / LAB5_LOGN=26 / LAB5_VARIANTS=3,4 narrow a profiling run
    dts = [getattr(torch, d) for d in os.environ.get("LAB5_DTYPES", "int32,float32,uint8").split(",")]
    lgs = [int(v) for v in os.environ.get("LAB5_LOGN", "16,20,24,26").split(",")]
    only = {int(v) for v in os.environ.get("LAB5_VARIANTS", "1,2,4,7,8").split(",")}
    for dt in dts:
        for lg in lgs:
            n = 1 << lg
            if dt == torch.uint8:
                src = torch.randint(0, 256, (n,), dtype=dt, device=dev)
            elif dt == torch.int32:
                src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=dt, device=dev)
            else:
                src = torch.randn(n, device=dev)
            ms, out = gpu_ms(ops.sort_, src)
            variants = {}
            if dt != torch.uint8:
                for v, nm in ((1, "onesweep"), (2, "reduce_scan"), (4, "reduce_scan_persistent_r2"),
                              (7, "lean_scatter"), (8, "lean_scatter_tile4096"), (9, "lean_rtn_rank"),
                              (10, "lean_rtn_rank_tile4096"), (20, "hot_rank"), (21, "hot_rank_tile4096"),
                              (22, "hot_rank_tile16384")):
                    if v not in only:
                        continue
                    try:
                        vms, vout = gpu_ms(lambda x, v=v: variant_sort(x, v), src)
                    except Exception as e:  # noqa: BLE001  (an older libmpx via MPX_LIB_PATH lacks the variant)
                        variants[nm] = {"error": str(e)[:80]}
                        continue
                    variants[nm] = {"ms": round(vms, 3), "ok": bool(torch.equal(vout, out))}
            vals, idx = torch.empty_like(src), torch.empty(src.shape, dtype=torch.int64, device=dev)
            tms, _ = gpu_ms(lambda x: torch.sort(x, out=(vals, idx)), src)
            ref = vals
            ok = torch.equal(out, ref)
            rec = {"workload": "lab5_sort", "dtype": str(dt).split(".")[-1], "n": n, "mpx_ms": round(ms, 3),
                   "torch_sort_ms": round(tms, 3), "torch_sort_note": "key+int64 index sort into preallocated out", "mkeys_s": round(n / ms / 1e3, 1), "verified_vs_torch": ok, "variants": variants}
            if lg <= 24:
                host = src.cpu()
                t0 = time.perf_counter()
                ops.sort_(host)
                rec["cpu_qsort_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
                rec["speedup_vs_cpu"] = round(rec["cpu_qsort_ms"] / ms, 1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
