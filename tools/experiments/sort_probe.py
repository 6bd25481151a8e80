"""Radix scatter attribution probe and the returning-add ranking
(sort variant 9) against the production lean scatter (variant 7).

1. knock-outs: mpx_sort_scatter_probe runs count + scan + lean scatter for the
   four digits of the SAME uniform keys with one ranking / staging step removed
   (radix_scatter_lean_kernel KNOCK bits) — under `rocprofv3 --pmc
   SQ_LDS_BANK_CONFLICT ...` the per-kernel counters attribute the conflict
   cycles per step; here the event times do the same for time.
2. variant 9 vs 7: full sorts of int32 / float32 at 2^24 and 2^26, every result
   compared with torch.sort, plus the distributions that stress stability
   (few distinct values, all equal, sorted, reversed, normal floats).
One JSON line per measurement. SORT_PROBE_ITERS (default 7) timed runs each,
SORT_PROBE_PARTS=knock,variants, SORT_PROBE_VARIANTS=7,9, SORT_PROBE_LOGN=24,26,
SORT_PROBE_CASES=float32_normal,... (default: every case) and
SORT_PROBE_SMALL=0|1 narrow a run."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cuda_mpi_openmp_amd import _native  # noqa: E402
from cuda_mpi_openmp_amd.ops.sort import DTYPES  # noqa: E402

ITERS = int(os.environ.get("SORT_PROBE_ITERS", "7"))
PARTS = set(os.environ.get("SORT_PROBE_PARTS", "knock,variants").split(","))
VARIANTS = [int(v) for v in os.environ.get("SORT_PROBE_VARIANTS", "7,9").split(",")]
LOGN = [int(v) for v in os.environ.get("SORT_PROBE_LOGN", "24,26").split(",")]
SMALL = os.environ.get("SORT_PROBE_SMALL", "1") == "1"  # the 2^22 + 37 stability cases
KNOCKS = {0: "production", 1: "linear staging", 6: "no counter read/add (table only)",
          12: "no table, no leader add", 14: "no ranking LDS at all", 16: "write-out without digit lookup",
          31: "all knocked"}


def timed(fn, reset=None, iters=ITERS):
    for _ in range(2):
        if reset:
            reset()
        fn()
    ts = []
    for _ in range(iters):
        if reset:
            reset()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    L = _native.lib()
    dev = torch.device("cuda:0")
    if "knock" in PARTS:
        n = 1 << 26
        x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
        nb = int(L.mpx_sort_workspace_bytes(n, DTYPES[torch.int32]))
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        st = _native.stream_of(x)
        for k, what in KNOCKS.items():
            med, mn = timed(lambda k=k: _native.check(_native.tune_lib().mpx_sort_scatter_probe(x.data_ptr(), n, ws.data_ptr(), nb, k, st)))
            print(json.dumps({"part": "knock", "knock": k, "what": what, "n": n,
                              "ms_4_passes": round(med, 4), "ms_min": round(mn, 4)}), flush=True)
    if "variants" in PARTS:
        cases = []
        for lg in LOGN:
            n = 1 << lg
            cases.append(("int32_uniform", torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)))
            cases.append(("float32_normal", torch.randn(n, device=dev)))
            # skewed digits (RANK 3's hot-digit ballots): passes 2 / 3 one digit, pass 1 four
            cases.append(("int32_range1000", torch.randint(0, 1000, (n,), dtype=torch.int32, device=dev)))
            cases.append(("float32_uniform01", torch.rand(n, device=dev)))
        n = (1 << 22) + 37
        cases += [] if not SMALL else [("int32_few", torch.randint(0, 4, (n,), dtype=torch.int32, device=dev)),
                  ("int32_equal", torch.full((n,), 7, dtype=torch.int32, device=dev)),
                  ("int32_sorted", torch.arange(n, dtype=torch.int32, device=dev)),
                  ("int32_reversed", torch.arange(n, 0, -1, dtype=torch.int32, device=dev)),
                  ("float32_few", (torch.randint(0, 3, (n,), device=dev) - 1).float() * 0.5),
                  ("int32_bytes_skewed", (torch.randint(0, 2, (n,), dtype=torch.int32, device=dev) << 24)
                   | torch.randint(0, 1 << 8, (n,), dtype=torch.int32, device=dev))]
        want = [c for c in os.environ.get("SORT_PROBE_CASES", "").split(",") if c]
        for name, src in cases:
            if want and name not in want:
                continue
            ref = torch.sort(src).values
            n = src.numel()
            dt = DTYPES[src.dtype]
            nb = int(L.mpx_sort_workspace_bytes(n, dt))
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            work = torch.empty_like(src)
            rec = {"part": "variants", "case": name, "n": n}
            for v in VARIANTS:
                def run(v=v):
                    _native.check(_native.tune_lib().mpx_sort_variant(work.data_ptr(), n, dt, ws.data_ptr(), nb, v,
                                                     _native.stream_of(work)))
                med, mn = timed(run, reset=lambda: work.copy_(src))
                rec[f"v{v}_ms"] = round(med, 4)
                rec[f"v{v}_min_ms"] = round(mn, 4)
                rec[f"v{v}_ok"] = bool(torch.equal(work, ref))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
