#!/usr/bin/env python3
"""Summarise gpurun_out/harness_cmp (tools/harness_compare.sh) as markdown:
median kernel ms per (bucket/n, timing, geometry), next to BASELINE.md."""
import glob
import os
import sys

import pandas as pd

# the reference's published medians (RTX A6000, one cold launch per process, ms)
BASELINE = {
    ("lab1", "1000"): {"CPU": 0.004, "[1, 32]": 0.14936, "[4, 64]": 0.14438, "[32, 128]": 0.14429,
                       "[512, 512]": 0.14653, "[1024, 1024]": 0.14592},
    ("lab1", "10000"): {"CPU": 0.081, "[1, 32]": 0.20557, "[4, 64]": 0.14816, "[32, 128]": 0.14064,
                        "[512, 512]": 0.14203, "[1024, 1024]": 0.14280},
    ("lab1", "1000000"): {"CPU": 8.338, "[1, 32]": 11.57053, "[4, 64]": 1.54635, "[32, 128]": 0.20198,
                          "[512, 512]": 0.13456, "[1024, 1024]": 0.13926},
    ("lab2", "small"): {"CPU": 0.001, "[[16, 16], [1024, 1024]]": 0.85797, "[[16, 16], [32, 32]]": 0.16846,
                        "[[2, 2], [16, 16]]": 0.16718, "[[32, 32], [16, 16]]": 0.16693, "[[32, 32], [64, 64]]": 0.17912},
    ("lab2", "medium"): {"CPU": 16.7635, "[[16, 16], [1024, 1024]]": 0.86232, "[[16, 16], [32, 32]]": 0.16573,
                         "[[2, 2], [16, 16]]": 0.26202, "[[32, 32], [16, 16]]": 0.17045, "[[32, 32], [64, 64]]": 0.18253},
    ("lab2", "large"): {"CPU": 37.891, "[[16, 16], [1024, 1024]]": 0.87987, "[[16, 16], [32, 32]]": 0.18054,
                        "[[2, 2], [16, 16]]": 0.51288, "[[32, 32], [16, 16]]": 0.17866, "[[32, 32], [64, 64]]": 0.19272},
}


def vs_baseline(out: "pd.DataFrame") -> None:
    """Per published configuration: reference median, ours cold / warm, cold speedup."""
    for (lab, size), ref in BASELINE.items():
        g = out[(out.lab == lab) & (out["size"] == size)]
        if g.empty:
            continue
        print(f"\n### {lab} {'n = ' + size if lab == 'lab1' else size + ' bucket'}\n")
        print("| launch geometry | reference RTX A6000 (cold) | MI355X cold | MI355X warm | cold speedup |")
        print("|---|---|---|---|---|")
        keys = list(ref) + sorted(k for k in set(g.geometry) if k not in ref and not k.startswith("CPU"))
        for k in keys:
            sel = g[g.geometry == k] if k != "CPU" else g[g.device.str.startswith("CPU")]
            cold = sel[sel.timing == "cold"].median_ms
            warm = sel[sel.timing == "warm"].median_ms
            c = float(cold.iloc[0]) if len(cold) else None
            w = float(warm.iloc[0]) if len(warm) else None
            r = ref.get(k)
            label = {"CPU": "CPU (serial -O0)", "[-1, -1]": "auto (tuned)", "[[0, 0], [0, 0]]": "auto (tuned)"}.get(k, k)
            sp = f"**{r / c:.1f}x**" if r and c else "—"
            fmt = lambda v: "—" if v is None else f"{v:.5f}"  # noqa: E731
            print(f"| {label} | {r if r is not None else '—'} | {fmt(c)} | {fmt(w)} | {sp} |")


args = [a for a in sys.argv[1:] if not a.startswith("--")]
root = args[0] if args else "gpurun_out/harness_cmp"
rows = []
for d in sorted(glob.glob(os.path.join(root, "*", "lab*"))):
    tag = os.path.basename(os.path.dirname(d))
    lab, size, timing, *variant = tag.split("_")  # <lab>_<bucket|n>_<timing>[_literal]
    if variant:
        timing = f"{timing}-{'-'.join(variant)}"
    for f in glob.glob(os.path.join(d, "src", "stats_*.csv")):
        df = pd.read_csv(f)
        dev = "CPU (-O0, 1 thread)" if os.path.basename(f).startswith("stats_cpu_") else "MI355X"
        for ks, g in df.groupby(df["kernel_size"].astype(str)):
            rows.append({"lab": lab, "size": size, "timing": timing, "device": dev, "geometry": ks,
                         "median_ms": g["time_kernel_exe_ms"].median(), "runs": len(g)})
out = pd.DataFrame(rows)
# published GPU/CPU speedups (BASELINE.md derived rows: CPU median / best GPU median)
PUBLISHED_SPEEDUP = {("lab2", "large"): 212.0, ("lab2", "medium"): 101.0, ("lab2", "small"): 0.006,
                     ("lab1", "1000000"): 62.0}
if "--speedups" in sys.argv:
    print("| lab | bucket / n | CPU median ms (serial -O0, this host) | best MI355X median ms cold / warm (geometry) "
          "| speedup cold / warm | published (RTX A6000 vs Xeon, cold) |")
    print("|---|---|---|---|---|---|")
    for (lab, size), g in out.groupby(["lab", "size"], sort=False):
        cpu = g[g.device.str.startswith("CPU")]
        gpu = g[~g.device.str.startswith("CPU")]
        if cpu.empty or gpu.empty:
            continue
        cells = []
        for timing in ("cold", "warm"):
            c = cpu[cpu.timing == timing].median_ms
            gg = gpu[gpu.timing == timing]
            if c.empty or gg.empty:
                cells.append(None)
                continue
            best = gg.loc[gg.median_ms.idxmin()]
            cells.append((float(c.iloc[0]), float(best.median_ms), best.geometry))
        cpu_ms = "/".join(f"{x[0]:.4g}" for x in cells if x)
        gpu_ms = " / ".join(f"{x[1]:.5f} ({x[2]})" for x in cells if x)
        sp = " / ".join(f"**{x[0] / x[1]:.1f}x**" for x in cells if x)
        pub = PUBLISHED_SPEEDUP.get((lab, size))
        print(f"| {lab} | {size} | {cpu_ms} | {gpu_ms} | {sp} | {str(pub) + 'x' if pub else '—'} |")
    sys.exit(0)
if "--like-for-like" in sys.argv:
    # lab2's published [[16,16],[1024,1024]] row under every methodology knob:
    # trimmed vs literal grid (MPX_GEOM_LITERAL=1), preloaded vs lazy code objects
    geo = "[[16, 16], [1024, 1024]]"
    cols = [("cold", "cold, trimmed grid, preloaded"), ("cold-literal", "cold, literal grid, preloaded"),
            ("cold-lazy", "cold, trimmed grid, lazy load"), ("cold-lazy-literal", "cold, literal grid, lazy load"),
            ("warm", "warm, trimmed"), ("warm-literal", "warm, literal")]
    print("| bucket | reference RTX A6000 (cold) | " + " | ".join(c[1] for c in cols) + " |")
    print("|---|---|" + "---|" * len(cols))
    for size in ("small", "medium", "large"):
        g = out[(out.lab == "lab2") & (out["size"] == size) & (out.geometry == geo) & (out.device == "MI355X")]
        cells = []
        for t, _ in cols:
            v = g[g.timing == t].median_ms
            cells.append(f"{float(v.iloc[0]):.5f}" if len(v) else "—")
        print(f"| {size} | {BASELINE[('lab2', size)][geo]} | " + " | ".join(cells) + " |")
    sys.exit(0)
if "--vs-baseline" in sys.argv:
    out["geometry"] = [("CPU" if d.startswith("CPU") else g) for d, g in zip(out.device, out.geometry)]
    vs_baseline(out)
    sys.exit(0)
for (lab, size), g in out.groupby(["lab", "size"], sort=False):
    print(f"\n### {lab} {size}\n")
    piv = g.pivot_table(index=["device", "geometry"], columns="timing", values="median_ms", aggfunc="first")
    print(piv.round(5).to_markdown())
