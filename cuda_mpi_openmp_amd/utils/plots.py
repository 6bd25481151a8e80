"""The framework's figures, in one place: the harness's median-time chart
(``Tester.plot``; the PNG the reference's tester.py:325-407 writes, same file
name and content) and the scaling figure of ``tools/scale.py``.

Data shaping is separate from drawing: :func:`median_groups` and
:func:`scaling_series` are plain pandas / list code (unit-tested without a
display), and the two drawing functions take their output. matplotlib is
imported lazily with the Agg backend; without it the drawing functions return
None and the caller keeps its CSV / JSON outputs.
"""

from __future__ import annotations

import json
from typing import Dict, List, Optional, Sequence, Tuple

import pandas as pd


def _pyplot():
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # noqa: BLE001  (no matplotlib: figures are optional)
        return None
    return plt


# ---------------------------------------------------------------- harness chart
def median_groups(df: pd.DataFrame, gpu_label: str = "HIP") -> pd.DataFrame:
    """One row per (device, launch geometry): median kernel ms and sample
    count, labelled ``CPU`` or ``<device>_<geometry json>``; GPU groups first in
    geometry order, the CPU last."""
    d = df.assign(geometry=df["kernel_size"].apply(json.dumps))
    g = (d.groupby(["device", "geometry"], sort=False)["time_kernel_exe_ms"]
         .agg(median_ms="median", samples="size").reset_index())
    g["label"] = [dev if dev == "CPU" else f"{dev}_{geo}" for dev, geo in zip(g["device"], g["geometry"])]
    g["cpu"] = g["device"] == "CPU"
    return g.sort_values(["cpu"], kind="stable").drop(columns="cpu").reset_index(drop=True)


def metadata_note(df: pd.DataFrame, columns: Sequence[str], groups: pd.DataFrame) -> str:
    """The side box: distinct values of the requested metadata columns, then
    the sample count of every bar."""
    lines: List[str] = []
    for col in columns:
        if col in df.columns:
            lines.append(f"{col}: [" + ", \n".join(map(str, df[col].unique())) + "]")
    lines += ["", "Sample Count by Group:"]
    lines += [f"{lab}: {n} samples" for lab, n in zip(groups["label"], groups["samples"])]
    return "\n".join(lines) + "\n"


def annotated_bars(labels: Sequence[str], values: Sequence[float], path: str, *, note: str = "",
                   xlabel: str = "", ylabel: str = "", title: str = "", dpi: int = 300) -> Optional[str]:
    """Bar chart with each value printed on its bar and an optional text box
    to the right of the axes."""
    plt = _pyplot()
    if plt is None:
        return None
    fig, ax = plt.subplots(figsize=(16, 6))
    bars = ax.bar(list(labels), list(values), color="skyblue")
    ax.bar_label(bars, labels=[f"{v:.5f}" for v in values], padding=2)
    if note:
        ax.text(1.02, 0.95, note, transform=ax.transAxes, fontsize=10, va="top",
                bbox=dict(facecolor="white", alpha=0.5))
    ax.set(xlabel=xlabel, ylabel=ylabel, title=title)
    fig.tight_layout()
    fig.savefig(path, dpi=dpi, bbox_inches="tight")
    plt.close(fig)
    return path


# ---------------------------------------------------------------- scaling figure
def scaling_series(rows: List[dict]) -> Tuple[Dict[str, List[Tuple[int, float]]], Dict[str, List[Tuple[int, float]]]]:
    """Per workload: weak-scaling points (N, throughput / 1-rank throughput;
    workloads have different units) and strong-scaling points (N, speedup)."""
    weak: Dict[str, List[Tuple[int, float]]] = {}
    strong: Dict[str, List[Tuple[int, float]]] = {}
    for name in sorted({r["name"] for r in rows}):
        mine = sorted((r for r in rows if r["name"] == name and r["status"] == "ok"), key=lambda r: r["n"])
        if mine and mine[0]["kind"] == "weak":
            base = [r["value"] for r in mine if r["n"] == 1 and r.get("value")]
            if base:
                weak[name] = [(r["n"], r["value"] / base[0]) for r in mine if r.get("value")]
        elif mine:
            pts = [(r["n"], r["speedup"]) for r in mine if r.get("speedup")]
            if pts:
                strong[name] = pts
    return weak, strong


def scaling_figure(rows: List[dict], path: str, title: str) -> Optional[str]:
    """Two panels against the ideal line: weak scaling (relative whole-job
    throughput) and strong scaling (speedup)."""
    plt = _pyplot()
    if plt is None:
        return None
    weak, strong = scaling_series(rows)
    ns = sorted({r["n"] for r in rows})
    fig, axes = plt.subplots(1, 2, figsize=(13, 5))
    panels = ((axes[0], weak, "whole-job throughput / 1-rank throughput", "weak scaling (dotted: ideal)"),
              (axes[1], strong, "speedup vs 1 GPU", "strong scaling: Jacobi 16384^2 fp64"))
    for ax, series, ylabel, sub in panels:
        for name, pts in series.items():
            ax.plot(*zip(*pts), marker="o", label=name)
        ax.plot(ns, ns, ls=":", color="gray", label="ideal")
        ax.set(xlabel="GPUs", ylabel=ylabel, title=sub, xticks=ns)
        ax.legend(fontsize=8)
    fig.suptitle(title)
    fig.tight_layout()
    fig.savefig(path, dpi=150)
    plt.close(fig)
    return path
