"""Experiment driver: k_times x kernel_sizes runs of the GPU binary (and of the
CPU binary without geometry), statistics, CSV files and the median-time plot
(reference tester.py:169-407, re-designed).

* Runs are executed strictly sequentially — which is what the reference's
  asyncio code effectively did — so GPU runs never
  contend; every run has an optional timeout (new).
* CSV: ``stats_<bin>.csv`` when every run verified, else ``failed_<bin>.csv``,
  in the GPU binary's directory, with the reference's columns plus ``device``,
  ``wall_ms`` and throughput columns (``gpixel_per_s`` for image labs,
  ``gb_per_s`` for lab1). A CPU binary sharing the GPU binary's name gets a
  ``cpu_`` prefix instead of overwriting its CSV.
* Plot: ``median_execution_time.png`` — median kernel ms per (device,
  kernel_size), legend listing ``metadata_columns2plot`` values and sample
  counts; the CPU/GPU speedup of every GPU group is printed as well.
"""

from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, List, Optional

import pandas as pd

from ..utils.plots import annotated_bars, median_groups, metadata_note
from .core import RunRecord, print_stats, run_binary


def _kernel_key(ks) -> str:
    return json.dumps(ks)


class Tester:
    def __init__(self, binary_path_gpu: str, k_times: int, kernel_sizes: List[List[Any]],
                 metadata_columns2plot: Optional[List[str]] = None, binary_path_cpu: Optional[str] = None,
                 return_inp: bool = False, return_task_res: bool = False, timeout: Optional[float] = None,
                 gpu_env: Optional[Dict[str, str]] = None, gpu_label: str = "HIP", compat: bool = False):
        self.binary_path_gpu = binary_path_gpu
        self.binary_path_cpu = binary_path_cpu
        self.k_times = int(k_times)
        self.kernel_sizes = kernel_sizes or [[None, None]]
        self.metadata_columns2plot = list(metadata_columns2plot or [])
        self.return_inp = return_inp
        self.return_task_res = return_task_res
        self.timeout = timeout
        self.gpu_env = gpu_env
        self.gpu_label = gpu_label
        # compat (run_test.py --compat): the reference's CSV schema and file
        # names for a literal replay (processors.COMPAT_DEVIATIONS)
        self.compat = bool(compat)
        self.dir2save = os.path.dirname(os.path.abspath(binary_path_gpu))

    # ------------------------------------------------------------------
    def run_experiment(self, binary_path: str, kernel_sizes, processor, device: str) -> pd.DataFrame:
        bin_name = os.path.splitext(os.path.basename(binary_path))[0]
        print(f"[Experiment bin_name=<{bin_name}>] START")
        t_start = time.time()
        rows: List[Dict[str, Any]] = []
        env = self.gpu_env if device == self.gpu_label else None
        for i in range(self.k_times):
            for k1, k2 in kernel_sizes:
                print(f"[Experiment bin_name=<{bin_name}> task={i} kernel_size=<{[k1, k2]}>] started")
                rec: RunRecord = run_binary(binary_path, processor, k1, k2, self.return_inp, self.timeout, env)
                row: Dict[str, Any] = {
                    "idx_run_time": i,
                    "bin_name": bin_name,
                    "kernel_size": [k1, k2],
                    "test_verification_result": rec.test_verification_result,
                    "time_kernel_exe_ms": rec.time_kernel_exe_ms,
                    "status": rec.status,
                    "err": rec.err,
                }
                if self.return_task_res:
                    row["task_result"] = rec.task_result
                if self.compat:  # reference order: asdict(SubProcessResult) puts task_result second
                    row = {k: row[k] for k in ("idx_run_time", "bin_name", "kernel_size", "test_verification_result",
                                               "task_result", "time_kernel_exe_ms", "status", "err") if k in row}
                row.update(processor.get_attr())
                row.update({k: v for k, v in rec.debug_data.items() if not (self.compat and k == "pixels")})
                row["time_exe_ms_from_start_run_time_bin_name"] = (time.time() - t_start) * 1e3
                if self.compat:
                    rows.append(row)
                    print(f"[Experiment bin_name=<{bin_name}> task={i} kernel_size=<{[k1, k2]}>] finished with "
                          f"`time_kernel_exe_ms`: {rec.time_kernel_exe_ms} ms")
                    continue
                row["wall_ms"] = rec.wall_ms
                row["device"] = device
                row["n_gpus"] = int((env or {}).get("MPX_NGPUS", 1)) if device == self.gpu_label else 0
                row["devices_used"] = int((env or {}).get("MPX_DEVICES_USED", row["n_gpus"] and 1)) \
                    if device == self.gpu_label else 0
                self._throughput(row)
                rows.append(row)
                print(f"[Experiment bin_name=<{bin_name}> task={i} kernel_size=<{[k1, k2]}>] finished with "
                      f"`time_kernel_exe_ms`: {rec.time_kernel_exe_ms} ms")
        df = pd.DataFrame(rows)
        ok = bool(rows) and all(bool(r["test_verification_result"]) for r in rows)
        prefix = "cpu_" if (not self.compat and device != self.gpu_label and self.binary_path_gpu and
                            os.path.basename(binary_path) == os.path.basename(self.binary_path_gpu)) else ""
        if ok:
            print_stats([r["time_kernel_exe_ms"] for r in rows])
            df.to_csv(os.path.join(self.dir2save, f"stats_{prefix}{bin_name}.csv"), index=False)
            print(f"[Experiment bin_name=<{bin_name}>] SUCCESS!")
            if self.compat:  # the plot groups by device, added after the CSV (reference tester.py:313-317)
                df = df.assign(device=device)
            return df
        failed = df[~df["test_verification_result"].fillna(False).astype(bool)] if len(df) else df
        print(f"[Experiment bin_name=<{bin_name}>] FAILED: len={len(failed)}!")
        failed.to_csv(os.path.join(self.dir2save, f"failed_{prefix}{bin_name}.csv"), index=False)
        return pd.DataFrame()

    @staticmethod
    def _throughput(row: Dict[str, Any]) -> None:
        t = row.get("time_kernel_exe_ms")
        if not t:
            return
        if row.get("pixels"):
            row["gpixel_per_s"] = row["pixels"] / (t * 1e-3) / 1e9
        if row.get("vector_size"):
            row["gb_per_s"] = 24.0 * row["vector_size"] / (t * 1e-3) / 1e9  # 2 reads + 1 write of fp64

    # ------------------------------------------------------------------
    def run_experiments(self, processor) -> pd.DataFrame:
        t0 = time.time()
        print("[Experiments] START")
        frames = [self.run_experiment(self.binary_path_gpu, self.kernel_sizes, processor, self.gpu_label)]
        if self.binary_path_cpu:
            frames.append(self.run_experiment(self.binary_path_cpu, [[None, None]], processor, "CPU"))
        df = pd.concat([f for f in frames if len(f)], ignore_index=True) if any(len(f) for f in frames) else \
            pd.DataFrame()
        if len(df):
            if not self.compat:
                self.report_speedup(df)
            self.plot(df)
        print(f"[Experiments] FINISH time exe: {time.time() - t0}")
        return df

    def report_speedup(self, df: pd.DataFrame) -> Optional[pd.DataFrame]:
        """CPU median / GPU median per GPU group (kernel_size, n_gpus): printed
        and persisted as ``speedup_<gpu bin>.csv`` next to the stats CSVs (SURVEY
        §5 ``speedup_vs_cpu``; the reference keeps every run attribute in CSV,
        reference tester.py:254-285)."""
        if "CPU" not in set(df["device"]) or self.gpu_label not in set(df["device"]):
            return None
        cpu_t = df[df["device"] == "CPU"]["time_kernel_exe_ms"]
        cpu = cpu_t.median()
        g = df[df["device"] == self.gpu_label].copy()
        g["ks"] = g["kernel_size"].apply(_kernel_key)
        if "n_gpus" not in g:
            g["n_gpus"] = 1
        rows = []
        for (ks, ng), grp in g.groupby(["ks", "n_gpus"]):
            med = grp["time_kernel_exe_ms"].median()
            if not med:
                continue
            print(f"[Speedup] CPU median {cpu:.5f} ms / {self.gpu_label}_{ks} median {med:.5f} ms = "
                  f"{cpu / med:.1f}x")
            rows.append({"device": self.gpu_label, "kernel_size": ks, "n_gpus": int(ng),
                         "gpu_runs": int(len(grp)), "gpu_median_ms": float(med),
                         "cpu_runs": int(len(cpu_t)), "cpu_median_ms": float(cpu),
                         "speedup_vs_cpu": float(cpu / med)})
        if not rows:
            return None
        out = pd.DataFrame(rows)
        bin_name = os.path.splitext(os.path.basename(self.binary_path_gpu))[0]
        out.to_csv(os.path.join(self.dir2save, f"speedup_{bin_name}.csv"), index=False)
        return out

    def plot(self, df: pd.DataFrame) -> Optional[str]:
        """``median_execution_time.png`` next to the GPU binary (utils/plots.py)."""
        groups = median_groups(df, self.gpu_label)
        return annotated_bars(groups["label"], groups["median_ms"], os.path.join(self.dir2save, "median_execution_time.png"),
                              note=metadata_note(df, self.metadata_columns2plot, groups),
                              xlabel="Device and Kernel Size", ylabel="Median Execution Time (ms)",
                              title="Median Execution Time by Device and Kernel Size")
