"""Harness primitives: the timing-line protocol, per-run records, statistics and
the subprocess runner (reference tester.py:16-166, re-designed).

Protocol: a lab binary prints ``... execution time:
<X ms>`` as the FIRST stdout line; the rest of stdout is the task payload.
"""

from __future__ import annotations

import os
import re
import subprocess
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Sequence

import numpy as np

TIMING_RE = re.compile(r"execution time: <([\d.]+) ms>")


def parse_timing(first_line: str) -> Optional[float]:
    m = TIMING_RE.search(first_line)
    return float(m.group(1)) if m else None


def split_stdout(stdout: str):
    """(timing line, payload) — line 0 is the timing line (reference tester.py:79-84)."""
    head, _, rest = stdout.partition("\n")
    return head, rest


def time_stats(values: Sequence[float]) -> Dict[str, float]:
    a = np.asarray([v for v in values if v is not None], dtype=np.float64)
    if a.size == 0:
        return {}
    return {"mean": float(a.mean()), "median": float(np.median(a)), "min": float(a.min()),
            "max": float(a.max()), "std": float(a.std())}


def print_stats(values: Sequence[float]) -> None:
    st = time_stats(values)
    if not st:
        print("no timings")
        return
    print(f"Mean: {st['mean']} ms")
    print(f"Median: {st['median']} ms")
    print(f"Min: {st['min']} ms")
    print(f"Max: {st['max']} ms")
    print(f"Standard Deviation: {st['std']} ms")


@dataclass
class RunRecord:
    """One binary invocation (reference TaskResult + SubProcessResult)."""

    test_verification_result: Optional[bool] = None
    task_result: Any = None
    time_kernel_exe_ms: Optional[float] = None
    status: bool = False
    err: Optional[str] = None
    debug_data: Dict[str, Any] = field(default_factory=dict)
    wall_ms: Optional[float] = None


def device_tag(binary_path: str, k1, k2) -> str:
    """Per-run output directory tag ``<bin>_<k1>_<k2>`` with the reference's
    character replacements (reference tester.py:103-109)."""
    tag = f"{os.path.basename(binary_path)}_{k1}_{k2}"
    for a, b in ((", ", "_"), (" ", "_"), ("[", "_"), ("]", "_")):
        tag = tag.replace(a, b)
    return tag


def geometry_prefix(k1, k2) -> str:
    """Launch-geometry lines prepended to stdin when both sizes are truthy; a
    list [a, b] becomes two lines (reference tester.py:113-121)."""
    if not (k1 and k2):
        return ""

    def lines(k):
        return f"{k[0]}\n{k[1]}" if isinstance(k, (list, tuple)) else f"{k}"

    return f"{lines(k1)}\n{lines(k2)}\n"


def run_binary(binary_path: str, processor, k1=None, k2=None, return_inp: bool = False,
               timeout: Optional[float] = None, env: Optional[Dict[str, str]] = None) -> RunRecord:
    rec = RunRecord()
    t0 = time.perf_counter()
    try:
        stdin_text, verify_kwargs, debug = processor.pre_process(device_info=device_tag(binary_path, k1, k2))
        rec.debug_data = dict(debug or {})
        binary = getattr(processor, "binary_io", False)
        if getattr(processor, "takes_geometry", True):
            prefix = geometry_prefix(k1, k2)
            stdin_text = (prefix.encode() + stdin_text) if binary else (prefix + stdin_text)
        if return_inp:
            rec.debug_data["input_str"] = stdin_text
        run_env = None
        proc_env = dict(getattr(processor, "env", None) or {})
        proc_env.update(env or {})
        if proc_env:
            run_env = dict(os.environ)
            run_env.update(proc_env)
        proc = subprocess.run([binary_path], input=stdin_text, text=not binary, capture_output=True, check=True,
                              timeout=timeout, env=run_env)
        if binary:
            # lab5: binary payload after a text timing line (benchmark personality only)
            raw = proc.stdout
            if raw.startswith(b"HIP execution time") or raw.startswith(b"CPU execution time"):
                head_b, _, payload = raw.partition(b"\n")
                head = head_b.decode(errors="replace")
            else:
                head, payload = "", raw
        else:
            head, payload = split_stdout(proc.stdout)
        rec.time_kernel_exe_ms = parse_timing(head)
        rec.task_result = processor.get_task_result(payload, **verify_kwargs)
        rec.test_verification_result = processor.verify_result(rec.task_result, **verify_kwargs)
        rec.status = True
    except subprocess.CalledProcessError as e:
        err = e.stderr or ""
        rec.err = (err.decode(errors="replace") if isinstance(err, bytes) else err).strip()
        print(f"[HIP ERROR] {rec.err}")
    except subprocess.TimeoutExpired:
        rec.err = f"timeout after {timeout} s"
        print(f"[TIMEOUT] {binary_path}: {rec.err}")
    except Exception:  # noqa: BLE001 - every failure becomes a failed row, like the reference
        rec.err = traceback.format_exc()
        traceback.print_exc()
    rec.wall_ms = (time.perf_counter() - t0) * 1e3
    return rec

