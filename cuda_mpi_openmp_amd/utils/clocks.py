"""Board clock / power / temperature sampler (VERDICT r4 Next #2).

A daemon thread that reads the GPU's SMU metrics table at a fixed rate
(default 200 Hz) while a benchmark runs, so a rate change between the timed
phases can be put next to what the board did at the same moment: graphics
clock (per XCD where reported), memory and fabric clocks, socket power,
hotspot / memory temperature, GFX activity and the throttle status word.

Sources, first that works:

* ``amdsmi`` (ROCm's SMI library, importable on this image):
  ``amdsmi_get_gpu_metrics_info`` — the SMU's gpu_metrics table;
* hwmon sysfs of the card (``freq1_input`` = SCLK in Hz, ``power1_average``
  or ``power1_input`` in uW, ``temp*_input`` in m°C).

Read-only: nothing here changes clocks, power caps or any other setting.
Every sample carries the node's CLOCK_MONOTONIC time in ns, the same clock
parallel/timing.py stamps the timed regions with.
"""

from __future__ import annotations

import glob
import os
import statistics
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

# metrics-table fields worth keeping (scalars; lists are averaged as <name>_mean
# and their max kept as <name>_max)
FIELDS = ("current_gfxclk", "current_gfxclks", "average_gfxclk_frequency", "current_uclk", "average_uclk_frequency",
          "current_fclk", "current_socclk", "current_socclks", "average_socket_power", "current_socket_power",
          "temperature_hotspot", "temperature_mem", "temperature_edge", "average_gfx_activity",
          "average_umc_activity", "throttle_status", "indep_throttle_status", "gfxclk_lock_status",
          "energy_accumulator", "accumulation_counter", "prochot_residency_acc", "ppt_residency_acc",
          "socket_thm_residency_acc", "vr_thm_residency_acc", "hbm_thm_residency_acc")


def _clock_ns() -> int:
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def _num(v) -> Optional[float]:
    if isinstance(v, bool):
        return float(v)
    if isinstance(v, (int, float)):
        # amdsmi marks unsupported fields with all-ones sentinels
        if v in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF, 0xFF):
            return None
        return float(v)
    return None


def _flatten(m: dict) -> Dict[str, float]:
    out: Dict[str, float] = {}
    for k in FIELDS:
        if k not in m:
            continue
        v = m[k]
        if isinstance(v, (list, tuple)):
            vals = [x for x in (_num(e) for e in v) if x is not None]
            if vals:
                out[k + "_mean"] = sum(vals) / len(vals)
                out[k + "_max"] = max(vals)
                out[k + "_min"] = min(vals)
        else:
            x = _num(v)
            if x is not None:
                out[k] = x
    return out


def _try(fn):
    try:
        return fn()
    except Exception:  # noqa: BLE001
        return None


def _bdf_match(full: Optional[str], bdf: str) -> bool:
    """``full`` ("0000:03:00.0") names the device ``bdf`` ("0000:03:00")?"""
    if not full:
        return False
    f, b = full.lower().strip(), bdf.lower().strip()
    return f == b or f.startswith(b + ".")


class _AmdSmi:
    def __init__(self, bdf: Optional[str]):
        import amdsmi

        self.a = amdsmi
        amdsmi.amdsmi_init()
        try:
            hs = amdsmi.amdsmi_get_processor_handles()
            if not hs:
                raise RuntimeError("amdsmi: no GPU handles")
            self.h = hs[0]
            if bdf:
                # the rank's own GPU or nothing (never another GPU's
                # clocks under this rank's name); amdsmi BDFs carry the PCI
                # function ("0000:03:00.0"), ours stop at the device
                mine = [h for h in hs if _bdf_match(_try(lambda h=h: amdsmi.amdsmi_get_gpu_device_bdf(h)), bdf)]
                if not mine:
                    raise RuntimeError(f"amdsmi: no GPU with BDF {bdf}")
                self.h = mine[0]
            self.read()  # fail here, not in the thread
        except Exception:
            self.close()  # the library was initialised: shut it down before falling back
            raise

    def read(self) -> Dict[str, float]:
        return _flatten(self.a.amdsmi_get_gpu_metrics_info(self.h))

    def close(self):
        try:
            self.a.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass


class _Hwmon:
    def __init__(self, bdf: Optional[str] = None):
        cands = sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*"))
        if bdf:  # the card whose PCI device is this rank's GPU, or nothing
            cands = [c for c in cands if _bdf_match(os.path.basename(os.path.realpath(c.split("/hwmon/")[0])), bdf)]
            if not cands:
                raise RuntimeError(f"hwmon: no card with BDF {bdf}")
        if not cands:
            raise RuntimeError("no hwmon directory for a GPU")
        self.d = cands[0]
        self.files = {}
        for name, key, scale in (("freq1_input", "current_gfxclk", 1e-6), ("freq2_input", "current_uclk", 1e-6),
                                 ("power1_average", "average_socket_power", 1e-6),
                                 ("power1_input", "current_socket_power", 1e-6),
                                 ("temp1_input", "temperature_edge", 1e-3), ("temp2_input", "temperature_hotspot", 1e-3),
                                 ("temp3_input", "temperature_mem", 1e-3)):
            p = os.path.join(self.d, name)
            if os.access(p, os.R_OK):
                self.files[key] = (p, scale)
        if not self.files:
            raise RuntimeError(f"{self.d}: nothing readable")
        self.read()

    def read(self) -> Dict[str, float]:
        out = {}
        for k, (p, sc) in self.files.items():
            try:
                with open(p) as f:
                    out[k] = float(f.read().strip()) * sc
            except (OSError, ValueError):
                pass
        return out

    def close(self):
        pass


class ClockSampler:
    """``with ClockSampler(hz=200) as cs: ...`` then ``cs.samples`` = [(t_ns, {field: value})].
    ``cs.source`` names the backend; ``cs.error`` says why sampling is off."""

    def __init__(self, hz: float = 200.0, bdf: Optional[str] = None):
        self.period = 1.0 / max(1.0, hz)
        self.samples: List[Tuple[int, Dict[str, float]]] = []
        self.read_us: List[float] = []
        self.source: Optional[str] = None
        self.error: Optional[str] = None
        self._src = None
        errs = []
        for name, mk in (("amdsmi", lambda: _AmdSmi(bdf)), ("hwmon", lambda: _Hwmon(bdf))):
            try:
                self._src = mk()
                self.source = name
                break
            except Exception as e:  # noqa: BLE001
                errs.append(f"{name}: {type(e).__name__}: {e}")
        if self._src is None:
            self.error = "; ".join(errs)
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def _loop(self):
        nxt = time.monotonic()
        while not self._stop.is_set():
            t0 = _clock_ns()
            try:
                m = self._src.read()
            except Exception as e:  # noqa: BLE001
                self.error = f"read: {type(e).__name__}: {e}"
                return
            t1 = _clock_ns()
            self.samples.append(((t0 + t1) // 2, m))
            self.read_us.append((t1 - t0) / 1e3)
            nxt += self.period
            d = nxt - time.monotonic()
            if d > 0:
                self._stop.wait(d)
            else:
                nxt = time.monotonic()

    def start(self) -> "ClockSampler":
        if self._src is not None and self._t is None:
            self._t = threading.Thread(target=self._loop, name="mpx-clock-sampler", daemon=True)
            self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2.0)
            if self._t.is_alive():  # still inside a read: never close the source under it
                self.error = (self.error or "") + "sampler thread did not exit within 2 s; source left open"
                return
        if self._src is not None:
            self._src.close()
            self._src = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def window(self, t0_ns: int, t1_ns: int, pad_ns: int = 0) -> List[Dict[str, float]]:
        return [m for t, m in self.samples if t0_ns - pad_ns <= t <= t1_ns + pad_ns]

    def summary(self, t0_ns: int, t1_ns: int, keys: Optional[List[str]] = None, pad_ns: int = 0) -> dict:
        """Median / min / max of each field over samples inside [t0, t1]."""
        ws = self.window(t0_ns, t1_ns, pad_ns)
        out: dict = {"samples": len(ws)}
        if not ws:
            return out
        ks = keys or sorted({k for m in ws for k in m})
        for k in ks:
            vals = [m[k] for m in ws if k in m]
            if vals:
                out[k] = {"med": round(statistics.median(vals), 3), "min": round(min(vals), 3),
                          "max": round(max(vals), 3)}
        return out

    def rate_hz(self) -> Optional[float]:
        if len(self.samples) < 2:
            return None
        return (len(self.samples) - 1) / ((self.samples[-1][0] - self.samples[0][0]) / 1e9)


class ProcessClockSampler(ClockSampler):
    """The same sampler in a child process (this file run as a script), so its
    reads never take the benchmark's GIL: a 100 Hz thread in the benchmark
    process cost the steady windows 2-3 % of their rate and made the first one
    up to 25 % slow (round 6, profiles/lab2_conv.md). The child appends one
    line per sample to a temporary file; ``stop()`` ends it (its exact PID)
    and reads the file back. The child reads the SMU through amdsmi / sysfs
    only; it never initialises the GPU's compute stack."""

    def __init__(self, hz: float = 200.0, bdf: Optional[str] = None, ready_s: float = 30.0):
        self.period = 1.0 / max(1.0, hz)
        self.samples = []
        self.read_us = []
        self.source = None
        self.error = None
        self._src = None
        self._t = None
        self._stop = threading.Event()
        self._hz, self._bdf, self._ready_s = hz, bdf, ready_s
        self._proc = None
        self._path = None

    def start(self) -> "ProcessClockSampler":
        import json
        import subprocess
        import sys
        import tempfile

        if self._proc is not None:
            return self
        fd, self._path = tempfile.mkstemp(prefix="mpx-clocks-", suffix=".txt")
        os.close(fd)
        cmd = [sys.executable, os.path.abspath(__file__), "--hz", str(self._hz), "--out", self._path]
        if self._bdf:
            cmd += ["--bdf", self._bdf]
        self._proc = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL,
                                      stderr=subprocess.DEVNULL)
        t_end = time.monotonic() + self._ready_s
        while time.monotonic() < t_end:  # the header line: source, or why there is none
            with open(self._path) as f:
                head = f.readline()
            if head.endswith("\n"):
                h = json.loads(head)
                self.source, self.error = h.get("source"), h.get("error")
                break
            if self._proc.poll() is not None:
                self.error = f"sampler process exited rc={self._proc.returncode} before its header"
                break
            time.sleep(0.01)
        else:
            self.error = f"sampler process not ready within {self._ready_s} s"
        return self

    def stop(self) -> None:
        import json

        p, self._proc = self._proc, None
        if p is None:
            return
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(timeout=5)
            except Exception:  # noqa: BLE001
                p.kill()
                p.wait(timeout=5)
        try:
            with open(self._path) as f:
                lines = f.read().splitlines()
        finally:
            os.unlink(self._path)
        for ln in lines[1:]:
            try:
                t, us, m = ln.split("\t", 2)
                self.samples.append((int(t), json.loads(m)))
                self.read_us.append(float(us))
            except ValueError:
                pass  # a line cut by the termination


def _child_main(argv=None) -> int:
    """``clocks.py --hz H --out FILE [--bdf B]``: ProcessClockSampler's child."""
    import argparse
    import json
    import signal

    ap = argparse.ArgumentParser()
    ap.add_argument("--hz", type=float, default=100.0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--bdf", default=None)
    a = ap.parse_args(argv)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    parent = os.getppid()  # a parent that dies without stop() must not leave this loop running
    cs = ClockSampler(hz=a.hz, bdf=a.bdf)
    with open(a.out, "a") as f:
        f.write(json.dumps({"source": cs.source, "error": cs.error}) + "\n")
        f.flush()
        if cs._src is None:
            return 0
        period = 1.0 / max(1.0, a.hz)
        nxt = time.monotonic()
        while not stop.is_set() and os.getppid() == parent:
            t0 = _clock_ns()
            try:
                m = cs._src.read()
            except Exception:  # noqa: BLE001
                break
            t1 = _clock_ns()
            f.write(f"{(t0 + t1) // 2}\t{(t1 - t0) / 1e3:.1f}\t{json.dumps(m)}\n")
            f.flush()
            nxt += period
            d = nxt - time.monotonic()
            if d > 0:
                stop.wait(d)
            else:
                nxt = time.monotonic()
    cs._src.close()
    return 0


def key_fields(summary: dict) -> dict:
    """The handful of fields that attribute a rate change, as flat medians."""
    pick = {}
    for k, name in (("current_gfxclks_mean", "gfxclk_mhz"), ("current_gfxclk", "gfxclk_mhz"),
                    ("average_gfxclk_frequency", "gfxclk_avg_mhz"), ("current_uclk", "uclk_mhz"),
                    ("current_fclk", "fclk_mhz"), ("current_socclks_mean", "socclk_mhz"),
                    ("current_socket_power", "power_w"), ("average_socket_power", "power_avg_w"),
                    ("temperature_hotspot", "hotspot_c"), ("temperature_mem", "mem_c"),
                    ("average_gfx_activity", "gfx_activity"), ("throttle_status", "throttle"),
                    ("indep_throttle_status", "indep_throttle")):
        if k in summary and name not in pick:
            pick[name] = summary[k]["med"]
    pick["samples"] = summary.get("samples", 0)
    return pick


def timed_with_clocks(fn: Callable[[], None], sampler: Optional[ClockSampler]) -> Tuple[int, int]:
    """Run fn between two CLOCK_MONOTONIC stamps (for sampler.summary)."""
    t0 = _clock_ns()
    fn()
    return t0, _clock_ns()


if __name__ == "__main__":
    raise SystemExit(_child_main())
