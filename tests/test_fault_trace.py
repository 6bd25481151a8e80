"""Failure detection (watchdog, async RCCL errors, fault injection) and roctx
tracing — host-side logic, runs on CPU."""

import subprocess
import sys
import time
import types

import pytest

from cuda_mpi_openmp_amd import parallel
from cuda_mpi_openmp_amd.utils import trace


class FakeNative:
    def __init__(self, fail=False):
        self.fail, self.aborted = fail, False

    def check(self):
        if self.fail:
            raise RuntimeError("RCCL asynchronous error: remote process exited")

    def abort(self):
        self.aborted = True


def _ctx(native=None):
    return types.SimpleNamespace(rank=3, native=native)


def test_watchdog_fires_on_silence():
    codes = []
    nat = FakeNative()
    wd = parallel.Watchdog(_ctx(nat), 0.2, exit_fn=codes.append)
    time.sleep(0.6)
    wd.stop()
    assert codes == [parallel.EXIT_HUNG] and nat.aborted and "no step completed" in wd.fired


def test_watchdog_quiet_while_beating():
    codes = []
    wd = parallel.Watchdog(_ctx(), 0.3, exit_fn=codes.append)
    for _ in range(10):
        time.sleep(0.05)
        wd.beat()
    wd.stop()
    assert codes == [] and wd.fired is None


def test_watchdog_fires_on_async_rccl_error():
    codes = []
    nat = FakeNative(fail=True)
    with parallel.Watchdog(_ctx(nat), 30.0, exit_fn=codes.append) as wd:
        time.sleep(1.3)
    assert codes == [parallel.EXIT_HUNG] and nat.aborted and "RCCL error" in wd.fired


def test_watchdog_disabled_with_zero_timeout():
    wd = parallel.Watchdog(_ctx(), 0)
    assert not wd._t.is_alive()
    wd.stop()


def test_watchdog_exits_process():
    """The real exit path: a child that stops beating exits with EXIT_HUNG."""
    code = ("import time, types; from cuda_mpi_openmp_amd import parallel; "
            "parallel.Watchdog(types.SimpleNamespace(rank=0, native=None), 0.2); time.sleep(30)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == parallel.EXIT_HUNG and "[mpx watchdog] rank 0" in r.stderr


def test_fault_hook(monkeypatch):
    monkeypatch.setenv("MPX_FAULT_INJECT", "1:4")
    parallel.fault_hook(0, 4)
    parallel.fault_hook(1, 3)
    with pytest.raises(parallel.FaultInjected):
        parallel.fault_hook(1, 4)


def test_trace_off_by_default_and_on(monkeypatch):
    monkeypatch.setattr(trace, "_enabled", None)
    monkeypatch.delenv("MPX_ROCTX", raising=False)
    assert not trace.enabled()
    with trace.range("x"):
        pass
    monkeypatch.setattr(trace, "_enabled", None)
    monkeypatch.setenv("MPX_ROCTX", "1")
    on = trace.enabled()  # libroctx64 loads without a GPU; ranges are no-ops without a profiler
    with trace.range("edge.step"):
        trace.mark("m")
    monkeypatch.setattr(trace, "_enabled", None)
    assert on or not __import__("os").path.exists("/opt/rocm/lib/libroctx64.so")
