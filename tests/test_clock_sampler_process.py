"""ProcessClockSampler (utils/clocks.py): the SMU sampler in a child process
that bench.py's steady windows use. On a host without a GPU the child reports
why there is no source, start() returns once its header arrived, stop() ends
the child and leaves no file behind; with a fake source the samples come back
with the shared clock's timestamps."""
import os
import time

from cuda_mpi_openmp_amd.utils import clocks


def test_process_sampler_without_source():
    s = clocks.ProcessClockSampler(hz=100).start()
    path = s._path
    assert s.source is None and s.error  # no GPU here: amdsmi / hwmon both refuse
    time.sleep(0.05)
    s.stop()
    assert s.samples == [] and not os.path.exists(path)
    s.stop()  # idempotent


def test_process_sampler_child_writes_samples(tmp_path, monkeypatch):
    """The child's loop with a fake source (run in-process): one header line,
    then one tab-separated line per sample that ProcessClockSampler.stop parses."""
    out = tmp_path / "s.txt"

    class Fake:
        def read(self):
            return {"current_gfxclk": 2100.0}

        def close(self):
            pass

    def init(self, hz=200.0, bdf=None):  # no amdsmi / hwmon probing (slow where they are absent)
        self._src, self.source, self.error = Fake(), "fake", None

    monkeypatch.setattr(clocks.ClockSampler, "__init__", init)
    import signal
    import threading

    t = threading.Timer(0.1, lambda: os.kill(os.getpid(), signal.SIGTERM))
    old = signal.getsignal(signal.SIGTERM)
    try:
        t.start()
        assert clocks._child_main(["--hz", "200", "--out", str(out)]) == 0
    finally:
        t.cancel()
        signal.signal(signal.SIGTERM, old)
    lines = out.read_text().splitlines()
    assert '"source": "fake"' in lines[0] and len(lines) >= 3
    ps = clocks.ProcessClockSampler(hz=200)
    ps._path = str(out)

    class Done:
        def poll(self):
            return 0

    ps._proc = Done()
    ps.stop()
    assert len(ps.samples) == len(lines) - 1 and all(m["current_gfxclk"] == 2100.0 for _, m in ps.samples)
    t0 = [t for t, _ in ps.samples]
    assert t0 == sorted(t0) and abs(t0[-1] - clocks._clock_ns()) < 10e9


def test_process_sampler_child_exits_with_its_parent(tmp_path, monkeypatch):
    """The child's loop ends when its parent is gone (os.getppid changes), so
    a benchmark that dies without stop() leaves no sampler behind."""
    out = tmp_path / "s.txt"

    class Fake:
        def read(self):
            return {"current_gfxclk": 2100.0}

        def close(self):
            pass

    def init(self, hz=200.0, bdf=None):
        self._src, self.source, self.error = Fake(), "fake", None

    monkeypatch.setattr(clocks.ClockSampler, "__init__", init)
    real = os.getppid()
    calls = [0]

    def ppid():
        calls[0] += 1
        return real if calls[0] < 5 else 1  # re-parented after a few samples
    monkeypatch.setattr(clocks.os, "getppid", ppid)
    t0 = time.monotonic()
    assert clocks._child_main(["--hz", "200", "--out", str(out)]) == 0
    assert time.monotonic() - t0 < 5
    assert 2 <= len(out.read_text().splitlines()) <= 6
