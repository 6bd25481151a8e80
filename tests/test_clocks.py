"""utils/clocks.py (VERDICT r4 Next #2): the board-metrics sampler's bookkeeping
on CPU — source selection degrades to an error string without a GPU, and the
per-phase summaries / key fields work on injected samples. The GPU box runs it
for real (bench.py --clocks, tools/experiments/sustain_clocks.py)."""

from cuda_mpi_openmp_amd.utils import clocks


def test_flatten_keeps_scalars_and_reduces_lists():
    m = {"current_gfxclks": [2400, 2390, 0xFFFF], "current_socket_power": 1400, "temperature_hotspot": 0xFFFF,
         "unrelated": 5, "throttle_status": True}
    f = clocks._flatten(m)
    assert f["current_gfxclks_mean"] == 2395 and f["current_gfxclks_min"] == 2390
    assert f["current_socket_power"] == 1400.0 and "temperature_hotspot" not in f and "unrelated" not in f
    assert f["throttle_status"] == 1.0


def test_summary_windows_and_key_fields():
    cs = clocks.ClockSampler.__new__(clocks.ClockSampler)
    cs.samples = [(t * 1_000_000, {"current_gfxclks_mean": 2400.0 - t, "current_socket_power": 300.0 + 10 * t})
                  for t in range(100)]
    s = cs.summary(10_000_000, 20_000_000)
    assert s["samples"] == 11 and s["current_gfxclks_mean"]["med"] == 2385.0
    assert s["current_socket_power"]["min"] == 400.0 and s["current_socket_power"]["max"] == 500.0
    assert cs.summary(10_500_000, 10_600_000)["samples"] == 0
    assert cs.summary(10_500_000, 10_600_000, pad_ns=1_000_000)["samples"] == 2
    k = clocks.key_fields(s)
    assert k["gfxclk_mhz"] == 2385.0 and k["power_w"] == 450.0 and k["samples"] == 11
    assert abs(cs.rate_hz() - 1000.0) < 1e-6


def test_sampler_without_gpu_reports_why():
    cs = clocks.ClockSampler(hz=50)
    try:
        if cs.source is None:
            assert cs.error and ("amdsmi" in cs.error or "hwmon" in cs.error)
        cs.start()
    finally:
        cs.stop()


def test_bdf_matching_is_strict():
    """a rank's clocks come from its own GPU or from nowhere."""
    assert clocks._bdf_match("0000:03:00.0", "0000:03:00") and clocks._bdf_match("0000:03:00.0", "0000:03:00.0")
    assert not clocks._bdf_match("0000:13:00.0", "0000:03:00") and not clocks._bdf_match(None, "0000:03:00")
    cs = clocks.ClockSampler(hz=50, bdf="ffff:ff:1f")  # no such device anywhere
    assert cs.source is None and cs.error


def test_stop_leaves_a_busy_source_open():
    """stop() never closes the metrics source under a read still in
    flight (the join timed out): it records why instead."""
    import threading
    import time

    gate = threading.Event()

    class Slow:
        closed = False

        def read(self):
            gate.wait(10)
            return {}

        def close(self):
            Slow.closed = True

    cs = clocks.ClockSampler.__new__(clocks.ClockSampler)
    cs.period, cs.samples, cs.read_us, cs.error, cs._src, cs.source = 0.01, [], [], None, Slow(), "fake"
    cs._stop, cs._t = threading.Event(), None
    cs.start()
    time.sleep(0.05)  # the thread is inside read()
    cs.stop()         # join(2 s) times out
    assert not Slow.closed and "did not exit" in cs.error
    gate.set()
    cs._t.join(5)
