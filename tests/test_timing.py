"""parallel/timing.py: the job-span arithmetic and the start-delay hook
(the multi-rank accounting itself runs in tests/test_bench_contract.py)."""

import time

import pytest

from cuda_mpi_openmp_amd.parallel import timing


def test_span_job_vs_slowest_rank():
    # rank 1 starts 300 µs late and runs 100 µs shorter: the job span charges
    # the skew, the slowest rank's own span does not
    s = timing.Span([1_000_000.0, 1_300_000.0], [2_000_000.0, 2_200_000.0])
    assert s.job_s == pytest.approx(1.2e-3)
    assert s.max_rank_s == pytest.approx(1.0e-3)
    assert s.start_skew_s == pytest.approx(0.3e-3)
    assert s.end_skew_s == pytest.approx(0.2e-3)
    f = s.fields(20, "_x")
    assert f["job_span_ms_x"] == pytest.approx(1.2) and f["max_rank_span_ms_x"] == pytest.approx(1.0)
    assert f["per_rank_ms_per_step_x"] == [pytest.approx(0.05), pytest.approx(0.045)]


def test_single_rank_span_has_no_skew():
    s = timing.Span([5.0], [5.0 + 2e6])
    assert s.job_s == s.max_rank_s == pytest.approx(2e-3)
    assert s.start_skew_s == s.end_skew_s == 0.0
    assert timing.Span([0.0], [4e6]).fields(0)["per_rank_ms_per_step"] == [pytest.approx(4.0)]  # steps 0 -> 1


def test_start_delay_hook(monkeypatch):
    monkeypatch.setenv("MPX_BENCH_START_DELAY", "1:20, 3:5")
    t = time.perf_counter()
    assert timing.start_delay(1) == pytest.approx(0.02)
    assert time.perf_counter() - t >= 0.019
    assert timing.start_delay(0) == 0.0
    assert timing.start_delay(3) == pytest.approx(0.005)
    monkeypatch.delenv("MPX_BENCH_START_DELAY")
    assert timing.start_delay(1) == 0.0


def test_aligned_start_is_immediate_without_ranks():
    class One:
        is_distributed = False

    t = timing.clock_ns()
    assert timing.aligned_start(One()) - t < 50_000_000  # no collective, no margin spin
