"""Job-span timing of N-rank benchmark regions (VERDICT r4 Next #1).

Every rank of a one-node job reads the same ``CLOCK_MONOTONIC``, so the
whole job's time for a timed region is directly computable: each rank records
``t0`` when it leaves the opening barrier + device sync and ``t1`` at its own
closing device sync; the job ran from the first rank's start to the last
rank's end, ``max(t1) - min(t0)``. Rates are computed from that span. The
slowest rank's own span ``max(t1_i - t0_i)`` (the round-4 figure) is kept
beside it: it never charges start skew between ranks (a rank that leaves the
barrier late, or whose first launch stalls, while its neighbours already run
independent steps), so it can only over-state the rate.

:func:`aligned_start` starts every rank at one agreed instant of that clock
after the opening barrier + device sync, so the ranks' host wake-up jitter
out of the barrier does not count as start skew.

Both need ONE clock: on a multi-node job (``LOCAL_WORLD_SIZE != WORLD_SIZE``
or differing host names, :func:`shared_clock`) the ranks' monotonic clocks are
unrelated, so :func:`aligned_start` falls back to the barrier alone and a
:class:`Span` reports the slowest rank's own span as the job time
(``clock: "per-rank"`` in its fields) instead of mixing clocks.

``MPX_BENCH_START_DELAY="rank:ms[,rank:ms...]"`` sleeps on the named ranks
between the aligned start and ``t0``: a fault-injection hook that creates a
known start skew for the tests (tests/test_bench_contract.py).

Reference: the reference times only events around one kernel launch
(/root/reference/lab2/src/to_plot.cu:101-122); it has no multi-rank timing.
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import List

from .collectives import all_gather_floats, max_over_ranks


def clock_ns() -> int:
    """The node-wide monotonic clock every rank shares."""
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


_SHARED: dict = {}


def shared_clock(ctx) -> bool:
    """Collective (once per world): do all ranks read one CLOCK_MONOTONIC, i.e.
    run on one host? False when the launcher reports fewer node-local ranks
    than ranks, or when the gathered host names differ."""
    if not getattr(ctx, "is_distributed", False):
        return True
    key = (ctx.world, ctx.rank)
    if key not in _SHARED:
        import socket

        from .collectives import all_gather_object

        lw = os.environ.get("LOCAL_WORLD_SIZE")
        local_ok = lw is None or int(lw) == ctx.world
        names = all_gather_object((socket.gethostname(), local_ok), ctx)
        _SHARED[key] = len({n for n, _ in names}) == 1 and all(ok for _, ok in names)
    return _SHARED[key]


def aligned_start(ctx, margin_ns: int = 1_000_000) -> int:
    """A common start instant for every rank: the latest rank's clock reading
    plus ``margin_ns``, agreed with one all-reduce, then each rank spins on the
    shared clock until it passes. A barrier's exit times differ by the host
    wake-up latencies (tens of µs — a sizeable share of a 20-step window at
    ~23 µs per step); this start differs by the spin's resolution. A rank that
    learns the agreed instant only after it has passed starts late, and the
    job span charges it. Returns this rank's start reading."""
    if not getattr(ctx, "is_distributed", False):
        return clock_ns()
    if not shared_clock(ctx):  # unrelated clocks: an agreed instant means nothing
        return clock_ns()
    t = max_over_ranks(float(clock_ns()), ctx) + margin_ns
    while clock_ns() < t:
        pass
    return clock_ns()


def start_delay(rank: int) -> float:
    """Seconds slept by the MPX_BENCH_START_DELAY hook on this rank (0 when unset)."""
    spec = os.environ.get("MPX_BENCH_START_DELAY", "").strip()
    if not spec:
        return 0.0
    for part in spec.split(","):
        r, _, ms = part.partition(":")
        if r.strip() and int(r) == rank:
            s = float(ms) / 1e3
            time.sleep(s)
            return s
    return 0.0


@dataclass
class Span:
    """One timed region of a job: every rank's (t0, t1) on the shared clock."""

    t0_ns: List[float]
    t1_ns: List[float]
    shared: bool = True  # every rank read one clock (one node)
    per_rank_s: List[float] = field(init=False)

    def __post_init__(self):
        self.per_rank_s = [(b - a) / 1e9 for a, b in zip(self.t0_ns, self.t1_ns)]

    @property
    def job_s(self) -> float:
        """First rank's start to last rank's end: the time the job took (the
        slowest rank's own span when the ranks' clocks are unrelated)."""
        if not self.shared:
            return self.max_rank_s
        return (max(self.t1_ns) - min(self.t0_ns)) / 1e9

    @property
    def max_rank_s(self) -> float:
        """The slowest rank's own span (does not charge start skew)."""
        return max(self.per_rank_s)

    @property
    def start_skew_s(self) -> float:
        return (max(self.t0_ns) - min(self.t0_ns)) / 1e9 if self.shared else float("nan")

    @property
    def end_skew_s(self) -> float:
        return (max(self.t1_ns) - min(self.t1_ns)) / 1e9 if self.shared else float("nan")

    def fields(self, steps: int, suffix: str = "") -> dict:
        """The JSON fields of this span: job_span_ms, max_rank_span_ms, per-rank
        ms per step and the start/end skews (all ms)."""
        k = max(1, steps)
        skew = (lambda v: round(v * 1e3, 5)) if self.shared else (lambda v: None)
        return {
            f"job_span_ms{suffix}": round(self.job_s * 1e3, 5),
            f"max_rank_span_ms{suffix}": round(self.max_rank_s * 1e3, 5),
            f"start_skew_ms{suffix}": skew(self.start_skew_s),
            f"end_skew_ms{suffix}": skew(self.end_skew_s),
            f"per_rank_ms_per_step{suffix}": [round(t * 1e3 / k, 5) for t in self.per_rank_s],
            f"clock{suffix}": "shared-monotonic" if self.shared else "per-rank",
        }


def gather_span(t0_ns: int, t1_ns: int, ctx) -> Span:
    """Collective: every rank's (t0, t1). Nanoseconds of CLOCK_MONOTONIC travel as
    float64: exact below 2^53 ns (104 days of uptime), rounded to 2 / 4 ns up to
    208 / 416 days — far below the µs-scale spans and skews reported."""
    return Span(all_gather_floats(float(t0_ns), ctx), all_gather_floats(float(t1_ns), ctx), shared_clock(ctx))
