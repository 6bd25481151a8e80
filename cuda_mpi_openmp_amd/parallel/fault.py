"""Failure detection for the multi-GPU tier (SURVEY §5 "failure detection /
recovery / fault injection").

A dead or hung rank leaves its neighbours blocked in RCCL forever. The
reference has no timeouts at all (its harness waits on subprocess.run). Here:

* :class:`Watchdog` — a daemon thread that expects :meth:`Watchdog.beat`
  every ``timeout_s`` seconds (one call per completed step). It also polls
  the native communicator's asynchronous error state (``ncclCommGetAsyncError``)
  once per period. On a missed deadline or an RCCL error it reports on
  stderr, aborts the communicator (``ncclCommAbort``, which releases the
  blocked RCCL kernels) and exits the process with :data:`EXIT_HUNG`, so a
  launcher sees a prompt, attributable failure instead of a silent hang.
* ``MPX_FAULT_INJECT="rank:iteration"`` (models/jacobi.py) raises
  :class:`FaultInjected` on one rank, which the tests use to check the path;
  ``MPX_FAULT_INJECT="halo:rank:iteration"`` instead corrupts that rank's
  received halo row before that iteration's sweep (silently wrong data; with
  peer mailboxes its first owned row, which reaches the neighbour one sweep
  later — models/jacobi.py), which the N-rank == one-device verification must
  catch.
* ``MPX_BENCH_START_DELAY="rank:ms"`` (parallel/timing.py) delays one rank's
  start of a timed region: the job-span accounting must charge it.
"""

from __future__ import annotations

import os
import sys
import threading
import time
from typing import Optional

EXIT_HUNG = 75  # EX_TEMPFAIL: the job did not fail by itself, a peer stopped answering


class FaultInjected(RuntimeError):
    """Raised by the MPX_FAULT_INJECT hook (tests of failure detection)."""


def fault_hook(rank: int, it: int) -> bool:
    """Raise on "rank:iteration"; return True on "halo:rank:iteration" (the
    caller corrupts its halo row); False otherwise."""
    spec = os.environ.get("MPX_FAULT_INJECT")
    if not spec:
        return False
    parts = spec.split(":")
    corrupt = parts[0] == "halo"
    r, i = (int(v) for v in parts[-2:])
    if r == rank and i == it:
        if corrupt:
            return True
        raise FaultInjected(f"injected fault on rank {rank} at iteration {it}")
    return False


class Watchdog:
    def __init__(self, ctx, timeout_s: float, what: str = "step", exit_fn=None):
        self.ctx = ctx
        self.timeout_s = float(timeout_s)
        self.what = what
        self.fired: Optional[str] = None
        self._exit = exit_fn if exit_fn is not None else os._exit
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="mpx-watchdog", daemon=True)
        if self.timeout_s > 0:
            self._t.start()

    def beat(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=5)

    def __enter__(self) -> "Watchdog":
        return self

    def __exit__(self, *exc) -> None:
        self.stop()

    def _fire(self, reason: str) -> None:
        self.fired = reason
        print(f"[mpx watchdog] rank {self.ctx.rank}: {reason}; aborting the communicator", file=sys.stderr,
              flush=True)
        nc = getattr(self.ctx, "native", None)
        if nc is not None:
            try:
                nc.abort()
            except Exception:  # noqa: BLE001 - best effort on the way out
                pass
        self._exit(EXIT_HUNG)

    def _run(self) -> None:
        period = max(0.05, min(1.0, self.timeout_s / 4))
        while not self._stop.wait(period):
            nc = getattr(self.ctx, "native", None)
            if nc is not None:
                try:
                    nc.check()
                except Exception as exc:  # noqa: BLE001 - asynchronous RCCL error
                    self._fire(f"RCCL error: {exc}")
                    return
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self._fire(f"no {self.what} completed for {idle:.1f} s (limit {self.timeout_s:.1f} s)")
                return
