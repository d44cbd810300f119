"""Budgeted post-measurement extras for ``bench.py``.

After the timed GEMM region ``bench.py`` runs optional extras: the RCCL sweep, the hand-written
one-/two-shot all-reduces, the xGMI probe, four cold-start variants and the control-plane
latencies. Any of them can be slow or, in the worst case, hang (a collective whose peer died, a
notebook pod that never becomes Ready). None of them may cost the headline JSON line, so:

* every extra runs in its own ``try``; an exception is recorded as ``<name>: error`` and the next
  extra runs;
* every extra has its own soft deadline (``deadline()`` inside the extra: cooperative code such as
  ``measure_cold_start`` stops starting runs at it) and the run has an overall budget: an extra whose
  estimate does not fit in what is left is recorded as ``skipped`` and not started;
* a watchdog thread enforces the hard limit: if an extra is still running ``grace_s`` after its own
  deadline (or the overall budget is spent) it is recorded as ``timeout``, rank 0 prints the JSON line
  with everything measured so far, and the process leaves with ``os._exit(124)`` (a hung collective
  cannot be interrupted from Python). Ranks other than 0 leave a few seconds later and print nothing.
  The exit status is 124 whatever the headline verdict: a hang is a failure the driver must see, not
  a footnote in ``extras_status``.

Collective extras (every rank participates) agree on run / skip through ``agree`` (a MIN all-reduce
over the CPU group supplied by bench.py), so no rank enters a collective the others skipped.

The verdict of every extra is in ``extras_status`` in the JSON line: ``ok``, ``error``, ``skipped``
or ``timeout``, with its wall time.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from typing import Callable


TIMEOUT_EXIT = 124  # the exit status of a run whose extra hung (as timeout(1))


class Extras:
    def __init__(self, budget_s: float, t_start: float | None = None, rank: int = 0,
                 emit: Callable[[dict], None] | None = None, agree: Callable[[bool], bool] | None = None,
                 grace_s: float = 10.0, nonzero_rank_delay_s: float = 5.0):
        self.t_start = time.time() if t_start is None else t_start
        self.budget_deadline = self.t_start + budget_s
        self.rank = rank
        self.emit = emit
        self.agree = agree
        self.grace_s = grace_s
        self.timed_out = False
        self.data: dict = {}
        self.status: dict[str, dict] = {}
        self._lock = threading.Lock()
        self._current: str | None = None
        self._current_deadline = float("inf")
        self._done = False
        self._emitted = False
        self._hard_delay = 0.0 if rank == 0 else nonzero_rank_delay_s
        self._wd = threading.Thread(target=self._watchdog, name="bench-extras-watchdog", daemon=True)
        self._wd.start()

    # --- what an extra sees -------------------------------------------------------------------
    def remaining(self) -> float:
        return self.budget_deadline - time.time()

    def deadline(self) -> float:
        """Soft deadline of the running extra (wall clock): stop starting new work after it."""
        return min(self._current_deadline, self.budget_deadline)

    # --- running ------------------------------------------------------------------------------
    def run(self, name: str, fn: Callable[["Extras"], dict | None], est_s: float = 0.0,
            timeout_s: float | None = None, collective: bool = False) -> bool:
        """Run ``fn(self)`` and merge the dict it returns into the report. Returns True when it ran
        to completion. ``est_s``: the least time it needs (skipped when less is left);
        ``timeout_s``: its own soft deadline (``deadline()``), hard limit + grace_s."""
        fits = self.remaining() >= est_s
        if collective and self.agree is not None:
            fits = bool(self.agree(fits))
        if not fits:
            self.status[name] = {"status": "skipped", "reason": f"{self.remaining():.0f} s left of the budget, needs {est_s:.0f} s"}
            return False
        t0 = time.time()
        with self._lock:
            self._current = name
            self._current_deadline = min(self.budget_deadline, t0 + timeout_s) if timeout_s else self.budget_deadline
        try:
            out = fn(self)
            if out:
                self.data.update(out)
            self.status[name] = {"status": "ok", "s": round(time.time() - t0, 2)}
            return True
        except Exception as e:  # noqa: BLE001 - reported, never fatal for the headline
            self.status[name] = {"status": "error", "s": round(time.time() - t0, 2), "error": f"{type(e).__name__}: {e}"[:2000]}
            return False
        finally:
            with self._lock:
                self._current = None
                self._current_deadline = float("inf")

    def skip(self, name: str, reason: str) -> None:
        self.status[name] = {"status": "skipped", "reason": reason}

    def report(self) -> dict:
        return {**self.data, "extras_status": dict(self.status),
                "extras_budget_s": round(self.budget_deadline - self.t_start, 1)}

    def finish(self) -> dict:
        """Stop the watchdog; returns the report for the JSON line."""
        with self._lock:
            self._done = True
        return self.report()

    def emit_once(self, extra: dict | None = None) -> None:
        with self._lock:
            if self._emitted:
                return
            self._emitted = True
        if self.rank == 0 and self.emit is not None:
            self.emit({**self.report(), **(extra or {})})

    # --- hard limit ---------------------------------------------------------------------------
    def _watchdog(self) -> None:
        while True:
            time.sleep(0.2)
            with self._lock:
                if self._done:
                    return
                cur, cur_dl = self._current, self._current_deadline
            hard = min(cur_dl + self.grace_s, self.budget_deadline + self.grace_s) + self._hard_delay
            if cur is not None and time.time() > hard:
                self.timed_out = True
                self.status[cur] = {"status": "timeout", "s": round(time.time() - self.t_start, 1),
                                    "error": "still running past its deadline; the process exits with what it has"}
                try:
                    self.emit_once()
                finally:
                    try:
                        sys.stdout.flush()
                        sys.stderr.flush()
                    finally:
                        os._exit(TIMEOUT_EXIT)


def print_line(line: dict) -> None:
    print(json.dumps(line), flush=True)
