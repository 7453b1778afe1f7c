"""Run watchdog: a bounded wall-clock budget per phase of a run, with a diagnostic dump on expiry.

The reference's host ``wait()`` spins on the NIC's done word forever (sw/mlp_mpi_example_f32.cpp:163-168) and the
author documents runs that "never complete" (hw/README:3-4). A multi-GPU run that hangs here (a stream parked on a
peer's flag, an RCCL collective whose peer died) must instead end on its own, non-zero, and say where it stood:

* ``arm(phase)`` starts the phase's budget; ``disarm()`` ends it. A phase that outlives its budget gets the
  ``dump()`` callback's text (the engine's ``debug_status()``: every request slot, the communicator's async error
  and rank count, the P2P flag words and stall counters — all read without blocking on the parked streams)
  written to stderr, then ``on_abort()`` (releases parked streams, aborts the communicator), then the process
  exits with ``exit_code`` via ``os._exit`` (no interpreter teardown that could block on the GPU).
* ``faulthandler.dump_traceback_later`` is armed with extra slack as a backstop that needs no GIL: if the dump
  itself cannot run (the main thread holds the GIL inside a blocking call), Python's C-level watchdog prints every
  thread's traceback and exits.
"""
from __future__ import annotations

import faulthandler
import json
import os
import sys
import threading
import time
from typing import Callable


class Watchdog:
    def __init__(self, timeout_s: float, dump: Callable[[], object] | None = None,
                 on_abort: Callable[[], None] | None = None, exit_code: int = 124, tag: str = "watchdog",
                 backstop_s: float = 60.0):
        self.timeout_s = float(timeout_s)
        self.dump = dump
        self.on_abort = on_abort
        self.exit_code = exit_code
        self.tag = tag
        self.backstop_s = backstop_s
        self.phase: str | None = None
        self.budget_s = self.timeout_s
        self._deadline = None
        self._cv = threading.Condition()
        self._stop = False
        self.fired = False
        self._th = None
        if self.timeout_s > 0:
            self._th = threading.Thread(target=self._run, name=f"{tag}-thread", daemon=True)
            self._th.start()

    def arm(self, phase: str, timeout_s: float | None = None):
        t = self.timeout_s if timeout_s is None else float(timeout_s)
        if t <= 0 or self._th is None:
            return
        with self._cv:
            self.phase = phase
            self.budget_s = t  # what _expire reports (a phase may carry its own budget)
            self._deadline = time.monotonic() + t
            self._cv.notify_all()
        faulthandler.dump_traceback_later(t + self.backstop_s, exit=True)

    def disarm(self):
        if self._th is None:
            return
        with self._cv:
            self.phase = None
            self._deadline = None
            self._cv.notify_all()
        faulthandler.cancel_dump_traceback_later()

    def close(self):
        self.disarm()
        with self._cv:
            self._stop = True
            self._cv.notify_all()

    def _run(self):
        with self._cv:
            while not self._stop:
                if self._deadline is None:
                    self._cv.wait()
                    continue
                left = self._deadline - time.monotonic()
                if left > 0:
                    self._cv.wait(left)
                    continue
                phase, budget = self.phase, self.budget_s
                break
            else:
                return
        self.fired = True
        self._expire(phase, budget)

    def _expire(self, phase, budget=None):
        err = sys.stderr
        budget = self.timeout_s if budget is None else budget
        print(f"[{self.tag}] phase '{phase}' exceeded {budget:.0f} s: dumping state and aborting",
              file=err, flush=True)
        if self.dump is not None:
            try:
                d = self.dump()
                print(f"[{self.tag}] debug_status " + (d if isinstance(d, str) else json.dumps(d, default=str)),
                      file=err, flush=True)
            except Exception as e:  # noqa: BLE001 - diagnostics must not mask the timeout
                print(f"[{self.tag}] debug_status unavailable: {e!r}", file=err, flush=True)
        if self.on_abort is not None:
            try:
                self.on_abort()
            except Exception as e:  # noqa: BLE001
                print(f"[{self.tag}] abort failed: {e!r}", file=err, flush=True)
        err.flush()
        os._exit(self.exit_code)
