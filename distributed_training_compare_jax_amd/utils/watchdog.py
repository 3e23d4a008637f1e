"""Fail-fast hang detection (the reference has no timeouts, signals or try/except).

Two layers:

* the process group is created with a finite ``timeout`` (``parallel/dist.py``), so a
  collective that never completes raises on every rank instead of blocking forever;
* :class:`Watchdog` — a daemon thread fed a heartbeat after every completed step.  If no step
  completes within ``timeout_s`` (a hung kernel, a peer that died mid-collective, a stuck data
  source) it prints which rank stalled at which step plus every thread's Python stack, then
  terminates the process with exit code 124 so the launcher (torchrun / ``main.py``'s spawn)
  tears the job down instead of leaving the other ranks spinning.
"""

from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time


class Watchdog:
    def __init__(self, rank: int, timeout_s: float, enabled: bool = True, exit_fn=None):
        self.rank = rank
        self.timeout_s = float(timeout_s)
        self.enabled = bool(enabled) and self.timeout_s > 0
        self.step = -1
        self.last = time.monotonic()
        self.fired = False
        self._stop = threading.Event()
        self._exit = exit_fn or (lambda code: os._exit(code))
        self._thread = None

    def start(self):
        if self.enabled and self._thread is None:
            self.last = time.monotonic()
            self._thread = threading.Thread(target=self._run, name=f"dtc-watchdog-r{self.rank}", daemon=True)
            self._thread.start()
        return self

    def beat(self, step: int):
        self.step = step
        self.last = time.monotonic()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def _run(self):
        poll = max(0.05, min(10.0, self.timeout_s / 4))
        while not self._stop.wait(poll):
            idle = time.monotonic() - self.last
            if idle > self.timeout_s:
                self.fired = True
                sys.stderr.write(f"[rank {self.rank}] watchdog: no training-step progress for {idle:.0f}s "
                                 f"(last completed step {self.step}); dumping stacks and aborting\n")
                sys.stderr.flush()
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                self._exit(124)
                return
