"""Step tracing: roctx ranges, per-step device time, and a Chrome-trace export.

The reference has no tracing beyond ``time.perf_counter`` around the host loop
(``train/train.py:73,84-85,94``).  Here ``profile: true`` in the train YAML turns on:

* **roctx ranges** (``libroctx64``) around every host phase — data, step enqueue, loss sync,
  checkpoint — visible on the timeline of ``rocprofv3 --marker-trace`` next to the kernels;
* **device step time**: a pair of HIP events around each step's enqueue (recorded on the
  stream outside any graph capture, so it also works when the step replays hipGraphs);
* a **Chrome trace** ``<output_dir>/trace/rank<r>.json`` (host spans + device step spans,
  open in ``chrome://tracing`` / Perfetto) and per-step device times in ``metrics.json``.

With ``profile: false`` every call below is a no-op (no events, no library load).
"""

from __future__ import annotations

import contextlib
import ctypes
import json
import os
import time
from typing import List, Optional

import torch

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX or None


class Tracer:
    def __init__(self, enabled: bool, out_dir: Optional[str] = None, rank: int = 0, device=None):
        self.enabled = bool(enabled)
        self.out_dir = out_dir
        self.rank = rank
        self.device = torch.device(device) if device is not None else None
        self.events: List[dict] = []
        self._t0 = time.perf_counter()
        self._pending = []  # (step, start_event, end_event, host_ts)
        self.device_ms: List[float] = []
        self._lib = _roctx() if self.enabled else None

    def _us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    @contextlib.contextmanager
    def span(self, name: str, **args):
        if not self.enabled:
            yield
            return
        if self._lib is not None:
            self._lib.roctxRangePushA(name.encode())
        ts = self._us()
        try:
            yield
        finally:
            if self._lib is not None:
                self._lib.roctxRangePop()
            self.events.append(dict(name=name, ph="X", ts=ts, dur=self._us() - ts, pid=self.rank, tid="host",
                                    args=args))

    def mark(self, name: str):
        if self.enabled and self._lib is not None:
            self._lib.roctxMarkA(name.encode())

    @contextlib.contextmanager
    def device_step(self, step: int):
        """Bracket one step's enqueue with HIP events (timed once the step has completed)."""
        on_gpu = self.enabled and self.device is not None and self.device.type == "cuda"
        if not on_gpu:
            with self.span(f"step {step}"):
                yield
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ts = self._us()
        with self.span(f"enqueue step {step}"):
            yield
        b.record()
        self._pending.append((step, a, b, ts))

    def collect(self):
        """Resolve finished device spans (call after a host sync, e.g. the loss read)."""
        keep = []
        for step, a, b, ts in self._pending:
            if b.query():
                ms = a.elapsed_time(b)
                self.device_ms.append(ms)
                self.events.append(dict(name=f"device step {step}", ph="X", ts=ts, dur=ms * 1e3, pid=self.rank,
                                        tid="device"))
            else:
                keep.append((step, a, b, ts))
        self._pending = keep

    def write(self) -> Optional[str]:
        if not self.enabled or not self.out_dir:
            return None
        if self._pending:
            torch.cuda.synchronize(self.device)
            self.collect()
        d = os.path.join(self.out_dir, "trace")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"rank{self.rank}.json")
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)
        return path
