"""Step programs: a training step as a static sequence of hipGraph segments and collectives.

The reference jit-compiles the whole step into one XLA program
(``train/create_train_step.py:28-50``) so the host issues one call per step.  The MI355X
analog is to capture the step's kernel stream into hipGraphs.  Collectives are kept OUT
of the graphs on purpose: RCCL calls are issued eagerly between graph segments on the
same stream order, which

* lets a DP gradient bucket's all-reduce run on RCCL's own stream while the NEXT backward
  segment replays (overlap without capturing RCCL),
* keeps PP send/recv and TP all-reduces on the well-trodden eager RCCL path.

``record(step_fn)`` runs ``step_fn`` once with capture on; every ``comm(fn)`` call the
step makes cuts the current graph, runs the collective for real (on whatever stale data
the buffers hold — the recording pass computes nothing) and opens the next graph.
``replay()`` then issues [graph, comm, graph, comm, ...] with one host call each.  With
``mode="eager"`` the same step code just executes (CPU/gloo path, first warmup steps).
All segments share one memory pool and are replayed in capture order, so activations
produced in one segment and consumed in a later one stay valid.
"""

from __future__ import annotations

import time
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch


class StepProgram:
    def __init__(self, device: torch.device, use_graph: bool):
        self.device = torch.device(device)
        self.use_graph = bool(use_graph) and self.device.type == "cuda"
        self.items: List[Tuple[str, Any, Optional[str]]] = []
        self.recording = False
        self.recorded = False
        self._graph = None
        self._pool = None
        self._handles: Dict[str, Any] = {}
        self._stream = torch.cuda.Stream(self.device) if self.use_graph else None
        # called before every cut/collective: forked streams (e.g. the backward side stream)
        # must re-join the capture stream before a graph segment ends / a collective reads data
        self.before_comm: List[Callable[[], None]] = []
        # observability (metrics.json comm_ms / comm_calls_per_step): with time_comms on, every
        # collective (and every wait on an async one) issued in eager mode or replay is bracketed
        # by timing events on the issuing stream, i.e. the EXPOSED time the step's stream spends
        # in it; a host clock on CPU (gloo is synchronous there)
        self.time_comms = False
        self.step_comms = 0
        self._ev: List[List[Any]] = []  # per step (FIFO): [(start, end) event pairs | host ms floats]

    def begin_step(self):
        self.step_comms = 0
        if self.time_comms:
            self._ev.append([])

    def _timed(self, fn):
        self.step_comms += 1
        if not self.time_comms or self.recording or not self._ev:
            return fn()
        if self.device.type == "cuda":
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            r = fn()
            e.record()
            self._ev[-1].append((s, e))
            return r
        t = time.perf_counter()
        r = fn()
        self._ev[-1].append(1e3 * (time.perf_counter() - t))
        return r

    def take_comm_ms(self) -> float:
        """Exposed collective time (ms) of the OLDEST timed step not yet taken (synchronises on that
        step's events only, so a step already queued behind it keeps running)."""
        if not self._ev:
            return 0.0
        ms = 0.0
        for x in self._ev.pop(0):
            if isinstance(x, float):
                ms += x
            else:
                s, e = x
                e.synchronize()
                ms += s.elapsed_time(e)
        return ms

    # -------------------------------------------------------------- step-code API
    def comm(self, fn: Callable[[], Any], name: Optional[str] = None):
        """Issue a collective.  ``fn`` may return an async Work handle, retrievable by ``wait(name)``."""
        for h in self.before_comm:
            h()
        if self.recording:
            self._cut()
            self.items.append(("comm", fn, name))
            res = fn()
            if name is not None:
                self._handles[name] = res
            self._begin()
            return res
        res = self._timed(fn)
        if name is not None:
            self._handles[name] = res
        return res

    def wait(self, name: str):
        for h in self.before_comm:
            h()
        if self.recording:
            self._cut()
            self.items.append(("wait", None, name))
            self._wait(name)
            self._begin()
        else:
            self._timed(lambda: self._wait(name))

    def _wait(self, name):
        h = self._handles.pop(name, None)
        if h is not None:
            if isinstance(h, (list, tuple)):
                for x in h:
                    x.wait()
            else:
                h.wait()

    # -------------------------------------------------------------- capture / replay
    def _begin(self):
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self._pool, capture_error_mode="thread_local")
        self._graph = g

    def _cut(self):
        g, self._graph = self._graph, None
        g.capture_end()
        self.items.append(("graph", g, None))

    def record(self, step_fn: Callable[[], Any]) -> Any:
        assert self.use_graph
        self.items = []
        torch.cuda.synchronize(self.device)
        cur = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(cur)
        self.recording = True
        try:
            with torch.cuda.stream(self._stream):
                self._begin()
                out = step_fn()
                for h in self.before_comm:
                    h()
                self._cut()
        except BaseException:
            import sys
            import traceback

            traceback.print_exc(file=sys.stderr)
            sys.stderr.flush()
            # never leave the stream in capture mode (the process would abort at teardown)
            for h in self.before_comm:
                try:
                    h()
                except Exception:
                    pass
            if self._graph is not None:
                try:
                    self._graph.capture_end()
                except Exception:
                    pass
                self._graph = None
            self.items = []
            raise
        finally:
            self.recording = False
        cur.wait_stream(self._stream)
        torch.cuda.synchronize(self.device)
        self.recorded = True
        return out

    def replay(self):
        for kind, obj, name in self.items:
            if kind == "graph":
                obj.replay()
            elif kind == "comm":
                res = self._timed(obj)
                if name is not None:
                    self._handles[name] = res
            else:
                self._timed(lambda: self._wait(name))

    @property
    def n_graphs(self) -> int:
        return sum(1 for k, _, _ in self.items if k == "graph")

    @property
    def n_comms(self) -> int:
        return sum(1 for k, _, _ in self.items if k != "graph")


class EagerProgram(StepProgram):
    def __init__(self, device):
        super().__init__(device, use_graph=False)
