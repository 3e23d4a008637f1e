"""Step programs: a training step as a static sequence of hipGraph segments and collectives.

The reference jit-compiles the whole step into one XLA program
(``train/create_train_step.py:28-50``) so the host issues one call per step.  The MI355X
analog is to capture the step's kernel stream into hipGraphs.  Collectives have two modes
(``TrainConfig.capture_comms``, decision and evidence in ``docs/CAPTURE.md``):

* **cut** (the default at world > 1): each collective cuts the graph and is issued eagerly
  between segments in stream order -- a DP bucket's all-reduce runs on RCCL's own stream while
  the NEXT backward segment replays, PP send/recv and TP RCCL calls stay on the eager path;
* **captured** (the default on a one-rank RCCL group, ``DTC_CAPTURE_COMMS=1`` anywhere): RCCL's
  kernels become nodes of the one step graph (below).

``record(step_fn)`` runs ``step_fn`` once with capture on; every ``comm(fn)`` call the
step makes cuts the current graph, stores ``fn`` WITHOUT running it (the recording pass
computes nothing, so a collective there would only move stale bytes and add a step of RCCL
traffic that the replays do not have) and opens the next graph.
``replay()`` then issues [graph, comm, graph, comm, ...] with one host call each.

Every collective also carries a signature (op, group ranks, tensor shapes/dtypes; for p2p the
peer and direction).  The first eager step and the recorded step gather every rank's list and
:func:`check_collective_sequences` proves that each group's members issue the same sequence and
that each send has the matching receive, in order — a mismatch (the classic hang of a rank-dependent
branch, or a PP schedule whose two sides disagree) raises on every rank instead of deadlocking.  With
``mode="eager"`` the same step code just executes (CPU/gloo path, first warmup steps).
All segments share one memory pool and are replayed in capture order, so activations
produced in one segment and consumed in a later one stay valid.

``capture_comms=True`` (``TrainConfig.capture_comms``, RCCL groups only): the recording pass runs every
collective INSIDE the capture instead of cutting the graph there -- RCCL's kernels (on its internal
stream, joined back by the captured event waits of ``Work.wait``) become nodes of the ONE step graph,
so a step replays with a single host call and no eager collective.  The recording pass then does move
(stale) bytes once, like the eager warmup step.
"""

from __future__ import annotations

import ctypes
import time
import warnings
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch


_RANKS: Dict[int, Tuple[int, ...]] = {}


def _group_ranks(group) -> Tuple[int, ...]:
    import torch.distributed as dist

    if not dist.is_initialized():  # nothing to check against (unit tests drive the code single-process)
        return ()
    key = id(group)
    if key not in _RANKS:
        g = group if group is not None else dist.group.WORLD
        _RANKS[key] = tuple(dist.get_process_group_ranks(g))
    return _RANKS[key]


def _meta(t) -> Tuple:
    return tuple(t.shape), str(t.dtype).replace("torch.", "")


def csig(op: str, group, *tensors) -> List[Tuple]:
    """Signature of one collective on ``group`` (the tensors that define its message size)."""
    return [("coll", op, _group_ranks(group), tuple(_meta(t) for t in tensors))]


def psig(direction: str, peer: int, t) -> List[Tuple]:
    """Signature of one point-to-point transfer (``direction`` = "send" | "recv", ``peer`` = global rank)."""
    return [(direction, int(peer), _meta(t))]


def check_collective_sequences(per_rank: List[List[Tuple]]) -> Optional[str]:
    """``per_rank[r]`` = rank r's collective signatures in issue order.  Returns None when every
    group's members issue identical sequences and every send (a -> b) sequence equals b's receive
    (from a) sequence, else a message naming the first disagreement."""
    colls: Dict[Tuple[int, ...], Dict[int, List]] = {}
    p2p: Dict[Tuple[int, int], Tuple[List, List]] = {}
    for r, seq in enumerate(per_rank):
        for e in seq:
            if e[0] == "coll":
                _, op, ranks, meta = e
                ranks = tuple(ranks)
                if r not in ranks:
                    return f"rank {r} issued {op} on group {ranks}, of which it is not a member"
                colls.setdefault(ranks, {}).setdefault(r, []).append((op, tuple(meta)))
            else:
                d, peer, meta = e
                key = (r, peer) if d == "send" else (peer, r)
                p2p.setdefault(key, ([], []))[0 if d == "send" else 1].append(tuple(meta))
    for ranks, by in sorted(colls.items()):
        ref = by.get(ranks[0], [])
        for r in ranks[1:]:
            seq = by.get(r, [])
            if seq != ref:
                k = next((i for i, (a, b) in enumerate(zip(ref, seq)) if a != b), min(len(ref), len(seq)))
                a = ref[k] if k < len(ref) else "nothing"
                b = seq[k] if k < len(seq) else "nothing"
                return (f"group {ranks}: collective #{k} is {a} on rank {ranks[0]} but {b} on rank {r} "
                        f"({len(ref)} vs {len(seq)} collectives per step)")
    for (a, b), (snd, rcv) in sorted(p2p.items()):
        if snd != rcv:
            k = next((i for i, (x, y) in enumerate(zip(snd, rcv)) if x != y), min(len(snd), len(rcv)))
            return (f"p2p {a} -> {b}: transfer #{k} sends {snd[k] if k < len(snd) else 'nothing'} but "
                    f"receives {rcv[k] if k < len(rcv) else 'nothing'} ({len(snd)} sends, {len(rcv)} receives)")
    return None


def _graph_nodes(g) -> int:
    from ..ops import _native as N

    n = ctypes.c_size_t(0)
    N.check(N.lib().dtc_graph_num_nodes(ctypes.c_void_p(g.raw_cuda_graph()), ctypes.byref(n)), "hipGraphGetNodes")
    return int(n.value)


class StepProgram:
    def __init__(self, device: torch.device, use_graph: bool, capture_comms: bool = False):
        self.device = torch.device(device)
        self.use_graph = bool(use_graph) and self.device.type == "cuda"
        self.capture_comms = bool(capture_comms) and self.use_graph
        self.items: List[Tuple[str, Any, Optional[str]]] = []
        self.recording = False
        self.recorded = False
        self._graph = None
        self._pool = None
        self._empty: List[Any] = []  # captured-empty segments (see _cut)
        self._handles: Dict[str, Any] = {}
        self._eager_names = set()  # named collectives issued eagerly between captured segments
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
        # collective signatures of the step being collected (None = not collecting)
        self.sigs: Optional[List[Tuple]] = None
        # sync_comms: wait every collective where it is issued (no collective in flight while later
        # kernels are enqueued).  Set for GPU tensors on a gloo group (the one-GPU multi-rank test rig):
        # gloo copies results back to the device from its WORKER thread, at a time no other rank can
        # predict, so that copy lands in a hardware queue behind whatever the main thread issued in
        # the meantime -- e.g. a P2P all-reduce barrier that spins on a peer whose own progress waits on
        # this rank's gloo result: a cycle whenever streams share a queue (parallel/dist.py).
        self.sync_comms = False

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
    def comm(self, fn: Callable[[], Any], name: Optional[str] = None, sig: Optional[List[Tuple]] = None,
             capturable: bool = True):
        """Issue a collective.  ``fn`` may return an async Work handle, retrievable by ``wait(name)``;
        ``sig`` (:func:`csig` / :func:`psig` entries) describes what it moves, for the cross-rank check.
        ``capturable=False``: never captured (``capture_comms``), always a graph cut + eager issue."""
        for h in self.before_comm:
            h()
        if self.sigs is not None and sig:
            self.sigs.extend(sig)
        if self.recording and self.capture_comms and not self.sync_comms and capturable:
            res = fn()  # captured into the current graph segment
            if name is not None:
                self._handles[name] = res
            return res
        if self.recording:
            if name is not None:
                self._eager_names.add(name)
            self._cut()
            self.items.append(("comm", fn, name))
            self._begin()
            return None
        res = self._timed(fn)
        if self.sync_comms and res is not None:
            self._wait_handle(res)
            res = None
        if name is not None:
            self._handles[name] = res
        return res

    def wait(self, name: str):
        for h in self.before_comm:
            h()
        if self.recording and self.capture_comms and not self.sync_comms and name not in self._eager_names:
            self._wait(name)  # the stream-side join is captured too
            return
        if self.recording:
            self._cut()
            self.items.append(("wait", None, name))
            self._wait(name)
            self._begin()
        else:
            self._timed(lambda: self._wait(name))

    # -------------------------------------------------------------- cross-rank sequence check
    def collect(self):
        self.sigs = []

    def verify(self, what: str = "step"):
        """Gather every rank's collected signatures and raise on any disagreement (all ranks raise)."""
        import torch.distributed as dist

        mine, self.sigs = self.sigs or [], None
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
            return
        allv: List[Any] = [None] * dist.get_world_size()
        dist.all_gather_object(allv, mine)
        err = check_collective_sequences(allv)
        if err is not None:
            raise RuntimeError(f"ranks disagree on the collectives of the {what}: {err}")

    def _wait(self, name):
        self._wait_handle(self._handles.pop(name, None))

    @staticmethod
    def _wait_handle(h):
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
        # keep_graph: the captured graph is inspected (node count) before it is instantiated
        g = torch.cuda.CUDAGraph(keep_graph=True)
        g.capture_begin(pool=self._pool, capture_error_mode="thread_local")
        self._graph = g

    def _cut(self):
        g, self._graph = self._graph, None
        with warnings.catch_warnings():
            warnings.filterwarnings("ignore", message=".*Graph is empty")
            g.capture_end()
        if _graph_nodes(g) == 0:  # nothing captured since the last cut (e.g. a collective, then its wait)
            # not replayed, but kept alive: releasing a graph drops its reference on the shared memory
            # pool, which the allocator asserts on at the next capture into that pool
            self._empty.append(g)
            return
        g.instantiate()
        self.items.append(("graph", g, None))

    def record(self, step_fn: Callable[[], Any]) -> Any:
        assert self.use_graph
        self.items = []
        torch.cuda.synchronize(self.device)
        cur = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(cur)
        self.recording = True
        # no cyclic garbage collection during the capture: a collected object of an earlier engine (its
        # graphs, its pool) must not be destroyed while this stream is capturing -- HIP aborts the process
        import gc

        gc.collect()
        gc_was = gc.isenabled()
        gc.disable()
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
            if gc_was:
                gc.enable()
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
                if self.sync_comms and res is not None:
                    self._wait_handle(res)
                    res = None
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
