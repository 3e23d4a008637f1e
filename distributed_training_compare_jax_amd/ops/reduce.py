"""Batched deferred gradient reductions: one kernel launch per backward layer.

A backward layer produces many small reductions that are NOT on its dgrad critical path:
split-K slabs of the weight-gradient GEMMs, LayerNorm dγ/dβ per-block partials, bias column
partials, and (single-rank) the layer's grad-norm partial.  Launched one by one they cost the
~5 µs floor of a replayed graph node each (measured: ~130 such kernels, ~0.8 ms of a 6.6 ms
step).  :class:`GradReducer` instead collects them as tasks while the layer's backward is
enqueued and :meth:`GradReducer.flush` finishes all of them with ONE ``reduce_tasks_kernel``
launch (``csrc/norm_reduce.hip``).  Numerics are unchanged: each output element is still summed
by one thread in ascending partial order (bitwise equal to the per-op kernels).

Memory: partial slabs live in a persistent arena (static addresses, so the hipGraph captured
after the eager warmup step replays against the same buffers); the arena is reused after every
flush — stream order guarantees the reduce kernel has consumed a slab before the next layer's
GEMM overwrites it.  Single-stream only (the backward side stream, when enabled, keeps the
immediate per-op reductions).

Grad-norm tasks (:meth:`add_sumsq`) read FINAL gradients, so a norm chunk queued after a layer
is launched with the NEXT flush (once the reductions producing it have run); ``flush_all``
drains everything at the end of backward.
"""

from __future__ import annotations

import ctypes
import os
from typing import List

import torch

from . import _native as N

RED_WIDE, RED_TALL, RED_SUMSQ = 0, 1, 2
_TALL_COLS = 32  # SR_COLS in csrc/norm_reduce.hip
_WIDE_COLS = 1024


class RedTask(ctypes.Structure):
    """Mirror of ``struct RedTask`` (csrc/common.h)."""

    _fields_ = [
        ("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("part", ctypes.c_void_p),
        ("C", ctypes.c_long), ("pstride", ctypes.c_long),
        ("P", ctypes.c_int), ("mode", ctypes.c_int), ("blk0", ctypes.c_int), ("nblk", ctypes.c_int),
        ("beta", ctypes.c_float), ("weight", ctypes.c_float),
    ]


MAX_TASKS = 48  # RED_MAX_TASKS
_TRACE = os.environ.get("DTC_RED_TRACE", "0") == "1"  # launch trace (diagnostic)


class RedBatch(ctypes.Structure):
    _fields_ = [("ntasks", ctypes.c_int), ("nblocks", ctypes.c_int), ("t", RedTask * MAX_TASKS)]


class GradReducer:
    def __init__(self, device, arena_mb: int = 256):
        self.device = torch.device(device)
        self.arena_bytes = int(arena_mb) << 20
        self.arena = None
        self.off = 0
        self.pending: List[tuple] = []   # reduction tasks of the current window
        self.sumsq: List[tuple] = []     # (ready_after_flush, task)
        self.nflush = 0
        self.launches = 0
        self._checked = False

    # ------------------------------------------------------------------ arena
    def alloc(self, nfloats: int) -> torch.Tensor:
        """fp32 scratch for one task's partials (valid until the next flush)."""
        nbytes = (int(nfloats) * 4 + 255) // 256 * 256
        if self.arena is None or self.off + nbytes > self.arena.numel():
            if self.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("GradReducer arena exhausted during graph capture (raise arena_mb)")
            if self.arena is not None and self.off > 0:
                raise RuntimeError(f"GradReducer window needs more than {self.arena.numel() >> 20} MB (raise arena_mb)")
            self.arena = torch.empty(max(self.arena_bytes, nbytes), dtype=torch.uint8, device=self.device)
        t = self.arena[self.off:self.off + nbytes].view(torch.float32)[:nfloats]
        self.off += nbytes
        return t

    # ------------------------------------------------------------------ tasks
    def add_wide(self, src: torch.Tensor, dst: torch.Tensor, P: int, beta: float):
        """dst[:] = beta·dst + Σ_p src[p] (src [P, dst.numel()], contiguous)."""
        C = dst.numel()
        self.pending.append((RED_WIDE, src.data_ptr(), dst.data_ptr(), 0, C, C, int(P), (C + _WIDE_COLS - 1) // _WIDE_COLS,
                             float(beta), 1.0))

    def add_tall(self, src_ptr: int, pstride: int, P: int, dst: torch.Tensor, beta: float):
        """dst[c] = beta·dst[c] + Σ_p src[p·pstride + c] for c < dst.numel()."""
        C = dst.numel()
        self.pending.append((RED_TALL, int(src_ptr), dst.data_ptr(), 0, C, int(pstride), int(P),
                             (C + _TALL_COLS - 1) // _TALL_COLS, float(beta), 1.0))

    def add_sumsq(self, data: torch.Tensor, weight: float, part: torch.Tensor):
        """part[b] = weight·Σ x² over block b's share of ``data`` (one grad-norm segment)."""
        assert part.dtype == torch.float32 and data.dtype == torch.float32
        task = (RED_SUMSQ, data.data_ptr(), 0, part.data_ptr(), data.numel(), 0, 1, part.numel(), 0.0, float(weight))
        ready_after = self.nflush if self.pending else self.nflush - 1
        self.sumsq.append((ready_after, task))

    # ------------------------------------------------------------------ launch
    def _launch(self, tasks):
        if _TRACE:  # DTC_RED_TRACE=1: one line per launch (diagnostic)
            names = {RED_WIDE: "wide", RED_TALL: "tall", RED_SUMSQ: "sumsq"}
            print(f"[reduce flush {self.nflush}] " + " ".join(f"{names[t[0]]}(C={t[4]},P={t[6]},blk={t[7]})"
                                                              for t in tasks), flush=True)
        L = N.lib()
        if not self._checked:
            assert L.dtc_red_task_bytes() == ctypes.sizeof(RedTask) and L.dtc_red_max_tasks() == MAX_TASKS
            self._checked = True
        for i in range(0, len(tasks), MAX_TASKS):
            chunk = tasks[i:i + MAX_TASKS]
            b = RedBatch()
            b.ntasks = len(chunk)
            blk = 0
            for j, (mode, src, dst, part, C, pstride, P, nblk, beta, weight) in enumerate(chunk):
                b.t[j] = RedTask(src, dst, part, C, pstride, P, mode, blk, nblk, beta, weight)
                blk += nblk
            b.nblocks = blk
            N.check(L.dtc_reduce_tasks(ctypes.byref(b), N.stream_ptr(self.device)), "dtc_reduce_tasks")
            self.launches += 1

    def flush(self):
        """Launch this window's reductions + every norm task whose inputs are final."""
        k = self.nflush
        ready = [t for (r, t) in self.sumsq if r < k]
        self.sumsq = [(r, t) for (r, t) in self.sumsq if r >= k]
        # long-running blocks first (they are dispatched first): norm chunks, then the many-partial
        # (TALL) columns, then the short split-K (WIDE) blocks fill in behind them; within a kind the
        # tasks with the most blocks first, so a flush of more than MAX_TASKS tasks leaves only the smallest
        # to its second launch (the wte + wpe norm chunk was last: a 99-block launch of 48 tiny chunks,
        # 18 us, ran before it)
        tasks = sorted(ready + self.pending, key=lambda t: ({RED_SUMSQ: 0, RED_TALL: 1, RED_WIDE: 2}[t[0]], -t[7]))
        self.pending = []
        if tasks:
            self._launch(tasks)
        self.off = 0
        self.nflush += 1

    def flush_all(self):
        self.flush()
        if self.sumsq:
            self.flush()
        assert not self.sumsq and not self.pending
