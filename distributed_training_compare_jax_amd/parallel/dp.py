"""Data-parallel gradient synchronisation: bucketed all-reduce over RCCL, overlapped with backward.

Reference DP (``parallel/sharding.py:25-27`` + GSPMD) replicates params and lets XLA insert
one implicit gradient all-reduce.  Here grads live in one flat fp32 buffer laid out in
backward order (``parallel/buffers.py``), so a bucket is a contiguous slice that becomes
complete the moment backward passes its last layer.  As soon as a bucket is complete its
all-reduce is issued (async, on RCCL's stream) and the next backward segment runs under
it; the step waits on all buckets only before the optimizer.

Bucket size is chosen for xGMI, not NVSwitch: a ring all-reduce on the 8×MI355X mesh is
per-link bound (~150 GB/s/link), so buckets are kept large (default 64 MB, a few per
step: enough to saturate RCCL's multi-channel rings, few enough that per-call latency
is noise).  Loss scaling makes the SUM equal the global-mean gradient (no extra pass).
"""

from __future__ import annotations

from typing import List, Tuple

import torch.distributed as dist

from .buffers import FlatParams


class GradBuckets:
    def __init__(self, flat: FlatParams, group, dp: int, program, bucket_mb: float = 64.0):
        self.flat = flat
        self.group = group
        self.dp = dp
        self.program = program
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        # param boundaries in flat (backward) order
        bounds: List[Tuple[int, int]] = []
        for s in flat.slots.values():
            bounds.append((s.offset, s.offset + s.numel))
        buckets: List[Tuple[int, int]] = []
        lo = None
        hi = 0
        for a, b in bounds:
            if lo is None:
                lo = a
            hi = b
            if hi - lo >= cap:
                buckets.append((lo, self._pad(hi)))
                lo = None
        if lo is not None:
            buckets.append((lo, self._pad(hi)))
        # make buckets tile the buffer contiguously (alignment gaps included)
        fixed = []
        prev = 0
        for i, (a, b) in enumerate(buckets):
            end = flat.numel if i == len(buckets) - 1 else b
            fixed.append((prev, end))
            prev = end
        self.buckets = fixed
        self.issued = [False] * len(fixed)

    def _pad(self, n: int) -> int:
        return min(self.flat.numel, (n + 63) // 64 * 64)

    def reset(self):
        self.issued = [False] * len(self.buckets)

    def ready_upto(self, offset: int):
        """All grads in flat[0:offset] are final → launch every complete, un-issued bucket."""
        if self.dp == 1:
            return
        for i, (a, b) in enumerate(self.buckets):
            if not self.issued[i] and b <= offset:
                self._issue(i)

    def ready_all(self):
        self.ready_upto(self.flat.numel)

    def _issue(self, i: int):
        a, b = self.buckets[i]
        view = self.flat.grads[a:b]
        g = self.group
        self.program.comm(lambda: dist.all_reduce(view, group=g, async_op=True), name=f"dp_bucket{i}")
        self.issued[i] = True

    def wait_all(self):
        if self.dp == 1:
            return
        for i in range(len(self.buckets)):
            if self.issued[i]:
                self.program.wait(f"dp_bucket{i}")
        self.reset()

    def layer_end_offset(self, layer: int) -> int:
        """End offset (exclusive) of layer ``layer``'s params in the flat buffer."""
        names = [n for n in self.flat.slots if n.startswith(f"h.{layer}.")]
        return self.flat.range_of(names)[1]

    def head_end_offset(self) -> int:
        names = [n for n in self.flat.slots if n.startswith("lm_head") or n.startswith("lnf")]
        return self.flat.range_of(names)[1] if names else 0
