"""Data-parallel gradient synchronisation: bucketed all-reduce over RCCL, overlapped with backward.

Reference DP (``parallel/sharding.py:25-27`` + GSPMD) replicates params and lets XLA insert
one implicit gradient all-reduce.  Here grads live in one flat fp32 buffer laid out in
backward order (``parallel/buffers.py``), so a bucket is a contiguous slice that becomes
complete the moment backward passes its last layer.  As soon as a bucket is complete its
all-reduce is issued (async, on RCCL's stream) and the next backward segment runs under
it; the step waits on all buckets only before the optimizer.

Bucket size is chosen for xGMI, not NVSwitch: a ring all-reduce on the 8×MI355X mesh is
per-link bound (~150 GB/s/link), so buckets are kept large (``dp_bucket_mb``, default 40 MB,
cut at layer boundaries, with a 16 MB ``dp_tail_mb`` last bucket because its all-reduce is
exposed: enough to saturate RCCL's multi-channel rings, few enough that per-call latency is
noise).  Loss scaling makes the SUM equal the global-mean gradient (no extra pass).
"""

from __future__ import annotations

from typing import List, Tuple

import torch.distributed as dist

import torch

from ..ops.payload import cast_bf16_to_f32, cast_to_bf16, shard_sum_bf16
from .buffers import FlatParams
from .program import csig


class _StreamJoin:
    """Work-like handle of a chain run on a side stream: wait() makes the current stream wait for it."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class GradBuckets:
    """Contiguous buckets over the flat grad buffer, issued in backward order.

    ``bucket_mb`` sizes the bulk buckets; the LAST bucket (complete only when backward ends,
    so its all-reduce is exposed) is cut to about ``tail_mb``.  ``local_names`` are params
    whose grads every rank computes identically on its own (the DP embedding gather); they must
    form the tail of the buffer and are excluded from the all-reduce.

    ``boundaries``: offsets where grads become final together (the head's and each layer's end,
    in backward order).  Buckets then end only there, so each is issued the moment its last layer
    is done; cut at arbitrary param boundaries, a bucket straddling two layers waits for the later
    one (for the reference model the second-to-last large bucket used to wait for the END of
    backward, its all-reduce fully exposed)."""

    def __init__(self, flat: FlatParams, group, dp: int, program, bucket_mb: float = 64.0, tail_mb: float = 16.0,
                 local_names=(), boundaries=None, payload: str = "fp32", active: bool = None):
        self.flat = flat
        self.group = group
        self.dp = dp
        # issue the collectives: dp > 1, or the one-member rehearsal group (TrainConfig.dp_comm_rehearsal)
        self.active = (dp > 1) if active is None else bool(active)
        self.program = program
        if payload not in ("fp32", "bf16"):
            raise ValueError(f"dp_grad_dtype={payload!r}: expected 'fp32' or 'bf16'")
        self.payload = payload
        self._bf16 = {}  # bucket -> (send, recv, reduced shard, gathered) bf16 buffers
        self._cs = None  # GPU: the stream the bf16 exchange chain runs on
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        tail_cap = max(1, int(tail_mb * 1024 * 1024 / 4))
        end = flat.numel
        if local_names:
            lo, _ = flat.range_of(list(local_names))
            rest = [s for n, s in flat.slots.items() if n not in local_names]
            if any(s.offset >= lo for s in rest):
                raise ValueError(f"local-grad params {local_names} must be the tail of the flat buffer")
            end = lo
        self.reduce_end = end
        bounds: List[Tuple[int, int]] = [(s.offset, s.offset + s.numel) for s in flat.slots.values()
                                         if s.offset < end]
        if boundaries:  # units = the spans between consecutive boundaries (layer-aligned buckets)
            xs = sorted({int(x) for x in boundaries if 0 < int(x) < end} | {end})
            bounds = list(zip([0] + xs[:-1], xs))
        # tail bucket: the last params adding up to ~tail_cap elements
        i_tail = len(bounds)
        acc = 0
        while i_tail > 1 and acc < tail_cap:
            u = bounds[i_tail - 1][1] - bounds[i_tail - 1][0]
            if boundaries and acc > 0 and acc + u > tail_cap:
                break  # layer-aligned: the tail stays within tail_mb (at least one unit)
            i_tail -= 1
            acc += u
        cuts: List[int] = []  # exclusive end offsets of each bucket
        lo = None
        for a, b in bounds[:i_tail]:
            lo = a if lo is None else lo
            if b - lo >= cap:
                cuts.append(self._pad(b))
                lo = None
        if lo is not None:  # leftover: its own bucket, or folded into the previous one if small
            c = self._pad(bounds[i_tail - 1][1])
            if cuts and c - lo < cap // 2:
                cuts[-1] = c
            else:
                cuts.append(c)
        cuts.append(end)
        # buckets tile [0, end) contiguously (alignment gaps included)
        self.buckets = []
        prev = 0
        for c in cuts:
            c = min(c, end)
            if c > prev:
                self.buckets.append((prev, c))
                prev = c
        self.issued = [False] * len(self.buckets)

    def _pad(self, n: int) -> int:
        return min(self.flat.numel, (n + 63) // 64 * 64)

    def reset(self):
        self.issued = [False] * len(self.buckets)

    def ready_upto(self, offset: int):
        """All grads in flat[0:offset] are final → launch every complete, un-issued bucket."""
        if not self.active:
            return
        for i, (a, b) in enumerate(self.buckets):
            if not self.issued[i] and b <= offset:
                self._issue(i)

    def ready_all(self):
        self.ready_upto(self.reduce_end)

    def _issue(self, i: int):
        a, b = self.buckets[i]
        view = self.flat.grads[a:b]
        g = self.group
        if self.payload == "bf16":
            self._issue_bf16(i, view)
        else:
            self.program.comm(lambda: dist.all_reduce(view, group=g, async_op=True), name=f"dp_bucket{i}",
                              sig=csig("all_reduce", g, view))
        self.issued[i] = True

    def _buffers(self, i: int, n: int):
        """Persistent bf16 buffers of bucket i (allocated at its first issue, i.e. in the eager warmup
        step, before any graph capture): the padded send image [dp*s] (pad stays zero), the all-to-all
        result [dp*s], this rank's reduced shard [s] and the all-gathered bucket [dp*s]."""
        if i not in self._bf16:
            s = -(-n // (self.dp * 64)) * 64
            kw = dict(dtype=torch.bfloat16, device=self.flat.device)
            self._bf16[i] = (torch.zeros(self.dp * s, **kw), torch.zeros(self.dp * s, **kw), torch.zeros(s, **kw),
                             torch.zeros(self.dp * s, **kw))
        return self._bf16[i]

    def _issue_bf16(self, i: int, view):
        """bf16 payload, fp32 accumulation: cast -> all-to-all (shard r of every rank to rank r) -> fixed-order
        fp32 sum of the dp shards -> all-gather of the bf16 shards -> cast back into the fp32 grads.  Half the
        bytes of an fp32 ring all-reduce, every rank-pair xGMI link busy at once, identical replicas.  On the
        GPU the chain runs on its own stream (the backward keeps going); the returned handle's wait() joins it."""
        n = view.numel()
        send, recv, red, gath = self._buffers(i, n)
        g, dp = self.group, self.dp

        def chain():
            cast_to_bf16(view, send[:n])
            dist.all_to_all_single(recv, send, group=g)
            shard_sum_bf16(recv, dp, red)
            dist.all_gather_into_tensor(gath, red, group=g)
            cast_bf16_to_f32(gath[:n], view)

        def fn():
            if not view.is_cuda:
                chain()
                return None
            if self._cs is None:
                self._cs = torch.cuda.Stream(view.device)
            cur = torch.cuda.current_stream(view.device)
            self._cs.wait_stream(cur)
            with torch.cuda.stream(self._cs):
                chain()
            ev = torch.cuda.Event()
            ev.record(self._cs)
            return _StreamJoin(ev)

        # NEVER captured (capture_comms or not): the chain issues its collectives from a side stream forked into
        # the capture, and an RCCL collective issued from a forked stream segfaults inside hipStreamEndCapture
        # (torch 2.10 / ROCm 7.0 / RCCL 2.26.6; minimal repro benchmarks/capture_side_stream_probe.py: the same
        # all_to_all_single from the capture's origin stream records and replays fine, from a stream joined by
        # wait_stream it crashes at capture_end; in the engine the PG watchdog then also trips over the event
        # recorded in the capturing stream).  It stays an eager item between graph segments.
        self.program.comm(fn, name=f"dp_bucket{i}", sig=csig("all_to_all", g, send) + csig("all_gather", g, red),
                          capturable=False)

    def wait_all(self):
        if not self.active:
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
