"""Optimizer: clip-by-global-norm(1.0) + AdamW(3e-4, wd 0.1) over the flat buffers.

Reference: ``train/create_optimizer.py:8-12`` (optax chain).  The global norm is computed
over exactly the reference's set of gradients:

* DP: grads are identical after the all-reduce → local Σg² is the global one.
* TP: sharded params' Σg² is summed over the TP group, replicated params (identical on
  every TP rank) are weighted 1/tp so the all-reduce counts them once.
* PP: ``pp_clip: local`` (default) clips with the stage-local norm exactly like the
  reference's per-stage ``tx.update`` (``create_train_step.py:189-191``);
  ``pp_clip: global`` all-reduces Σg² over the pipeline (what a single-device run does).
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..config.schema import OptimConfig
from ..ops import optim as O
from ..ops.reduce import GradReducer
from ..parallel.buffers import FlatParams
from ..parallel.program import csig

# DTC_ADAMW_TR: the transposed bf16 weight mirror written by the AdamW update itself (one segmented
# element-wise launch + one tiled launch) instead of a transpose pass re-reading the fresh mirror
_ADAMW_TR = os.environ.get("DTC_ADAMW_TR", "1") == "1"


def merge_segments(segs, total: int):
    """Coalesce per-parameter (offset, len, weight) into maximal ranges of equal weight.

    Alignment gaps between params are zero in the grad buffer, so each range may absorb the gap
    up to the next param; at tp=1 the whole buffer becomes ONE range (a single streaming pass)."""
    segs = sorted(segs)
    out = []
    for i, (o, n, w) in enumerate(segs):
        end = segs[i + 1][0] if i + 1 < len(segs) else total
        if out and out[-1][2] == w and out[-1][0] + out[-1][1] == o:
            out[-1] = (out[-1][0], end - out[-1][0], w)
        else:
            out.append((o, end - o, w))
    return out


def _subtract_ranges(segs, ranges):
    """``segs`` [(offset, n, weight)] minus the flat ranges [(offset, n)] (sorted, disjoint)."""
    out = []
    for (o, n, w) in segs:
        cur = o
        end = o + n
        for (ro, rn) in ranges:
            re_ = ro + rn
            if re_ <= cur or ro >= end:
                continue
            if ro > cur:
                out.append((cur, ro - cur, w))
            cur = max(cur, re_)
            if cur >= end:
                break
        if cur < end:
            out.append((cur, end - cur, w))
    return out


class FusedAdamW:
    def __init__(self, flat: FlatParams, cfg: OptimConfig, program, tp_size: int = 1, tp_group=None,
                 pp_group=None, pp_global_clip: bool = False):
        self.flat = flat
        self.cfg = cfg
        self.program = program
        self._aw_plans = {}  # (lo, hi) -> fused AdamW + transpose launch lists
        self.tp_size, self.tp_group = tp_size, tp_group
        self.pp_group = pp_group if pp_global_clip else None
        dev = flat.device
        w = (lambda spec: 1.0 if spec.tp != "rep" else 1.0 / tp_size)
        self._merged = merge_segments(flat.segments(w), flat.numel)
        self.segments = O.make_segments(self._merged, dev)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.chunks = []  # incremental-norm chunks: [segments, lo, hi, partial view, reducer tasks]
        self._done = []
        self.reducer = None  # GradReducer of the model stage (single-stream GPU backward)
        self.tp_comm = None  # parallel.tp.TPComm: the TP norm partial through its P2P path when it has one
        self._fused = ([], 0)  # flat ranges whose Σg² arrives precomputed (set_fused_sumsq), slot count
        self._cuts = None
        self.fused_part = None

    # -- incremental global norm ------------------------------------------------------
    def set_chunks(self, cuts, elems_per_block: int = 16384):
        """Split Σg² into flat ranges [0,c0), [c0,c1), ... (cuts ascending, 4-aligned, last =
        numel).  A chunk whose grads are final can be reduced early (:meth:`ready_upto` /
        :meth:`chunk_ready`, typically on the backward side stream) so only the last chunk and a
        fixed-order finish remain between backward and the AdamW pass."""
        f = self.flat
        assert cuts and cuts[-1] == f.numel and all(c % 4 == 0 for c in cuts)
        self._cuts = list(cuts)
        fused, nfused = self._fused
        specs, lo = [], 0
        for hi in cuts:
            segs = [(max(o, lo), min(o + n, hi) - max(o, lo), wt) for (o, n, wt) in self._merged
                    if o < hi and o + n > lo]
            segs = _subtract_ranges(segs, fused)
            # partial slots per segment (a batched-reducer task each; one block per ~16K elements so
            # no block of the batched launch streams more than 64 KB), >= 8 per chunk in total
            nbs = [max(1, (n + elems_per_block - 1) // elems_per_block) for (_, n, _) in segs]
            if nbs:
                nbs[-1] += max(0, 8 - sum(nbs))
            specs.append((segs, lo, hi, nbs))
            lo = hi
        nchunk = sum(sum(s[3]) for s in specs)
        self.part = torch.zeros(nchunk + nfused, dtype=torch.float32, device=f.device)
        self.fused_part = self.part[nchunk:] if nfused else None
        self.chunks, off = [], 0
        for segs, lo, hi, nbs in specs:
            nb = sum(nbs)
            part = self.part[off:off + nb]
            tasks, o2 = [], 0
            for (o, n, w), k in zip(segs, nbs):
                tasks.append((o, n, w, part[o2:o2 + k]))
                o2 += k
            self.chunks.append((O.make_segments(segs, f.device) if segs else None, lo, hi, part, tasks))
            off += nb
        self._done = [False] * len(self.chunks)

    def set_fused_sumsq(self, ranges, nslots: int) -> torch.Tensor:
        """The Σg² of the flat ranges ``[(offset, n), ...]`` arrives as ``nslots`` per-tile partials written
        by the grouped weight-gradient epilogue (``ops.gemm.wgrad_group(sq=...)``): the norm chunks skip
        those ranges and the finish sums the partials after theirs (one fixed order).  Returns the partial
        buffer (a view of the norm's partial array) for the writer.  Call after :meth:`set_chunks`, only
        for grads that are final where they are written (dp == 1) and whose norm weight is 1."""
        assert self._cuts is not None, "set_fused_sumsq needs the incremental-norm chunks"
        ranges = sorted((int(o), int(n)) for o, n in ranges)
        for o, n in ranges:
            for (so, sn, wt) in self._merged:
                if so < o + n and so + sn > o and wt != 1.0:
                    raise ValueError(f"fused Σg² range at {o} overlaps a weight-{wt} segment")
        self._fused = (ranges, int(nslots))
        self.set_chunks(self._cuts)
        return self.fused_part

    def chunk_ready(self, i: int, runner=None):
        """Σg² partials of chunk i (its grads must be final).  ``runner``: a ``GradReducer``
        (queued into its next batched launch), a callable taking a thunk, or None (run now)."""
        if self._done[i]:
            return
        segs, _, _, part, tasks = self.chunks[i]
        if segs is None:  # every grad of the chunk is covered by the fused partials
            self._done[i] = True
            return
        g = self.flat.grads
        if isinstance(runner, GradReducer):
            for o, n, w, pt in tasks:
                runner.add_sumsq(g[o:o + n], w, pt)
        else:
            fn = lambda: O.sumsq_partial(g, segs, part)
            runner(fn) if runner is not None else fn()
        self._done[i] = True

    def ready_upto(self, offset: int, runner=None):
        for i, ch in enumerate(self.chunks):
            if ch[2] <= offset:
                self.chunk_ready(i, runner)

    def norm(self):
        """Global Σg² (all chunks, fixed order) + step counter bump (+ TP/PP all-reduce)."""
        f = self.flat
        red = self.reducer
        if self.chunks:
            for i in range(len(self.chunks)):
                self.chunk_ready(i, red)
            if red is not None:
                red.flush_all()  # every remaining chunk in one launch
            O.sum_finish(self.part, self.sumsq, step=self.step_t)
            self._done = [False] * len(self.chunks)
        else:
            if red is not None:
                red.flush_all()  # grads must be final
            O.sumsq_segments(f.grads, self.segments, self.sumsq, step=self.step_t)
        if self.tp_size > 1:
            if self.tp_comm is not None and self.tp_comm.p2p is not None:
                self.tp_comm.all_reduce_(self.sumsq)  # in-graph one-shot (no graph cut)
            else:
                g = self.tp_group
                s = self.sumsq
                self.program.comm(lambda: dist.all_reduce(s, group=g), sig=csig("all_reduce", g, s))
        if self.pp_group is not None:
            g = self.pp_group
            s = self.sumsq
            self.program.comm(lambda: dist.all_reduce(s, group=g), sig=csig("all_reduce", g, s))

    def update_range(self, lo: int, hi: int, enable=None, max_blocks: int = 0):
        """Clip + AdamW over flat[lo:hi] (4-aligned) with the norm/step of the last :meth:`norm`
        (skipped on device when ``enable[0] == 0``; ``max_blocks`` caps the kernel's grid)."""
        f, c = self.flat, self.cfg
        if hi <= lo:
            return
        nm = (min(max(f.n_mirror - lo, 0), hi - lo) if f.use_mirror else 0)
        if nm > 0 and enable is None and max_blocks == 0 and f.params.is_cuda and f.mirror_t and _ADAMW_TR:
            # the transposed mirror written by the update itself (ops/optim.py adamw_tr)
            key = (lo, hi)
            if key not in self._aw_plans:
                self._aw_plans[key] = O.adamw_tr_plan(lo, hi, f.transposed_in(lo, hi))
            plan = self._aw_plans[key]
            if plan is not None:
                O.adamw_tr(f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.mirror, f.n_mirror, plan, self.step_t,
                           self.sumsq, c.lr, c.b1, c.b2, c.eps, c.weight_decay, c.grad_clip)
                return
        O.adamw_flat(f.params[lo:hi], f.grads[lo:hi], f.exp_avg[lo:hi], f.exp_avg_sq[lo:hi],
                     f.mirror[lo:lo + max(nm, 4)] if nm > 0 else None, nm, self.step_t, self.sumsq, c.lr, c.b1, c.b2,
                     c.eps, c.weight_decay, c.grad_clip, enable=enable, max_blocks=max_blocks)
        if nm > 0:
            f.refresh_transposed(lo, hi)

    def step(self):
        self.norm()
        self.update_range(0, self.flat.numel)

    def grad_norm(self) -> float:
        return float(self.sumsq.item()) ** 0.5


class ShardedAdamW:
    """ZeRO-1 over the data-parallel group: each DP rank owns 1/dp of the Adam state.

    Not in the reference (SURVEY §2.2 lists ZeRO/FSDP as absent and optional; the reference
    replicates the optax state on every device, ``train.py:44-52``).  Step:

    1. one in-place ``reduce_scatter`` of the flat grad buffer over the DP group (same bytes on
       the xGMI ring as half an all-reduce): rank r ends with the summed grads of its slice
       ``[r·S, (r+1)·S)``; the small remainder ``[dp·S, numel)`` is all-reduced and owned by all;
    2. Σg² of the owned slice (+ the shared tail weighted 1/dp), one scalar all-reduce → the
       global clip norm, exactly the replicated optimizer's;
    3. fused clip+AdamW (the same HIP kernel) on the owned slice with shard-sized m/v;
    4. one in-place ``all_gather`` of the updated params, then the bf16 compute mirror is rebuilt.

    Adam m/v shrink from 8·numel to 8·(numel/dp) bytes per rank.  ``flat.exp_avg``/``exp_avg_sq``
    are replaced by the shard buffers, so checkpoints hold each rank's shard (resume at the
    same dp)."""

    def __init__(self, flat: FlatParams, cfg: OptimConfig, program, dp_group, dp: int, dp_idx: int):
        self.flat, self.cfg, self.program = flat, cfg, program
        self.group, self.dp, self.rank = dp_group, dp, dp_idx
        align = 64
        self.S = (flat.numel // dp) // align * align
        self.lo, self.hi = dp_idx * self.S, (dp_idx + 1) * self.S
        self.n_rs = dp * self.S  # [0, n_rs) reduce-scattered, [n_rs, numel) all-reduced
        self.n_tail = flat.numel - self.n_rs
        dev = flat.device
        n_own = self.S + self.n_tail
        flat.exp_avg = torch.zeros(n_own, dtype=torch.float32, device=dev)
        flat.exp_avg_sq = torch.zeros(n_own, dtype=torch.float32, device=dev)
        segs = [(self.lo, self.S, 1.0)] if self.S else []
        if self.n_tail:
            segs.append((self.n_rs, self.n_tail, 1.0 / dp))
        self.segments = O.make_segments(segs, dev)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.reducer = None
        # gloo on device tensors (the 2-ranks-on-one-GPU test rig) lacks the in-place tensor
        # collectives: emulate them with all_reduce / list all_gather (same results)
        self._emulate = dev.type == "cuda" and dist.get_backend(dp_group) == "gloo"

    def _adamw(self, lo: int, hi: int, mlo: int):
        f, c = self.flat, self.cfg
        if hi <= lo:
            return
        O.adamw_flat(f.params[lo:hi], f.grads[lo:hi], f.exp_avg[mlo:mlo + hi - lo], f.exp_avg_sq[mlo:mlo + hi - lo],
                     None, 0, self.step_t, self.sumsq, c.lr, c.b1, c.b2, c.eps, c.weight_decay, c.grad_clip)

    def step(self):
        if self.reducer is not None:
            self.reducer.flush_all()  # grads must be final
        f, grp = self.flat, self.group
        g, p = f.grads, f.params
        lo, hi, n = self.lo, self.hi, self.n_rs
        if n and self._emulate:
            self.program.comm(lambda: dist.all_reduce(g[:n], group=grp), sig=csig("all_reduce", grp, g[:n]))
        elif n:
            self.program.comm(lambda: dist.reduce_scatter_tensor(g[lo:hi], g[:n], group=grp),
                              sig=csig("reduce_scatter", grp, g[:n]))
        if self.n_tail:
            self.program.comm(lambda: dist.all_reduce(g[n:], group=grp), sig=csig("all_reduce", grp, g[n:]))
        O.sumsq_segments(g, self.segments, self.sumsq, step=self.step_t)
        s = self.sumsq
        self.program.comm(lambda: dist.all_reduce(s, group=grp), sig=csig("all_reduce", grp, s))
        self._adamw(lo, hi, 0)
        self._adamw(n, f.numel, self.S)
        if n and self._emulate:
            S = self.S
            self.program.comm(lambda: dist.all_gather([p[i * S:(i + 1) * S] for i in range(self.dp)],
                                                      p[lo:hi].clone(), group=grp),
                              sig=csig("all_gather", grp, p[lo:hi]))
        elif n:
            self.program.comm(lambda: dist.all_gather_into_tensor(p[:n], p[lo:hi], group=grp),
                              sig=csig("all_gather", grp, p[lo:hi]))
        f.refresh_mirror()

    def grad_norm(self) -> float:
        return float(self.sumsq.item()) ** 0.5
