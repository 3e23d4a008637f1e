"""Pipeline-parallel schedules over RCCL point-to-point send/recv.

Reference PP (``train/create_train_step.py:55-195``): GPipe fill/drain expressed as a
``lax.scan`` over ``M+S-1`` clocks where EVERY stage runs ``lax.cond``-gated work on every
clock and ``ppermute`` shifts activations, labels and a valid flag each clock (also on
bubble clocks); backward is autodiff of the scan.  Here the schedule is a host-side
static program:

* only valid (stage, microbatch) work exists — no bubble-clock compute or traffic;
* labels never travel (every rank reads its own rows; reference ppermutes them, ``:165``);
* activations travel as fp32 ``[mb·T, D]`` (the residual stream) with
  ``isend``/``irecv``; the receiver waits right before the consuming segment;
* ``gpipe`` = reference order (all forwards, then all backwards), ``1f1b`` = PipeDream-flush
  order (activation memory bounded by S microbatches instead of M).

Loss/gradient scaling is exact: each microbatch's CE is scaled by ``1/(mb·T·M)`` so the
sum over microbatches is the full-batch mean (reference: ``psum(loss_sum / M)``, ``:187``).
"""

from __future__ import annotations

from typing import Dict, List

import torch
import torch.distributed as dist

from ..ops.optim import cast_to_bf16, fill_
from .dist import staged_p2p


class _HostSend:
    """isend of a device tensor through a host copy (gloo backend); ``wait()`` like a Work."""

    def __init__(self, t, dst):
        self.host = t.detach().to("cpu")
        self.work = dist.isend(self.host, dst)

    def wait(self):
        self.work.wait()
        self.host = None


def _host_recv(buf, src):
    host = torch.empty(buf.shape, dtype=buf.dtype)
    dist.recv(host, src)
    buf.copy_(host)


def _schedule(kind: str, S: int, s: int, M: int) -> List[tuple]:
    """List of ('F', mb) / ('B', mb) for stage s of S."""
    if kind == "gpipe" or S == 1:
        return [("F", i) for i in range(M)] + [("B", i) for i in reversed(range(M))]
    if kind != "1f1b":
        raise ValueError(f"unknown pp_schedule {kind}")
    warm = min(S - s - 1, M)
    ops = [("F", i) for i in range(warm)]
    f, b = warm, 0
    while f < M:
        ops.append(("F", f))
        f += 1
        ops.append(("B", b))
        b += 1
    while b < M:
        ops.append(("B", b))
        b += 1
    return ops


def run_pipeline(eng) -> None:
    m = eng.mesh
    st = eng.stage
    prog = eng.program
    S, s, M = m.pp, m.pp_idx, eng.n_micro
    T, rows = eng.T, eng.mb_rows
    first, last = s == 0, s == S - 1
    step = eng.opt.step_t
    ctxs: Dict[int, Dict] = {i: {} for i in range(M)}
    outs: Dict[int, torch.Tensor] = {}
    grad_scale = 1.0 / (rows * T * M * m.dp)
    loss_scale = 1.0 / (rows * T * M)
    order = _schedule(eng.tcfg.pp_schedule, S, s, M)
    n_bwd_done = 0
    sends = []
    if not last:
        fill_(eng.loss, 0.0)

    staged = staged_p2p() and eng.device.type == "cuda"

    def isend(t, dst, tag):
        name = f"send_{tag}"
        if staged:  # gloo carries host tensors only: stage through pinned host memory
            prog.comm(lambda: _HostSend(t, dst), name=name)
        else:
            prog.comm(lambda: dist.isend(t, dst), name=name)
        sends.append(name)

    def recv(buf, src, tag):
        name = f"recv_{tag}"
        if staged:
            prog.comm(lambda: _host_recv(buf, src), name=None)
            return
        prog.comm(lambda: dist.irecv(buf, src), name=name)
        prog.wait(name)

    for kind, i in order:
        ids = eng.ids[i * rows:(i + 1) * rows]
        labels = eng.labels[i * rows:(i + 1) * rows]
        row0 = eng.row0 + i * rows
        ctx = ctxs[i]
        if kind == "F":
            if first:
                h = st.embed_forward(ids, step, row0, ctx)
            else:
                recv(eng.recv_x[i], m.pp_prev, f"f{i}")
                h = eng.recv_x[i]
            h = st.stage_forward(h, rows, ctx)
            if last:
                st.head_forward(h, labels, loss_scale, ctx, loss_out=eng.loss, accumulate=(i > 0))
            else:
                outs[i] = h
                isend(h, m.pp_next, f"f{i}")
        else:
            beta = 0.0 if n_bwd_done == 0 else 1.0
            n_bwd_done += 1
            if last:
                dx, dx_c = st.head_backward(ctx, grad_scale, beta)
            else:
                recv(eng.recv_dx[i], m.pp_next, f"b{i}")
                dx = eng.recv_dx[i]
                dx_c = eng.recv_dx_c[i]
                if dx_c is not dx:
                    cast_to_bf16(dx, dx_c)
            dx, dx_c = st.stage_backward(ctx, dx, dx_c, beta)
            if first:
                st.embed_backward(ctx, dx, step, beta)
            else:
                isend(dx, m.pp_prev, f"b{i}")
            outs.pop(i, None)
    for name in sends:
        prog.wait(name)
