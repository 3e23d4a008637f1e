"""Fused clip-by-global-norm + AdamW over flat fp32 buffers.

Reference: ``train/create_optimizer.py:8-12`` —
``optax.chain(clip_by_global_norm(1.0), adamw(lr=3e-4, weight_decay=0.1))`` with optax
defaults (b1 0.9, b2 0.999, eps 1e-8, eps_root 0, bias correction, decoupled decay on
ALL params, no mask):

    g ← g·min(1, max_norm/‖g‖)         (optax: where(‖g‖ < max, g, g/‖g‖·max))
    m ← b1·m + (1−b1)·g ;  v ← b2·v + (1−b2)·g²
    p ← p − lr·( m/(1−b1ᵗ) / (√(v/(1−b2ᵗ)) + eps) + wd·p )

GPU path (``csrc/optim.hip``): (1) a deterministic two-stage Σg² over a segment table
(each segment carries a weight so TP-replicated params are counted once across ranks),
whose finalize kernel also bumps the device step counter; (2) ONE streaming kernel over
the whole flat buffer that applies clip+AdamW and writes the bf16 compute mirror of the
weights — no per-parameter launches, no host sync (graph-capturable).
"""

from __future__ import annotations

import ctypes

from typing import Optional

import torch

from . import _native as N
from .gemm import _workspace


def make_segments(segments, device) -> torch.Tensor:
    """segments: list of (offset, length, weight) → packed float64 tensor [S, 3] for the kernel."""
    t = torch.tensor([[float(o), float(n), float(w)] for (o, n, w) in segments], dtype=torch.float64)
    return t.to(device)


def sumsq_segments(flat: torch.Tensor, segments: torch.Tensor, out: torch.Tensor,
                   step: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[0] = Σ_s w_s·Σ_{i∈s} flat[i]²  (fp32).  If ``step`` is given it is incremented by 1."""
    if not flat.is_cuda:
        acc = torch.zeros((), dtype=torch.float64)
        for o, n, w in segments.tolist():
            seg = flat[int(o):int(o) + int(n)].double()
            acc += w * (seg * seg).sum()
        out.fill_(float(acc))
        if step is not None:
            step.add_(1)
        return out
    L = N.lib()
    ws = _workspace(flat.device, int(L.dtc_sumsq_workspace_bytes()))
    N.check(L.dtc_sumsq_segments(flat.data_ptr(), segments.data_ptr(), segments.shape[0], out.data_ptr(),
                                 N.ptr(step), ws.data_ptr(), ws.numel(), N.stream_ptr(flat.device)),
            "dtc_sumsq_segments")
    return out


def sumsq_partial(flat: torch.Tensor, segments: torch.Tensor, part: torch.Tensor):
    """part[:] = per-block partial Σ w·g² over ``segments`` (one chunk of an incremental norm)."""
    if not flat.is_cuda:
        acc = torch.zeros((), dtype=torch.float64)
        for o, n, w in segments.tolist():
            seg = flat[int(o):int(o) + int(n)].double()
            acc += w * (seg * seg).sum()
        part.zero_()
        part[0] = float(acc)
        return part
    N.check(N.lib().dtc_sumsq_partial(flat.data_ptr(), segments.data_ptr(), segments.shape[0], part.data_ptr(),
                                      part.numel(), N.stream_ptr(flat.device)), "dtc_sumsq_partial")
    return part


def sum_finish(part: torch.Tensor, out: torch.Tensor, step: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[0] = Σ part (fixed order, fp64 accumulate); bumps ``step`` if given."""
    if not part.is_cuda:
        out.fill_(float(part.double().sum()))
        if step is not None:
            step.add_(1)
        return out
    N.check(N.lib().dtc_sum_finish(part.data_ptr(), part.numel(), out.data_ptr(), N.ptr(step),
                                   N.stream_ptr(part.device)), "dtc_sum_finish")
    return out


def adamw_flat(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
               mirror: Optional[torch.Tensor], n_mirror: int, step: torch.Tensor, sumsq: torch.Tensor,
               lr: float, b1: float, b2: float, eps: float, wd: float, max_norm: float,
               enable: Optional[torch.Tensor] = None, max_blocks: int = 0):
    """In-place AdamW on flat fp32 buffers; ``mirror[:n_mirror] = bf16(p[:n_mirror])``.

    ``step`` (int64 [1], already incremented) gives t for the bias correction; ``sumsq``
    (fp32 [1]) is the global Σg² for the clip.  ``enable`` (fp32 [1], optional): the update is
    skipped when ``enable[0] == 0`` (device-side switch for the deferred optimizer).  ``max_blocks``
    (GPU, > 0): cap the grid (grid-stride loop) so the pass shares the CUs with concurrent kernels."""
    n = p.numel()
    if not p.is_cuda:
        if enable is not None and float(enable.item()) == 0.0:
            return
        t = float(step.item())
        norm = float(sumsq.item()) ** 0.5
        scale = 1.0 if (max_norm <= 0 or norm < max_norm) else max_norm / norm
        gg = g * scale
        m.mul_(b1).add_(gg, alpha=1 - b1)
        v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
        mhat = m / (1 - b1 ** t)
        vhat = v / (1 - b2 ** t)
        p.sub_(lr * (mhat / (vhat.sqrt() + eps) + wd * p))
        if mirror is not None and n_mirror > 0:
            mirror[:n_mirror].copy_(p[:n_mirror])
        return
    N.check(N.lib().dtc_adamw(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), N.ptr(mirror), n, n_mirror,
                              step.data_ptr(), sumsq.data_ptr(), lr, b1, b2, eps, wd, max_norm, N.ptr(enable),
                              int(max_blocks), N.stream_ptr(p.device)), "dtc_adamw")


def cast_to_bf16(src: torch.Tensor, dst: torch.Tensor):
    if not src.is_cuda:
        dst.copy_(src)
        return
    N.check(N.lib().dtc_cast_f32_bf16(src.data_ptr(), dst.data_ptr(), src.numel(), N.stream_ptr(src.device)),
            "dtc_cast_f32_bf16")


class _TrTask(ctypes.Structure):
    """Mirror of ``struct TrTask`` (csrc/elementwise.hip)."""

    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("rows", ctypes.c_int), ("cols", ctypes.c_int),
                ("blk0", ctypes.c_int), ("pad", ctypes.c_int)]


_TR_MAX = 32


class _TrBatch(ctypes.Structure):
    _fields_ = [("ntasks", ctypes.c_int), ("nblocks", ctypes.c_int), ("t", _TrTask * _TR_MAX)]


def transpose_batch(pairs):
    """dst = src.T for each (src [rows, cols], dst [cols, rows]) bf16 pair: one launch per 32 matrices
    on GPU (the transposed weight mirror), torch on CPU."""
    if not pairs:
        return
    if not pairs[0][0].is_cuda:
        for src, dst in pairs:
            dst.copy_(src.t())
        return
    L = N.lib()
    assert L.dtc_tr_task_bytes() == ctypes.sizeof(_TrTask) and L.dtc_tr_max_tasks() == _TR_MAX
    for i in range(0, len(pairs), _TR_MAX):
        chunk = pairs[i:i + _TR_MAX]
        b = _TrBatch()
        b.ntasks = len(chunk)
        blk = 0
        for j, (src, dst) in enumerate(chunk):
            rows, cols = src.shape
            assert tuple(dst.shape) == (cols, rows) and src.is_contiguous() and dst.is_contiguous()
            b.t[j] = _TrTask(src.data_ptr(), dst.data_ptr(), rows, cols, blk, 0)
            blk += ((rows + 63) // 64) * ((cols + 63) // 64)
        b.nblocks = blk
        N.check(L.dtc_transpose_batch(ctypes.byref(b), N.stream_ptr(src.device)), "dtc_transpose_batch")


class _AwSeg(ctypes.Structure):
    """Mirror of ``struct AwSeg`` (csrc/elementwise.hip)."""

    _fields_ = [("lo", ctypes.c_long), ("n", ctypes.c_long), ("blk0", ctypes.c_int), ("pad", ctypes.c_int)]


_AW_SEG_MAX, _AW_TASK_MAX = 96, 64


class _AwSegs(ctypes.Structure):
    _fields_ = [("nseg", ctypes.c_int), ("nblocks", ctypes.c_int), ("s", _AwSeg * _AW_SEG_MAX)]


class _AwtTask(ctypes.Structure):
    _fields_ = [("off", ctypes.c_long), ("dst", ctypes.c_void_p), ("rows", ctypes.c_int), ("cols", ctypes.c_int),
                ("blk0", ctypes.c_int), ("pad", ctypes.c_int)]


class _AwtBatch(ctypes.Structure):
    _fields_ = [("ntasks", ctypes.c_int), ("nblocks", ctypes.c_int), ("t", _AwtTask * _AW_TASK_MAX)]


def adamw_tr_plan(lo: int, hi: int, mats):
    """Launch lists of :func:`adamw_tr` over flat[lo:hi]: ``mats`` = [(offset, rows, cols, W^T tensor)] of the
    weights that keep a transposed mirror (inside the range).  Returns [(segments, tiles)] chunks (each
    within the kernels' list capacities), or None when a shape does not fit the tiled kernel."""
    mats = sorted(mats, key=lambda x: x[0])
    if any(r % 8 or c % 4 or o % 4 for o, r, c, _ in mats):
        return None
    segs, cur = [], lo
    for o, r, c, _ in mats:
        if o > cur:
            segs.append((cur, o - cur))
        cur = o + r * c
    if hi > cur:
        segs.append((cur, hi - cur))
    if any(a % 4 or n % 4 for a, n in segs):
        return None
    chunks = []
    while segs or mats:
        sb, tb = _AwSegs(), _AwtBatch()
        blk = 0
        take = segs[:_AW_SEG_MAX]
        segs = segs[_AW_SEG_MAX:]
        for j, (a, n) in enumerate(take):
            sb.s[j] = _AwSeg(a, n, blk, 0)
            blk += (n + 4095) // 4096
        sb.nseg, sb.nblocks = len(take), blk
        blk = 0
        tk = mats[:_AW_TASK_MAX]
        mats = mats[_AW_TASK_MAX:]
        for j, (o, r, c, dst) in enumerate(tk):
            assert tuple(dst.shape) == (c, r) and dst.is_contiguous()
            tb.t[j] = _AwtTask(o, dst.data_ptr(), r, c, blk, 0)
            blk += ((r + 63) // 64) * ((c + 63) // 64)
        tb.ntasks, tb.nblocks = len(tk), blk
        chunks.append((sb, tb))
    return chunks


def adamw_tr(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, mirror: torch.Tensor, n_mirror: int,
             plan, step: torch.Tensor, sumsq: torch.Tensor, lr: float, b1: float, b2: float, eps: float, wd: float,
             max_norm: float):
    """AdamW over the flat buffers (absolute offsets in ``plan``, :func:`adamw_tr_plan`) with the transposed
    bf16 mirror of the tiled weights written by the update itself (no separate transpose pass).  GPU only;
    bitwise equal to :func:`adamw_flat` + :func:`transpose_batch`."""
    L = N.lib()
    assert L.dtc_aw_seg_bytes() == ctypes.sizeof(_AwSeg) and L.dtc_aw_task_bytes() == ctypes.sizeof(_AwtTask)
    assert L.dtc_aw_max_seg() == _AW_SEG_MAX and L.dtc_aw_max_tasks() == _AW_TASK_MAX
    for sb, tb in plan:
        N.check(L.dtc_adamw_tr(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), mirror.data_ptr(), n_mirror,
                               ctypes.byref(sb), ctypes.byref(tb), step.data_ptr(), sumsq.data_ptr(), lr, b1, b2, eps,
                               wd, max_norm, N.stream_ptr(p.device)), "dtc_adamw_tr")


def fill_(t: torch.Tensor, value: float):
    """t[:] = value (fp32; graph-capturable on GPU)."""
    if not t.is_cuda:
        t.fill_(value)
        return t
    N.check(N.lib().dtc_fill_f32(t.data_ptr(), value, t.numel(), N.stream_ptr(t.device)), "dtc_fill_f32")
    return t
