"""Fused lm_head + softmax cross-entropy (reference ``model/GPTModel.py:71-72`` and
``train/create_train_step.py:32-34``: ``softmax_cross_entropy_with_integer_labels(...).mean()``).

Forward (GPU): ONE MFMA GEMM ``logits = h·Wᵀ + b`` whose epilogue also emits, per row and
per 128-column tile, the partial ``(max, Σexp)`` of the fp32 accumulators and captures the
label logit — the 4096×50304 fp32 logits (823 MB in the reference) are never re-read for
the forward loss.  Logits are kept only as bf16 (412 MB, trivially resident in 288 GB
HBM) for the backward, which is one streaming pass ``dlogits = (softmax − onehot)·scale``
written in place, followed by the two GEMMs of the Dense backward.

The vocab is padded (``ModelConfig.padded_vocab``); pad columns get ``-inf`` logits, so
their probability and gradient are exactly 0 — identical loss to the unpadded reference.
Vocab-parallel TP: each rank owns columns ``[vocab_start, vocab_start+V_local)``; rows'
``(max, Σexp)`` and label logits are combined across ranks (``parallel/tp.py``).
"""

from __future__ import annotations

import torch

from . import _native as N


def lmhead_logits_partials(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, labels: torch.Tensor,
                           vocab_start: int, n_valid: int, combine: bool = True):
    """Returns ``(logits [M,Vl], rowstat [M,2] (max,Σexp), label_logit [M])`` for the local vocab shard.

    ``n_valid`` = number of real (non-pad) columns in this shard; ``label_logit`` is 0 for rows
    whose label is outside the shard.  ``combine=False`` returns the GEMM's raw per-tile partials
    ``[P, M, 2]`` instead of ``rowstat`` (a single-shard loss feeds them straight to
    :func:`ce_finalize`: one combine launch instead of two)."""
    M, D = h.shape
    Vl = w.shape[0]
    if N.library_path(h):
        logits = h.float() @ w.float().t() + b.float()
        if n_valid < Vl:
            logits[:, n_valid:] = float("-inf")
        mx = logits.max(-1).values
        se = torch.exp(logits - mx[:, None]).sum(-1)
        loc = labels.long() - vocab_start
        inside = (loc >= 0) & (loc < n_valid)
        lab = torch.where(inside, logits.gather(1, loc.clamp(0, Vl - 1)[:, None])[:, 0], torch.zeros(M, device=h.device))
        rs = torch.stack([mx, se], -1)
        return logits.to(h.dtype), (rs if combine else rs.unsqueeze(0)), lab
    L = N.lib()
    f32 = h.dtype == torch.float32  # exact-fp32 parity mode: fp32 logits (csrc/gemm_f32.hip)
    P = int(L.dtc_lmhead_nparts_f32(M, Vl, D) if f32 else L.dtc_lmhead_nparts(M, Vl, D))
    logits = torch.empty(M, Vl, dtype=h.dtype, device=h.device)
    part = torch.empty(P, M, 2, dtype=torch.float32, device=h.device)  # part-major (coalesced epilogue writes)
    # a single shard (combine=False) holds every row's label: the epilogue writes all of lab
    lab = (torch.zeros if combine else torch.empty)(M, dtype=torch.float32, device=h.device)
    from .gemm import _gemm_native

    _gemm_native(0, M, Vl, D, h, h.stride(0), w, w.stride(0), logits, Vl, epi=N.EPI_LMHEAD, bias=b,
                 labels=labels, vocab_start=vocab_start, n_valid=n_valid, part=part, label_out=lab)
    if not combine:
        return logits, part, lab
    rowstat = torch.empty(M, 2, dtype=torch.float32, device=h.device)
    N.check(L.dtc_ce_combine(part.data_ptr(), M, P, 1, M, None, None, rowstat.data_ptr(), 0.0, None, 0,
                             N.stream_ptr(h.device)), "dtc_ce_combine")
    return logits, rowstat, lab


def ce_finalize(rowstats: torch.Tensor, label_logit: torch.Tensor, loss_scale: float,
                loss_out: torch.Tensor | None = None, accumulate: bool = False):
    """rowstats [R, M, 2] (R vocab shards) + label_logit [M] → (lse [M], loss).

    ``loss = scale·Σ(lse − label)`` (1-element fp32), written to / accumulated into ``loss_out``."""
    R, M, _ = rowstats.shape
    if loss_out is None:
        loss_out = torch.zeros(1, dtype=torch.float32, device=rowstats.device)
    if not rowstats.is_cuda:
        mx = rowstats[..., 0].max(0).values
        s = (rowstats[..., 1] * torch.exp(rowstats[..., 0] - mx[None])).sum(0)
        lse = mx + torch.log(s)
        loss = (lse - label_logit).sum() * loss_scale
        if accumulate:
            loss_out.add_(loss)
        else:
            loss_out.fill_(float(loss))
        return lse, loss_out
    lse = torch.empty(M, dtype=torch.float32, device=rowstats.device)
    assert rowstats.is_contiguous()
    N.check(N.lib().dtc_ce_combine(rowstats.data_ptr(), M, R, 1, M, label_logit.data_ptr(), lse.data_ptr(), None,
                                   loss_scale, loss_out.data_ptr(), 1 if accumulate else 0,
                                   N.stream_ptr(rowstats.device)), "dtc_ce_combine")
    return lse, loss_out


def ce_backward_inplace(logits: torch.Tensor, lse: torch.Tensor, labels: torch.Tensor, vocab_start: int,
                        n_valid: int, grad_scale: float, colpart: bool = False):
    """logits → dlogits = (exp(logits − lse) − onehot)·grad_scale (pad columns 0), in place.

    ``colpart=True`` also returns fp32 column partial sums of dlogits ``[R, V]`` (R row chunks)
    from the same pass — the lm_head bias gradient is their column sum (``gemm.colsum``)."""
    M, Vl = logits.shape
    if N.library_path(logits):
        p = torch.exp(logits.float() - lse[:, None])
        if n_valid < Vl:
            p[:, n_valid:] = 0.0
        loc = labels.long() - vocab_start
        inside = (loc >= 0) & (loc < n_valid)
        # one-hot subtraction without a data-dependent shape (graph-capturable on the GPU fp32 path)
        rows = torch.arange(M, device=logits.device)
        p.index_put_((rows, loc.clamp(0, Vl - 1)), -inside.to(p.dtype), accumulate=True)
        logits.copy_((p * grad_scale).to(logits.dtype))
        if colpart:
            return logits, (p * grad_scale).sum(0, keepdim=True)
        return logits
    L = N.lib()
    cp = None
    if colpart:
        R = (M + int(L.dtc_ce_colsum_rows()) - 1) // int(L.dtc_ce_colsum_rows())
        cp = torch.empty(R, Vl, dtype=torch.float32, device=logits.device)
    fn = L.dtc_ce_bwd_f32 if logits.dtype == torch.float32 else L.dtc_ce_bwd
    N.check(fn(logits.data_ptr(), logits.stride(0), lse.data_ptr(), labels.data_ptr(), M, Vl, vocab_start,
               n_valid, grad_scale, N.ptr(cp), N.stream_ptr(logits.device)), "dtc_ce_bwd")
    return (logits, cp) if colpart else logits


def ce_dgrad_fused(logits: torch.Tensor, lse: torch.Tensor, labels: torch.Tensor, vocab_start: int, n_valid: int,
                   grad_scale: float, wt: torch.Tensor, want_dlogits: bool = True):
    """The lm_head backward's first half in ONE kernel (``csrc/gemm.hip`` ce_dgrad256_kernel): the
    cross-entropy backward applied to the logits as they are staged into the dgrad GEMM.

    Returns ``(dx, dlogits, colpart)``: dx = dlogits·W (fp32 [M, d], ``wt`` = Wᵀ [d, V] bf16),
    dlogits (bf16 [M, V], bitwise equal to :func:`ce_backward_inplace`'s, for the weight gradient)
    and the column partial sums of dlogits (fp32 [R, V], the bias gradient's input — summed from
    the bf16 dlogits, where :func:`ce_backward_inplace` sums the fp32 values before rounding).
    The logits are left untouched.  GPU bf16 path only."""
    from .gemm import _workspace

    M, Vl = logits.shape
    D = wt.shape[0]
    assert wt.shape[1] == Vl and logits.dtype == torch.bfloat16 and wt.dtype == torch.bfloat16
    assert logits.is_contiguous() and wt.is_contiguous()
    L = N.lib()
    dl = torch.empty_like(logits) if want_dlogits else None
    cp = torch.empty(int(L.dtc_ce_dgrad_colpart_rows(M)), Vl, dtype=torch.float32, device=logits.device) \
        if want_dlogits else None
    dx = torch.empty(M, D, dtype=torch.float32, device=logits.device)
    nbytes = int(L.dtc_ce_dgrad_workspace_bytes(M, D, Vl))
    ws = _workspace(logits.device, nbytes)
    N.check(L.dtc_ce_dgrad(logits.data_ptr(), logits.stride(0), lse.data_ptr(), labels.data_ptr(), vocab_start, n_valid,
                           grad_scale, wt.data_ptr(), wt.stride(0), N.ptr(dl), 0 if dl is None else dl.stride(0),
                           N.ptr(cp),
                           dx.data_ptr(), M, D, Vl, ws.data_ptr(), ws.numel(), N.stream_ptr(logits.device)),
            "dtc_ce_dgrad")
    return dx, dl, cp


