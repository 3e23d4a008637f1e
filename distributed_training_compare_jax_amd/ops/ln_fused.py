"""LayerNorm fused into the layer GEMMs around it (GPU, bf16, tp = pp = 1).

Reference sites: the two pre-LN LayerNorms of every block and the final one
(``model/TransformerBlock.py:16,22``, ``model/GPTModel.py:71``).  Unfused, each LayerNorm is its own
launch and its own full pass over the [tokens, d_model] fp32 residual stream, forward and backward.
Here:

* :func:`linear_resid_ln` — the GEMM that produces the residual stream (out_proj / fc2 forward,
  ``x = resid + a·Wᵀ + b``) also emits ``y = LN(x)`` in bf16 plus the row mean / rstd: the operand of
  the next qkv / fc1 / lm_head GEMM.
* :func:`dgrad_ln_bwd` — the NT dgrad that produces a LayerNorm's output gradient
  (``dy = dY·W`` of fc1 / qkv, on the transposed weight mirror) finishes the LayerNorm backward in its
  epilogue: ``dx = dres + LN'(dy)`` (fp32 + bf16 copy) and the dγ / dβ (/ upstream bias) column
  partials; ``dy`` itself is never stored.

A row of ``d_model`` columns spans ``d_model / 64`` blocks, so the row statistics are exchanged
inside the launch (``csrc/gemm.hip`` "LayerNorm fused into the layer GEMM epilogue"): write-through
partials plus one epoch flag per block in ``sync`` (a zero-initialised int64 buffer shared by all
sites of a stage); epoch = ``step`` (the device step counter) * ``nsites`` + ``site`` (the call's index
in execution order) + 1.  A timed-out wait sets ``err`` and makes the affected rows NaN (never a
hang).  Numerics match the unfused kernels to fp32 rounding (forward: per-chunk mean/M2 combined
with Chan's formula instead of one two-pass row).  Only the backward fusion is on by default
(``DTC_LN_FUSE``, ``profiles/r2_ab_ln_fuse.log``).
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _native as N
from . import gemm as G
from . import layernorm as LN


class LnSync:
    """Granule buffer + error word + site numbering for one model stage's fused LayerNorms."""

    def __init__(self, device, M: int, D: int, nsites: int, step: torch.Tensor):
        words = int(N.lib().dtc_gemm_ln_sync_words(M, D))
        self.buf = torch.zeros(words, dtype=torch.int64, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.M, self.D, self.nsites, self.step = M, D, int(nsites), step

    def check(self):
        if int(self.err.item()) != 0:
            raise RuntimeError("fused LayerNorm: a row-statistics wait timed out (outputs were NaN)")


def supported(M: int, D: int, K: int) -> bool:
    """Shapes the fused kernels take AND where they pay: at most 512 tiles of 128 x 64, i.e. where the
    unfused NT dgrad runs the same 8-wave 128 x 64 plan (csrc/gemm.hip dmaw_plan).  Beyond that (GPT-2
    small / medium at T = 1024: 768 / 1024 tiles) the fused launch measured slower than the unfused
    dgrad + LayerNorm kernels (15.53 vs 14.87 and 37.96 vs 36.81 ms/step)."""
    return (M % 128 == 0 and D % 256 == 0 and D <= 1024 and K % 64 == 0
            and (M // 128) * (D // 64) <= 512)


def _args(bwd: int, a: torch.Tensor, w: torch.Tensor, c: torch.Tensor, sync: LnSync, site: int, **kw) -> "N.LnArgs":
    M, K = a.shape
    D = w.shape[0]
    assert w.shape[1] == K and c.shape == (M, D) and (M, D) == (sync.M, sync.D), (a.shape, w.shape, c.shape)
    assert a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and a.stride(1) == 1 and w.stride(1) == 1
    assert 0 <= site < sync.nsites
    return N.LnArgs(bwd=bwd, M=M, N=D, K=K, A=a.data_ptr(), lda=a.stride(0), B=w.data_ptr(), ldb=w.stride(0),
                    C=c.data_ptr(), sync=sync.buf.data_ptr(), step=sync.step.data_ptr(), site=site,
                    nsites=sync.nsites, err=sync.err.data_ptr(), **kw)


def linear_resid_ln(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], resid: torch.Tensor,
                    gamma: torch.Tensor, beta: torch.Tensor, eps: float, sync: Optional[LnSync] = None,
                    site: int = 0) -> Tuple[torch.Tensor, Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """``x = resid + a·Wᵀ + bias`` (fp32) and ``(LN(x) bf16, mean, rstd)``.  Without ``sync`` (CPU,
    fp32 parity mode): the unfused ops."""
    if sync is None or N.library_path(a):
        x = G.linear_resid(a, w, bias, resid)
        return x, LN.layernorm_fwd(x, gamma, beta, eps, a.dtype)
    M, _ = a.shape
    D = w.shape[0]
    assert resid.dtype == torch.float32 and resid.is_contiguous() and resid.shape == (M, D)
    x = torch.empty(M, D, dtype=torch.float32, device=a.device)
    y = torch.empty(M, D, dtype=torch.bfloat16, device=a.device)
    mean = torch.empty(M, dtype=torch.float32, device=a.device)
    rstd = torch.empty_like(mean)
    args = _args(0, a, w, x, sync, site, bias=N.ptr(bias), resid=resid.data_ptr(), gamma=gamma.data_ptr(),
                 beta=beta.data_ptr(), y=y.data_ptr(), mean=mean.data_ptr(), rstd=rstd.data_ptr(), eps=eps)
    N.check(N.lib().dtc_gemm_ln(args, N.stream_ptr(a.device)), "dtc_gemm_ln(fwd)")
    return x, (y, mean, rstd)


def dgrad_ln_bwd(dY: torch.Tensor, wt: torch.Tensor, x: torch.Tensor, gamma: torch.Tensor, mean: torch.Tensor,
                 rstd: torch.Tensor, dres: Optional[torch.Tensor], dg: torch.Tensor, db: torch.Tensor, beta: float,
                 dbias: Optional[torch.Tensor] = None, red=None, sync: Optional[LnSync] = None,
                 site: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """``dy = dY·wtᵀ`` (``wt`` = the transposed weight mirror [d_model, K]) followed by the LayerNorm
    backward of :func:`layernorm.layernorm_bwd`: returns ``(dx fp32, dx bf16)`` and writes
    ``dg / db (/ dbias) = β·old + Σ_rows`` (through ``red``'s batched launch when given)."""
    if sync is None or N.library_path(dY):
        dy = G.linear_resid(dY, wt, None, None)
        dx_c = None if dY.dtype == torch.float32 else torch.empty(dy.shape, dtype=dY.dtype, device=dy.device)
        dx = LN.layernorm_bwd(dy, x, gamma, mean, rstd, dres, dg, db, beta, out_c=dx_c, dbias=dbias, red=red)
        return dx, (dx if dx_c is None else dx_c)
    M, _ = dY.shape
    D = wt.shape[0]
    assert x.dtype == torch.float32 and x.is_contiguous() and x.shape == (M, D)
    if dres is not None:
        assert dres.dtype == torch.float32 and dres.is_contiguous() and dres.shape == (M, D)
    dx = torch.empty(M, D, dtype=torch.float32, device=dY.device)
    dx_c = torch.empty(M, D, dtype=torch.bfloat16, device=dY.device)
    nslab = 3 if dbias is not None else 2
    P = M // 128
    words = P * nslab * D
    part = red.alloc(words) if red is not None else torch.empty(words, dtype=torch.float32, device=dY.device)
    args = _args(1, dY, wt, dx, sync, site, resid=N.ptr(dres), gamma=gamma.data_ptr(), y=dx_c.data_ptr(),
                 mean=mean.data_ptr(), rstd=rstd.data_ptr(), x=x.data_ptr(), part=part.data_ptr(), nslab=nslab)
    N.check(N.lib().dtc_gemm_ln(args, N.stream_ptr(dY.device)), "dtc_gemm_ln(bwd)")
    acc = 1.0 if beta != 0.0 else 0.0
    outs = (dg, db, dbias)[:nslab]
    if red is not None:  # partials [P][nslab][D]: one ordered column reduction per slab (batched launch)
        for s, dst in enumerate(outs):
            red.add_tall(part.data_ptr() + s * D * 4, nslab * D, P, dst, acc)
    else:  # standalone use (tests)
        for s, dst in enumerate(outs):
            pv = part.view(P, nslab, D)[:, s]
            if acc != 0.0:
                dst.add_(pv.sum(0))
            else:
                dst.copy_(pv.sum(0))
    return dx, dx_c
