"""LayerNorm (flax ``nn.LayerNorm`` defaults: eps 1e-6, learned scale and bias).

Reference sites: ``model/TransformerBlock.py:16,22`` and the final LN ``model/GPTModel.py:71``.
Input is the fp32 residual stream; output is the GEMM operand dtype (bf16 on GPU).  The
backward fuses the residual-gradient add (``dx = dres + LN'(dy)``) and emits per-row-block
partials for ``dγ, dβ`` that are reduced deterministically (no float atomics).
GPU path: ``csrc/layernorm.hip`` (one wave64 per row, vectorised 16-B loads).
"""

from __future__ import annotations

from typing import Optional

import torch

from . import _native as N
from .gemm import _workspace


def layernorm_fwd(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float,
                  out_dtype: Optional[torch.dtype] = None):
    M, D = x.shape
    out_dtype = out_dtype or x.dtype
    if not x.is_cuda:
        xf = x.float()
        mean = xf.mean(-1)
        var = (xf - mean[:, None]).pow(2).mean(-1)
        rstd = torch.rsqrt(var + eps)
        y = (xf - mean[:, None]) * rstd[:, None] * g.float() + b.float()
        return y.to(out_dtype), mean, rstd
    assert x.dtype == torch.float32 and x.is_contiguous()
    y = torch.empty(M, D, dtype=out_dtype, device=x.device)
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    N.check(N.lib().dtc_layernorm_fwd(x.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                      rstd.data_ptr(), M, D, eps, 1 if out_dtype == torch.float32 else 0,
                                      N.stream_ptr(x.device)), "dtc_layernorm_fwd")
    return y, mean, rstd


def add_layernorm_fwd(d: torch.Tensor, resid: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float,
                      out_dtype: Optional[torch.dtype] = None):
    """``x = d + resid`` (fp32, written over ``d``) and ``(LN(x), mean, rstd)``: the residual add of the
    layer that produced ``d`` (its GEMM stores ``a·Wᵀ + bias``), done in the LayerNorm pass that reads
    the row anyway instead of in the GEMM epilogue.  Same arithmetic as the fused epilogue
    (``(acc + bias) + resid``).  Returns ``(x, (y, mean, rstd))``.

    ``d`` bf16 (a bf16 GEMM output, ``DTC_FWD_BF16``): ``x = float(d) + resid`` goes to a new fp32 tensor."""
    M, D = d.shape
    out_dtype = out_dtype or resid.dtype
    if d.dtype == torch.bfloat16:
        if not d.is_cuda:
            x = d.float() + resid
            return x, layernorm_fwd(x, g, b, eps, out_dtype)
        assert d.is_contiguous() and resid.dtype == torch.float32 and resid.is_contiguous()
        x = torch.empty(M, D, dtype=torch.float32, device=d.device)
        y = torch.empty(M, D, dtype=out_dtype, device=d.device)
        mean = torch.empty(M, dtype=torch.float32, device=d.device)
        rstd = torch.empty_like(mean)
        N.check(N.lib().dtc_add_layernorm_fwd_bf16(d.data_ptr(), resid.data_ptr(), x.data_ptr(), g.data_ptr(),
                                                   b.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), M, D,
                                                   eps, 1 if out_dtype == torch.float32 else 0,
                                                   N.stream_ptr(d.device)), "dtc_add_layernorm_fwd_bf16")
        return x, (y, mean, rstd)
    if not d.is_cuda:
        d.add_(resid)
        return d, layernorm_fwd(d, g, b, eps, out_dtype)
    assert d.dtype == torch.float32 and d.is_contiguous() and resid.dtype == torch.float32 and resid.is_contiguous()
    y = torch.empty(M, D, dtype=out_dtype, device=d.device)
    mean = torch.empty(M, dtype=torch.float32, device=d.device)
    rstd = torch.empty_like(mean)
    N.check(N.lib().dtc_add_layernorm_fwd(d.data_ptr(), resid.data_ptr(), d.data_ptr(), g.data_ptr(), b.data_ptr(),
                                          y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), M, D, eps,
                                          1 if out_dtype == torch.float32 else 0, N.stream_ptr(d.device)),
            "dtc_add_layernorm_fwd")
    return d, (y, mean, rstd)


def layernorm_bwd(dy: torch.Tensor, x: torch.Tensor, g: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor,
                  dres: Optional[torch.Tensor], dg: torch.Tensor, db: torch.Tensor, beta: float = 0.0,
                  out: Optional[torch.Tensor] = None, out_c: Optional[torch.Tensor] = None,
                  dbias: Optional[torch.Tensor] = None, red=None) -> torch.Tensor:
    """Returns fp32 ``dx = dres + dLN/dx·dy``; writes ``dg/db = β·(dg/db) + Σ_rows`` (β ∈ {0, 1}).

    ``out`` may alias ``dres`` (in-place residual-gradient update); ``out_c`` (optional)
    receives a compute-dtype (bf16) copy of ``dx`` — the next dgrad/wgrad GEMM operand.
    ``dbias`` (optional) receives ``β·dbias + Σ_rows dx``: the bias gradient of the layer whose
    output gradient ``dx`` is (out_proj.b / fc2.b), fused into the same pass."""
    M, D = x.shape
    if not x.is_cuda:
        xhat = (x.float() - mean[:, None]) * rstd[:, None]
        dyf = dy.float()
        gdy = dyf * g.float()
        c1 = gdy.mean(-1, keepdim=True)
        c2 = (gdy * xhat).mean(-1, keepdim=True)
        dx = (gdy - c1 - xhat * c2) * rstd[:, None]
        if dres is not None:
            dx = dx + dres
        sg = (dyf * xhat).sum(0)
        sb = dyf.sum(0)
        if beta != 0.0:
            dg.mul_(beta).add_(sg)
            db.mul_(beta).add_(sb)
        else:
            dg.copy_(sg)
            db.copy_(sb)
        if dbias is not None:
            if beta != 0.0:
                dbias.mul_(beta).add_(dx.sum(0))
            else:
                dbias.copy_(dx.sum(0))
        if out_c is not None:
            out_c.copy_(dx)
        if out is not None:
            out.copy_(dx)
            return out
        return dx
    assert x.is_contiguous() and dy.is_contiguous()
    if out is None:
        out = torch.empty(M, D, dtype=torch.float32, device=x.device)
    L = N.lib()
    nbytes = int(L.dtc_layernorm_bwd_workspace_bytes(M, D))
    ws = _workspace(x.device, nbytes) if red is None else red.alloc(nbytes // 4)
    N.check(L.dtc_layernorm_bwd(dy.data_ptr(), 1 if dy.dtype == torch.float32 else 0, x.data_ptr(), g.data_ptr(),
                                mean.data_ptr(), rstd.data_ptr(), N.ptr(dres), out.data_ptr(), N.ptr(out_c),
                                dg.data_ptr(), db.data_ptr(), N.ptr(dbias), M, D, 1 if beta != 0.0 else 0,
                                ws.data_ptr(), nbytes if red is not None else ws.numel(), 1 if red is not None else 0,
                                N.stream_ptr(x.device)), "dtc_layernorm_bwd")
    if red is not None:  # partials [blocks][nslab][D]: one ordered column reduction per slab
        nslab = 3 if dbias is not None else 2
        blocks = nbytes // 4 // (3 * D)
        for s, dst in enumerate((dg, db, dbias)[:nslab]):
            red.add_tall(ws.data_ptr() + s * D * 4, nslab * D, blocks, dst, 1.0 if beta != 0.0 else 0.0)
    return out
