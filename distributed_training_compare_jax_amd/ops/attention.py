"""Causal multi-head self-attention core.

Reference: ``model/CausalSelfAttention.py:34-44`` — ``softmax(QKᵀ·hd^-½ + mask)·V`` with an
additive ``-1e9`` causal mask (``model/GPTModel.py:50-51``) and the full ``[B,H,T,T]`` fp32
score tensor materialised.  Here the mask is an in-kernel predicate (``-1e9`` then ``exp``
is exactly 0 in fp32, so the semantics are identical) and the scores never leave the chip:
``csrc/attention.hip`` is a flash-style kernel (online softmax, LSE saved for backward,
P recomputed in backward) on ``mfma_f32_16x16x32_bf16`` with head_dim = 32 = one MFMA K.
fp32 tensors (the exact-fp32 parity mode) run ``csrc/attention_f32.hip``: the same algorithm on
``v_mfma_f32_32x32x2_f32`` (exact f32), again with no ``[B,H,T,T]`` tensor anywhere.

Layout: the fused QKV GEMM writes ``qkv[B, T, 3, H, hd]`` (bf16); attention reads Q/K/V
in place with strides and writes ``o[B, T, H, hd]`` which is directly the out_proj input.
"""

from __future__ import annotations


import torch

from . import _native as N
from .gemm import _workspace


def attn_fwd(qkv: torch.Tensor, n_heads: int, scale: float | None = None, flags: int = 0):
    """qkv [B,T,3*H*hd] → (o [B,T,H*hd], lse [B,H,T] fp32, natural-log units).  ``flags`` (A/B switches of
    ``dtc_attn_fwd``): bit 0 the resident kernel's plain wave → query-group order; bit 2 the 16-row chunked
    kernel; bit 4 the round-4 32-row kernel; bit 5 the round-5 forward at 2 waves per SIMD (the default
    runs it at 3); bit 6 its heavy-first block order (the default assigns query blocks to CU slots
    longest-processing-time-first)."""
    B, T, C3 = qkv.shape
    hd = C3 // (3 * n_heads)
    scale = scale if scale is not None else hd ** -0.5
    if N.library_path(qkv):
        q, k, v = qkv.float().view(B, T, 3, n_heads, hd).unbind(2)
        s = torch.einsum("bthd,bshd->bhts", q, k) * scale
        mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril()
        s = s.masked_fill(~mask, float("-inf"))
        lse = torch.logsumexp(s, -1)
        p = torch.exp(s - lse[..., None])
        o = torch.einsum("bhts,bshd->bthd", p, v).reshape(B, T, n_heads * hd)
        return o.to(qkv.dtype), lse
    assert qkv.dtype in (torch.bfloat16, torch.float32) and qkv.is_contiguous()
    if hd != 32 and hd != 64:
        raise NotImplementedError(f"attention kernel supports head_dim 32/64, got {hd}")
    o = torch.empty(B, T, n_heads * hd, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(B, n_heads, T, dtype=torch.float32, device=qkv.device)
    if qkv.dtype == torch.float32:
        N.check(N.lib().dtc_attn_f32_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, T, n_heads, hd, scale,
                                         N.stream_ptr(qkv.device)), "dtc_attn_f32_fwd")
        return o, lse
    N.check(N.lib().dtc_attn_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, T, n_heads, hd, int(flags), scale,
                                 N.stream_ptr(qkv.device)), "dtc_attn_fwd")
    return o, lse


def attn_bwd(qkv: torch.Tensor, o: torch.Tensor, lse: torch.Tensor, do: torch.Tensor, n_heads: int,
             scale: float | None = None, flags: int = 0) -> torch.Tensor:
    """Returns dqkv [B,T,3*H*hd] (same dtype as qkv).  ``flags`` bit 0 forces the two-round resident
    kernels instead of the fused single-round one (A/B and tests)."""
    B, T, C3 = qkv.shape
    hd = C3 // (3 * n_heads)
    scale = scale if scale is not None else hd ** -0.5
    if N.library_path(qkv):
        q, k, v = qkv.float().view(B, T, 3, n_heads, hd).unbind(2)
        dof = do.float().view(B, T, n_heads, hd)
        s = torch.einsum("bthd,bshd->bhts", q, k) * scale
        mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril()
        s = s.masked_fill(~mask, float("-inf"))
        p = torch.exp(s - lse[..., None])
        dv = torch.einsum("bhts,bthd->bshd", p, dof)
        dp = torch.einsum("bthd,bshd->bhts", dof, v)
        delta = (dof * o.float().view(B, T, n_heads, hd)).sum(-1).permute(0, 2, 1)  # [B,H,T]
        ds = p * (dp - delta[..., None]) * scale
        dq = torch.einsum("bhts,bshd->bthd", ds, k)
        dk = torch.einsum("bhts,bthd->bshd", ds, q)
        return torch.stack([dq, dk, dv], 2).reshape(B, T, C3).to(qkv.dtype)
    assert do.is_contiguous() and o.is_contiguous()
    dqkv = torch.empty_like(qkv)
    L = N.lib()
    if qkv.dtype == torch.float32:
        assert do.dtype == torch.float32 and o.dtype == torch.float32
        ws = _workspace(qkv.device, int(L.dtc_attn_f32_bwd_workspace_bytes(B, T, n_heads, hd)))
        N.check(L.dtc_attn_f32_bwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(), dqkv.data_ptr(), B, T,
                                   n_heads, hd, scale, ws.data_ptr(), ws.numel(), N.stream_ptr(qkv.device)),
                "dtc_attn_f32_bwd")
        return dqkv
    ws = _workspace(qkv.device, int(L.dtc_attn_bwd_workspace_bytes(B, T, n_heads, hd)))
    N.check(L.dtc_attn_bwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(), dqkv.data_ptr(), int(flags),
                           B, T, n_heads, hd, scale, ws.data_ptr(), ws.numel() * ws.element_size(),
                           N.stream_ptr(qkv.device)),
            "dtc_attn_bwd")
    return dqkv


def attn_flops(B: int, T: int, H: int, hd: int, causal: bool = True) -> float:
    f = 4.0 * B * H * T * T * hd
    return f / 2 if causal else f

