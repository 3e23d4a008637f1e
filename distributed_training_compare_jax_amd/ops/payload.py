"""bf16 communication payloads with fp32 accumulation (``csrc/payload.hip``).

Used by the DP gradient exchange (``parallel/dp.py``, ``dp_grad_dtype: bf16``) and the PP activation /
gradient messages (``parallel/pp.py``, ``pp_comm_dtype: bf16``).  CPU tensors (the gloo test path) use
the same arithmetic in torch: fp32 sums in shard order, one bf16 rounding.
"""

from __future__ import annotations

import torch

from . import _native as N
from .optim import cast_to_bf16

__all__ = ["cast_to_bf16", "cast_bf16_to_f32", "shard_sum_bf16"]


def cast_bf16_to_f32(src: torch.Tensor, dst: torch.Tensor):
    """dst (fp32) = src (bf16); numel % 8 == 0 on GPU."""
    if not src.is_cuda:
        dst.copy_(src.float())
        return dst
    N.check(N.lib().dtc_cast_bf16_f32(src.data_ptr(), dst.data_ptr(), src.numel(), N.stream_ptr(src.device)),
            "dtc_cast_bf16_f32")
    return dst


def shard_sum_bf16(src: torch.Tensor, nshards: int, out: torch.Tensor):
    """out[i] = bf16(Σ_j src[j·s + i]) with s = out.numel(): fp32 accumulation in shard order."""
    s = out.numel()
    if not src.is_cuda:
        out.copy_(src[:nshards * s].view(nshards, s).float().sum(0).to(torch.bfloat16))
        return out
    N.check(N.lib().dtc_shard_sum_bf16(src.data_ptr(), int(nshards), s, out.data_ptr(), N.stream_ptr(src.device)),
            "dtc_shard_sum_bf16")
    return out
