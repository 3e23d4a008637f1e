"""Tensor-parallel communication (Megatron-style 1-D TP over RCCL).

Replaces the GSPMD-inserted collectives of the reference TP mode
(``model/CausalSelfAttention.py:28-31,49-50``, ``model/MLP.py:17-18,23-24``,
``parallel/sharding.py:29-60``) with the four explicit all-reduces per block
(out_proj and fc2 outputs in forward; the q/k/v and fc1 input grads in backward) plus the
vocab-parallel cross-entropy reduction (all-gather of per-row (max, Σexp) — 16 KB per
rank — and an all-reduce of the label logit instead of gathering 823 MB of logits).

The row-parallel bias and the residual are folded into ONE rank's GEMM epilogue so the
all-reduce output is directly the new residual stream (no extra elementwise pass).
"""

from __future__ import annotations

import torch
import torch.distributed as dist


class TPComm:
    """``p2p`` (optional :class:`parallel.p2p.P2PAllReduce`) takes the fp32 activation
    all-reduces as in-graph xGMI kernels; everything else goes through RCCL (a graph cut)."""

    def __init__(self, group, size: int, rank: int, program, p2p=None):
        self.group = group
        self.size = size
        self.rank = rank
        self.program = program
        self.p2p = p2p

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return t
        if self.p2p is not None and self.p2p.supports(t):
            return self.p2p.all_reduce_(t)
        g = self.group
        self.program.comm(lambda: dist.all_reduce(t, group=g))
        return t

    def all_gather_stack(self, t: torch.Tensor) -> torch.Tensor:
        """[...] → [size, ...] (shard-major)."""
        if self.size == 1:
            return t.unsqueeze(0)
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        outs = list(out.unbind(0))
        g = self.group
        self.program.comm(lambda: dist.all_gather(outs, t, group=g))
        return out
