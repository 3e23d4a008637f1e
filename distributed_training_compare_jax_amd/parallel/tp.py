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

from .program import csig


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
        if self.p2p is not None and t.dtype == torch.float32 and t.numel() < 4 and t.is_contiguous():
            # a scalar (the grad-norm partial): through a zero-padded 4-float buffer, in-graph
            from ..ops.optim import fill_

            if not hasattr(self, "_pad4"):
                self._pad4 = torch.zeros(4, dtype=torch.float32, device=t.device)
            fill_(self._pad4, 0.0)
            self._pad4[:t.numel()].copy_(t.view(-1))
            self.p2p.all_reduce_(self._pad4)
            t.view(-1).copy_(self._pad4[:t.numel()])
            return t
        g = self.group
        self.program.comm(lambda: dist.all_reduce(t, group=g), sig=csig("all_reduce", g, t))
        return t

    def reduce_to(self, part: torch.Tensor, resid=None, bias=None) -> torch.Tensor:
        """fp32 ``resid + bias + Σ_ranks part`` for a bf16 partial (``tp_comm_dtype: bf16``): the partial
        travels as bf16 and is summed in fp32; the residual and the bias are added once, after the sum, on
        every rank (the residual stream is never rounded).  P2P kernels on GPU; otherwise an fp32
        all-reduce of the bf16-rounded partial (same arithmetic up to summation order)."""
        out = torch.empty(part.shape, dtype=torch.float32, device=part.device)
        if self.size > 1 and self.p2p is not None and self.p2p.supports_bf16(part) and \
                (bias is None or part.shape[-1] % 8 == 0):
            return self.p2p.all_reduce_bf16(part, out, resid, bias)
        out.copy_(part)
        self.all_reduce_(out)
        if resid is not None:
            out.add_(resid)
        if bias is not None:
            out.add_(bias)
        return out

    def partial_out(self, rows: int, cols: int, bias=None):
        """Where a row-parallel GEMM should write its bf16 partial [rows, cols] so the P2P all-reduce
        needs no stage copy (the own half of the P2P buffer, an ``ops.gemm.RawOut``), or None (no P2P,
        size, or a bias the kernels cannot index).  Follow it by :meth:`reduce_staged`."""
        if self.size == 1 or self.p2p is None or (bias is not None and cols % 8):
            return None
        return self.p2p.staged_out(rows * cols)

    def reduce_staged(self, rows: int, cols: int, resid=None, bias=None, device=None) -> torch.Tensor:
        """fp32 ``resid + bias + Σ_ranks partial`` for the partial a GEMM wrote into :meth:`partial_out`."""
        out = torch.empty(rows, cols, dtype=torch.float32, device=device or self.p2p.device)
        return self.p2p.all_reduce_bf16(None, out, resid, bias)

    def all_gather_stack(self, t: torch.Tensor) -> torch.Tensor:
        """[...] → [size, ...] (shard-major).  With the P2P path: every rank writes its slot of a
        zeroed [size, ...] buffer and the buffer is summed (x + 0 = x exactly, so it IS the gather),
        in-graph, no RCCL call."""
        if self.size == 1:
            return t.unsqueeze(0)
        if self.p2p is not None and t.dtype == torch.float32 and (t.numel() * self.size) % 4 == 0 \
                and t.numel() * self.size * 4 <= self.p2p.half:
            from ..ops.optim import fill_

            out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            fill_(out, 0.0)
            out[self.rank].copy_(t)
            self.p2p.all_reduce_(out.view(-1))
            return out
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        outs = list(out.unbind(0))
        g = self.group
        self.program.comm(lambda: dist.all_gather(outs, t, group=g), sig=csig("all_gather", g, t))
        return out

    # ---- sequence parallelism (TrainConfig.tp_sequence_parallel): the residual stream, the LayerNorms and
    # the embedding output live on rows/size rows per rank; the all-reduce after a row-parallel GEMM becomes
    # a reduce-scatter and the LayerNorm output feeding a column-parallel GEMM is all-gathered (Megatron-LM
    # sequence parallelism: the same bytes as the all-reduce, LN / residual work divided by tp)
    def _rccl(self) -> bool:
        return dist.get_backend(self.group) == "nccl"

    def reduce_scatter_rows(self, part: torch.Tensor, resid=None, bias=None) -> torch.Tensor:
        """fp32 [rows/size, cols] = resid + bias + Σ_ranks part[this rank's rows] for a [rows, cols] partial
        (bf16 or fp32)."""
        rows, cols = part.shape
        rl = rows // self.size
        out = torch.empty(rl, cols, dtype=torch.float32, device=part.device)
        if self.p2p is not None and part.is_cuda and part.is_contiguous() and \
                self.p2p.supports_rs(rows, cols, part.dtype) and (bias is None or cols % 8 == 0):
            return self.p2p.reduce_scatter(part, rows, cols, part.dtype, out, resid, bias)
        full = part.float() if part.dtype != torch.float32 else part.clone()
        g = self.group
        if self._rccl():
            self.program.comm(lambda: dist.reduce_scatter_tensor(out, full, group=g),
                              sig=csig("reduce_scatter", g, full))
        else:  # gloo: no reduce-scatter; all-reduce and keep the own rows (same sum)
            self.program.comm(lambda: dist.all_reduce(full, group=g), sig=csig("all_reduce", g, full))
            out.copy_(full[self.rank * rl:(self.rank + 1) * rl])
        if resid is not None:
            out.add_(resid)
        if bias is not None:
            out.add_(bias)
        return out

    def partial_out_rows(self, rows: int, cols: int, dtype, bias=None):
        """Where a row-parallel GEMM writes its [rows, cols] partial for :meth:`reduce_scatter_staged` (the
        own P2P buffer half), or None."""
        if self.p2p is None or not self.p2p.supports_rs(rows, cols, dtype) or (bias is not None and cols % 8):
            return None
        return self.p2p.staged_out(rows * cols, dtype)

    def reduce_scatter_staged(self, rows: int, cols: int, dtype, resid=None, bias=None, device=None):
        out = torch.empty(rows // self.size, cols, dtype=torch.float32, device=device or self.p2p.device)
        return self.p2p.reduce_scatter(None, rows, cols, dtype, out, resid, bias)

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        """[rows, ...] on every rank → [size * rows, ...] (rank-major)."""
        out = torch.empty((self.size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        if self.p2p is not None and self.p2p.supports_ag(x):
            return self.p2p.all_gather(x.contiguous(), out)
        g = self.group
        xc = x.contiguous()
        if self._rccl():
            self.program.comm(lambda: dist.all_gather_into_tensor(out, xc, group=g), sig=csig("all_gather", g, xc))
        else:
            outs = list(out.chunk(self.size, 0))
            self.program.comm(lambda: dist.all_gather(outs, xc, group=g), sig=csig("all_gather", g, xc))
        return out

