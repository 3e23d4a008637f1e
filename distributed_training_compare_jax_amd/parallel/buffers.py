"""Flat per-rank parameter / gradient / optimizer-state buffers.

One contiguous fp32 buffer each for master params, grads, Adam m and v (+ a bf16 mirror
of the GEMM-side params) replaces the reference's pytree of 22 leaves.  This is what
makes the MI355X step cheap:

* the fused clip+AdamW (``ops/optim.py``) is ONE launch over the whole buffer;
* DP gradient buckets are plain contiguous slices (grads are laid out in backward
  order), so each RCCL all-reduce / reduce-scatter is one large message;
* wgrad GEMM epilogues write straight into their slice (no autograd accumulation copy);
* checkpoints are a handful of tensors plus an index.

Offsets are 64-element (256-B) aligned for 16-byte vector access.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

from ..models.params import ParamSpec, init_full, local_shape, shard

ALIGN = 64


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class Slot:
    spec: ParamSpec
    offset: int
    shape: Tuple[int, ...]

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


class FlatParams:
    def __init__(self, specs: List[ParamSpec], tp_rank: int, tp_size: int, device, compute_dtype=torch.bfloat16):
        self.specs = specs
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.slots: Dict[str, Slot] = {}
        off = 0
        n_mirror = 0
        seen_nonmirror = False
        for s in specs:
            shp = local_shape(s, tp_size, tp_rank)
            slot = Slot(s, off, shp)
            self.slots[s.name] = slot
            off = _align(off + slot.numel)
            if s.mirror:
                assert not seen_nonmirror, "mirrored params must precede non-mirrored ones"
                n_mirror = off
            else:
                seen_nonmirror = True
        self.numel = max(off, ALIGN)
        self.n_mirror = n_mirror
        f32 = dict(dtype=torch.float32, device=self.device)
        self.params = torch.zeros(self.numel, **f32)
        self.grads = torch.zeros(self.numel, **f32)
        self.exp_avg = torch.zeros(self.numel, **f32)
        self.exp_avg_sq = torch.zeros(self.numel, **f32)
        self.use_mirror = compute_dtype != torch.float32
        self.mirror = (torch.zeros(max(n_mirror, ALIGN), dtype=compute_dtype, device=self.device)
                       if self.use_mirror else None)
        # transposed compute mirror (enable_transposed): name -> (slot, [in, out] bf16 view)
        self.mirror_t: Dict[str, Tuple[Slot, torch.Tensor]] = {}
        self._mirror_t_buf = None

    # -- init -----------------------------------------------------------------
    def init_canonical(self, seed: int):
        for name, slot in self.slots.items():
            full = init_full(slot.spec, seed)
            loc = shard(slot.spec, full, self.tp_rank, self.tp_size)
            self.p(name).copy_(loc.to(self.device))
        self.refresh_mirror()

    def refresh_mirror(self):
        if self.use_mirror and self.n_mirror > 0:
            from ..ops.optim import cast_to_bf16

            cast_to_bf16(self.params[: self.n_mirror], self.mirror[: self.n_mirror])
            self.refresh_transposed()

    # -- transposed mirror --------------------------------------------------------
    def enable_transposed(self, names: List[str]):
        """Keep a transposed bf16 copy ``[in, out]`` of these 2-D mirrored weights (each rebuilt from
        the mirror after every update: :meth:`refresh_transposed`).  With it a Dense's dgrad
        dX = dY·W runs as an NT GEMM (both operands K-major) on the 8-wave kernels instead of reading
        W k-strided (csrc/gemm.hip; measured in the step, profiles/r2_ab_dgrad_nt.log)."""
        names = [n for n in names if n in self.slots and self.slots[n].spec.mirror and len(self.slots[n].shape) == 2]
        if not names or not self.use_mirror:
            return
        total = sum(self.slots[n].numel for n in names)
        self._mirror_t_buf = torch.zeros(total, dtype=self.compute_dtype, device=self.device)
        off = 0
        for n in names:
            sl = self.slots[n]
            rows, cols = sl.shape
            self.mirror_t[n] = (sl, self._mirror_t_buf[off:off + sl.numel].view(cols, rows))
            off += sl.numel
        self.refresh_transposed()

    def refresh_transposed(self, lo: int = 0, hi: int = None):
        """Rebuild the transposed copies of the weights inside flat[lo:hi] from the bf16 mirror."""
        if not self.mirror_t:
            return
        from ..ops.optim import transpose_batch

        hi = self.numel if hi is None else hi
        transpose_batch([(self._view(self.mirror, n), t) for n, (sl, t) in self.mirror_t.items()
                         if sl.offset >= lo and sl.offset + sl.numel <= hi])

    def transposed_in(self, lo: int, hi: int):
        """[(flat offset, rows, cols, W^T)] of the transposed-mirror weights inside flat[lo:hi]."""
        return [(sl.offset, sl.shape[0], sl.shape[1], t) for sl, t in self.mirror_t.values()
                if sl.offset >= lo and sl.offset + sl.numel <= hi]

    def wt(self, name: str):
        """Transposed bf16 view ``[in, out]`` of a weight, or None when not kept."""
        e = self.mirror_t.get(name)
        return None if e is None else e[1]

    # -- views ----------------------------------------------------------------
    def _view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        s = self.slots[name]
        return buf[s.offset: s.offset + s.numel].view(s.shape)

    def p(self, name: str) -> torch.Tensor:
        return self._view(self.params, name)

    def g(self, name: str) -> torch.Tensor:
        return self._view(self.grads, name)

    def w(self, name: str) -> torch.Tensor:
        """Compute-dtype view (bf16 mirror on GPU, fp32 master otherwise)."""
        if self.use_mirror and self.slots[name].spec.mirror:
            return self._view(self.mirror, name)
        return self.p(name)

    def has(self, name: str) -> bool:
        return name in self.slots

    def range_of(self, names: List[str]) -> Tuple[int, int]:
        lo = min(self.slots[n].offset for n in names)
        hi = max(_align(self.slots[n].offset + self.slots[n].numel) for n in names)
        return lo, hi

    def segments(self, weight_fn) -> List[Tuple[int, int, float]]:
        return [(s.offset, s.numel, float(weight_fn(s.spec))) for s in self.slots.values()]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {"params": self.params, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}
