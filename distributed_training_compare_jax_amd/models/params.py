"""Parameter inventory, canonical initialisation and tensor-parallel sharding rules.

Reference parameter tree (flax, ``model/*.py``): ``wte``, ``wpe`` (nn.Embed,
``GPTModel.py:30-34``), per layer ``LayerNorm_0/1``, ``q_proj/k_proj/v_proj/out_proj``
(``CausalSelfAttention.py:18-46``), ``fc1/fc2`` (``MLP.py:13-20``), stacked on a leading
layer axis by ``nn.scan`` (``GPTModel.py:58-64``), then the final ``LayerNorm`` and
``lm_head`` (``GPTModel.py:71-72``).  Here:

* Dense kernels are stored ``[out, in]`` (transpose of flax) and q/k/v are fused into one
  ``qkv.w [3D, D]`` (same lecun-normal fan_in = D distribution as three separate kernels).
* ``lm_head`` is padded to ``padded_vocab`` rows (zero rows, masked logits).
* **Canonical init**: every full tensor is drawn from a generator seeded by
  ``(seed, crc32(name))`` and then sliced, so DP, TP, PP and hybrid layouts start from
  bit-identical weights (the reference's PP init differs from DP/TP,
  ``train/train.py:120-153``; SURVEY App. B "fix").
* TP rules mirror ``parallel/sharding.py:29-60`` (column-parallel qkv/fc1, row-parallel
  out/fc2, vocab-parallel lm_head) except that column-parallel BIASES are sharded with
  their kernels (no extra comm) and the vocab is padded so N=4/8 work.
* Attention is sharded by whole HEADS (``CausalSelfAttention.py:28-31``): qkv rows and out_proj
  input columns follow :func:`head_split`, which also covers a head count the TP degree does not
  divide (GPT-2 small's 12 heads on 8 ranks: 2,2,2,2,1,1,1,1 -- the reference cannot shard it at
  all).  Everything else (fc1/fc2, the padded vocab) splits evenly.

Flat-buffer order = the order backward produces gradients (head → layers L-1..0 →
embeddings), so DP buckets are contiguous ranges that become ready in sequence.
"""

from __future__ import annotations

import math
import zlib
from dataclasses import dataclass
from typing import List, Tuple

import torch

from ..config.schema import ModelConfig

_TRUNC = 0.87962566103423978  # std of a unit normal truncated to [-2, 2]


@dataclass(frozen=True)
class ParamSpec:
    name: str
    shape: Tuple[int, ...]     # full (unsharded) shape
    init: str                  # embed | dense | zeros | ones
    fan_in: int
    tp: str                    # rep | rows | cols | qkv_rows | head_cols
    layer: int                 # -1 embed, -2 head, else layer index
    mirror: bool               # has a bf16 compute copy (GEMM weight / bias / LN)
    valid_rows: int = -1       # for padded lm_head: rows >= valid_rows are zero
    heads: int = 0             # head-sharded (qkv_rows / head_cols): attention heads along the split dim
    # (part, parts): the lm_head vocab split over the last `parts` PIPELINE stages (pp_head_split), applied
    # before the TP split: this stage holds rows [part * Vp / parts, (part + 1) * Vp / parts)
    vpart: Tuple[int, int] = (0, 1)


def layer_param_specs(cfg: ModelConfig, l: int) -> List[ParamSpec]:
    D, F, H = cfg.d_model, cfg.d_ff, cfg.n_heads
    p = f"h.{l}."
    # backward production order inside a block
    return [
        ParamSpec(p + "fc2.w", (D, F), "dense", F, "cols", l, True),
        ParamSpec(p + "fc2.b", (D,), "zeros", F, "rep", l, True),
        ParamSpec(p + "fc1.w", (F, D), "dense", D, "rows", l, True),
        ParamSpec(p + "fc1.b", (F,), "zeros", D, "rows", l, True),
        ParamSpec(p + "ln2.g", (D,), "ones", D, "rep", l, True),
        ParamSpec(p + "ln2.b", (D,), "zeros", D, "rep", l, True),
        ParamSpec(p + "out.w", (D, D), "dense", D, "head_cols", l, True, heads=H),
        ParamSpec(p + "out.b", (D,), "zeros", D, "rep", l, True),
        ParamSpec(p + "qkv.w", (3 * D, D), "dense", D, "qkv_rows", l, True, heads=H),
        ParamSpec(p + "qkv.b", (3 * D,), "zeros", D, "qkv_rows", l, True, heads=H),
        ParamSpec(p + "ln1.g", (D,), "ones", D, "rep", l, True),
        ParamSpec(p + "ln1.b", (D,), "zeros", D, "rep", l, True),
    ]


def head_param_specs(cfg: ModelConfig, part: int = 0, parts: int = 1) -> List[ParamSpec]:
    """lm_head (+ the final LayerNorm on part 0); ``parts`` > 1: this pipeline stage's vocab slice of a head
    split over the last ``parts`` stages (``pp_head_split``)."""
    D, Vp = cfg.d_model, cfg.padded_vocab
    vp = (int(part), int(parts))
    out = [
        ParamSpec("lm_head.w", (Vp, D), "dense", D, "rows", -2, True, valid_rows=cfg.vocab_size, vpart=vp),
        ParamSpec("lm_head.b", (Vp,), "zeros", D, "rows", -2, True, valid_rows=cfg.vocab_size, vpart=vp),
    ]
    if part == 0:
        out += [ParamSpec("lnf.g", (D,), "ones", D, "rep", -2, True),
                ParamSpec("lnf.b", (D,), "zeros", D, "rep", -2, True)]
    return out


def embed_param_specs(cfg: ModelConfig) -> List[ParamSpec]:
    D = cfg.d_model
    return [
        ParamSpec("wpe", (cfg.max_seq_len, D), "embed", D, "rep", -1, False),
        ParamSpec("wte", (cfg.vocab_size, D), "embed", D, "rep", -1, False),
    ]


def all_param_specs(cfg: ModelConfig) -> List[ParamSpec]:
    out = head_param_specs(cfg)
    for l in reversed(range(cfg.n_layers)):
        out += layer_param_specs(cfg, l)
    return out + embed_param_specs(cfg)


def stage_param_specs(cfg: ModelConfig, layers: range, has_embed: bool, has_head: bool,
                      head_part: Tuple[int, int] = (0, 1)) -> List[ParamSpec]:
    out: List[ParamSpec] = []
    if has_head:
        out += head_param_specs(cfg, *head_part)
    for l in reversed(list(layers)):
        out += layer_param_specs(cfg, l)
    if has_embed:
        out += embed_param_specs(cfg)
    return out


def _gen(seed: int, name: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((int(seed) * 1_000_003 + zlib.crc32(name.encode())) & 0x7FFFFFFFFFFFFFFF)
    return g


def init_full(spec: ParamSpec, seed: int) -> torch.Tensor:
    """Canonical fp32 init of the FULL tensor (flax defaults, see module docstring)."""
    shape = spec.shape
    if spec.init == "zeros":
        return torch.zeros(shape)
    if spec.init == "ones":
        return torch.ones(shape)
    g = _gen(seed, spec.name)
    if spec.init == "embed":  # flax default_embed_init: normal, std 1/sqrt(features)
        return torch.randn(shape, generator=g) * (1.0 / math.sqrt(spec.shape[-1]))
    if spec.init == "dense":  # lecun_normal: truncated normal [-2σ, 2σ], σ = sqrt(1/fan_in)/0.8796
        lo, hi = 0.5 * (1 + math.erf(-2 / math.sqrt(2))), 0.5 * (1 + math.erf(2 / math.sqrt(2)))
        u = torch.rand(shape, generator=g, dtype=torch.float64) * (hi - lo) + lo
        z = torch.erfinv(2 * u - 1) * math.sqrt(2.0)
        t = (z * (math.sqrt(1.0 / spec.fan_in) / _TRUNC)).float()
        if spec.valid_rows >= 0:
            t[spec.valid_rows:] = 0.0
        return t
    raise ValueError(spec.init)


def head_split(n_heads: int, tp_size: int) -> List[Tuple[int, int]]:
    """(first head, heads) of each TP rank: whole heads, the first ``n_heads % tp`` ranks one more."""
    if n_heads < tp_size:
        raise ValueError(f"n_heads {n_heads} < tp {tp_size}: every TP rank needs at least one attention head")
    base, rem = divmod(n_heads, tp_size)
    out, h0 = [], 0
    for r in range(tp_size):
        n = base + (1 if r < rem else 0)
        out.append((h0, n))
        h0 += n
    return out


def _head_range(spec: ParamSpec, width: int, tp_rank: int, tp_size: int) -> Tuple[int, int]:
    """[lo, hi) of a head-sharded dimension of ``width`` = heads * head_dim owned by ``tp_rank``."""
    hd = width // spec.heads
    h0, n = head_split(spec.heads, tp_size)[tp_rank]
    return h0 * hd, (h0 + n) * hd


def local_shape(spec: ParamSpec, tp_size: int, tp_rank: int = 0) -> Tuple[int, ...]:
    s = list(spec.shape)
    if spec.vpart[1] > 1:
        assert s[0] % spec.vpart[1] == 0, f"{spec.name}: dim0 {s[0]} not divisible by {spec.vpart[1]} head stages"
        s[0] //= spec.vpart[1]
    if tp_size == 1 or spec.tp == "rep":
        return tuple(s)
    if spec.tp == "qkv_rows" and spec.heads:
        lo, hi = _head_range(spec, s[0] // 3, tp_rank, tp_size)
        s[0] = 3 * (hi - lo)
    elif spec.tp == "head_cols":
        lo, hi = _head_range(spec, s[1], tp_rank, tp_size)
        s[1] = hi - lo
    elif spec.tp in ("rows", "qkv_rows"):
        assert s[0] % tp_size == 0, f"{spec.name}: dim0 {s[0]} not divisible by tp={tp_size}"
        s[0] //= tp_size
    elif spec.tp == "cols":
        assert s[1] % tp_size == 0, f"{spec.name}: dim1 {s[1]} not divisible by tp={tp_size}"
        s[1] //= tp_size
    return tuple(s)


def shard(spec: ParamSpec, full: torch.Tensor, tp_rank: int, tp_size: int) -> torch.Tensor:
    if spec.vpart[1] > 1:  # this stage's vocab slice first, then the TP split of it
        full = full.chunk(spec.vpart[1], 0)[spec.vpart[0]].contiguous()
    if tp_size == 1 or spec.tp == "rep":
        return full
    if spec.tp == "rows":
        return full.chunk(tp_size, 0)[tp_rank].contiguous()
    if spec.tp == "cols":
        return full.chunk(tp_size, 1)[tp_rank].contiguous()
    if spec.tp == "head_cols":
        lo, hi = _head_range(spec, full.shape[1], tp_rank, tp_size)
        return full[:, lo:hi].contiguous()
    if spec.tp == "qkv_rows":  # [3D, ...] -> per q/k/v slab, heads split
        three = full.reshape(3, full.shape[0] // 3, *full.shape[1:])
        if spec.heads:
            lo, hi = _head_range(spec, three.shape[1], tp_rank, tp_size)
            return three[:, lo:hi].reshape(-1, *full.shape[1:]).contiguous()
        return three.chunk(tp_size, 1)[tp_rank].reshape(-1, *full.shape[1:]).contiguous()
    raise ValueError(spec.tp)


def unshard(spec: ParamSpec, shards: List[torch.Tensor]) -> torch.Tensor:
    """Inverse of :func:`shard` (checkpoint re-sharding / tests)."""
    if len(shards) == 1 or spec.tp == "rep":
        return shards[0]
    if spec.tp == "rows":
        return torch.cat(shards, 0)
    if spec.tp in ("cols", "head_cols"):
        return torch.cat(shards, 1)
    if spec.tp == "qkv_rows":
        parts = [s.reshape(3, s.shape[0] // 3, *s.shape[1:]) for s in shards]
        return torch.cat(parts, 1).reshape(-1, *shards[0].shape[1:])
    raise ValueError(spec.tp)
