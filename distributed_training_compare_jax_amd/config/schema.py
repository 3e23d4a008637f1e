"""Configuration schema.

Mirrors the three frozen dataclasses of the reference (``config/schema.py:7-38``):
``ModelConfig``, ``OptimConfig`` and ``TrainConfig`` keep every reference field with
the same name and meaning, so the reference YAML files load unchanged.  New fields
are optional and default to the reference behaviour:

* ``ModelConfig.vocab_pad_multiple`` — the vocab is padded (masked pad logits) to a
  multiple of this so TP works at 4 and 8 GPUs (reference quirk: 50258 = 2*13*1933,
  ``parallel/sharding.py:35``).
* ``TrainConfig.dtype`` — ``bf16`` (MFMA bf16, fp32 master/accum) or ``fp32``.
* ``TrainConfig.dp/tp/pp`` — explicit mesh degrees for hybrid runs (reference: one
  1-D axis, ``train/train.py:29``).
* ``TrainConfig.pp_schedule`` (``gpipe`` | ``1f1b`` | ``zb``: 1F1B with the backward split into the
  input-gradient chain and the deferred weight gradients, the latter placed in the pipeline's idle gaps,
  ``parallel/pp.py``), ``pp_clip`` (``local`` is the
  reference's stage-local global-norm clip, ``create_train_step.py:190``; ``global``
  all-reduces the norm across stages).
* ``TrainConfig.data`` (``synthetic`` | ``fineweb``), ``use_graph``, ``profile`` (roctx
  ranges, device step times and a Chrome trace under ``<output_dir>/trace/``, see
  ``utils/trace.py``), ``watchdog_s`` (abort a rank whose step stalls that long, 0 = off),
  ``dp_bucket_mb`` / ``dp_tail_mb`` (DP grad bucket sizes, cut at layer boundaries and issued as
  soon as their last layer's grads are final; the last bucket is kept small because its
  all-reduce is exposed: for the reference model 98 / 48 / 48 / 36 / 12 MB), ``dp_embed_gather`` (DP: all-gather the embedding
  output grads and rebuild wte/wpe grads locally instead of all-reducing the 103 MB table),
  ``warmup_steps`` (reference hard-codes 5, ``train/train.py:64``), ``ckpt_every``/``resume``,
  ``tp_comm`` (``auto`` | ``p2p`` | ``rccl``: TP activation all-reduces as in-graph xGMI
  peer-to-peer kernels, ``parallel/p2p.py``; ``auto`` = p2p on a GPU RCCL group),
  ``defer_optimizer`` / ``defer_groups`` (run the non-embedding AdamW under the next step's
  forward in that many layer groups, on its own stream with a capped grid, ``DTC_DEFER_BLOCKS``;
  exact, off by default: measured slower at the reference size because the forward GEMMs run
  ~2x slower while the AdamW blocks share their CUs, ``profiles/r2_ab_defer_optimizer.log``),
  ``zero_stage`` (1 = ZeRO-1 Adam-state sharding over the DP group, ``ShardedAdamW``; pure DP only),
  ``wgrad_group`` (weight gradients deferred to grouped launches of that many layers, 0 = the whole
  stage plus the lm_head in one launch, -1 = each Dense's right after its dgrad; None = auto: 0 at
  dp = 1, 2 under DP so each group's buckets overlap the rest of the backward), ``pp_split``
  (``cost``: the contiguous layer split minimising the most expensive stage, counting lm_head + CE as
  ``pp_head_cost`` blocks on the last stage -- default from FLOPs, ``parallel/mesh.py``; ``even``: the
  remainder layers to the earliest stages), ``dp_grad_dtype`` / ``pp_comm_dtype`` / ``tp_comm_dtype`` (``bf16``: the DP
  gradient buckets / PP stage messages / TP partial sums travel as bf16 and are summed in fp32,
  ``ops/payload.py``, ``parallel/tp.py reduce_to``; the TP residual is added after the sum, unrounded).
"""

from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field, replace
from typing import Any, Dict, Optional

PyTree = Any

# GPT-2 BPE (50257) + the added <pad> token (reference data/fineweb_edu.py:8-12, main.py:17-18).
REFERENCE_VOCAB_SIZE = 50258


@dataclass(frozen=True)
class ModelConfig:
    vocab_size: int
    d_model: int
    n_layers: int
    n_heads: int
    d_ff: int
    max_seq_len: int
    dropout: float
    parallel: str = "none"
    # --- extensions (defaults = reference behaviour) ---
    vocab_pad_multiple: int = 128
    layernorm_eps: float = 1e-6  # flax nn.LayerNorm default
    name: str = "gpt-ref-89M"

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def padded_vocab(self) -> int:
        m = max(1, int(self.vocab_pad_multiple))
        return ((self.vocab_size + m - 1) // m) * m

    def num_params(self) -> int:
        """Parameter count of the reference architecture (unpadded vocab)."""
        D, F, V, T, L = self.d_model, self.d_ff, self.vocab_size, self.max_seq_len, self.n_layers
        per_layer = 4 * D * D + 4 * D + D * F + F + F * D + D + 4 * D
        return V * D + T * D + L * per_layer + 2 * D + D * V + V

    def flops_per_token(self, causal: bool = True) -> float:
        """Matmul FLOPs per token, fwd+bwd: 6 * N_matmul + attention.  ``causal`` (default): the useful
        work of the causal attention, (T + 1) / 2 keys per query on average; ``causal=False``: the full
        T x T count SURVEY §2.4 / BASELINE.md's 1.715 TFLOP/step estimate use."""
        D, F, V, T, L = self.d_model, self.d_ff, self.vocab_size, self.max_seq_len, self.n_layers
        mm = L * (4 * D * D + 2 * D * F) + D * V
        keys = (T + 1) / 2.0 if causal else float(T)
        attn = L * 2 * keys * D  # QK^T + PV multiply-adds per token
        return 6.0 * mm + 3.0 * 2.0 * attn


@dataclass(frozen=True)
class OptimConfig:
    lr: float
    weight_decay: float
    grad_clip: float
    # optax.adamw defaults (optax 0.2.6)
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8


@dataclass(frozen=True)
class TrainConfig:
    seed: int
    parallel: str
    # batching
    batch: int
    # steps
    steps: int
    log_every: int
    # output
    output_dir: str
    # pipeline parallelism
    pp_microbatches: int = 1
    # --- extensions ---
    dtype: str = "bf16"
    dp: Optional[int] = None
    tp: Optional[int] = None
    pp: Optional[int] = None
    pp_schedule: str = "gpipe"
    pp_clip: str = "local"
    data: str = "synthetic"
    use_graph: bool = True
    profile: bool = False
    watchdog_s: float = 900.0
    tp_comm: str = "auto"
    defer_optimizer: bool = False
    defer_groups: int = 4
    dp_bucket_mb: float = 40.0
    dp_tail_mb: float = 16.0
    dp_embed_gather: bool = True
    zero_stage: int = 0  # 1 = ZeRO-1: Adam state sharded over the DP group (train/optimizer.py)
    wgrad_group: Optional[int] = None  # deferred grouped weight gradients (models/gpt.py set_wgrad_group)
    pp_split: str = "cost"  # cost | even: PP layer split (parallel/mesh.py split_layers)
    dp_grad_dtype: str = "fp32"  # fp32 | bf16: DP gradient payload (bf16: all-to-all + fp32 shard sums)
    # fp32 | bf16 | auto: PP activation / gradient messages; auto = bf16 when the compute dtype is bf16 (5000-step
    # pp2 curve: the same gap to dp1 as fp32 messages; half the bytes of the latency-bound pp8 hops)
    pp_comm_dtype: str = "auto"
    # fp32 | bf16 | auto: TP row-parallel / input-gradient partials (fp32 sums either way); auto = bf16 when the
    # compute dtype is bf16 (5000-step tp2 curve: the same gap to dp1 as fp32, profiles/r5_cross_strategy.md)
    tp_comm_dtype: str = "auto"
    # Megatron-style sequence parallelism over the TP group (pp == 1, batch % tp == 0): the residual stream,
    # LayerNorms and embedding output on batch/tp sequences per rank; reduce-scatter + all-gather in place of
    # each TP all-reduce (models/gpt.py enable_sequence_parallel).  None = auto: on whenever it applies
    tp_sequence_parallel: Optional[bool] = None
    pp_head_cost: Optional[float] = None  # lm_head + CE in blocks (None: parallel/mesh.py head_cost_blocks)
    # lm_head + CE split by vocab over the last two pipeline stages (1f1b / zb, tp == 1; parallel/pp.py
    # _head_split).  None = auto: on when the head alone outweighs an even share of the model (pp >= 4)
    pp_head_split: Optional[bool] = None
    warmup_steps: int = 5
    ckpt_every: int = 0
    resume: bool = False
    deterministic: bool = False
    # DP collective rehearsal: at dp == 1 on an initialised (one-rank) process group, run the DP code path
    # anyway -- bucket all-reduces, embedding-grad all-gather, loss all-reduce, ZeRO-1 reduce-scatter /
    # all-gather, bf16 all-to-all payloads -- on a one-member communicator (identities: same math as dp1).
    # The one-GPU box uses it to execute the exact RCCL call sequence of a DP step (tests/test_rccl_gpu.py)
    dp_comm_rehearsal: bool = False
    # capture the step's collectives INTO its hipGraph (one graph per step) instead of cutting the graph at
    # each collective and issuing it eagerly between segments (parallel/program.py).  None = auto: on for a
    # ONE-rank RCCL process group (the rehearsal, where it was measured: 11.39-11.41 ms/step captured vs
    # 11.62-11.64 cut, profiles/r5_rccl_rehearsal.md), off at world > 1 until capture has run against real
    # peers (docs/CAPTURE.md), off for gloo; DTC_CAPTURE_COMMS=1 / 0 force it
    capture_comms: Optional[bool] = None
    device: str = "auto"  # auto | cuda | cpu
    batch_is_global: bool = True  # reference: `batch` is the global batch


# Named model presets.  "ref" is the reference's configs/model_config.yaml.
MODEL_PRESETS: Dict[str, Dict[str, Any]] = {
    "ref": dict(d_model=512, n_layers=12, n_heads=16, d_ff=2048, max_seq_len=512, dropout=0.1,
                name="gpt-ref-89M"),
    "gpt2-small": dict(d_model=768, n_layers=12, n_heads=12, d_ff=3072, max_seq_len=1024, dropout=0.1,
                       name="gpt2-small-124M"),
    "gpt2-medium": dict(d_model=1024, n_layers=24, n_heads=16, d_ff=4096, max_seq_len=1024, dropout=0.1,
                        name="gpt2-medium-355M"),
    "tiny": dict(d_model=64, n_layers=2, n_heads=2, d_ff=256, max_seq_len=64, dropout=0.1, name="tiny"),
}


def model_config_from_preset(preset: str, vocab_size: int = REFERENCE_VOCAB_SIZE, **overrides) -> ModelConfig:
    d = dict(MODEL_PRESETS[preset])
    d.update(overrides)
    return ModelConfig(vocab_size=vocab_size, **d)


def _filter_fields(cls, d: Dict[str, Any]) -> Dict[str, Any]:
    names = {f.name for f in dataclasses.fields(cls)}
    unknown = set(d) - names
    if unknown:
        raise TypeError(f"{cls.__name__}: unknown config keys {sorted(unknown)}")
    return d


def load_yaml(path: str) -> Dict[str, Any]:
    import yaml

    with open(path) as f:
        return yaml.safe_load(f) or {}


def build_configs(train_config_path: str, model_config_path: str = "configs/model_config.yaml",
                  optim_config_path: str = "configs/optim_config.yaml",
                  vocab_size: int = REFERENCE_VOCAB_SIZE):
    """Same assembly as reference main.py:14-30: vocab injected, parallel copied into ModelConfig."""
    mdict = load_yaml(model_config_path)
    mdict["vocab_size"] = vocab_size
    tdict = load_yaml(train_config_path)
    train_config = TrainConfig(**_filter_fields(TrainConfig, tdict))
    mdict["parallel"] = train_config.parallel
    model_config = ModelConfig(**_filter_fields(ModelConfig, mdict))
    opt_config = OptimConfig(**_filter_fields(OptimConfig, load_yaml(optim_config_path)))
    return train_config, model_config, opt_config


__all__ = [
    "PyTree", "ModelConfig", "OptimConfig", "TrainConfig", "MODEL_PRESETS", "REFERENCE_VOCAB_SIZE",
    "model_config_from_preset", "build_configs", "load_yaml", "replace", "field",
]
