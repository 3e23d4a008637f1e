"""Pure-torch autograd oracle of the reference GPT (fp32, no fusion, no parallelism).

A line-by-line statement of the reference semantics (``model/GPTModel.py``,
``TransformerBlock.py``, ``CausalSelfAttention.py``, ``MLP.py``,
``train/create_train_step.py:30-34``) used only by tests: the explicit fused
forward/backward of ``models/gpt.py`` (CPU path and HIP path) and every parallel layout
must agree with the gradients autograd computes here.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..config.schema import ModelConfig
from ..ops.embedding import dropout_keep_mask


def _gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def oracle_loss(cfg: ModelConfig, params: dict, ids: torch.Tensor, labels: torch.Tensor, seed: int, step: int,
                row0: int = 0) -> torch.Tensor:
    """params: name → fp32 tensor (full shapes, [out,in] Dense layout), requires_grad allowed."""
    B, T = ids.shape
    D, H = cfg.d_model, cfg.n_heads
    hd = D // H
    eps = cfg.layernorm_eps
    h = params["wte"][ids.long()] + params["wpe"][:T][None]
    if cfg.dropout > 0:
        keep = dropout_keep_mask(B * T, D, row0 * T, cfg.dropout, seed, step).view(B, T, D).to(h.device)
        h = torch.where(keep, h / (1 - cfg.dropout), torch.zeros_like(h))
    mask = torch.tril(torch.ones(T, T, device=h.device))
    add_mask = torch.where(mask == 1, 0.0, -1e9)  # GPTModel.py:50-51
    for l in range(cfg.n_layers):
        p = lambda n: params[f"h.{l}.{n}"]  # noqa: E731
        r = h
        x = F.layer_norm(h, (D,), p("ln1.g"), p("ln1.b"), eps)
        qkv = x @ p("qkv.w").t() + p("qkv.b")
        q, k, v = qkv.view(B, T, 3, H, hd).unbind(2)
        s = torch.einsum("bthd,bshd->bhts", q, k) * hd ** -0.5 + add_mask
        a = torch.softmax(s, -1)
        o = torch.einsum("bhts,bshd->bthd", a, v).reshape(B, T, D)
        h = o @ p("out.w").t() + p("out.b") + r
        r = h
        x = F.layer_norm(h, (D,), p("ln2.g"), p("ln2.b"), eps)
        x = _gelu_tanh(x @ p("fc1.w").t() + p("fc1.b"))
        h = x @ p("fc2.w").t() + p("fc2.b") + r
    x = F.layer_norm(h, (D,), params["lnf.g"], params["lnf.b"], eps)
    V = cfg.vocab_size
    logits = x @ params["lm_head.w"][:V].t() + params["lm_head.b"][:V]
    return F.cross_entropy(logits.reshape(-1, V), labels.reshape(-1).long())
