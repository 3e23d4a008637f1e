"""Grouped weight gradients (csrc/gemm.hip gemm8p_group_kernel, ops/gemm.py wgrad_group): one launch of
whole 256^2 tiles over several problems that share K (the tokens) -- dW = beta*dW + dY^T X and
db = beta*db + colsum(dY) -- against the fp32 PyTorch reference of the same op, on the GPT-2 small layer
shapes (+ the lm_head's, a ragged width and a TP-shard width) and with beta = 1 (pipeline
microbatch accumulation)."""

import pytest
import torch

from distributed_training_compare_jax_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def _r(*shape, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    t = torch.randn(*shape, generator=g) + 0.1 * torch.rand(*shape, generator=g)
    return t.to("cuda").to(dtype)


def _close(a, b, rtol, name):
    err = (a.float() - b.float()).abs().max().item()
    ref = b.float().abs().max().item() + 1e-6
    assert err <= rtol * ref, f"{name}: max abs err {err:.3e} vs ref max {ref:.3e}"


# (out features M, in features N) of a GPT-2 small layer's four Dense + out-of-pattern widths
SHAPES = [(768, 3072), (3072, 768), (768, 768), (2304, 768), (200, 768), (384, 96)]


@pytest.mark.parametrize("K", [8192, 1024])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_group_matches_reference(cuda, K, beta):
    items, refs = [], []
    for i, (M, Nn) in enumerate(SHAPES):
        dy, x = _r(K, M, seed=3 * i), _r(K, Nn, seed=3 * i + 1)
        dw = _r(M, Nn, seed=3 * i + 2, dtype=torch.float32)
        db = _r(M, seed=7 * i + 5, dtype=torch.float32) if i % 2 == 0 else None
        rw = beta * dw + dy.float().t() @ x.float()
        rb = None if db is None else beta * db + dy.float().sum(0)
        items.append((dy, x, dw, db))
        refs.append((rw, rb))
    G.wgrad_group(items, beta)
    torch.cuda.synchronize()
    for (dy, x, dw, db), (rw, rb), (M, Nn) in zip(items, refs, SHAPES):
        _close(dw, rw, 2e-3, f"dW {M}x{Nn} K={K}")
        if db is not None:
            _close(db, rb, 2e-3, f"db {M} K={K}")


def test_wgrad_group_lmhead_and_layers(cuda):
    """The step's group: twelve GPT-2 small layers' four weight gradients + the lm_head's (49 problems,
    1887 tiles) in one launch, spot-checked against fp32 per problem."""
    K = 8192
    shapes = [(768, 3072), (3072, 768), (768, 768), (2304, 768)] * 12 + [(50304, 768)]
    xs = {Nn: _r(K, Nn, seed=Nn) for Nn in (768, 3072)}
    dys = {M: _r(K, M, seed=M + 1) for M in (768, 3072, 2304, 50304)}
    items = [(dys[M], xs[Nn], torch.empty(M, Nn, device="cuda"), torch.empty(M, device="cuda") if M != 50304 else None)
             for (M, Nn) in shapes]
    G.wgrad_group(items, 0.0)
    torch.cuda.synchronize()
    for k in (0, 1, 2, 3, 47, 48):
        dy, x, dw, db = items[k]
        _close(dw, dy.float().t() @ x.float(), 2e-3, f"problem {k}")
        if db is not None:
            _close(db, dy.float().sum(0), 2e-3, f"bias {k}")


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_group_tail_split(cuda, monkeypatch, beta):
    """DTC_WG_TAIL_SPLIT: the step's group (1887 tiles = 7 rounds + 95 on 256 CUs) with its last 95 tiles --
    the bias-free lm_head's, sorted last -- as 2 K-pieces each, finished by wg_tail_reduce: dW against fp32
    torch and against the unsplit launch, bias sums unchanged, and the per-tile grad-norm partials still sum
    to sum(dW^2) over every problem."""
    K = 8192
    shapes = [(768, 3072), (3072, 768), (768, 768), (2304, 768)] * 12 + [(50304, 768)]
    xs = {Nn: _r(K, Nn, seed=Nn) for Nn in (768, 3072)}
    dys = {M: _r(K, M, seed=M + 1) for M in (768, 3072, 2304, 50304)}
    tiles = sum(G.wgrad_tiles(M, Nn) for M, Nn in shapes)
    out = {}
    for tail in (1, 0):
        monkeypatch.setattr(G, "_WG_TAIL", tail)
        items = [(dys[M], xs[Nn], _r(M, Nn, seed=5, dtype=torch.float32),
                  _r(M, seed=6, dtype=torch.float32) if M != 50304 else None) for (M, Nn) in shapes]
        start = [(dw.clone(), None if db is None else db.clone()) for _, _, dw, db in items]
        sq = torch.zeros(G.WG_SQ_SLOTS * tiles, device="cuda")
        G.wgrad_group(items, beta, sq=sq)
        torch.cuda.synchronize()
        total = sum((dw.double() ** 2).sum().item() for _, _, dw, _ in items)
        assert sq.double().sum().item() == pytest.approx(total, rel=1e-5), tail
        for k in (0, 3, 47, 48):
            dy, x, dw, db = items[k]
            _close(dw, beta * start[k][0] + dy.float().t() @ x.float(), 2e-3, f"tail={tail} problem {k}")
            if db is not None:
                _close(db, beta * start[k][1] + dy.float().sum(0), 2e-3, f"tail={tail} bias {k}")
        out[tail] = [dw for _, _, dw, _ in items]
    for a, b in zip(out[1], out[0]):
        _close(a, b, 1e-5, "tail split vs whole tiles")
