"""CPU tests: reference semantics of the model, data, config and optimizer (no GPU)."""

import math

import numpy as np
import pytest
import torch

from distributed_training_compare_jax_amd.config.schema import (OptimConfig, TrainConfig, build_configs,
                                                                 model_config_from_preset)
from distributed_training_compare_jax_amd.data.synthetic import SyntheticTokenStream, get_batch_iterator, get_tokenizer
from distributed_training_compare_jax_amd.models.gpt import GPTStage, StageLayout
from distributed_training_compare_jax_amd.models.params import all_param_specs, init_full, shard, unshard
from distributed_training_compare_jax_amd.models.reference import oracle_loss
from distributed_training_compare_jax_amd.ops import embedding as E
from distributed_training_compare_jax_amd.ops import gemm as G
from distributed_training_compare_jax_amd.ops import optim as O
from distributed_training_compare_jax_amd.parallel.buffers import FlatParams
from distributed_training_compare_jax_amd.parallel.mesh import resolve_degrees, split_layers


def test_reference_configs_load():
    tc, mc, oc = build_configs("configs/train_config_pp.yaml", vocab_size=len(get_tokenizer()))
    assert (mc.vocab_size, mc.d_model, mc.n_layers, mc.n_heads, mc.d_ff, mc.max_seq_len) == (50258, 512, 12, 16, 2048, 512)
    assert mc.dropout == 0.1 and mc.parallel == "pp" and tc.pp_microbatches == 2
    assert (oc.lr, oc.weight_decay, oc.grad_clip) == (3e-4, 0.1, 1.0)
    assert mc.padded_vocab % 128 == 0 and mc.padded_vocab >= 50258
    assert abs(mc.num_params() - 89.61e6) < 0.01e6  # 89.61 M params
    for s in ("dp", "tp"):
        tc, _, _ = build_configs(f"configs/train_config_{s}.yaml")
        assert tc.parallel == s and tc.batch == 8 and tc.steps == 5000 and tc.log_every == 50


def test_unknown_key_rejected(tmp_path):
    p = tmp_path / "t.yaml"
    p.write_text("batch: 8\nlog_every: 1\noutput_dir: x\nparallel: dp\nseed: 0\nsteps: 1\nbogus: 3\n")
    with pytest.raises(TypeError):
        build_configs(str(p))


def test_strategy_resolution():
    assert resolve_degrees("dp", 8, None, None, None) == (8, 1, 1)
    assert resolve_degrees("tp", 8, None, None, None) == (1, 8, 1)
    assert resolve_degrees("pp", 4, None, None, None) == (1, 1, 4)
    assert resolve_degrees("dp", 8, None, 2, None) == (4, 2, 1)
    with pytest.raises(ValueError):
        resolve_degrees("zz", 2, None, None, None)
    # reference quirk fix: 12 layers over 8 stages keeps all 12 layers
    r = split_layers(12, 8)
    assert sum(len(x) for x in r) == 12 and r[0].start == 0 and r[-1].stop == 12


@pytest.mark.parametrize("L,pp,head", [(12, 2, 2.9), (12, 4, 2.9), (12, 8, 2.9), (24, 8, 2.2), (12, 8, 4.5), (4, 4, 1.0)])
def test_cost_aware_pp_split(L, pp, head):
    """split_layers(weights=(embed, head)) is contiguous, keeps every layer, puts >= 1 layer on every
    non-last stage and minimises the most expensive stage (checked against brute force)."""
    import itertools

    from distributed_training_compare_jax_amd.parallel.mesh import stage_costs

    w = (0.05, head)
    r = split_layers(L, pp, w)
    assert len(r) == pp and r[0].start == 0 and r[-1].stop == L
    assert all(a.stop == b.start for a, b in zip(r, r[1:]))
    assert all(len(x) >= 1 for x in r[:-1])
    if pp <= 4:  # brute force over the non-last stage sizes
        best = min(max(stage_costs([range(0, k) for k in ks], w))  # only lengths matter
                   for ks in itertools.product(range(1, L + 1), repeat=pp - 1) if sum(ks) <= L
                   for ks in [ks + (L - sum(ks),)])
        assert max(stage_costs(r, w)) == pytest.approx(best)
    assert max(stage_costs(r, w)) <= max(stage_costs(split_layers(L, pp), w)) + 1e-9


def test_synthetic_data_contract():
    it = get_batch_iterator(8, 513)
    a = next(it)
    assert a.shape == (8, 513) and a.dtype == np.int32
    assert a.min() >= 0 and a.max() < 50257  # pad id never appears
    # row-sliced iterator (a DP rank) is bit-identical to slicing the global batch
    b = next(get_batch_iterator(8, 513, row0=2, nrows=3))
    assert np.array_equal(a[2:5], b)
    # deterministic and non-trivial
    assert np.array_equal(a, next(get_batch_iterator(8, 513)))
    assert not np.array_equal(a, next(it))
    s = SyntheticTokenStream()
    t = s.tokens(0, 20000)
    follow = (s.succ[t[:-1]] == t[1:]).mean()
    # P(e_t = succ[e_{t-1}]) = p_follow * P(e_{t-1} was not itself a follow) ~ 0.25: learnable structure
    assert 0.2 < follow < 0.35


def test_init_statistics():
    mc = model_config_from_preset("ref")
    specs = {s.name: s for s in all_param_specs(mc)}
    wte = init_full(specs["wte"], 0)
    assert abs(wte.std().item() - 1 / math.sqrt(512)) < 1e-3
    w = init_full(specs["h.0.fc2.w"], 0)  # fan_in 2048, truncated normal
    sigma = math.sqrt(1 / 2048) / 0.87962566103423978
    assert w.abs().max().item() <= 2 * sigma + 1e-6
    assert abs(w.std().item() - math.sqrt(1 / 2048)) < 2e-4
    lm = init_full(specs["lm_head.w"], 0)
    assert lm[mc.vocab_size:].abs().max().item() == 0.0
    assert init_full(specs["h.3.ln1.g"], 0).eq(1).all() and init_full(specs["h.3.qkv.b"], 0).eq(0).all()
    # canonical init: same tensors for the same seed, different for another
    assert torch.equal(init_full(specs["h.0.qkv.w"], 0), init_full(specs["h.0.qkv.w"], 0))
    assert not torch.equal(init_full(specs["h.0.qkv.w"], 0), init_full(specs["h.0.qkv.w"], 1))


@pytest.mark.parametrize("name", ["h.0.qkv.w", "h.0.qkv.b", "h.0.fc1.w", "h.0.fc2.w", "h.0.out.w", "lm_head.w"])
def test_tp_shard_roundtrip(name):
    mc = model_config_from_preset("tiny", vocab_size=1000)
    spec = {s.name: s for s in all_param_specs(mc)}[name]
    full = init_full(spec, 3)
    if spec.init == "zeros":
        full = torch.randn(spec.shape)
    tp = 2 if spec.heads else 4  # head-sharded params: whole heads (the tiny preset has 2)
    parts = [shard(spec, full, r, tp) for r in range(tp)]
    assert torch.equal(unshard(spec, parts), full)


@pytest.mark.parametrize("tp", [3, 5, 8, 12])
@pytest.mark.parametrize("name", ["h.0.qkv.w", "h.0.qkv.b", "h.0.out.w"])
def test_uneven_head_shard_roundtrip(name, tp):
    """12 heads on tp ranks that do not divide it: whole heads per rank (head_split), exact round trip."""
    from distributed_training_compare_jax_amd.models.params import head_split, local_shape

    mc = model_config_from_preset("gpt2-small", vocab_size=1000, n_layers=1)
    spec = {s.name: s for s in all_param_specs(mc)}[name]
    full = torch.randn(spec.shape)
    parts = [shard(spec, full, r, tp) for r in range(tp)]
    split = head_split(12, tp)
    assert sum(n for _, n in split) == 12 and max(n for _, n in split) - min(n for _, n in split) <= 1
    for r, t in enumerate(parts):
        assert tuple(t.shape) == local_shape(spec, tp, r)
        width = t.shape[0] // 3 if spec.tp == "qkv_rows" else t.shape[1]
        assert width == split[r][1] * 64
    assert torch.equal(unshard(spec, parts), full)


def test_head_split_rejects_too_many_ranks():
    from distributed_training_compare_jax_amd.models.params import head_split

    with pytest.raises(ValueError):
        head_split(2, 4)


def test_gelu_is_tanh_approx():
    x = torch.linspace(-6, 6, 101)
    assert torch.allclose(G.gelu_tanh(x), torch.nn.functional.gelu(x, approximate="tanh"), atol=1e-6)
    x.requires_grad_(True)
    torch.nn.functional.gelu(x, approximate="tanh").sum().backward()
    assert torch.allclose(G.gelu_tanh_grad(x.detach()), x.grad, atol=1e-5)


def test_philox_known_answer_and_rate():
    # Philox4x32-10 known-answer vector (Random123 kat: ctr=0, key=0)
    out = E.philox4x32(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    keep = E.dropout_keep_mask(512, 512, 0, 0.1, seed=0, step=0)
    assert abs(keep.float().mean().item() - 0.9) < 0.005
    # layout invariance: a token slice of the global mask equals the mask of that slice
    sub = E.dropout_keep_mask(100, 512, 37, 0.1, seed=0, step=0)
    assert torch.equal(sub, keep[37:137])


@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_explicit_backward_matches_autograd(dropout):
    mc = model_config_from_preset("tiny", vocab_size=1000, dropout=dropout)
    specs = all_param_specs(mc)
    flat = FlatParams(specs, 0, 1, "cpu", compute_dtype=torch.float32)
    flat.init_canonical(0)
    st = GPTStage(mc, flat, StageLayout(range(mc.n_layers), True, True), act_dtype=torch.float32, dropout_seed=5)
    b = next(get_batch_iterator(4, mc.max_seq_len + 1, vocab=999))
    ids, lab = torch.from_numpy(b[:, :-1]).contiguous(), torch.from_numpy(b[:, 1:]).contiguous()
    step = torch.tensor([3])
    ctx = {}
    T = mc.max_seq_len
    h = st.embed_forward(ids, step, 0, ctx)
    h = st.stage_forward(h, 4, ctx)
    loss = st.head_forward(h, lab, 1 / (4 * T), ctx)
    dx, dxc = st.head_backward(ctx, 1 / (4 * T), 0.0)
    dx, dxc = st.stage_backward(ctx, dx, dxc, 0.0)
    st.embed_backward(ctx, dx, step, 0.0)
    params = {n: flat.p(n).clone().requires_grad_(True) for n in flat.slots}
    lo = oracle_loss(mc, params, ids, lab, 5, 3)
    lo.backward()
    assert abs(loss.item() - lo.item()) < 1e-5
    for n in flat.slots:
        assert torch.allclose(flat.g(n), params[n].grad, rtol=1e-4, atol=1e-6), n
    assert not ctx  # every saved activation consumed


def test_adamw_matches_optax_semantics():
    n = 256
    torch.manual_seed(0)
    p0 = torch.randn(n)
    grads = [torch.randn(n) * s for s in (0.01, 5.0, 0.3)]  # second step triggers clipping
    p, m, v = p0.clone(), torch.zeros(n), torch.zeros(n)
    step, ss = torch.zeros(1, dtype=torch.int64), torch.zeros(1)
    segs = O.make_segments([(0, n, 1.0)], "cpu")
    rp, rm, rv = p0.clone().double(), torch.zeros(n).double(), torch.zeros(n).double()
    for t, g in enumerate(grads, 1):
        O.sumsq_segments(g, segs, ss, step)
        O.adamw_flat(p, g, m, v, None, 0, step, ss, 3e-4, 0.9, 0.999, 1e-8, 0.1, 1.0)
        gd = g.double()
        nrm = gd.norm()
        gd = gd if nrm < 1.0 else gd / nrm * 1.0  # optax clip_by_global_norm
        rm = 0.9 * rm + 0.1 * gd
        rv = 0.999 * rv + 0.001 * gd * gd
        mh, vh = rm / (1 - 0.9 ** t), rv / (1 - 0.999 ** t)
        rp = rp - 3e-4 * (mh / (vh.sqrt() + 1e-8) + 0.1 * rp)
        assert step.item() == t
    assert torch.allclose(p.double(), rp, atol=1e-6)


def test_transposed_mirror_tracks_updates():
    """FlatParams.enable_transposed: the [in, out] copy equals the mirror's transpose after init and
    after every optimizer range update (CPU: fp32 'mirror' is the params; exercised via bf16 on GPU)."""
    from distributed_training_compare_jax_amd.models.params import stage_param_specs
    from distributed_training_compare_jax_amd.ops import optim as O
    from distributed_training_compare_jax_amd.parallel.buffers import FlatParams

    mc = model_config_from_preset("tiny", vocab_size=1000)
    specs = stage_param_specs(mc, range(mc.n_layers), True, True)
    f = FlatParams(specs, 0, 1, "cpu", compute_dtype=torch.bfloat16)
    f.enable_transposed(["h.0.fc1.w", "h.1.qkv.w"])
    f.init_canonical(0)
    for n in ("h.0.fc1.w", "h.1.qkv.w"):
        assert torch.equal(f.wt(n), f.w(n).t())
    f.params.add_(0.5)
    f.refresh_mirror()
    assert torch.equal(f.wt("h.0.fc1.w"), f.w("h.0.fc1.w").t())
    assert f.wt("h.0.qkv.w") is None
    pairs = [(torch.randn(24, 40).bfloat16(), torch.empty(40, 24, dtype=torch.bfloat16))]
    O.transpose_batch(pairs)
    assert torch.equal(pairs[0][1], pairs[0][0].t())


def test_ln_fused_cpu_fallback_and_site_order():
    """ops/ln_fused.py without a granule buffer (CPU / fp32 parity) is exactly the unfused pair of ops, and
    the fused LayerNorm sites of a stage are numbered in execution order (forward, then backward in
    reverse layer order), each once — the epoch-tag scheme relies on consecutive uses differing."""
    from distributed_training_compare_jax_amd.ops import layernorm as LN
    from distributed_training_compare_jax_amd.ops import ln_fused as LF

    g = torch.Generator().manual_seed(0)
    M, K, D = 64, 48, 32
    a, w = torch.randn(M, K, generator=g), torch.randn(D, K, generator=g) * 0.1
    b, res = torch.randn(D, generator=g), torch.randn(M, D, generator=g)
    gam, bet = torch.randn(D, generator=g), torch.randn(D, generator=g)
    x, (y, mu, rs) = LF.linear_resid_ln(a, w, b, res, gam, bet, 1e-6)
    xr = G.linear_resid(a, w, b, res)
    yr, mur, rsr = LN.layernorm_fwd(xr, gam, bet, 1e-6)
    assert torch.equal(x, xr) and torch.equal(y, yr) and torch.equal(mu, mur) and torch.equal(rs, rsr)
    dY, wt = torch.randn(M, K, generator=g), torch.randn(D, K, generator=g) * 0.1
    dres = torch.randn(M, D, generator=g)
    dg, db, dbias = torch.zeros(D), torch.zeros(D), torch.zeros(D)
    dx, dxc = LF.dgrad_ln_bwd(dY, wt, x, gam, mu, rs, dres, dg, db, 0.0, dbias=dbias)
    dgr, dbr, dbiasr = torch.zeros(D), torch.zeros(D), torch.zeros(D)
    dxr = LN.layernorm_bwd(G.linear_resid(dY, wt, None, None), x, gam, mu, rs, dres, dgr, dbr, 0.0, dbias=dbiasr)
    assert torch.allclose(dx, dxr) and torch.allclose(dg, dgr) and torch.allclose(db, dbr)
    assert torch.allclose(dbias, dbiasr) and dxc is dx
    assert LF.supported(4096, 512, 2048) and not LF.supported(4096, 64, 512) and not LF.supported(1000, 512, 512)
    assert not LF.supported(8192, 768, 3072) and not LF.supported(8192, 1024, 4096)  # GPT-2 small / medium: slower

    mc = build_configs("configs/train_config_dp.yaml")[1]
    for layers in (range(0, 12), range(4, 8)):
        st = GPTStage.__new__(GPTStage)
        st.layout = StageLayout(layers, True, True)
        order = [st._ln_site(l, k, False) for l in layers for k in (0, 1)]
        order += [st._ln_site(l, k, True) for l in reversed(layers) for k in (0, 1)]
        assert order == list(range(4 * len(layers))), order
    assert mc.d_model == 512


@pytest.mark.parametrize("chunk", [256, 384])
def test_vocab_chunked_head_matches_unchunked(monkeypatch, chunk):
    """DTC_CE_CHUNK: the vocab-chunked lm_head + CE (per-chunk row statistics combined like vocab
    shards, logits recomputed chunk by chunk in the backward) gives the unchunked loss and gradients;
    1000 real columns (padded to 1024) -> chunks of 256 (4, the last one 232 valid) or 384 (3, ragged)."""
    from distributed_training_compare_jax_amd.models import gpt as GPTMOD

    mc = model_config_from_preset("tiny", vocab_size=1000, dropout=0.0)
    specs = all_param_specs(mc)
    b = next(get_batch_iterator(4, mc.max_seq_len + 1, vocab=999))
    ids, lab = torch.from_numpy(b[:, :-1]).contiguous(), torch.from_numpy(b[:, 1:]).contiguous()
    T = mc.max_seq_len
    res = []
    for ch in (0, chunk):
        monkeypatch.setattr(GPTMOD, "_CE_CHUNK", ch)
        flat = FlatParams(specs, 0, 1, "cpu", compute_dtype=torch.float32)
        flat.init_canonical(0)
        st = GPTStage(mc, flat, StageLayout(range(mc.n_layers), True, True), act_dtype=torch.float32)
        step = torch.tensor([3])
        ctx = {}
        h = st.embed_forward(ids, step, 0, ctx)
        h = st.stage_forward(h, 4, ctx)
        loss = st.head_forward(h, lab, 1 / (4 * T), ctx)
        assert (ctx["head"][4] is None) == (ch > 0)  # chunked: no logits kept for the backward
        dx, dxc = st.head_backward(ctx, 1 / (4 * T), 0.0)
        dx, dxc = st.stage_backward(ctx, dx, dxc, 0.0)
        st.embed_backward(ctx, dx, step, 0.0)
        res.append((loss.item(), {n: flat.g(n).clone() for n in flat.slots}))
    assert abs(res[0][0] - res[1][0]) < 1e-5
    for n in res[0][1]:
        assert torch.allclose(res[0][1][n], res[1][1][n], rtol=1e-4, atol=1e-6), n
