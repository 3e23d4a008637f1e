"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU).

Inputs are bf16-rounded first, so the reference sees exactly the kernel's operands and the
only difference is accumulation order / fp32 vs bf16 output rounding.  Operands are
asymmetric random data (cdna_hip_programming.md §3: a symmetric operand hides transposes).
"""

import math

import pytest
import torch

from distributed_training_compare_jax_amd.ops import attention as A
from distributed_training_compare_jax_amd.ops import embedding as E
from distributed_training_compare_jax_amd.ops import gemm as G
from distributed_training_compare_jax_amd.ops import layernorm as LN
from distributed_training_compare_jax_amd.ops import optim as O
from distributed_training_compare_jax_amd.ops import xent as X

pytestmark = pytest.mark.gpu


def _r(*shape, scale=1.0, dev="cuda", seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    t = (torch.randn(*shape, generator=g) * scale + 0.1 * torch.rand(*shape, generator=g))
    return t.to(dev).to(dtype)


def _close(a, b, rtol, name=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= rtol * ref, f"{name}: max abs err {err:.3e} vs ref max {ref:.3e} (rel {err / ref:.2e})"


GEMM_SHAPES = [(4096, 1536, 512), (4096, 512, 512), (4096, 2048, 512), (4096, 512, 2048), (256, 384, 128), (512, 768, 96),
               (200, 136, 64), (4096, 50304, 512), (2000, 33000, 128), (8192, 2304, 768)]


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
def test_gemm_nt_bias(cuda, M, N, K):
    x, w = _r(M, K, seed=1), _r(N, K, scale=0.05, seed=2)
    b = _r(N, dtype=torch.float32, seed=3)
    y = G.linear(x, w, b)
    ref = x.float() @ w.float().t() + b
    _close(y, ref, 1e-2, "nt")


def test_gemm_resid_gelu(cuda):
    M, N, K = 512, 768, 256
    x, w = _r(M, K, seed=1), _r(N, K, scale=0.05, seed=2)
    b = _r(N, dtype=torch.float32, seed=3)
    res = _r(M, N, dtype=torch.float32, seed=4)
    y = G.linear_resid(x, w, b, res)
    _close(y, res + x.float() @ w.float().t() + b, 2e-3, "resid")
    y2 = G.linear_resid(x, w, None, None)
    _close(y2, x.float() @ w.float().t(), 2e-3, "store_f32")
    u, g = G.linear_gelu(x, w, b)
    uref = x.float() @ w.float().t() + b
    _close(u, G.gelu_tanh_grad(uref), 1e-2, "gelu_grad")
    _close(g, G.gelu_tanh(uref), 1e-2, "gelu_g")


@pytest.mark.parametrize("N,K", [(512, 512), (512, 2048), (2048, 512), (1536, 512)])
def test_gemm_reference_shape_epilogues(cuda, N, K):
    """Every forward / dgrad epilogue at the reference model's Dense shapes (4096 tokens): these are
    the shapes the 8-wave DMA kernels (csrc/gemm.hip gemm_dmaw_kernel) are planned for."""
    M = 4096
    x, w = _r(M, K, seed=41), _r(N, K, scale=0.05, seed=42)
    b = _r(N, dtype=torch.float32, seed=43)
    res = _r(M, N, dtype=torch.float32, seed=44)
    ref = x.float() @ w.float().t() + b
    _close(G.linear(x, w, b), ref, 1e-2, "store_bf16")
    _close(G.linear_resid(x, w, b, res), res + ref, 2e-3, "resid")
    u, g = G.linear_gelu(x, w, b)
    _close(u, G.gelu_tanh_grad(ref), 1e-2, "gelu_grad")
    _close(g, G.gelu_tanh(ref), 1e-2, "gelu")
    dy = _r(M, N, seed=45)  # dgrad through the same weight: [M, N] . [N, K]
    _close(G.matmul_nn(dy, w), dy.float() @ w.float(), 2e-3, "nn_f32")
    _close(G.matmul_nn(dy, w, out_dtype=torch.bfloat16), dy.float() @ w.float(), 1e-2, "nn_bf16")
    uu = _r(M, K, seed=46)
    _close(G.matmul_nn_dgelu(dy, w, uu), (dy.float() @ w.float()) * uu.float(), 1e-2, "dgelu")


@pytest.mark.parametrize("M,N,K", [(4096, 512, 50304), (2048, 256, 50304), (4096, 512, 20480)])
def test_gemm_nt_splitk_vocab(cuda, M, N, K):
    """The lm_head dgrad as an NT GEMM on the transposed weight (K = vocab): 256^2 tiles, split-K slabs."""
    dy, wt = _r(M, K, seed=47), _r(N, K, scale=0.05, seed=48)
    _close(G.linear_resid(dy, wt, None, None), dy.float() @ wt.float().t(), 2e-3, "nt_splitk")


@pytest.mark.parametrize("M,N,K", [(4096, 512, 1536), (4096, 2048, 512), (4096, 512, 50304), (256, 128, 64), (256, 64, 96),
                                   (256, 32, 64), (2000, 384, 40000)])
def test_gemm_nn(cuda, M, N, K):
    dy, w = _r(M, K, seed=5), _r(K, N, scale=0.05, seed=6)
    dx = G.matmul_nn(dy, w)
    _close(dx, dy.float() @ w.float(), 2e-3, "nn")
    u = _r(M, N, seed=7)
    du = G.matmul_nn_dgelu(dy, w, u)
    _close(du, (dy.float() @ w.float()) * u.float(), 1e-2, "dgelu")


@pytest.mark.parametrize("Mtok,N,K", [(4096, 1536, 512), (4096, 512, 512), (4096, 2048, 512), (4096, 512, 2048),
                                      (4096, 50304, 512), (128, 64, 64), (512, 200, 96), (3072, 50000, 384),
                                      (4096, 45000, 512), (1024, 32768, 512)])
def test_gemm_wgrad(cuda, Mtok, N, K):
    """Weight gradients; the vocab-sized ones (32768-50304 rows) run on the 256^2 kernel."""
    dy, x = _r(Mtok, N, seed=8), _r(Mtok, K, seed=9)
    dw = torch.full((N, K), 3.0, device=cuda)
    G.wgrad(dy, x, dw, beta=0.0)
    ref = dy.float().t() @ x.float()
    _close(dw, ref, 2e-3, "wgrad")
    G.wgrad(dy, x, dw, beta=1.0)
    _close(dw, 2 * ref, 2e-3, "wgrad_acc")


def test_colsum(cuda):
    dy = _r(4096, 1536, seed=10)
    db = torch.zeros(1536, device=cuda)
    G.colsum(dy, db)
    _close(db, dy.float().sum(0), 1e-4, "colsum")
    G.colsum(dy, db, beta=1.0)
    _close(db, 2 * dy.float().sum(0), 1e-4, "colsum_acc")
    d32 = _r(1000, 520, dtype=torch.float32, seed=11)
    db2 = torch.zeros(520, device=cuda)
    G.colsum(d32, db2)
    _close(db2, d32.sum(0), 1e-5, "colsum_f32")


@pytest.mark.parametrize("D", [512, 768, 64])
def test_layernorm(cuda, D):
    M = 1024
    x = _r(M, D, dtype=torch.float32, seed=12) * 3 + 1
    g = _r(D, dtype=torch.float32, seed=13)
    b = _r(D, dtype=torch.float32, seed=14)
    y, mu, rs = LN.layernorm_fwd(x, g, b, 1e-6, torch.bfloat16)
    yc, muc, rsc = LN.layernorm_fwd(x.cpu(), g.cpu(), b.cpu(), 1e-6, torch.float32)
    _close(y.cpu(), yc, 1e-2, "ln_fwd")
    _close(rs.cpu(), rsc, 1e-5, "ln_rstd")
    dy = _r(M, D, seed=15)
    dres = _r(M, D, dtype=torch.float32, seed=16)
    dg, db = torch.zeros(D, device=cuda), torch.zeros(D, device=cuda)
    dxc = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
    dx = LN.layernorm_bwd(dy, x, g, mu, rs, dres, dg, db, 0.0, out_c=dxc)
    dgc, dbc = torch.zeros(D), torch.zeros(D)
    dxr = LN.layernorm_bwd(dy.cpu().float(), x.cpu(), g.cpu(), muc, rsc, dres.cpu(), dgc, dbc, 0.0)
    _close(dx.cpu(), dxr, 1e-4, "ln_dx")
    _close(dxc.cpu(), dxr, 1e-2, "ln_dx_bf16")
    _close(dg.cpu(), dgc, 1e-4, "ln_dg")
    _close(db.cpu(), dbc, 1e-4, "ln_db")


@pytest.mark.parametrize("D", [512, 768, 1024])
def test_add_layernorm(cuda, D):
    """Residual add in the LayerNorm pass (models/gpt.py DTC_ADD_LN): x = d + resid written over d
    (bitwise the fp32 sum), LN(x) as the plain LayerNorm of that sum."""
    M = 1000
    d = _r(M, D, dtype=torch.float32, seed=17)
    r = _r(M, D, dtype=torch.float32, seed=18) * 3 + 1
    g, b = _r(D, dtype=torch.float32, seed=19), _r(D, dtype=torch.float32, seed=20)
    want = d + r
    d2 = d.clone()
    x, (y, mu, rs) = LN.add_layernorm_fwd(d2, r, g, b, 1e-6, torch.bfloat16)
    assert x.data_ptr() == d2.data_ptr() and torch.equal(x, want)
    y0, mu0, rs0 = LN.layernorm_fwd(want, g, b, 1e-6, torch.bfloat16)
    assert torch.equal(y, y0) and torch.equal(mu, mu0) and torch.equal(rs, rs0)
    # bf16 branch output (DTC_FWD_BF16): x = float(d) + resid into a new fp32 tensor
    db = d.to(torch.bfloat16)
    want = db.float() + r
    x, (y, mu, rs) = LN.add_layernorm_fwd(db, r, g, b, 1e-6, torch.bfloat16)
    assert x.dtype == torch.float32 and x.data_ptr() != db.data_ptr() and torch.equal(x, want)
    y0, mu0, rs0 = LN.layernorm_fwd(want, g, b, 1e-6, torch.bfloat16)
    assert torch.equal(y, y0) and torch.equal(mu, mu0) and torch.equal(rs, rs0)


@pytest.mark.parametrize("D", [128, 768, 1280])
def test_embedding_dropout_bits(cuda, D):
    B, T, V = 4, 64, 1000
    ids = torch.randint(0, V, (B, T), dtype=torch.int32)
    wte = _r(V, D, dtype=torch.float32, seed=17)
    wpe = _r(T, D, dtype=torch.float32, seed=18)
    step = torch.tensor([7], dtype=torch.int64)
    h = E.embed_fwd(ids.to(cuda), wte, wpe, 0.1, 1234, step.to(cuda), row0=3)
    hc = E.embed_fwd(ids, wte.cpu(), wpe.cpu(), 0.1, 1234, step, row0=3)
    assert torch.equal((h.cpu() == 0), (hc == 0)), "dropout mask differs between HIP Philox and CPU Philox"
    _close(h.cpu(), hc, 1e-6, "embed_fwd")
    dh = _r(B * T, D, dtype=torch.float32, seed=19)
    dwte, dwpe = torch.full((V, D), 5.0, device=cuda), torch.zeros(T, D, device=cuda)
    E.embed_bwd(ids.to(cuda), dh, dwte, dwpe, 0.1, 1234, step.to(cuda), 3, 0.0)
    dwc, dpc = torch.zeros(V, D), torch.zeros(T, D)
    E.embed_bwd(ids, dh.cpu(), dwc, dpc, 0.1, 1234, step, 3, 0.0)
    _close(dwte.cpu(), dwc, 1e-5, "dwte")
    _close(dwpe.cpu(), dpc, 1e-5, "dwpe")


@pytest.mark.parametrize("B,T,D,V,skew", [(8, 512, 512, 50304, True), (64, 512, 128, 50304, True),
                                           (3, 100, 64, 300, False), (80, 512, 64, 1000, True)])
def test_embedding_bwd_sorted_deterministic(cuda, B, T, D, V, skew):
    """Sorted segment-sum backward: exact vs index_add (fp64), bitwise repeatable, accumulate mode.
    ``skew`` draws Zipf-like ids so one id spans many 64-key tiles (the multi-piece path)."""
    g = torch.Generator().manual_seed(3)
    if skew:
        r = torch.rand(B * T, generator=g)
        ids = torch.minimum((V ** r).long() - 1, torch.tensor(V - 1)).to(torch.int32).view(B, T)
        ids.view(-1)[: 3 * 64 + 5] = 7  # one long run crossing tile boundaries
    else:
        ids = torch.randint(0, V, (B, T), generator=g, dtype=torch.int32)
    step = torch.tensor([3], dtype=torch.int64)
    dh = _r(B * T, D, dtype=torch.float32, seed=21)
    keys = None
    if B * T <= E.SORT_MAX:  # else: the row-chunked path sorts each chunk itself
        keys = E.embed_sort_keys(ids.to(cuda), V)
        nb = max(1, (B * T - 1).bit_length())
        kc = keys.cpu().long() & 0xFFFFFFFF
        assert torch.equal(kc >> nb, ids.view(-1).long().sort().values), "sorted ids"
        assert torch.equal(torch.sort(kc & ((1 << nb) - 1)).values, torch.arange(B * T)), "token permutation"
    outs = []
    for _ in range(2):
        dwte, dwpe = torch.full((V, D), 5.0, device=cuda), torch.zeros(T, D, device=cuda)
        E.embed_bwd(ids.to(cuda), dh, dwte, dwpe, 0.1, 99, step.to(cuda), 2, 0.0, keys=keys)
        outs.append((dwte.clone(), dwpe.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), "not bitwise repeatable"
    keep = E.dropout_keep_mask(B * T, D, 2 * T, 0.1, 99, 3)
    gd = torch.where(keep, dh.cpu().double() / 0.9, torch.zeros((), dtype=torch.float64))
    ref_w = torch.zeros(V, D, dtype=torch.float64).index_add_(0, ids.view(-1).long(), gd)
    ref_p = gd.view(B, T, D).sum(0)
    _close(outs[0][0].cpu(), ref_w, 2e-6, "dwte")
    _close(outs[0][1].cpu(), ref_p, 2e-6, "dwpe")
    # accumulate (beta = 1): adds onto the existing grads
    dwte, dwpe = outs[0][0].clone(), outs[0][1].clone()
    E.embed_bwd(ids.to(cuda), dh, dwte, dwpe, 0.1, 99, step.to(cuda), 2, 1.0, keys=keys)
    _close(dwte.cpu(), 2 * ref_w, 2e-6, "dwte_acc")
    _close(dwpe.cpu(), 2 * ref_p, 2e-6, "dwpe_acc")


@pytest.mark.parametrize("B,T,H,hd", [(2, 512, 4, 32), (1, 256, 2, 64), (2, 128, 3, 32), (2, 200, 3, 32), (1, 520, 2, 32),
                                      (1, 1024, 2, 64), (1, 1000, 2, 64), (1, 700, 3, 32)])
def test_attention(cuda, B, T, H, hd):
    qkv = _r(B, T, 3 * H * hd, seed=20)
    o, lse = A.attn_fwd(qkv, H)
    oc, lsec = A.attn_fwd(qkv.cpu().float(), H)
    _close(o.cpu(), oc, 2e-2, "attn_o")
    _close(lse.cpu(), lsec, 1e-3, "attn_lse")
    do = _r(B, T, H * hd, seed=21)
    dqkv = A.attn_bwd(qkv, o, lse, do, H)
    dref = A.attn_bwd(qkv.cpu().float(), o.cpu().float(), lse.cpu(), do.cpu().float(), H)
    d3, r3 = dqkv.cpu().float().view(B, T, 3, -1), dref.view(B, T, 3, -1)
    for i, n in enumerate("qkv"):
        _close(d3[:, :, i], r3[:, :, i], 3e-2, f"attn_d{n}")


@pytest.mark.parametrize("spike", [False, True])
@pytest.mark.parametrize("B,T,H", [(2, 1024, 3), (1, 777, 2)])
def test_attention_fwd32_vs_chunk_and_reference(cuda, B, T, H, spike):
    """head_dim 64 forward on the 32-query-per-wave 32x32x16 kernel (default) against the 16-row chunked
    kernel (flags bit 2) and the fp32 reference.  ``spike``: one key scaled up mid-sequence so the
    running max jumps by far more than the deferred-max threshold (2^8) at a late tile -- the rescale
    branch runs on most rows (cdna_hip_programming.md §5.4 rule 26)."""
    hd = 64
    qkv = _r(B, T, 3 * H * hd, seed=40)
    if spike:
        v = qkv.view(B, T, 3, H, hd)
        v[:, T // 2 + 5, 1] *= 12.0  # key row T/2+5 of every head: its scores dominate later queries
    o, lse = A.attn_fwd(qkv, H)
    o4, lse4 = A.attn_fwd(qkv, H, flags=4)
    oc, lsec = A.attn_fwd(qkv.cpu().float(), H)
    _close(o.cpu(), oc, 2e-2, "attn32_o")
    _close(lse.cpu(), lsec, 1e-3, "attn32_lse")
    _close(o.float(), o4.float(), 2e-2, "attn32_vs_chunk")
    o4r, lse4r = A.attn_fwd(qkv, H, flags=16)  # the round-4 32-row kernel (the default is the round-5 pipeline)
    _close(o4r.cpu(), oc, 2e-2, "attn32r4_o")
    _close(lse4r.cpu(), lsec, 1e-3, "attn32r4_lse")
    assert torch.equal(o, A.attn_fwd(qkv, H)[0])  # deterministic
    # backward: the 32x32x16 dQ and dK/dV kernels (default) vs the 16-row chunked ones vs fp32
    do = _r(B, T, H * hd, seed=41)
    d = A.attn_bwd(qkv, o, lse, do, H)
    d4 = A.attn_bwd(qkv, o, lse, do, H, flags=4)
    d8 = A.attn_bwd(qkv, o, lse, do, H, flags=8)  # merged: delta pass + dK/dV and dQ blocks in one launch
    dref = A.attn_bwd(qkv.cpu().float(), o.cpu().float(), lse.cpu(), do.cpu().float(), H)
    d3, r3, o3 = d.cpu().float().view(B, T, 3, -1), dref.view(B, T, 3, -1), d4.cpu().float().view(B, T, 3, -1)
    m3 = d8.cpu().float().view(B, T, 3, -1)
    for i, n in enumerate("qkv"):
        _close(d3[:, :, i], r3[:, :, i], 3e-2, f"attn32_d{n}")
        _close(d3[:, :, i], o3[:, :, i], 3e-2, f"attn32_vs_chunk_d{n}")
        _close(m3[:, :, i], r3[:, :, i], 3e-2, f"attn32_merged_d{n}")
    assert torch.equal(d, A.attn_bwd(qkv, o, lse, do, H))  # deterministic
    assert torch.equal(d8, A.attn_bwd(qkv, o, lse, do, H, flags=8))


def test_attention_fwd_balanced_order_bitwise(cuda):
    """GPT-2 small shape (B8 T1024 H12: 768 blocks = one round at 3 per CU): the CU-balanced block order
    (default) computes every (query block, b, h) exactly once, bitwise equal to the heavy-first order (flags
    bit 6) and to the 2-waves-per-SIMD form (bit 5, heavy-first)."""
    B, T, H, hd = 8, 1024, 12, 64
    qkv = _r(B, T, 3 * H * hd, seed=44)
    o, lse = A.attn_fwd(qkv, H)
    o6, lse6 = A.attn_fwd(qkv, H, flags=64)
    o5, lse5 = A.attn_fwd(qkv, H, flags=32)
    assert torch.equal(o, o6) and torch.equal(lse, lse6)
    assert torch.equal(o, o5) and torch.equal(lse, lse5)
    # one head of one sequence against the fp32 reference (the order only moves whole blocks)
    one = qkv[:1].view(1, T, 3, H, hd)[:, :, :, :1].reshape(1, T, 3 * hd)
    oc, lsec = A.attn_fwd(one.cpu().float(), 1)
    _close(o[:1, :, :hd].cpu(), oc, 2e-2, "attn_bal_o")
    _close(lse[:1, :1].cpu(), lsec, 1e-3, "attn_bal_lse")


@pytest.mark.parametrize("B,T,H", [(2, 512, 4), (1, 200, 3), (2, 64, 2)])
def test_attention_bwd_fused_matches_two_round(cuda, B, T, H):
    """The fused single-round backward and the two-round resident kernels compute the same
    gradients (different summation orders only) and both match the fp32 reference."""
    qkv = _r(B, T, 3 * H * 32, seed=30)
    do = _r(B, T, H * 32, seed=31)
    o, lse = A.attn_fwd(qkv, H)
    d_fused = A.attn_bwd(qkv, o, lse, do, H)
    d_two = A.attn_bwd(qkv, o, lse, do, H, flags=1)
    dref = A.attn_bwd(qkv.cpu().float(), o.cpu().float(), lse.cpu(), do.cpu().float(), H)
    _close(d_fused.cpu().float(), dref, 3e-2, "attn_bwd_fused")
    _close(d_fused.cpu().float(), d_two.cpu().float(), 2e-2, "fused_vs_two_round")
    # deterministic: a second launch is bitwise identical
    assert torch.equal(d_fused, A.attn_bwd(qkv, o, lse, do, H))


@pytest.mark.parametrize("M,D,V,Vp", [(512, 128, 1000, 1024), (2048, 256, 50258, 50304)])
def test_lmhead_ce(cuda, M, D, V, Vp):
    """Second case runs the 256x256 DMA-staged kernel (>= 512 tiles), incl. its ragged last N tile."""
    h = _r(M, D, seed=22)
    w = _r(Vp, D, scale=0.2, seed=23)
    b = _r(Vp, dtype=torch.float32, seed=24)
    labels = torch.randint(0, V, (M,), dtype=torch.int32)
    logits, rowstat, lab = X.lmhead_logits_partials(h, w, b, labels.to(cuda), 0, V)
    lse, loss = X.ce_finalize(rowstat.unsqueeze(0).contiguous(), lab, 1.0 / M)
    ref = torch.nn.functional.cross_entropy(h.float().cpu() @ w.float().cpu()[:V].t() + b.cpu()[:V], labels.long())
    assert abs(loss.item() - ref.item()) < 2e-2 * abs(ref.item()), (loss.item(), ref.item())
    lg2 = logits.clone()
    lg0 = logits.float().cpu()  # the kernel's bf16 logits (-inf pads): the reference for the bias grad
    X.ce_backward_inplace(logits, lse, labels.to(cuda), 0, V, 1.0 / M)
    lg2, cp = X.ce_backward_inplace(lg2, lse, labels.to(cuda), 0, V, 1.0 / M, colpart=True)
    assert torch.equal(lg2, logits)  # the fused column-partial variant writes the same dlogits
    db = torch.zeros(Vp, device=cuda)
    G.colsum(cp, db)
    lf = h.float().cpu() @ w.float().cpu().t() + b.cpu()
    lf[:, V:] = float("-inf")
    p = torch.softmax(lf, -1)
    p[torch.arange(M), labels.long()] -= 1
    _close(logits.cpu(), p / M, 3e-2, "dlogits")
    pb = torch.softmax(lg0, -1)
    pb[torch.arange(M), labels.long()] -= 1
    _close(db.cpu(), (pb / M).sum(0), 2e-3, "dbias")
    assert logits[:, V:].abs().max().item() == 0.0


@pytest.mark.parametrize("M,D,V,Vp,vstart", [(4096, 512, 50258, 50304, 0), (1024, 256, 25129, 25152, 25129), (1000, 256, 30000, 30016, 0),
                                             (512, 256, 1000, 1024, 0)])
def test_ce_dgrad_fused_matches_unfused(cuda, M, D, V, Vp, vstart):
    """ce_dgrad_fused (CE backward inside the lm_head dgrad's operand staging) == ce_backward_inplace +
    the NT dgrad on W^T: identical dlogits bits, the same dX up to summation order, and column
    sums of the (rounded) dlogits.  vstart > 0: a vocab-parallel shard (labels outside it too)."""
    g = torch.Generator().manual_seed(31)
    logits = (torch.randn(M, Vp, generator=g) * 3).to(torch.bfloat16)
    logits[:, V:] = float("-inf")
    logits = logits.to(cuda)
    lse = torch.logsumexp(logits.float(), -1).contiguous()
    labels = torch.randint(0, 2 * V if vstart else V, (M,), dtype=torch.int32, generator=g).to(cuda)
    wt = _r(D, Vp, scale=0.05, seed=32)
    dx, dl, cp = X.ce_dgrad_fused(logits, lse, labels, vstart, V, 1.0 / M, wt)
    ref_dl, ref_cp = X.ce_backward_inplace(logits.clone(), lse, labels, vstart, V, 1.0 / M, colpart=True)
    assert torch.equal(dl, ref_dl)
    _close(dx, dl.float() @ wt.float().t(), 2e-3, "dx")
    _close(cp.sum(0), dl.float().sum(0), 1e-4, "colsum")
    _close(cp.sum(0), ref_cp.sum(0), 5e-3, "colsum_vs_fp32")



def test_lmhead_raw_partials_match_combined(cuda):
    """combine=False (one vocab shard: raw per-tile partials, a label logit written for every row,
    no zero-fill) gives the same logits, label logits and loss as the combined row statistics."""
    M, D, V, Vp = 2048, 256, 50258, 50304
    h = _r(M, D, seed=27)
    w = _r(Vp, D, scale=0.2, seed=28)
    b = _r(Vp, dtype=torch.float32, seed=29)
    labels = torch.randint(0, V, (M,), dtype=torch.int32).to(cuda)
    lg1, rs, lab1 = X.lmhead_logits_partials(h, w, b, labels, 0, V)
    lg2, part, lab2 = X.lmhead_logits_partials(h, w, b, labels, 0, V, combine=False)
    assert torch.equal(lg1, lg2) and torch.equal(lab1, lab2)
    lse1, loss1 = X.ce_finalize(rs.unsqueeze(0).contiguous(), lab1, 1.0 / M)
    lse2, loss2 = X.ce_finalize(part, lab2, 1.0 / M)
    torch.testing.assert_close(lse1, lse2, rtol=1e-5, atol=1e-5)
    assert abs(loss1.item() - loss2.item()) < 1e-4 * abs(loss1.item())


def test_adamw_matches_cpu(cuda):
    n = 10_000 * 64
    p = _r(n, dtype=torch.float32, seed=25)
    g = _r(n, dtype=torch.float32, seed=26) * 0.01
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    mirror = torch.zeros(n, dtype=torch.bfloat16, device=cuda)
    segs = O.make_segments([(0, n // 2, 1.0), (n // 2, n // 2, 0.5)], cuda)
    ss, step = torch.zeros(1, device=cuda), torch.zeros(1, dtype=torch.int64, device=cuda)
    O.sumsq_segments(g, segs, ss, step)
    gc = g.cpu()
    ref_ss = (gc[: n // 2].double() ** 2).sum() + 0.5 * (gc[n // 2:].double() ** 2).sum()
    assert abs(ss.item() - ref_ss.item()) < 1e-4 * ref_ss.item()
    assert step.item() == 1
    pc, mc, vc = p.cpu().clone(), torch.zeros(n), torch.zeros(n)
    for it in range(3):
        O.adamw_flat(p, g, m, v, mirror, n, step, ss, 3e-4, 0.9, 0.999, 1e-8, 0.1, 1.0)
        O.adamw_flat(pc, gc, mc, vc, None, 0, step.cpu(), ss.cpu(), 3e-4, 0.9, 0.999, 1e-8, 0.1, 1.0)
        step += 1
    _close(p.cpu(), pc, 1e-6, "adamw_p")
    _close(mirror.cpu(), pc, 1e-2, "adamw_mirror")
    _close(v.cpu(), vc, 1e-5, "adamw_v")
    # capped grid (grid-stride loop, the deferred optimizer's form) is bitwise the same update
    p2, m2, v2, mir2 = p.clone(), m.clone(), v.clone(), mirror.clone()
    O.adamw_flat(p, g, m, v, mirror, n, step, ss, 3e-4, 0.9, 0.999, 1e-8, 0.1, 1.0)
    O.adamw_flat(p2, g, m2, v2, mir2, n, step, ss, 3e-4, 0.9, 0.999, 1e-8, 0.1, 1.0, max_blocks=7)
    assert torch.equal(p, p2) and torch.equal(m, m2) and torch.equal(v, v2) and torch.equal(mirror, mir2)


@pytest.mark.parametrize("R", [1, 197, 788, 1000])
def test_ce_combine_rows(cuda, R):
    """Row (max, Σexp) partials of R vocab tiles / shards -> lse and loss against a float64 torch reference:
    the register path (R <= 896: every partial loaded once) and the two-pass path (R > 896); empty partials
    (Σexp = 0, max -inf: tiles past a row's valid vocab) must not contribute."""
    from distributed_training_compare_jax_amd.ops import xent as X

    M = 1000
    g = torch.Generator().manual_seed(R)
    mx = torch.randn(R, M, generator=g) * 4
    se = torch.rand(R, M, generator=g) * 60 + 1
    if R > 1:
        mx[-1, :50], se[-1, :50] = -float("inf"), 0.0
    st = torch.stack([mx, se], -1).contiguous()
    lab = torch.randn(M, generator=g)
    lse, loss = X.ce_finalize(st.to(cuda), lab.to(cuda), 0.5)
    m64 = st[..., 0].double().max(0).values
    ref = m64 + torch.log((st[..., 1].double() * torch.exp(st[..., 0].double() - m64)).sum(0))
    assert torch.allclose(lse.cpu().double(), ref, rtol=0, atol=2e-5), (lse.cpu().double() - ref).abs().max()
    assert float(loss.item()) == pytest.approx(float(0.5 * (ref - lab.double()).sum()), rel=1e-5)


def test_batched_reducer_matches_per_op(cuda):
    """ops/reduce.py: wgrad split-K slabs, colsum and LN partials finished by one batched launch
    are bitwise equal to the per-op kernels; the grad-norm task matches torch."""
    from distributed_training_compare_jax_amd.ops.reduce import GradReducer

    red = GradReducer(cuda, arena_mb=64)
    dy, x = _r(4096, 512, seed=21), _r(4096, 2048, seed=22)
    for beta in (0.0, 1.0):
        dw_a = _r(512, 2048, dtype=torch.float32, seed=23)
        dw_b = dw_a.clone()
        G.wgrad(dy, x, dw_a, beta=beta)
        G.wgrad(dy, x, dw_b, beta=beta, red=red)
        db_a = _r(2048, dtype=torch.float32, seed=24)
        db_b = db_a.clone()
        G.colsum(x, db_a, beta=beta)
        G.colsum(x, db_b, beta=beta, red=red)
        D = 512
        xx, g = _r(4096, D, dtype=torch.float32, seed=25), _r(D, dtype=torch.float32, seed=26)
        mu, rs = xx.mean(-1), torch.rsqrt(xx.var(-1, unbiased=False) + 1e-6)
        dyl = _r(4096, D, dtype=torch.float32, seed=27)
        outs = []
        for r in (None, red):
            dg, dbb, dbias = (_r(D, dtype=torch.float32, seed=28 + i) for i in range(3))
            dx = LN.layernorm_bwd(dyl, xx, g, mu, rs, None, dg, dbb, beta, dbias=dbias, red=r)
            outs.append((dx, dg, dbb, dbias))
        assert red.pending, "tasks should be queued until flush"
        red.flush()
        assert torch.equal(dw_a, dw_b), "wgrad split-K via reducer"
        assert torch.equal(db_a, db_b), "colsum via reducer"
        for a, b in zip(*outs):
            assert torch.equal(a, b), "layernorm_bwd via reducer"
    data = _r(1_000_003, dtype=torch.float32, seed=30)
    part = torch.zeros(37, device=cuda)
    red.add_sumsq(data, 0.5, part)
    red.flush_all()
    ref = 0.5 * (data.double() ** 2).sum()
    assert abs(part.double().sum().item() - ref.item()) <= 1e-5 * ref.item()


@pytest.mark.parametrize("Mtok,N,K", [(4096, 2048, 512), (4096, 1536, 512), (4096, 512, 512), (256, 200, 96)])
def test_wgrad_fused_bias_grad(cuda, Mtok, N, K):
    """wgrad(..., db=) sums the bias gradient inside the GEMM (register-staged path) — equals the
    standalone colsum to fp32 reassociation, dW unchanged."""
    from distributed_training_compare_jax_amd.ops.reduce import GradReducer

    red = GradReducer(cuda, arena_mb=64)
    dy, x = _r(Mtok, N, seed=31), _r(Mtok, K, seed=32)
    for beta in (0.0, 1.0):
        dw, db = _r(N, K, dtype=torch.float32, seed=33), _r(N, dtype=torch.float32, seed=34)
        dw0, db0 = dw.clone(), db.clone()
        G.wgrad(dy, x, dw, beta=beta, red=red, db=db)
        red.flush()
        _close(dw, beta * dw0 + dy.float().t() @ x.float(), 2e-3, "dW")
        _close(db, beta * db0 + dy.float().sum(0), 1e-5, "db")


def test_host_sort_keys_match_device(cuda):
    """The host-side embedding sort keys (shipped with the batch) equal the device bitonic sort."""
    import numpy as np

    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 50258, (8, 512), generator=g, dtype=torch.int32)
    ids[0, :100] = 7  # long run of one id
    dev = E.embed_sort_keys(ids.to(cuda), 50258)
    host = E.embed_sort_keys_host(ids.numpy())
    assert np.array_equal(dev.cpu().numpy(), host)


@pytest.mark.parametrize("M,Nout,Kin,mode", [(4096, 512, 2048, "dgelu"), (4096, 2048, 512, "f32"),
                                              (4096, 512, 512, "bf16"), (4096, 1536, 512, "f32"),
                                              (512, 384, 256, "f32")])
def test_linear_backward_pair(cuda, M, Nout, Kin, mode):
    """G.linear_backward (dgrad + weight gradient [+ bias gradient] in one paired launch) equals the
    two separate GEMMs bitwise (same tile programs, same summation orders)."""
    from distributed_training_compare_jax_amd.ops.reduce import GradReducer

    red = GradReducer(cuda, arena_mb=128)
    dy, w, x = _r(M, Nout, seed=41), _r(Nout, Kin, scale=0.05, seed=42), _r(M, Kin, seed=43)
    u = _r(M, Kin, seed=44) if mode == "dgelu" else None
    od = torch.bfloat16 if mode == "bf16" else torch.float32
    for beta in (0.0, 1.0):
        dw_a, db_a = _r(Nout, Kin, dtype=torch.float32, seed=45), _r(Nout, dtype=torch.float32, seed=46)
        dw_b, db_b = dw_a.clone(), db_a.clone()
        dx_b = G.linear_backward(dy, w, x, dw_b, beta, red=red, db=db_b, dgelu_u=u, out_dtype=od)
        red.flush()
        dx_a = G.matmul_nn_dgelu(dy, w, u) if u is not None else G.matmul_nn(dy, w, out_dtype=od)
        G.wgrad(dy, x, dw_a, beta, red=red, db=db_a)
        red.flush()
        assert torch.equal(dx_a, dx_b), "dgrad"
        assert torch.equal(dw_a, dw_b), "wgrad"
        assert torch.equal(db_a, db_b), "bias grad"
    ref = dy.float().t() @ x.float()  # last iteration: beta = 1 onto the seed-45 tensor
    _close(dw_b, _r(Nout, Kin, dtype=torch.float32, seed=45) + ref, 2e-3, "wgrad vs fp32")


@pytest.mark.parametrize("M,D,K", [(4096, 512, 512), (4096, 512, 2048), (1024, 768, 256), (2048, 1024, 128)])
def test_gemm_resid_ln_fused(cuda, M, D, K):
    """Residual-stream GEMM + LayerNorm in one launch (ops/ln_fused.py) vs the fp32 reference; two calls
    on one granule buffer with an advancing step (stale tags of the first call must not satisfy the second)."""
    from distributed_training_compare_jax_amd.ops import ln_fused as LF

    a, w = _r(M, K, seed=31), _r(D, K, scale=0.05, seed=32)
    b = _r(D, dtype=torch.float32, seed=33)
    res = _r(M, D, dtype=torch.float32, seed=34) * 2 + 0.5
    g, be = _r(D, dtype=torch.float32, seed=35), _r(D, dtype=torch.float32, seed=36)
    step = torch.zeros(1, dtype=torch.int64, device=cuda)
    sync = LF.LnSync(cuda, M, D, nsites=2, step=step)
    for it in range(2):
        x, (y, mu, rs) = LF.linear_resid_ln(a, w, b, res, g, be, 1e-6, sync, site=it)
        xr = res + a.float() @ w.float().t() + b
        _close(x, xr, 2e-5, "x")
        mr = xr.mean(-1)
        rr = torch.rsqrt((xr - mr[:, None]).pow(2).mean(-1) + 1e-6)
        _close(mu, mr, 1e-5, "mean")
        _close(rs, rr, 1e-4, "rstd")
        _close(y, (xr - mr[:, None]) * rr[:, None] * g + be, 1e-2, "y")
        a = _r(M, K, seed=40 + it)  # new data for the second call
        step += 1
    torch.cuda.synchronize()
    sync.check()


@pytest.mark.parametrize("M,D,K,nslab", [(4096, 512, 2048, 3), (4096, 512, 1536, 2), (1024, 768, 256, 3)])
def test_dgrad_ln_bwd_fused(cuda, M, D, K, nslab):
    """NT dgrad + LayerNorm backward in one launch vs the unfused dgrad + ln_bwd kernels."""
    from distributed_training_compare_jax_amd.ops import ln_fused as LF

    dY, wt = _r(M, K, seed=51), _r(D, K, scale=0.05, seed=52)
    x = _r(M, D, dtype=torch.float32, seed=53) * 3 + 1
    g = _r(D, dtype=torch.float32, seed=54)
    _, mu, rs = LN.layernorm_fwd(x, g, g, 1e-6, torch.bfloat16)
    dres = _r(M, D, dtype=torch.float32, seed=55)
    step = torch.full((1,), 7, dtype=torch.int64, device=cuda)
    sync = LF.LnSync(cuda, M, D, nsites=3, step=step)
    outs = [torch.zeros(D, device=cuda) for _ in range(3)]
    dbias = outs[2] if nslab == 3 else None
    dx, dxc = LF.dgrad_ln_bwd(dY, wt, x, g, mu, rs, dres, outs[0], outs[1], 0.0, dbias=dbias, sync=sync, site=2)
    refs = [torch.zeros(D, device=cuda) for _ in range(3)]
    dy = G.linear_resid(dY, wt, None, None)
    dxr = LN.layernorm_bwd(dy, x, g, mu, rs, dres, refs[0], refs[1], 0.0, dbias=refs[2] if nslab == 3 else None)
    _close(dx, dxr, 1e-4, "dx")
    _close(dxc, dxr, 1e-2, "dx_bf16")
    for s, name in enumerate(("dgamma", "dbeta", "dbias")[:nslab]):
        _close(outs[s], refs[s], 1e-4, name)
    # accumulate mode (beta = 1) adds onto the existing gradients
    dx2, _ = LF.dgrad_ln_bwd(dY, wt, x, g, mu, rs, None, outs[0], outs[1], 1.0, dbias=dbias, sync=sync, site=0)
    _close(outs[0], 2 * refs[0], 1e-4, "dgamma_acc")
    _close(dx2, dxr - dres, 1e-4, "dx_no_dres")
    torch.cuda.synchronize()
    sync.check()
