"""Exact-fp32 kernels (dtype: fp32 parity mode, csrc/gemm_f32.hip + csrc/attention_f32.hip) against a
plain PyTorch reference of the same op computed in float64 on the CPU.

These kernels run v_mfma_f32_32x32x2_f32 (exact f32 products, fp32 accumulation), so the only
difference from the float64 reference is fp32 rounding of the sums: the tolerance is 1e-5 of the
output's magnitude (3e-5 for the K = vocab contraction).  Operands are asymmetric random data.
"""

import pytest
import torch

from distributed_training_compare_jax_amd.ops import attention as A
from distributed_training_compare_jax_amd.ops import gemm as G
from distributed_training_compare_jax_amd.ops import xent as X

pytestmark = pytest.mark.gpu


def _r(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale + 0.1 * torch.rand(*shape, generator=g)).float()


def _close(out, ref64, rtol, name=""):
    out = out.detach().double().cpu()
    err = (out - ref64).abs().max().item()
    mag = ref64.abs().max().item() + 1e-30
    assert err <= rtol * mag, f"{name}: max abs err {err:.3e} vs ref max {mag:.3e} (rel {err / mag:.2e})"


# the reference model's and GPT-2 small's Dense shapes, ragged edges, the lm_head forward
SHAPES = [(4096, 1536, 512), (4096, 512, 2048), (512, 512, 4096), (1000, 200, 48), (130, 70, 32),
          (4096, 50304, 512)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_f32_gemm_forward_epilogues(cuda, M, N, K):
    x, w, b = _r(M, K, seed=1), _r(N, K, scale=0.05, seed=2), _r(N, seed=3)
    xd, wd, bd = x.double(), w.double(), b.double()
    ref = xd @ wd.t() + bd
    xc, wc, bc = x.to(cuda), w.to(cuda), b.to(cuda)
    y = G.linear(xc, wc, bc)
    _close(y, ref, 1e-5, "nt+bias")
    if M * N <= 4096 * 2048:
        res = _r(M, N, seed=4)
        _close(G.linear_resid(xc, wc, bc, res.to(cuda)), ref + res.double(), 1e-5, "nt+bias+resid")
        u, g = G.linear_gelu(xc, wc, bc)
        # the epilogue is checked at the kernel's own pre-activation (same accumulation as y): the
        # fp32 sum's own rounding, amplified by gelu'', is not the epilogue's error
        yd = y.double().cpu()
        _close(u, G.gelu_tanh_grad(yd), 2e-6, "gelu'")
        _close(g, G.gelu_tanh(yd), 2e-6, "gelu")


@pytest.mark.parametrize("M,N,K", [(4096, 512, 512), (4096, 512, 2048), (4096, 2048, 512), (300, 136, 64),
                                   (4096, 50304, 512)])
def test_f32_gemm_dgrad_nn(cuda, M, N, K):
    """dX[M,K] = dY[M,N] . W[N,K] (layout nn), plain and fused with the GELU backward."""
    dy, w = _r(M, N, seed=5), _r(N, K, scale=0.05, seed=6)
    ref = dy.double() @ w.double()
    dyc, wc = dy.to(cuda), w.to(cuda)
    _close(G.matmul_nn(dyc, wc), ref, 3e-5 if N > 8192 else 1e-5, "nn")
    if M * K <= 4096 * 2048:
        u = _r(M, K, seed=7)
        _close(G.matmul_nn_dgelu(dyc, wc, u.to(cuda)), ref * u.double(), 1e-5, "nn*dgelu")


@pytest.mark.parametrize("M,N,K", [(4096, 512, 512), (4096, 2048, 512), (4096, 512, 2048), (4096, 1536, 512),
                                   (777, 96, 160), (4096, 50304, 512)])
def test_f32_gemm_wgrad_tn_splitk(cuda, M, N, K):
    """dW[N,K] = beta*dW + dY[M,N]^T . X[M,K] (layout tn; split-K slabs + ordered reduce) and db."""
    dy, x = _r(M, N, seed=8), _r(M, K, seed=9)
    dw0, db0 = _r(N, K, seed=10), _r(N, seed=11)
    for beta in (0.0, 1.0):
        dw, db = dw0.clone().to(cuda), db0.clone().to(cuda)
        G.wgrad(dy.to(cuda), x.to(cuda), dw, beta=beta, db=db)
        ref = dy.double().t() @ x.double() + beta * dw0.double()
        _close(dw, ref, 1e-5, f"wgrad beta={beta}")
        _close(db, dy.double().sum(0) + beta * db0.double(), 1e-5, f"db beta={beta}")


@pytest.mark.parametrize("M,V,D,valid", [(512, 1024, 64, 1000), (4096, 50304, 512, 50258)])
def test_f32_lmhead_ce(cuda, M, V, D, valid):
    """lm_head logits + CE partials epilogue, the combine, and the fp32 CE backward (+ bias partials)."""
    h, w, b = _r(M, D, seed=12), _r(V, D, scale=0.05, seed=13), _r(V, seed=14)
    g = torch.Generator().manual_seed(15)
    lab = torch.randint(0, valid, (M,), generator=g, dtype=torch.int32)
    logits, part, labl = X.lmhead_logits_partials(h.to(cuda), w.to(cuda), b.to(cuda), lab.to(cuda), 0, valid,
                                                  combine=False)
    lse, loss = X.ce_finalize(part, labl, 1.0 / M)
    ref = h.double() @ w.double().t() + b.double()
    ref[:, valid:] = float("-inf")
    _close(logits[:, :valid], ref[:, :valid], 1e-5, "logits")
    assert torch.isinf(logits[:, valid:]).all()
    lse_ref = torch.logsumexp(ref, -1)
    _close(lse, lse_ref, 1e-6, "lse")
    loss_ref = (lse_ref - ref.gather(1, lab.long()[:, None])[:, 0]).mean()
    assert abs(loss.item() - loss_ref.item()) <= 1e-6 * abs(loss_ref.item()), (loss.item(), loss_ref.item())
    dl, cp = X.ce_backward_inplace(logits, lse, lab.to(cuda), 0, valid, 1.0 / M, colpart=True)
    p = torch.softmax(ref, -1)
    p[torch.arange(M), lab.long()] -= 1.0
    p /= M
    _close(dl, p, 1e-5, "dlogits")
    _close(cp.sum(0), p.sum(0), 1e-5, "bias partials")


@pytest.mark.parametrize("B,T,H,hd", [(2, 512, 4, 32), (1, 1024, 2, 64), (2, 200, 3, 32), (1, 64, 2, 64),
                                      (2, 192, 2, 64)])
def test_f32_flash_attention(cuda, B, T, H, hd):
    """Causal flash attention forward (O, LSE) and backward (dQ, dK, dV) vs the materialised
    float64 softmax(QK^T * hd^-1/2 + causal mask) V of model/CausalSelfAttention.py:34-44."""
    qkv = _r(B, T, 3 * H * hd, seed=16)
    do = _r(B, T, H * hd, seed=17)
    o, lse = A.attn_fwd(qkv.to(cuda), H)
    q, k, v = (t.clone().requires_grad_(True) for t in qkv.double().view(B, T, 3, H, hd).unbind(2))
    s = torch.einsum("bthd,bshd->bhts", q, k) * hd ** -0.5
    mask = torch.ones(T, T, dtype=torch.bool).tril()
    s = s.masked_fill(~mask, float("-inf"))
    oref = torch.einsum("bhts,bshd->bthd", torch.softmax(s, -1), v).reshape(B, T, H * hd)
    _close(o, oref.detach(), 1e-5, "o")
    _close(lse, torch.logsumexp(s, -1).detach(), 1e-6, "lse")
    oref.backward(do.double())
    dqkv = A.attn_bwd(qkv.to(cuda), o, lse, do.to(cuda), H).view(B, T, 3, H, hd)
    for i, (name, t) in enumerate((("dq", q), ("dk", k), ("dv", v))):
        _close(dqkv[:, :, i], t.grad, 1e-5, name)
