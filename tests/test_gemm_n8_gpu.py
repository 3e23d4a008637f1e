"""Layer-GEMM kernel on 128 x 192 / 128 x 256 tiles (csrc/gemm.hip gemm8n_kernel: 8 waves, 4- / 3-stage
LDS-DMA ring, phase-interleaved main loop).  Every epilogue the layer GEMMs use (bf16 + bias, fp32
residual, GELU pair, dGELU, fp32 dgrad) on the GPT-2 small / medium shapes it is selected for, forward
(NT) and dgrad (NN, W MN-major) layouts, against the fp32 PyTorch reference of the same op and against
the 128^2 / 256^2 kernels the same call takes with the path switched off (DTC_GEMM8N=0)."""

import pytest
import torch

from distributed_training_compare_jax_amd.ops import _native as N
from distributed_training_compare_jax_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def _r(*shape, scale=1.0, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    t = torch.randn(*shape, generator=g) * scale + 0.1 * torch.rand(*shape, generator=g)
    return t.to("cuda").to(dtype)


def _close(a, b, rtol, name):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= rtol * ref, f"{name}: max abs err {err:.3e} vs ref max {ref:.3e}"


@pytest.fixture
def n8(cuda):
    L = N.lib()
    old = L.dtc_gemm_set_n8(7)  # every whole-round shape (the default takes one-round shapes)
    yield L
    L.dtc_gemm_set_n8(old)


# (M, N, K): GPT-2 small qkv / out_proj / fc1 / fc2 (8192 tokens), ragged M (8100 -> 64 M-tiles),
# GPT-2 medium out_proj (CB 4) and fc1 (CB 4, 4 rounds)
FWD = [(8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072), (8100, 768, 768),
       (8192, 1024, 1024), (8192, 4096, 1024)]


@pytest.mark.parametrize("M,Nn,K", FWD)
def test_n8_forward_epilogues(n8, M, Nn, K):
    x, w = _r(M, K, seed=1), _r(Nn, K, scale=0.05, seed=2)
    b = _r(Nn, seed=3, dtype=torch.float32)
    ref = x.float() @ w.float().t() + b
    y = G.linear(x, w, b)
    _close(y, ref, 1e-2, "store_bf16")
    res = _r(M, Nn, seed=4, dtype=torch.float32)
    yr = G.linear_resid(x, w, b, res)
    _close(yr, ref + res, 2e-3, "resid_f32")
    u, g = G.linear_gelu(x, w, b)
    _close(u, G.gelu_tanh_grad(ref), 1e-2, "gelu_grad")
    _close(g, G.gelu_tanh(ref), 1e-2, "gelu")
    # NT dgrad on a transposed weight (fp32 out), as the fc1 / qkv backward runs it
    _close(G.linear(x, w, out_dtype=torch.float32), ref - b, 2e-3, "nt_f32")
    # the 128^2 / 256^2 kernels agree closely (same bf16 operands, fp32 accumulation, other k order)
    n8.dtc_gemm_set_n8(0)
    yr0 = G.linear_resid(x, w, b, res)
    n8.dtc_gemm_set_n8(7)
    _close(yr, yr0, 1e-4, "n8_vs_tiled")
    assert torch.equal(yr, G.linear_resid(x, w, b, res)), "not run-to-run deterministic"


DGRAD = [(8192, 768, 3072), (8192, 768, 768), (8192, 3072, 768), (8192, 1024, 4096)]


@pytest.mark.parametrize("M,Nn,K", DGRAD)
def test_n8_dgrad(n8, M, Nn, K):
    """dX[M, K] = dY[M, Nn] . W[Nn, K] (layout nn: W is the MN-major operand), plain and dGELU."""
    dy, w = _r(M, Nn, seed=5), _r(Nn, K, scale=0.05, seed=6)
    ref = dy.float() @ w.float()
    _close(G.matmul_nn(dy, w), ref, 2e-3, "nn_f32")
    _close(G.matmul_nn(dy, w, out_dtype=torch.bfloat16), ref, 1e-2, "nn_bf16")
    u = _r(M, K, seed=7)
    _close(G.matmul_nn_dgelu(dy, w, u), ref * u.float(), 1e-2, "dgelu")
    # fused with the GELU backward as NT on W^T
    _close(G.matmul_nt_dgelu(dy, w.t().contiguous(), u), ref * u.float(), 1e-2, "nt_dgelu")


def test_n8_selection(n8):
    """The plan takes exactly the whole-round layer shapes."""
    L = n8
    assert L.dtc_gemm_set_n8(7) == 7
    # the dgrad of a pairable Dense no longer pairs when gemm8n owns its dgrad (checked via the
    # python path: linear_backward still returns the right dX and dW)
    M, Nn, K = 8192, 768, 3072
    dy, w, x = _r(M, Nn, seed=8), _r(Nn, K, scale=0.05, seed=9), _r(M, K, seed=10)
    from distributed_training_compare_jax_amd.ops.reduce import GradReducer
    red = GradReducer(torch.device("cuda"), arena_mb=64)
    dw = torch.zeros(Nn, K, device="cuda")
    dx = G.linear_backward(dy, w, x, dw, red=red)
    red.flush_all()
    torch.cuda.synchronize()
    _close(dx, dy.float() @ w.float(), 2e-3, "pair_dx")
    _close(dw, dy.float().t() @ x.float(), 2e-3, "pair_dw")


WGRAD = [(2304, 768, 8192), (3072, 768, 8192), (768, 3072, 8192), (768, 768, 8192)]


@pytest.mark.parametrize("Nn,K,M", WGRAD)
def test_wgrad_split256(cuda, Nn, K, M):
    """Layer weight gradients split-K on the 256^2 kernel (DTC_WGRAD256): fp32 slabs summed by the
    reducer, bias gradient by the separate column sum; against fp32 torch and the default plan."""
    from distributed_training_compare_jax_amd.ops.reduce import GradReducer
    L = N.lib()
    dy, x = _r(M, Nn, seed=11), _r(M, K, seed=12)
    ref = dy.float().t() @ x.float()
    outs = []
    for on in (1, 0):
        old = L.dtc_gemm_set_wgrad256(on)
        try:
            red = GradReducer(torch.device("cuda"), arena_mb=128)
            dw = torch.full((Nn, K), 0.5, device="cuda")
            db = torch.full((Nn,), 0.25, device="cuda")
            G.wgrad(dy, x, dw, beta=1.0, red=red, db=db)
            red.flush_all()
            torch.cuda.synchronize()
        finally:
            L.dtc_gemm_set_wgrad256(old)
        _close(dw, ref + 0.5, 2e-3, f"dw(w256={on})")
        _close(db, dy.float().sum(0) + 0.25, 2e-3, f"db(w256={on})")
        outs.append(dw)
    _close(outs[0], outs[1], 1e-4, "split256_vs_default")



def test_lmhead_dgrad_cb3(cuda):
    """The lm_head dgrad through the vocabulary (GPT-2 small: M 8192, N 768, K 50304, NT on W^T, split-K
    fp32 slabs): the 256 x 192 plan (DTC_BIG_CB3, 128 tiles x split 2 = one block per CU) against fp32
    torch and against the 256^2 plan (96 tiles x split 2)."""
    L = N.lib()
    M, Nn, K = 8192, 768, 50304
    dy, wt = _r(M, K, scale=0.05, seed=21), _r(Nn, K, scale=0.05, seed=22)
    ref = dy.float() @ wt.float().t()
    outs = []
    for on in (1, 0):
        old = L.dtc_gemm_set_big_cb3(on)
        try:
            out = G.linear(dy, wt, out_dtype=torch.float32)
            torch.cuda.synchronize()
        finally:
            L.dtc_gemm_set_big_cb3(old)
        _close(out, ref, 2e-3, f"lm_head dgrad (cb3={on})")
        outs.append(out)
    _close(outs[0], outs[1], 1e-5, "cb3_vs_256")


# gemm8r (DTC_GEMM8R): 256-row tiles of two widths in one launch.  (M, N, K): qkv forward (256 x 256 tiles on
# columns 0..2047 + 256 x 64 on the rest), fc1 forward / fc2 NT dgrad (N 3072), out_proj (N 768: narrow
# tiles only), GPT-2 medium qkv (N 3072, K 1024)
R8 = [(8192, 2304, 768), (8192, 3072, 768), (8192, 768, 768), (4096, 3072, 1024)]


@pytest.mark.parametrize("M,Nn,K", R8)
def test_r8_epilogues(cuda, M, Nn, K):
    """Every epilogue gemm8r takes (bf16 + bias, GELU pair, NT dGELU, fp32 + bias with mask bit 2) against
    fp32 torch and against the same call with the plan off."""
    L = N.lib()
    x, w = _r(M, K, seed=31), _r(Nn, K, scale=0.05, seed=32)
    b = _r(Nn, seed=33, dtype=torch.float32)
    ref = x.float() @ w.float().t() + b
    dy, u = _r(M, K, seed=34), _r(M, Nn, seed=35)
    # NT dGELU: dU[M, Nn] = (dy[M, K] . w^T) * u, w [Nn, K] the transposed weight operand
    dref = (dy.float() @ w.float().t()) * u.float()
    wkn = w.t().contiguous()  # [K, Nn] row-major: the NN dgrad layout (mask bit 4)
    outs = {}
    for mask in (7, 0):
        old = L.dtc_gemm_set_r8(mask)
        try:
            y = G.linear(x, w, b)
            gg, g = G.linear_gelu(x, w, b)
            yf = G.linear(x, w, b, out_dtype=torch.float32)
            dg = G.matmul_nt_dgelu(dy, w, u)
            dn = G.matmul_nn_dgelu(dy, wkn, u)
            torch.cuda.synchronize()
        finally:
            L.dtc_gemm_set_r8(old)
        _close(y, ref, 1e-2, f"store_bf16 r8={mask}")
        _close(gg, G.gelu_tanh_grad(ref), 1e-2, f"gelu_grad r8={mask}")
        _close(g, G.gelu_tanh(ref), 1e-2, f"gelu r8={mask}")
        _close(yf, ref, 2e-3, f"store_f32 r8={mask}")
        _close(dg, dref, 1e-2, f"nt_dgelu r8={mask}")
        _close(dn, dref, 1e-2, f"nn_dgelu r8={mask}")
        outs[mask] = (y, g, yf, dg, dn)
    for a, c, name in zip(outs[7], outs[0], ("store_bf16", "gelu", "store_f32", "nt_dgelu", "nn_dgelu")):
        _close(a, c, 1e-2, f"r8_vs_default {name}")


@pytest.mark.parametrize("M,Nn,K", R8[:2])
def test_r8_interleaved_order_bitwise(cuda, M, Nn, K):
    """DTC_R8_ILV only changes which block computes which tile: every output bit is unchanged."""
    L = N.lib()
    x, w = _r(M, K, seed=51), _r(Nn, K, scale=0.05, seed=52)
    b = _r(Nn, seed=53, dtype=torch.float32)
    dy, u = _r(M, K, seed=54), _r(M, Nn, seed=55)
    wkn = w.t().contiguous()
    outs = {}
    for ilv in (1, 0):
        old = L.dtc_gemm_set_r8_ilv(ilv)
        try:
            outs[ilv] = (G.linear(x, w, b), *G.linear_gelu(x, w, b), G.matmul_nt_dgelu(dy, w, u),
                         G.matmul_nn_dgelu(dy, wkn, u))
            torch.cuda.synchronize()
        finally:
            L.dtc_gemm_set_r8_ilv(old)
    for a, c in zip(outs[1], outs[0]):
        assert torch.equal(a, c)
