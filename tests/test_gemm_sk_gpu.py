"""Stream-K GEMM (csrc/gemm.hip gemm_sk_kernel): every CU runs an equal contiguous stretch of the
(tile, K-step) stream; tiles cut between blocks are combined by the last arriving piece, in piece
order.  Checked against the fp32 PyTorch reference of the same op, against the tiled kernels, and
for bitwise run-to-run determinism, on shapes whose K-step counts do not divide the grid evenly
(so tiles are cut into 2-4 pieces), with ragged M and every forward / dgrad epilogue."""

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
def sk(cuda):
    L = N.lib()
    old = L.dtc_gemm_set_sk(3)
    yield L
    L.dtc_gemm_set_sk(old)


# GPT-2 small layer shapes (8192 tokens), a reference-model shape, a cut-heavy one (K-steps per
# tile > K-steps per CU), ragged M
SHAPES = [(8192, 2304, 768), (8192, 3072, 768), (8192, 768, 3072), (8192, 768, 768), (4096, 1536, 512),
          (2000, 1024, 1024)]


@pytest.mark.parametrize("M,Nn,K", SHAPES)
def test_sk_forward_epilogues(sk, M, Nn, K):
    x, w = _r(M, K, seed=1), _r(Nn, K, scale=0.05, seed=2)
    b = _r(Nn, seed=3, dtype=torch.float32)
    ref = x.float() @ w.float().t() + b
    y = G.linear(x, w, b)
    _close(y, ref, 1e-2, "store_bf16")
    res = _r(M, Nn, seed=4, dtype=torch.float32)
    _close(G.linear_resid(x, w, b, res), ref + res, 2e-3, "resid_f32")
    u, g = G.linear_gelu(x, w, b)
    _close(u, G.gelu_tanh_grad(ref), 1e-2, "gelu_grad")
    _close(g, G.gelu_tanh(ref), 1e-2, "gelu")
    # the same problem on the tiled kernels agrees, and stream-K is bitwise deterministic
    sk.dtc_gemm_set_sk(0)
    y_tiled = G.linear_resid(x, w, b, res)
    sk.dtc_gemm_set_sk(3)
    y1, y2 = G.linear_resid(x, w, b, res), G.linear_resid(x, w, b, res)
    assert torch.equal(y1, y2)
    _close(y1, y_tiled, 1e-4, "sk_vs_tiled")


@pytest.mark.parametrize("M,Nn,K", SHAPES)
def test_sk_dgrad(sk, M, Nn, K):
    """dX = dY . W (layout nn, W MN-major), plain and fused with the GELU backward."""
    dy, w = _r(M, Nn, seed=5), _r(Nn, K, scale=0.05, seed=6)
    ref = dy.float() @ w.float()
    _close(G.matmul_nn(dy, w), ref, 2e-3, "nn_f32")
    _close(G.matmul_nn(dy, w, out_dtype=torch.bfloat16), ref, 1e-2, "nn_bf16")
    u = _r(M, K, seed=7)
    _close(G.matmul_nn_dgelu(dy, w, u), ref * u.float(), 1e-2, "dgelu")
