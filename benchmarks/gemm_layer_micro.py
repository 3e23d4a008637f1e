"""Layer-GEMM shapes for counter profiling (rocprofv3 --pmc ... -- python benchmarks/gemm_layer_micro.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import gemm as G  # noqa: E402

M, D, F = 4096, 512, 2048
g = torch.Generator().manual_seed(0)
r = lambda *s: (torch.randn(*s, generator=g) * 0.1).to("cuda").to(torch.bfloat16)
x, w1, w2, hmid = r(M, D), r(F, D), r(D, F), r(M, F)
b1, b2 = torch.zeros(F, device="cuda"), torch.zeros(D, device="cuda")
res = torch.zeros(M, D, device="cuda")
dw = torch.zeros(F, D, device="cuda")
for _ in range(5):
    u, ga = G.linear_gelu(x, w1, b1)                 # fc1 fwd  [4096 x 2048 x 512]
    y = G.linear_resid(hmid, w2, b2, res)            # fc2 fwd  [4096 x 512 x 2048]
    G.wgrad(hmid, x, dw, 0.0)                        # fc1 wgrad [2048 x 512 x 4096]
torch.cuda.synchronize()
print("ok")
