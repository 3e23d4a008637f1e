"""Attention kernels at the reference shape, for counter profiling:
    rocprofv3 --pmc ... -- python benchmarks/attn_micro.py
ATTN_SHAPE=medium: the GPT-2 medium shape (T 1024, head_dim 64: the tiled kernels)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import attention as A

B, T, H, hd = (8, 1024, 16, 64) if os.environ.get("ATTN_SHAPE") == "medium" else (8, 512, 16, 32)
g = torch.Generator().manual_seed(0)
qkv = (torch.randn(B, T, 3 * H * hd, generator=g) * 0.5).to("cuda").to(torch.bfloat16)
do = (torch.randn(B, T, H * hd, generator=g) * 0.5).to("cuda").to(torch.bfloat16)
for _ in range(5):
    o, lse = A.attn_fwd(qkv, H)
    dq = A.attn_bwd(qkv, o, lse, do, H)
torch.cuda.synchronize()
print("ok", float(o.float().abs().mean()), float(dq.float().abs().mean()))
