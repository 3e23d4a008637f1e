"""Attention kernels for counter profiling:
    rocprofv3 --pmc ... -- python benchmarks/attn_micro.py
ATTN_SHAPE=gpt2s (default): B8 T1024 H12 hd64, both the default kernels and the 16-row chunked ones
(flags bit 2) so one pass profiles both; ATTN_SHAPE=ref: B8 T512 H16 hd32; ATTN_SHAPE=medium: H16 hd64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import attention as A

shape = os.environ.get("ATTN_SHAPE", "gpt2s")
B, T, H, hd = {"gpt2s": (8, 1024, 12, 64), "medium": (8, 1024, 16, 64), "ref": (8, 512, 16, 32)}[shape]
g = torch.Generator().manual_seed(0)
qkv = torch.randn(B, T, 3 * H * hd, generator=g).to("cuda").to(torch.bfloat16)
do = torch.randn(B, T, H * hd, generator=g).to("cuda").to(torch.bfloat16)
for flags in ((0, 4, 16) if hd == 64 else (0,)):  # 16: the round-4 forward
    for _ in range(5):
        o, lse = A.attn_fwd(qkv, H, flags=flags)
        dq = A.attn_bwd(qkv, o, lse, do, H, flags=flags)
torch.cuda.synchronize()
print("ok", float(o.float().abs().mean()), float(dq.float().abs().mean()))
