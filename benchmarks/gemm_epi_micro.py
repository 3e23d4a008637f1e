"""Epilogue cost of the N=2048 layer GEMMs: fc1 fwd plain vs +GELU (2 outputs), fc2 dgrad plain vs
+dGELU, timed as a replayed hipGraph of 20 back-to-back launches (the training step's conditions).

    python benchmarks/gemm_epi_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import gemm as G  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
r = lambda *s: (torch.randn(*s, generator=g) * 0.1).to(dev).to(torch.bfloat16)  # noqa: E731
M, D, F = 4096, 512, 2048
x, w1, w2, u, dy = r(M, D), r(F, D), r(D, F), r(M, F), r(M, D)
b1 = torch.zeros(F, device=dev)
G.reserve_workspace(dev, 64 << 20)
REP = 20


def graphed(fn):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(REP):
            fn()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        gr.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (10 * REP)


cases = {
    "fc1 fwd plain bf16 [4096x2048x512]": lambda: G.linear(x, w1, b1),
    "fc1 fwd +gelu (u,g)": lambda: G.linear_gelu(x, w1, b1),
    "fc2 dgrad plain f32 [4096x2048x512]": lambda: G.matmul_nn(dy, w2),
    "fc2 dgrad plain bf16": lambda: G.matmul_nn(dy, w2, out_dtype=torch.bfloat16),
    "fc2 dgrad +dgelu": lambda: G.matmul_nn_dgelu(dy, w2, u),
}
for name, fn in cases.items():
    us = graphed(fn)
    print(f"{name:40s} {us:7.2f} us  {2 * M * F * D / us / 1e6:7.1f} TF/s", flush=True)
