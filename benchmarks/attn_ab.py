"""In-process A/B of the attention backward variants at the reference shape (B8 T512 H16 hd32):
fused single-round kernel (default) vs the two-round resident kernels (flags bit 0), interleaved
rounds, plus the forward.  Also checks that both backward variants agree.

    python benchmarks/attn_ab.py [--rounds 7] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import attention as A  # noqa: E402


def timeit(fn, reps):
    """GPU time per call: `reps` calls captured in one hipGraph, replayed (host launch cost excluded)."""
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        gr.capture_begin()
        for _ in range(reps):
            fn()
        gr.capture_end()
    torch.cuda.current_stream().wait_stream(st)
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    B, T, H, hd = 8, 512, 16, 32
    g = torch.Generator().manual_seed(0)
    qkv = (torch.randn(B, T, 3 * H * hd, generator=g) * 0.5).cuda().bfloat16()
    do = (torch.randn(B, T, H * hd, generator=g) * 0.5).cuda().bfloat16()
    o, lse = A.attn_fwd(qkv, H)
    d_new = A.attn_bwd(qkv, o, lse, do, H)
    d_old = A.attn_bwd(qkv, o, lse, do, H, flags=1)
    torch.cuda.synchronize()
    diff = (d_new.float() - d_old.float()).abs().max().item()
    ref = d_old.float().abs().max().item()
    print(f"max |fused - two-round| = {diff:.3e} (max |d| {ref:.3e})", flush=True)
    o1, l1 = A.attn_fwd(qkv, H, flags=1)
    torch.cuda.synchronize()
    print(f"fwd zig vs plain order: max |do| {(o.float() - o1.float()).abs().max().item():.3e}, "
          f"max |dlse| {(lse - l1).abs().max().item():.3e}", flush=True)
    res = {"fwd": [], "fwd plain order": [], "bwd fused": [], "bwd two-round": []}
    for _ in range(a.rounds):
        res["fwd"].append(timeit(lambda: A.attn_fwd(qkv, H), a.reps))
        res["fwd plain order"].append(timeit(lambda: A.attn_fwd(qkv, H, flags=1), a.reps))
        res["bwd fused"].append(timeit(lambda: A.attn_bwd(qkv, o, lse, do, H), a.reps))
        res["bwd two-round"].append(timeit(lambda: A.attn_bwd(qkv, o, lse, do, H, flags=1), a.reps))
    for k, v in res.items():
        v = sorted(v)
        print(f"{k:15s} median {v[len(v) // 2]:7.2f} us  min {v[0]:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
