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
    ap.add_argument("--shape", default="gpt2s", choices=["ref", "gpt2s"])
    a = ap.parse_args()
    B, T, H, hd = (8, 512, 16, 32) if a.shape == "ref" else (8, 1024, 12, 64)
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(B, T, 3 * H * hd, generator=g).cuda().bfloat16()
    do = torch.randn(B, T, H * hd, generator=g).cuda().bfloat16()
    o, lse = A.attn_fwd(qkv, H)
    fwd_flops = 4.0 * B * H * T * T * hd / 2  # causal: half of QK^T and PV
    if a.shape == "ref":
        variants = {"fwd": lambda: A.attn_fwd(qkv, H), "fwd plain order": lambda: A.attn_fwd(qkv, H, flags=1),
                    "bwd fused": lambda: A.attn_bwd(qkv, o, lse, do, H),
                    "bwd two-round": lambda: A.attn_bwd(qkv, o, lse, do, H, flags=1)}
    else:
        o4, _ = A.attn_fwd(qkv, H, flags=4)
        o5, lse5 = A.attn_fwd(qkv, H, flags=16)
        torch.cuda.synchronize()
        print(f"fwd 32-row vs 16-row kernel: max |do| {(o.float() - o4.float()).abs().max().item():.3e}", flush=True)
        print(f"fwd round-4 32-row kernel vs round-5 default: max |do| {(o.float() - o5.float()).abs().max().item():.3e} "
              f"max |dlse| {(lse - lse5).abs().max().item():.3e}", flush=True)
        o6, lse6 = A.attn_fwd(qkv, H, flags=32)
        torch.cuda.synchronize()
        print(f"fwd 2 waves/SIMD vs default (3): max |do| {(o.float() - o6.float()).abs().max().item():.3e} "
              f"max |dlse| {(lse - lse6).abs().max().item():.3e}", flush=True)
        o7, lse7 = A.attn_fwd(qkv, H, flags=64)
        torch.cuda.synchronize()
        print(f"fwd heavy-first vs CU-balanced (default) order: max |do| {(o.float() - o7.float()).abs().max().item():.3e} "
              f"max |dlse| {(lse - lse7).abs().max().item():.3e}", flush=True)
        variants = {"fwd (default, 3 waves/SIMD)": lambda: A.attn_fwd(qkv, H),
                    "fwd heavy-first order": lambda: A.attn_fwd(qkv, H, flags=64),
                    "fwd (2 waves/SIMD, round 5)": lambda: A.attn_fwd(qkv, H, flags=32),
                    "fwd (round 4: 32 q/wave)": lambda: A.attn_fwd(qkv, H, flags=16),
                    "fwd (16 q/wave chunk)": lambda: A.attn_fwd(qkv, H, flags=4),
                    "bwd (32 rows/wave)": lambda: A.attn_bwd(qkv, o, lse, do, H),
                    "bwd merged (delta + 1 launch)": lambda: A.attn_bwd(qkv, o, lse, do, H, flags=8),
                    "bwd (16-row chunk)": lambda: A.attn_bwd(qkv, o, lse, do, H, flags=4)}
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, fn in variants.items():
            res[k].append(timeit(fn, a.reps))
    for k, v in res.items():
        v = sorted(v)
        fl = fwd_flops * (2.5 if k.startswith("bwd") else 1.0)
        print(f"{k:28s} median {v[len(v) // 2]:7.2f} us  min {v[0]:7.2f} us  ({fl / v[len(v) // 2] / 1e6:6.1f} TF/s)",
              flush=True)


if __name__ == "__main__":
    main()
