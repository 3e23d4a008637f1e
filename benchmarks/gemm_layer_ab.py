"""In-process A/B of the layer-GEMM plans at a model's training shapes (every NT-layout GEMM the step
runs: the forwards and the dgrads on transposed weights), interleaved rounds, with hipBLASLt
(torch.matmul on the same bf16 operands) as a yardstick and a numerics check of every variant
against an fp32 torch reference.

    python benchmarks/gemm_layer_ab.py [--model gpt2-small] [--rounds 5] [--reps 30]

``--cold``: every call follows a 512 MB buffer write, so its operands come from HBM as in the step.  The
warm (default) mode misranked a candidate kernel in round 4 (gemm4w: ahead warm, profiles/r4_gemm4w_ab.log;
behind cold and in the step, profiles/r4_gemm_cold_ab.log / r4_ab_step_knobs.log): rank candidates cold.
To A/B a kernel variant, build it into another library (scripts/build_variant.py) and run this script
under DTC_KERNEL_LIB for each.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import _native as N  # noqa: E402
from distributed_training_compare_jax_amd.ops import gemm as G  # noqa: E402


def graph_time(fn, reps, pre=None):
    """GPU time per call: `reps` calls captured in one hipGraph, replayed (host launch cost excluded).
    ``pre``: a cache-flushing op captured before every call; its own time (measured alone) is subtracted."""
    if pre is not None:
        both = graph_time(lambda: (pre(), fn()), reps)
        return both - graph_time(pre, reps)
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
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="", help="comma list of plan variants: n8, n8w3, n8w4, n8k768, r8, r8f, r8nn, nor8")
    ap.add_argument("--cold", action="store_true",
                    help="write a 512 MB buffer before every call (operands come from HBM, as in the step)")
    a = ap.parse_args()
    from distributed_training_compare_jax_amd.config.schema import model_config_from_preset

    mc = model_config_from_preset(a.model)
    M, D, F = 8 * mc.max_seq_len, mc.d_model, mc.d_ff
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=0.5: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
    cases = []
    pre = None
    if a.cold:
        flush = torch.empty(128 << 20, dtype=torch.float32, device=dev)
        pre = lambda: flush.fill_(1.0)  # noqa: E731

    def add(name, flops, fn, ref, blas):
        if not a.only or any(o in name for o in a.only.split(",")):
            cases.append((name, flops, fn, ref, blas))

    for (n, k, tag) in [(3 * D, D, "qkv"), (D, D, "out"), (F, D, "fc1"), (D, F, "fc2")]:
        x, w, b = r(M, k), r(n, k, sc=0.05), torch.randn(n, device=dev, generator=g) * 0.1
        fl = 2.0 * M * n * k
        if tag in ("out", "fc2"):  # as the step runs them (DTC_ADD_LN): fp32 a·Wᵀ + b, residual added by the LN
            add(f"fwd {tag} [{M}x{n}x{k}] f32+b", fl, lambda x=x, w=w, b=b: G.linear(x, w, b, out_dtype=torch.float32),
                lambda x=x, w=w, b=b: x.float() @ w.float().t() + b, lambda x=x, w=w: x @ w.t())
        elif tag == "fc1":
            add(f"fwd {tag} [{M}x{n}x{k}] gelu", fl, lambda x=x, w=w, b=b: G.linear_gelu(x, w, b)[1],
                lambda x=x, w=w, b=b: G.gelu_tanh(x.float() @ w.float().t() + b), lambda x=x, w=w: x @ w.t())
            # the same GEMM with one plain bf16 output (what the yardstick computes): the dual-output GELU
            # epilogue's share of the gap
            add(f"fwd {tag} [{M}x{n}x{k}] plain", fl, lambda x=x, w=w, b=b: G.linear(x, w, b),
                lambda x=x, w=w, b=b: x.float() @ w.float().t() + b, lambda x=x, w=w: x @ w.t())
        else:
            add(f"fwd {tag} [{M}x{n}x{k}]", fl, lambda x=x, w=w, b=b: G.linear(x, w, b),
                lambda x=x, w=w, b=b: x.float() @ w.float().t() + b, lambda x=x, w=w: x @ w.t())
        dy, wt = r(M, n), w.t().contiguous()
        if tag in ("qkv", "fc1"):  # DTC_DGRAD_BF16: the input gradient stored bf16
            add(f"ntdgrad {tag} [{M}x{k}x{n}] bf16", fl, lambda dy=dy, wt=wt: G.linear(dy, wt),
                lambda dy=dy, w=w: dy.float() @ w.float(), lambda dy=dy, w=w: dy @ w)
        if tag in ("out", "fc2"):  # DTC_FWD_BF16: the forward stored bf16 + bias
            add(f"fwd {tag} [{M}x{n}x{k}] bf16+b", fl, lambda x=x, w=w, b=b: G.linear(x, w, b),
                lambda x=x, w=w, b=b: x.float() @ w.float().t() + b, lambda x=x, w=w: x @ w.t())
        if tag == "fc2":
            u = r(M, k)
            add(f"ntdgrad {tag} [{M}x{k}x{n}] dgelu", fl, lambda dy=dy, wt=wt, u=u: G.matmul_nt_dgelu(dy, wt, u),
                lambda dy=dy, w=w, u=u: (dy.float() @ w.float()) * u.float(), lambda dy=dy, w=w: dy @ w)
            # the same on the row-major weight (NN: what the step runs)
            add(f"nndgrad {tag} [{M}x{k}x{n}] dgelu", fl, lambda dy=dy, w=w, u=u: G.matmul_nn_dgelu(dy, w, u),
                lambda dy=dy, w=w, u=u: (dy.float() @ w.float()) * u.float(), lambda dy=dy, w=w: dy @ w)
        elif tag == "out":
            add(f"ntdgrad {tag} [{M}x{k}x{n}] bf16", fl, lambda dy=dy, wt=wt: G.linear(dy, wt),
                lambda dy=dy, w=w: dy.float() @ w.float(), lambda dy=dy, w=w: dy @ w)
        else:
            add(f"ntdgrad {tag} [{M}x{k}x{n}] f32", fl, lambda dy=dy, wt=wt: G.linear(dy, wt, out_dtype=torch.float32),
                lambda dy=dy, w=w: dy.float() @ w.float(), lambda dy=dy, w=w: dy @ w)

    # plan variants switched in-process: (gemm8n layout mask, gemm8n tile width) -- "n8" = the persistent
    # 128 x 64CB kernel for multi-round problems too (DTC_GEMM8N bit 4), "n8w4" = with 128 x 256 tiles
    L = N.lib()
    # "n8k768": one-round gemm8n problems down to K = 768 (the out_proj forward / dgrad)
    # "r8": the mixed-width 256-row plan (DTC_GEMM8R=1, bf16 epilogues), "r8f": also fp32 outputs (=3)
    r8_default = L.dtc_gemm_set_r8(0)
    variants = {"ours": (3, 0, 1024, r8_default)}
    for v in [x for x in a.variants.split(",") if x]:
        variants[v] = {"n8": (7, 0, 1024, 0), "n8w3": (7, 3, 1024, 0), "n8w4": (7, 4, 1024, 0),
                       "n8k768": (3, 0, 768, 0), "r8": (3, 0, 1024, 1), "r8f": (3, 0, 1024, 3),
                       "r8nn": (3, 0, 1024, 5), "nor8": (3, 0, 1024, 0), "r8ilv": None}[v]

    ilv_default = L.dtc_gemm_set_r8_ilv(0)
    L.dtc_gemm_set_r8_ilv(ilv_default)
    if "r8ilv" in variants:
        variants["r8ilv"] = variants["ours"] + (1,)

    def use(v):
        L.dtc_gemm_set_r8_ilv(v[4] if len(v) > 4 else ilv_default)
        L.dtc_gemm_set_n8(v[0])
        L.dtc_gemm_set_n8_cb(v[1])
        L.dtc_gemm_set_n8_mink(v[2])
        L.dtc_gemm_set_r8(v[3])

    for name, _, fn, ref, _ in cases:
        want = ref().float()
        for vn, v in variants.items():
            use(v)
            got = fn().float()
            err = ((got - want).norm() / want.norm()).item()
            print(f"check {name:36s} {vn:8s} rel err {err:.2e}", flush=True)
            assert err < 1e-2, (name, vn, err)
    res = {(c[0], v): [] for c in cases for v in list(variants) + ["hipBLASLt"]}
    for _ in range(a.rounds):
        for name, _, fn, _, blas in cases:
            for vn, v in variants.items():
                use(v)
                res[(name, vn)].append(graph_time(fn, a.reps, pre))
            use(variants["ours"])
            res[(name, "hipBLASLt")].append(graph_time(blas, a.reps, pre))
    for name, fl, *_ in cases:
        row = []
        for vn in list(variants) + ["hipBLASLt"]:
            v = sorted(res[(name, vn)])
            med = v[len(v) // 2]
            row.append(f"{vn} {med:7.1f} us ({fl / med / 1e6:6.0f} TF/s)")
        print(f"{name:36s} " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
