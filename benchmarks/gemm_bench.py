"""Per-shape timing of the HIP GEMM (every Dense of the reference GPT, fwd/dgrad/wgrad) and of the
other hot kernels, in TFLOP/s / TB/s.  torch.matmul (hipBLASLt) is timed on the same bf16 operands
as a yardstick only — it is never used by the training path.

    python benchmarks/gemm_bench.py [--reps 50] [--json out.json] [--model ref|gpt2-small|gpt2-medium]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import attention as A  # noqa: E402
from distributed_training_compare_jax_amd.ops import gemm as G  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    ap.add_argument("--model", default="ref")
    ap.add_argument("--only", default="", help="comma list: run only ops whose name contains one of these")
    ap.add_argument("--no-ref", action="store_true", help="skip the hipBLASLt yardstick (clean PMC runs)")
    a = ap.parse_args()
    only = [x for x in a.only.split(",") if x]
    want = lambda name: not only or any(o in name for o in only)  # noqa: E731
    dev = torch.device("cuda")
    from distributed_training_compare_jax_amd.config.schema import model_config_from_preset

    mc = model_config_from_preset(a.model)
    M, D, F, V = 8 * mc.max_seq_len, mc.d_model, mc.d_ff, mc.padded_vocab
    H, T = mc.n_heads, mc.max_seq_len
    r = lambda *s: (torch.randn(*s, device=dev) * 0.5).to(torch.bfloat16)  # noqa: E731
    rows = []

    def tm(name, fn, ref=None):
        """(us, hipBLASLt us) of `name`, or None when filtered out"""
        if not want(name):
            return None
        return timeit(fn, a.reps), (None if (ref is None or a.no_ref) else timeit(ref, a.reps))

    def rec(name, us, flops, ref_us=None):
        tf = flops / us / 1e6
        rows.append(dict(op=name, us=round(us, 2), tflops=round(tf, 1),
                         hipblaslt_us=None if ref_us is None else round(ref_us, 2)))
        print(f"{name:38s} {us:9.1f} us {tf:8.1f} TF/s" + ("" if ref_us is None else f"   (hipBLASLt {ref_us:8.1f} us)"),
              flush=True)

    for (n, k, tag) in [(3 * D, D, "qkv"), (D, D, "out"), (F, D, "fc1"), (D, F, "fc2"), (V, D, "lm_head")]:
        x, w = r(M, k), r(n, k) * 0.05
        b = torch.zeros(n, device=dev)
        res = torch.zeros(M, n, device=dev)
        if tag in ("out", "fc2"):
            f = lambda: G.linear_resid(x, w, b, res)  # noqa: E731
        elif tag == "fc1":
            f = lambda: G.linear_gelu(x, w, b)  # noqa: E731
        elif tag == "lm_head":
            from distributed_training_compare_jax_amd.ops import xent as X
            lab = torch.randint(0, 50257, (M,), device=dev, dtype=torch.int32)
            f = lambda: X.lmhead_logits_partials(x, w, b, lab, 0, 50257)  # noqa: E731
        else:
            f = lambda: G.linear(x, w, b)  # noqa: E731
        nm = f"fwd  {tag} [{M}x{n}x{k}]"
        t = tm(nm, f, lambda: x @ w.t())
        if t:
            rec(nm, t[0], 2 * M * n * k, t[1])
        dy = r(M, n)
        if tag == "fc2":
            u = r(M, k)
            f = lambda: G.matmul_nn_dgelu(dy, w, u)  # noqa: E731
        else:
            f = lambda: G.matmul_nn(dy, w)  # noqa: E731
        nm = f"dgrad {tag} [{M}x{k}x{n}]"
        t = tm(nm, f, lambda: dy @ w)
        if t:
            rec(nm, t[0], 2 * M * n * k, t[1])
        if tag in ("qkv", "fc1"):  # the NT dgrad on the transposed weight (fp32 out), as the step runs it
            wt = w.t().contiguous()
            nm = f"ntdgrad {tag} [{M}x{k}x{n}]"
            t = tm(nm, lambda: G.linear(dy, wt, out_dtype=torch.float32), lambda: dy @ w)
            if t:
                rec(nm, t[0], 2 * M * n * k, t[1])
        dw = torch.zeros(n, k, device=dev)
        nm = f"wgrad {tag} [{n}x{k}x{M}]"
        t = tm(nm, lambda: G.wgrad(dy, x, dw), lambda: dy.t() @ x)
        if t:
            rec(nm, t[0], 2 * M * n * k, t[1])
        db = torch.zeros(n, device=dev)
        t = tm(f"colsum {tag}", lambda: G.colsum(dy, db))
        if t:
            rows.append(dict(op=f"colsum {tag}", us=round(t[0], 2)))
            print(f"colsum {tag:31s} {t[0]:9.1f} us", flush=True)
    # lm_head forward without the CE epilogue (isolates the epilogue cost)
    x, w = r(M, D), r(V, D) * 0.05
    nm = f"fwd  lm_head plain-epilogue [{M}x{V}x{D}]"
    t = tm(nm, lambda: G.linear(x, w, None))
    if t:
        rec(nm, t[0], 2 * M * V * D)
    qkv = r(8, T, 3 * D)
    o, lse = A.attn_fwd(qkv, H)
    fl = A.attn_flops(8, T, H, D // H)
    nm = f"attn fwd  B8 T{T} H{H} hd{D // H}"
    t = tm(nm, lambda: A.attn_fwd(qkv, H))
    if t:
        rec(nm, t[0], fl)
    do = r(8, T, D)
    nm = f"attn bwd  B8 T{T} H{H} hd{D // H}"
    t = tm(nm, lambda: A.attn_bwd(qkv, o, lse, do, H))
    if t:
        rec(nm, t[0], 2.5 * fl)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
