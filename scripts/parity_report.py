"""bf16 vs exact-fp32 loss curves of the same 5000-step run (scripts/parity_runs.sh) -> markdown.

    python scripts/parity_report.py gpurun_out/parity [--out profiles/r3_parity_bf16_vs_fp32.md]

Per 500-step window: mean |loss_bf16 - loss_fp32| and both window means; plus the last-50 means
(the reference's headline loss statistic) and step-0 losses.
"""

import argparse
import os

import numpy as np
import pandas as pd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    b = pd.read_csv(os.path.join(a.root, "bf16", "log.csv"))
    f = pd.read_csv(os.path.join(a.root, "fp32", "log.csv"))
    n = min(len(b), len(f))
    lb, lf = b.loss.values[:n], f.loss.values[:n]
    d = np.abs(lb - lf)
    lines = ["# bf16 vs exact-fp32 training curves (reference model, DP, 5000 timed steps, same data and init)", "",
             "Both runs: `main.py --train_config_path configs/train_config_dp.yaml` (5 warmup + 5000 timed steps), "
             "synthetic FineWeb-shaped tokens, canonical init (seed 0).  bf16 = MFMA bf16 with fp32 master weights "
             "and fp32 accumulation; fp32 = every GEMM / attention / CE on the exact-fp32 MFMA kernels "
             "(`csrc/gemm_f32.hip`, `csrc/attention_f32.hip`), the reference's precision.", "",
             f"* step 0 loss: bf16 {lb[0]:.4f}, fp32 {lf[0]:.4f} (|d| {abs(lb[0] - lf[0]):.2e})",
             f"* last-50 mean: bf16 {lb[-50:].mean():.4f}, fp32 {lf[-50:].mean():.4f} "
             f"(|d| {abs(lb[-50:].mean() - lf[-50:].mean()):.4f})",
             f"* last-500 mean: bf16 {lb[-500:].mean():.4f}, fp32 {lf[-500:].mean():.4f}",
             f"* avg step (ms, the reference's timed span): bf16 {1e3 * b.elapsed_time.values[n - 1] / n:.2f}, "
             f"fp32 {1e3 * f.elapsed_time.values[n - 1] / n:.2f}", "",
             "| steps | mean loss bf16 | mean loss fp32 | mean abs diff | max abs diff |", "|---|---|---|---|---|"]
    for s in range(0, n, 500):
        e = min(n, s + 500)
        lines.append(f"| {s}-{e - 1} | {lb[s:e].mean():.4f} | {lf[s:e].mean():.4f} | {d[s:e].mean():.4f} | "
                     f"{d[s:e].max():.4f} |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
