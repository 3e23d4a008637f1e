"""Cross-strategy loss agreement of long runs (scripts/cross_strategy_runs.sh) -> markdown + loss.png.

    python scripts/cross_strategy_report.py gpurun_out/curves --out profiles/r4_cross_strategy.md [--png ...]

Per 100-step window: mean |loss_tp - loss_dp| and mean |loss_pp - loss_dp|; the last-50 means (the
reference's headline loss statistic) and the step-0 losses of every run.  The reference's
own criterion is "the loss remains consistent across all strategies" (README.md:51); its published
DP-TP gap is 4.3e-5 mean over the first 100 steps and 7.0e-3 over the last 100.
"""

import argparse
import os

import numpy as np
import pandas as pd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    ap.add_argument("--png", default=None)
    ap.add_argument("--window", type=int, default=100)
    a = ap.parse_args()
    runs = {k: pd.read_csv(os.path.join(a.root, k, "log.csv")) for k in ("dp", "tp", "tp_bf16", "tp_sp", "pp", "pp_zb", "pp_bf16")
            if os.path.exists(os.path.join(a.root, k, "log.csv"))}
    n = min(len(d) for d in runs.values())
    L = {k: d.loss.values[:n] for k, d in runs.items()}
    ms = {k: 1e3 * d.elapsed_time.values[n - 1] / n for k, d in runs.items()}
    lines = ["# Cross-strategy loss curves (reference model, one MI355X)", "",
             f"{n} timed steps each after 5 warmup steps, `main.py` with the reference YAMLs: dp = 1 process; tp = 2 "
             "processes, TP all-reduces on the in-graph P2P kernels (fp32 partials; tp_bf16: bf16 partials, fp32 "
             "sums; tp_sp: bf16 partials + sequence parallelism, reduce-scatter / all-gather); pp = 2 processes, 1F1B with 8 microbatches (`configs/train_config_pp_1f1b.yaml`; pp_zb: the "
             "zero-bubble B/W split; pp_bf16: bf16 stage messages).  The 2-process runs share one GPU over gloo, so their step times "
             "measure nothing about multi-GPU scaling.  Same synthetic data stream and canonical init in every run.", "",
             "| run | step-0 loss | last-50 mean | avg step (ms, shared GPU) |", "|---|---|---|---|"]
    for k in L:
        lines.append(f"| {k} | {L[k][0]:.4f} | {L[k][-50:].mean():.4f} | {ms[k]:.2f} |")
    others = [k for k in L if k != "dp"]
    lines += ["", "| steps | " + " | ".join(f"mean abs({k} - dp)" for k in others) + " | "
              + " | ".join(f"max abs({k} - dp)" for k in others) + " |",
              "|---|" + "---|" * (2 * len(others))]
    for s in range(0, n, a.window):
        e = min(n, s + a.window)
        row = [f"{np.abs(L[k][s:e] - L['dp'][s:e]).mean():.2e}" for k in others]
        row += [f"{np.abs(L[k][s:e] - L['dp'][s:e]).max():.2e}" for k in others]
        lines.append(f"| {s}-{e - 1} | " + " | ".join(row) + " |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)
    if a.png:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        plt.figure(figsize=(8, 4))
        for k, c in zip(L, ("red", "green", "orange", "brown", "blue", "purple", "cyan")):
            plt.plot(L[k], label=k, alpha=0.5, color=c)
        plt.xlabel("step")
        plt.ylabel("loss")
        plt.legend()
        plt.tight_layout()
        plt.savefig(a.png, dpi=100)


if __name__ == "__main__":
    main()
