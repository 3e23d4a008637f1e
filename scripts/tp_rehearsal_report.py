"""Per-rank kernel sums of the TP=8 one-GPU rehearsal (scripts/tp8_rehearsal.sh) -> markdown.

    python scripts/tp_rehearsal_report.py gpurun_out/tp8_fp32 gpurun_out/tp8_bf16 ... [--out profiles/x.md]

Each directory holds rocprofv3 kernel traces of the 8 bench.py ranks (one process each).  One step = the
kernels between a rank's last two ``adamw`` launches.  Kernel classes: P2P collectives (their time includes
the barrier spin while the 7 other processes' kernels occupy the shared GPU -- not an xGMI number), and the
compute kernels (GEMM, attention, LayerNorm, the rest), whose per-rank sums ARE what one GPU of a TP=8 node
runs per step.
"""

import argparse
import glob
import os
import re

import pandas as pd

CLASSES = [("p2p", r"p2p_|barrier"), ("gemm", r"gemm"), ("attention", r"attn"), ("layernorm", r"ln_|layernorm"),
           ("adamw", r"adamw"), ("ce/lm_head", r"ce_|lmhead|xent")]


def classify(name: str) -> str:
    for c, pat in CLASSES:
        if re.search(pat, name):
            return c
    return "other"


def rank_steps(d):
    files = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    out = []
    for f in files:  # one file per rank process
        pid = os.path.basename(f).split("_")[0]
        tp = pd.read_csv(f).sort_values("Start_Timestamp").reset_index(drop=True)
        idx = tp.index[tp.Kernel_Name.str.contains("adamw")].tolist()
        if len(idx) < 2:
            continue
        step = tp.loc[idx[-2] + 1: idx[-1]].copy()
        step["dur_us"] = (step.End_Timestamp - step.Start_Timestamp) / 1e3
        step["cls"] = step.Kernel_Name.map(classify)
        out.append((pid, step))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = ["# TP=8 one-GPU rehearsal: per-rank kernel sums per step", "",
             "8 bench.py ranks (GPT-2 small, global batch 8, tp8) share ONE MI355X; P2P time includes barrier "
             "spins behind the other ranks' kernels. Compute classes are per-rank work.", ""]
    cls = [c for c, _ in CLASSES if c != "p2p"] + ["other"]
    lines.append("| layout | ranks | kernels/step | p2p launches | compute µs/rank (mean) | " +
                 " | ".join(f"{c} µs" for c in cls) + " |")
    lines.append("|---|---|---|---|---|" + "---|" * len(cls))
    for d in a.dirs:
        rs = rank_steps(d)
        if not rs:
            lines.append(f"| {os.path.basename(d)} | 0 | (no trace) |")
            continue
        n = len(rs)
        kern = sum(len(s) for _, s in rs) / n
        p2p = sum((s.cls == "p2p").sum() for _, s in rs) / n
        comp = sum(s.loc[s.cls != "p2p", "dur_us"].sum() for _, s in rs) / n
        per = {c: sum(s.loc[s.cls == c, "dur_us"].sum() for _, s in rs) / n for c in cls}
        lines.append(f"| {os.path.basename(d)} | {n} | {kern:.0f} | {p2p:.0f} | {comp:.0f} | " +
                     " | ".join(f"{per[c]:.0f}" for c in cls) + " |")
    md = "\n".join(lines) + "\n"
    print(md)
    if a.out:
        with open(a.out, "w") as f:
            f.write(md)


if __name__ == "__main__":
    main()
