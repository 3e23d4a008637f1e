"""Comparison plots — same two figures as the reference ``plot.py:6-38`` plus two extras.

* ``outputs/loss.png``: loss vs step for dp/tp/pp (alpha 0.5, red/green/blue).
* ``outputs/average_elapsed_time.png``: bar of Σ(cumulative elapsed_time) per strategy —
  reproduced as-is for parity (the reference sums the cumulative column, which is
  ≈ steps²/2 × step time, not an average).
* ``outputs/step_time.png`` (new): the true average step time in ms.
* ``outputs/scaling.png`` (new, if ``outputs/scaling.json`` exists): tokens/s vs GPUs.
"""

from __future__ import annotations

import json
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

ROOT = "outputs/"
NAMES = ["dp", "tp", "pp"]
COLORS = ["red", "green", "blue"]


def main():
    dfs = {}
    for n in NAMES:
        p = os.path.join(ROOT, n, "log.csv")
        if os.path.exists(p):
            dfs[n] = pd.read_csv(p)
    if not dfs:
        raise SystemExit("no outputs/{dp,tp,pp}/log.csv found")
    for n, c in zip(NAMES, COLORS):
        if n in dfs:
            plt.plot(dfs[n]["step"], dfs[n]["loss"], label=n, alpha=0.5, color=c)
    plt.xlabel("step")
    plt.ylabel("loss")
    plt.legend()
    plt.savefig(os.path.join(ROOT, "loss.png"))
    plt.cla()

    labels = [n for n in NAMES if n in dfs]
    colors = [c for n, c in zip(NAMES, COLORS) if n in dfs]
    plt.bar(labels, [np.sum(dfs[n]["elapsed_time"]) for n in labels], color=colors)
    plt.xlabel("method")
    plt.ylabel("time [sec]")
    plt.savefig(os.path.join(ROOT, "average_elapsed_time.png"))
    plt.cla()

    avg_ms = [1e3 * dfs[n]["elapsed_time"].iloc[-1] / len(dfs[n]) for n in labels]
    plt.bar(labels, avg_ms, color=colors)
    plt.xlabel("method")
    plt.ylabel("average step time [ms]")
    plt.savefig(os.path.join(ROOT, "step_time.png"))
    plt.cla()

    sp = os.path.join(ROOT, "scaling.json")
    if os.path.exists(sp):
        data = json.load(open(sp))  # {"dp": {"1": tok/s, "2": ...}, ...}
        for n, c in zip(NAMES, COLORS):
            if n in data:
                xs = sorted(int(k) for k in data[n])
                plt.plot(xs, [data[n][str(x)] for x in xs], "o-", color=c, label=n)
        plt.xlabel("GPUs")
        plt.ylabel("tokens/s")
        plt.legend()
        plt.savefig(os.path.join(ROOT, "scaling.png"))


if __name__ == "__main__":
    main()
