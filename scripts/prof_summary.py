"""Summarise a rocprofv3 kernel trace (csv) into a per-step table (markdown).

    python scripts/prof_summary.py gpurun_out/prof/prof_kernel_trace.csv [--out profiles/x.md] [--step-marker adamw]

One training step = the kernels between two consecutive optimizer (``adamw``) launches.
"""

import argparse
import re

import pandas as pd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default=None)
    ap.add_argument("--step-marker", default="adamw_kernel")
    ap.add_argument("--title", default="rocprofv3 kernel trace")
    a = ap.parse_args()
    t = pd.read_csv(a.trace).sort_values("Start_Timestamp").reset_index(drop=True)  # rows are not in time order
    t["dur_us"] = (t.End_Timestamp - t.Start_Timestamp) / 1e3
    t["kernel"] = t.Kernel_Name.map(lambda s: re.sub(r"\(anonymous namespace\)::", "", s))
    t["kernel"] = t.kernel.map(lambda s: re.sub(r"\(.*", "", s)[:70])
    t["blocks"] = t.Grid_Size_X // t.Workgroup_Size_X.clip(lower=1)
    idx = t.index[t.Kernel_Name.str.contains(a.step_marker)].tolist()
    if len(idx) < 2:
        raise SystemExit("need >= 2 optimizer launches in the trace")
    step = t.loc[idx[-2] + 1: idx[-1]]
    wall = (step.End_Timestamp.max() - step.Start_Timestamp.min()) / 1e3
    busy = step.dur_us.sum()
    g = step.groupby(["kernel", "blocks"]).dur_us.agg(["count", "mean", "sum"]).sort_values("sum", ascending=False)
    g["pct"] = 100 * g["sum"] / busy
    lines = [f"# {a.title}", "", f"One step (last complete step in the trace): **{len(step)} kernels**, "
             f"GPU-busy {busy / 1e3:.3f} ms, wall (first start → last end) {wall / 1e3:.3f} ms.", "",
             "| kernel | blocks | calls | mean µs | total µs | % |", "|---|---|---|---|---|---|"]
    for (k, b), r in g.iterrows():
        lines.append(f"| `{k}` | {b} | {int(r['count'])} | {r['mean']:.1f} | {r['sum']:.1f} | {r['pct']:.1f} |")
    md = "\n".join(lines) + "\n"
    print(md)
    if a.out:
        with open(a.out, "w") as f:
            f.write(md)


if __name__ == "__main__":
    main()
