"""Per-step timeline of a rocprofv3 kernel trace: kernel sequence with queue, start offset,
duration, plus idle-gap statistics.  python scripts/timeline.py <trace.csv> [--marker adamw_kernel] [--out f]"""
import argparse
import re

import pandas as pd

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="adamw_kernel")
ap.add_argument("--out", default=None)
a = ap.parse_args()
t = pd.read_csv(a.trace)
t["k"] = t.Kernel_Name.map(lambda s: re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", s))[:60])
t["blocks"] = t.Grid_Size_X // t.Workgroup_Size_X.clip(lower=1)
t = t.sort_values("Start_Timestamp").reset_index(drop=True)
idx = t.index[t.Kernel_Name.str.contains(a.marker)].tolist()
s = t.loc[idx[-2] + 1: idx[-1]].copy()
t0 = s.Start_Timestamp.min()
s["st"] = (s.Start_Timestamp - t0) / 1e3
s["en"] = (s.End_Timestamp - t0) / 1e3
s["d"] = s.en - s.st
iv = sorted(zip(s.st, s.en))
cur = iv[0][1]
idle = 0.0
gaps = []
for x, y in iv[1:]:
    if x > cur:
        idle += x - cur
        gaps.append(x - cur)
    cur = max(cur, y)
print(f"kernels {len(s)}  wall {cur:.1f} us  busy {s.d.sum():.1f} us  idle {idle:.1f} us in {len(gaps)} gaps")
g = s.groupby(["k", "blocks"]).d.agg(["count", "mean", "sum"]).sort_values("sum", ascending=False)
print(g.head(40).to_string())
if a.out:
    with open(a.out, "w") as f:
        for _, r in s.iterrows():
            f.write(f"{r.st:8.1f} {r.d:7.1f} q{r.Queue_Id} {r.blocks:6d} {r.k}\n")
