"""Aggregate bench.py JSON lines of a scaling sweep (scripts/scale_sweep.sh).

    python scripts/scaling_report.py outputs/scaling_raw.jsonl [--json outputs/scaling.json] [--md outputs/scaling.md]

scaling.json is what plot.py draws ({"dp": {"1": tokens/s, ...}, ...}); the markdown table adds
ms/step and the efficiency vs the same strategy at N=1: weak scaling (dp: per-GPU batch fixed)
eff = value_N / (N * value_1); strong scaling (tp, pp: global batch fixed) eff = value_N / (N * value_1)
as well (ideal strong scaling multiplies tokens/s by N).
"""

import argparse
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("raw")
    ap.add_argument("--json", default=None)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = [json.loads(l) for l in open(a.raw) if l.strip()]
    table = defaultdict(dict)
    extra = []
    failed = [r["failed"] for r in rows if "failed" in r]
    for r in rows:
        if "failed" in r:
            continue
        par = r["config"]["parallelism"]
        strat = "".join(c for c in par if c.isalpha())
        if "x" in par:
            extra.append(r)
            continue
        table[strat][str(r["n_gpus"])] = r
    out = {s: {n: v["value"] for n, v in d.items()} for s, d in table.items()}
    lines = ["| strategy | GPUs | model | global batch | ms/step | tokens/s | scaling | efficiency vs N=1 |",
             "|---|---|---|---|---|---|---|---|"]
    for s in ("dp", "tp", "pp"):
        d = table.get(s, {})
        base = d.get("1")
        for n in sorted(d, key=int):
            r = d[n]
            eff = r["value"] / (int(n) * base["value"]) if base else None
            lines.append(f"| {s} | {n} | {r['config']['model'].split(' ')[0]} | {r['config']['global_batch']} | "
                         f"{r['ms_per_step']:.3f} | {r['value']:,.0f} | {r['scaling']} | "
                         f"{'' if eff is None else f'{100 * eff:.1f} %'} |")
    for r in extra:
        lines.append(f"| {r['config']['parallelism']} | {r['n_gpus']} | {r['config']['model'].split(' ')[0]} | "
                     f"{r['config']['global_batch']} | {r['ms_per_step']:.3f} | {r['value']:,.0f} | {r['scaling']} | |")
    if failed:
        lines.append("")
        lines.append("failed runs: " + ", ".join(failed))
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=2)
    if a.md:
        open(a.md, "w").write(txt)


if __name__ == "__main__":
    main()
