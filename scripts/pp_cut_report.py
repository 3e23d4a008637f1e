"""Collective calls (= graph cuts of a replayed step) per stage per step of the PP programs, round 3
(parallel/pp.py: grouped exchanges, one call per run of p2p items) vs the round-2 executor (receive =
post + wait, send = post, sends waited at the end), for the pipeline shapes the engine runs.

    python scripts/pp_cut_report.py [--out profiles/r3_pp_cuts.md]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.parallel import pp as PP  # noqa: E402


def runs(prog):
    n, prev = 0, False
    for it in prog:
        c = it[0] in ("post", "wait")
        n += c and not prev
        prev = c
    return n


def round2(kind, S, s, M):
    """round-2 executor: per F (non-first) recv = comm(irecv) + wait, per send one comm, waits at the
    end one per send; same for B"""
    n, sends = 0, 0
    for k, _ in PP._schedule(kind, S, s, M):
        if (k == "F" and s > 0) or (k == "B" and s < S - 1):
            n += 2
        if (k == "F" and s < S - 1) or (k == "B" and s > 0):
            n += 1
            sends += 1
    return n + sends


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = ["# PP: collective calls (graph cuts) per stage per step, round 2 vs round 3", "",
             "Max over stages; the whole pipeline's programs also pass `pp.simulate` (RCCL semantics).", "",
             "| schedule | S | M | round 2 | round 3 | ratio |", "|---|---|---|---|---|---|"]
    for kind in ("gpipe", "1f1b"):
        for S, M in ((2, 2), (2, 4), (4, 4), (4, 8), (8, 8), (8, 16)):
            r2 = max(round2(kind, S, s, M) for s in range(S))
            r3 = max(runs(PP.pp_program(kind, S, s, M)) for s in range(S))
            PP.simulate(kind, S, M)
            lines.append(f"| {kind} | {S} | {M} | {r2} | {r3} | {r2 / r3:.1f}x |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
