"""Predicted PP step of GPT-2 small at 8 stages (BASELINE.json config 4) from the schedule simulator.

    PYTHONPATH=. python scripts/pp_estimate.py [--block-ms 0.081] [--head 3.07] > profiles/r5_pp8_estimate.md

Costs: one block's F + B + W for one one-sequence microbatch = ``--block-ms`` (0.650 ms per block for the
8-sequence 1-GPU step / 8, profiles/r5_gemm8r step profile), split F : B : W = 1 : 1 : 1; the head (lm_head
+ CE forward and backward) = ``--head`` blocks (measured: lm_head fwd 633 + dgrad 501 + wgrad ~559 + CE
backward 279 + combine 21 us = 1.99 ms vs 0.65 ms per block).  Messages: one microbatch's [1024, 768]
residual (fp32 3.1 MB, bf16 1.6 MB) over one xGMI link at ~54 GB/s (70 % of 76.8 GB/s per direction) =
58 / 29 us; the head split's row-statistics exchange ~10 us (latency).
"""

import argparse

from distributed_training_compare_jax_amd.parallel.mesh import split_layers, stage_costs
from distributed_training_compare_jax_amd.parallel.pp import estimate, stage_item_costs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block-ms", type=float, default=0.650 / 8)
    ap.add_argument("--head", type=float, default=3.07)
    ap.add_argument("--S", type=int, default=8)
    ap.add_argument("--M", type=int, default=8)
    a = ap.parse_args()
    blk, hc, S, M = a.block_ms, a.head, a.S, a.M
    print(f"# Predicted pp{S} step, GPT-2 small, M = {M} one-sequence microbatches\n")
    print("`scripts/pp_estimate.py` (timed replay of the real stage programs, `parallel/pp.py timeline`). "
          f"Block F+B+W = {blk * 1e3:.0f} us per microbatch, head = {hc} blocks.  Ideal (one GPU's whole "
          f"step / {S}): {12 * blk * M / S + hc * blk * M / S:.2f} ms.\n")
    print("| head | split | schedule | messages | step ms | bubble |")
    print("|---|---|---|---|---|---|")
    for hs in (1, 2):
        r = split_layers(12, S, (0.05, hc), head_stages=hs)
        c = stage_item_costs(S, stage_costs(r, (0.05, hc), hs), head_half=hc / 2 if hs == 2 else 0.0)
        for kind in ("1f1b", "zb"):
            for name, fb in (("free", 0.0), ("bf16 29 us", 0.029), ("fp32 58 us", 0.058)):
                comm = {"f": fb / blk, "b": fb / blk, "s": (0.010 / blk) if fb else 0.0}
                e = estimate(kind, S, M, c, comm=comm, head_split=hs == 2)
                print(f"| {'split over 2 stages' if hs == 2 else 'last stage'} | {[len(x) for x in r]} | {kind} | "
                      f"{name} | {e['makespan'] * blk:.2f} | {100 * e['bubble']:.0f} % |")


if __name__ == "__main__":
    main()
