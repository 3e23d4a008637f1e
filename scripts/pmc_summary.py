"""Per-kernel hardware-counter table of one training step from scripts/pmc_step.sh output.

    python scripts/pmc_summary.py gpurun_out [--out profiles/x.md]

Derived columns (gfx950, 256 CUs x 4 SIMDs, 2.4 GHz):
* MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (duration * 2.4e9 * 1024): the counter counts busy cycles
  per SIMD (16 per 16x16x32 bf16 MFMA = 1024 FLOP/cycle/SIMD), so busy * 1024 = the MFMA FLOPs and
  the ratio is the fraction of the 2.5 PF/s dense bf16 peak.
* HBM GB/s = (2 * FETCH_SIZE + WRITE_SIZE) KiB / duration: FETCH_SIZE reports half the bytes of
  wide coalesced reads on gfx950 (MI355X_MICROARCH.md), so it is doubled (an upper bound for
  narrow reads).  Durations are the PMC run's own dispatch timestamps (counters serialise
  dispatches, so they are slightly longer than in the free-running step).
* Last column: the raw ratio of the two SQ counters (extra conflict cycles over LDS-instruction
  issue cycles; different units, so a relative indicator between kernels, not a percentage).
One step = the dispatches after the second-to-last ``adamw_kernel`` / ``adamw_seg_kernel`` up to the last one.
"""

import argparse
import glob
import os

import pandas as pd

CLK, SIMDS = 2.4e9, 1024
SIMDS_FLOP = 1024  # bf16 16x16x32: 1024 FLOP per MFMA-busy cycle per SIMD


def load(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        raise SystemExit(f"no counter_collection.csv under {d}")
    x = pd.read_csv(fs[0])
    return x


def last_step(x):
    disp = x.drop_duplicates("Dispatch_Id").sort_values("Dispatch_Id")
    ad = disp[disp.Kernel_Name.str.contains("adamw_seg_kernel|adamw_kernel", regex=True)].Dispatch_Id.tolist()
    lo, hi = ad[-2], ad[-1]
    return x[(x.Dispatch_Id > lo) & (x.Dispatch_Id <= hi)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tag", default="step", help="pmc_<tag>{1,2,3} directories (scripts/pmc_step.sh PMC_TAG)")
    ap.add_argument("--fp32", action="store_true",
                    help="exact-fp32 step: MFMA busy cycles are v_mfma_f32_32x32x2_f32 (64 FLOP/cycle/SIMD, 157 TF peak)")
    ap.add_argument("--title", default="Whole-step hardware counters (rocprofv3 --pmc, 3 passes, one step of bench.py)")
    a = ap.parse_args()
    flop_cyc = 64 if a.fp32 else SIMDS_FLOP
    frames = []
    for i in (1, 2, 3):
        s = last_step(load(os.path.join(a.root, f"pmc_{a.tag}{i}")))
        s = s.assign(order=s.Dispatch_Id.rank(method="dense").astype(int))
        frames.append(s)
    # the three passes run the same dispatch sequence: align them by position within the step
    wide = []
    for s in frames:
        p = s.pivot_table(index=["order", "Kernel_Name"], columns="Counter_Name", values="Counter_Value",
                          aggfunc="sum")
        dur = s.drop_duplicates("Dispatch_Id").set_index("order")
        p = p.reset_index().set_index("order")
        p["dur_ns"] = (dur.End_Timestamp - dur.Start_Timestamp).reindex(p.index)
        wide.append(p)
    base = wide[0]
    for w in wide[1:]:
        for c in w.columns:
            if c not in ("Kernel_Name", "dur_ns"):
                base[c] = w[c].reindex(base.index)
    base["name"] = base.Kernel_Name.str.replace("(anonymous namespace)::", "", regex=False).str.replace(
        r"\(.*", "", regex=True).str.slice(0, 72)
    g = base.groupby("name").agg(calls=("dur_ns", "size"), dur_us=("dur_ns", lambda v: v.sum() / 1e3),
                                 mfma=("SQ_VALU_MFMA_BUSY_CYCLES", "sum"), fetch=("FETCH_SIZE", "sum"),
                                 write=("WRITE_SIZE", "sum"), ldsc=("SQ_LDS_BANK_CONFLICT", "sum"),
                                 ldsa=("SQ_ACTIVE_INST_LDS", "sum"))
    g = g.sort_values("dur_us", ascending=False)
    tot = g.dur_us.sum()
    lines = [f"# {a.title}", "",
             f"{int(g.calls.sum())} dispatches, {tot:.0f} us summed dispatch time under PMC; step MFMA FLOPs "
             f"{g.mfma.sum() * flop_cyc / 1e12:.3f} TFLOP, HBM traffic {(2 * g.fetch.sum() + g.write.sum()) * 1024 / 1e9:.2f} GB.",
             "", "MFMA util = MFMA-busy fraction of all SIMD cycles" + (
                 " (exact-fp32 MFMA: 100 % = 157 TF/s)" if a.fp32 else " (bf16: 100 % = 2.5 PF/s dense)"), "",
             "| kernel | calls | us | % | MFMA util | MFMA TF/s | HBM GB/s | SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS |",
             "|---|---|---|---|---|---|---|---|"]
    for n, r in g.iterrows():
        s = r.dur_us * 1e-6
        util = r.mfma / (s * CLK * SIMDS) if s > 0 else 0
        tf = r.mfma * flop_cyc / s / 1e12 if s > 0 else 0
        bw = (2 * r.fetch + r.write) * 1024 / s / 1e9 if s > 0 else 0
        lc = f"{r.ldsc / r.ldsa:.3f}" if r.ldsa > 0 else "-"
        lines.append(f"| `{n}` | {int(r.calls)} | {r.dur_us:.1f} | {100 * r.dur_us / tot:.1f} | "
                     f"{100 * util:.1f} % | {tf:.0f} | {bw:.0f} | {lc} |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
