"""GPT-2 medium (d1024 L24 H16 T1024, BASELINE.json config 5's model) at its real shape under the
dp2 x tp2 mesh, rehearsed with 4 ranks sharing ONE GPU (gloo: RCCL refuses two ranks per device),
against a single-process run of the same global batch: losses per step and the parameter updates
(reassembled from the TP shards) must agree to bf16 reduction-order noise.

    python scripts/rehearse_medium.py [--steps 3] [--batch 4] [--out gpurun_out/rehearse_medium.json]
"""

import argparse
import json
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(steps, batch, kw, out_dir):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed
    from distributed_training_compare_jax_amd.train.loop import train

    mc = model_config_from_preset("gpt2-medium")
    tc = TrainConfig(seed=0, parallel="dp", batch=batch, steps=steps, log_every=1000, output_dir="/tmp/unused",
                     device="cuda", warmup_steps=2, **kw)
    d = init_distributed("cuda")
    r = train(tc, mc, OptimConfig(lr=3e-4, weight_decay=0.1, grad_clip=1.0), d, quiet=True, write_csv=False)
    eng = r["engine"]
    torch.save({"losses": r["history"], "graphs": r["n_graphs"], "comms": r["n_comms"],
                "named": {n: eng.flat.p(n).detach().float().cpu() for n in eng.flat.slots},
                "tp_idx": eng.mesh.tp_idx, "dp_idx": eng.mesh.dp_idx, "avg_step_ms": r["avg_step_ms"]},
               os.path.join(out_dir, f"rank{d.rank}.pt"))
    destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--out", default="gpurun_out/rehearse_medium.json")
    a = ap.parse_args()
    from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
    from distributed_training_compare_jax_amd.models.params import all_param_specs, unshard
    from distributed_training_compare_jax_amd.parallel.dist import DistInfo, spawn
    from distributed_training_compare_jax_amd.train.engine import Engine

    runs = {}
    for tag, world, kw in (("single", 1, {}), ("dp2xtp2", 4, {"tp": 2})):
        with tempfile.TemporaryDirectory() as td:
            if world == 1:
                for k in ("WORLD_SIZE", "RANK"):
                    os.environ.pop(k, None)
                _worker(a.steps, a.batch, kw, td)
            else:
                spawn(_worker, world, args=(a.steps, a.batch, kw, td))
            runs[tag] = [torch.load(os.path.join(td, f"rank{r}.pt")) for r in range(world)]
        print(tag, "losses", runs[tag][0]["losses"], "graphs", runs[tag][0]["graphs"], "comms", runs[tag][0]["comms"],
              flush=True)
    mc = model_config_from_preset("gpt2-medium")
    specs = {s.name: s for s in all_param_specs(mc)}

    def full(res):
        pieces = {}
        for r in res:
            if r["dp_idx"] == 0:
                for n, t in r["named"].items():
                    pieces.setdefault(n, {})[r["tp_idx"]] = t
        return {n: unshard(specs[n], [p[k] for k in sorted(p)]) for n, p in pieces.items()}

    dev = torch.device("cuda", 0)
    tc = TrainConfig(seed=0, parallel="dp", batch=a.batch, steps=1, log_every=1000, output_dir="/tmp/unused",
                     device="cuda")
    eng = Engine(mc, tc, OptimConfig(lr=3e-4, weight_decay=0.1, grad_clip=1.0), DistInfo(0, 1, 0, dev, "nccl"))
    p0 = {n: eng.flat.p(n).detach().float().cpu() for n in eng.flat.slots}
    del eng
    one, hyb = full(runs["single"]), full(runs["dp2xtp2"])
    worst, errs = 0.0, {}
    for n in one:
        a_, b_, z = hyb[n], one[n], p0[n]
        if n.endswith("qkv.b"):
            a_, b_, z = (x.view(3, -1)[[0, 2]] for x in (a_, b_, z))
        e = ((a_ - z - (b_ - z)).norm() / ((b_ - z).norm() + 1e-12)).item()
        errs[n] = e
        worst = max(worst, e)
    la, lb = runs["dp2xtp2"][0]["losses"], runs["single"][0]["losses"]
    rep = {"model": "gpt2-medium (d1024 L24 H16 F4096 T1024 V50258)", "global_batch": a.batch, "steps": a.steps,
           "mesh": "dp2 x tp2 (4 gloo ranks on one MI355X) vs 1 rank", "losses_dp2xtp2": la, "losses_single": lb,
           "max_abs_loss_diff": max(abs(x - y) for x, y in zip(la, lb)),
           "worst_param_update_rel_diff": worst,
           "worst_params": sorted(errs, key=errs.get)[-5:],
           "graphs_per_step_hybrid": runs["dp2xtp2"][0]["graphs"], "collectives_per_step_hybrid": runs["dp2xtp2"][0]["comms"]}
    print(json.dumps(rep, indent=1))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(rep, open(a.out, "w"), indent=1)
    ok = rep["max_abs_loss_diff"] < 2e-2 and worst < 0.15
    print("REHEARSAL", "OK" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
