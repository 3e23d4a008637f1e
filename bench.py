"""Headline benchmark: GPT training throughput on N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--parallel dp|tp|pp] [--tp T] [--model gpt2-small|ref|gpt2-medium]

Metric (BASELINE.json): avg step time (ms) + tokens/sec of **GPT-2 small** (the model every
BASELINE.json config names: d_model 768, 12 layers, 12 heads, d_ff 3072, seq 1024, vocab 50258,
124 M params) trained with AdamW + global-norm clip, bf16 MFMA compute / fp32 master weights,
synthetic FineWeb-shaped tokens (no network) and random-init weights.  ``--model ref`` measures the
reference repo's own 89.6 M model (``configs/model_config.yaml``: d512 L12 H16 F2048 T512).

``vs_baseline`` divides by the only published throughput, the reference's fp32 run of its 89.6 M
model (DP 27,887 / TP 27,919 / PP 19,978 tokens/s, unpublished NVIDIA GPU).  For
GPT-2 small that comparator is conservative: GPT-2 small costs ~2.8x the FLOPs per token of the
reference model (854 M vs 302 M FLOP/token, fwd+bwd), so its tokens/s would be lower on the
reference's own hardware.  The JSON names the comparator (``baseline_comparator``).

Timed span.  W untimed warmup steps first (the first one eager, then hipGraph capture), then TWO
timed loops of K steps, each bracketed by barrier + device sync on both sides, MAX over ranks:

* **blocking** -- ``value`` / ``ms_per_step``: the reference's timed loop (``train/train.py:75-85``)
  step for step: next host batch -> H2D -> full forward + backward + gradient collectives + clip +
  AdamW -> blocking read of THIS step's loss before the next step is issued.  The next batch's host
  work (pinned-buffer fill, embedding sort keys: ``Engine.stage_batch``) runs while the step is on the
  GPU, as a host data loader's would; its H2D copies and the next launch come after the loss read;
* **pipelined** -- ``ms_per_step_pipelined``: the same steps, but step i's loss is read after step
  i+1 is enqueued (the host never leaves the GPU idle between steps; every loss is still read).

``value`` is whole-job tokens/s of the blocking loop.  ``tflops_per_gpu`` counts the causal
attention's useful FLOPs (``ModelConfig.flops_per_token``).

Scaling: ``dp`` keeps 8 sequences per GPU (weak scaling, global batch 8·N); ``tp`` and
``pp`` keep the reference global batch of 8 (strong scaling; pp uses 2·N microbatches).
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOKENS_PER_S = {"dp": 27887.0, "tp": 27919.0, "pp": 19978.0}  # BASELINE.md (4096 tok/step)
METRIC = "avg step time (ms) + tokens/sec, GPT-2-small DP/TP/PP at 1/2/4/8 MI355X"
DEFAULT_MODEL = "gpt2-small"  # BASELINE.json configs 1-4 name GPT-2 small


def _overrides(items):
    """KEY=VALUE strings -> TrainConfig kwargs (value parsed as the field's type)."""
    import dataclasses

    from distributed_training_compare_jax_amd.config.schema import TrainConfig

    types = {f.name: f.type for f in dataclasses.fields(TrainConfig)}
    out = {}
    for it in items:
        k, v = it.split("=", 1)
        if k not in types:
            raise SystemExit(f"unknown TrainConfig field {k!r}")
        t = str(types[k])
        if "bool" in t:
            out[k] = v.lower() in ("1", "true", "yes")
        elif "int" in t:
            out[k] = int(v)
        elif "float" in t:
            out[k] = float(v)
        else:
            out[k] = v
    return out


def _ref_fp32_point(dinfo, steps: int = 20, warmup: int = 3):
    """ms/step and tokens/s of the reference's model (configs/model_config.yaml: d512 L12 H16 F2048 T512,
    batch 8 = 4096 tokens) trained at the reference's precision (exact fp32 MFMA kernels), same timed span
    as the headline's blocking loop, against the published DP number (146.88 ms, 27,887 tok/s)."""
    import torch

    from distributed_training_compare_jax_amd.config.schema import (OptimConfig, TrainConfig,
                                                                     model_config_from_preset)
    from distributed_training_compare_jax_amd.data.synthetic import get_batch_iterator
    from distributed_training_compare_jax_amd.parallel.dist import barrier
    from distributed_training_compare_jax_amd.train.engine import Engine

    mc = model_config_from_preset("ref")
    tc = TrainConfig(seed=0, parallel="dp", batch=8 * dinfo.world, steps=steps, log_every=10 ** 9,
                     output_dir="/tmp/bench", dtype="fp32")
    e = Engine(mc, tc, OptimConfig(lr=3e-4, weight_decay=0.1, grad_clip=1.0), dinfo)
    data = get_batch_iterator(tc.batch, mc.max_seq_len + 1, seed=0, row0=e.feed_row0, nrows=e.feed_rows)
    for _ in range(max(warmup, 2)):
        e.set_batch(next(data))
        e.run_step()
        e.loss_value()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        e.set_batch(next(data))
        e.run_step()
        loss = e.read_loss(e.loss_handle())
    e.flush_optimizer()
    torch.cuda.synchronize()
    barrier()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    tok = 8 * mc.max_seq_len / (ms / 1e3)  # per GPU
    del e
    torch.cuda.empty_cache()
    return {"model": "gpt-ref-89M (d512 L12 H16 F2048 T512 V50258)", "dtype": "fp32", "steps": steps,
            "ms_per_step": round(ms, 3), "tokens_per_s_per_gpu": round(tok, 1), "final_loss": round(loss, 4),
            "reference_ms_per_step": 146.88, "vs_reference": round(tok / BASELINE_TOKENS_PER_S["dp"], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--parallel", default="dp", choices=["dp", "tp", "pp"])
    ap.add_argument("--tp", type=int, default=1,
                    help="with --parallel dp: hybrid DP x TP mesh (BASELINE.json config 5 is dp4 x tp2)")
    ap.add_argument("--model", default=DEFAULT_MODEL)
    ap.add_argument("--batch_per_gpu", type=int, default=8)
    ap.add_argument("--no_graph", action="store_true")
    # zb + the auto head split: the schedule the pp8 estimate ranks best (profiles/r5_pp8_estimate.md:
    # 2.42 ms vs 3.09-3.58 for 1F1B); the JSON reports which schedule and split ran
    ap.add_argument("--pp_schedule", default="zb", choices=["gpipe", "1f1b", "zb"])
    ap.add_argument("--ref32", default="auto", choices=["auto", "on", "off"],
                    help="also time the reference's own model (d512 L12 T512) at the reference's precision (exact "
                         "fp32) and report it as ref_fp32 next to the headline (auto: on for a 1-GPU run)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="extra TrainConfig overrides for A/B runs, e.g. --set defer_optimizer=false")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from distributed_training_compare_jax_amd.config.schema import (OptimConfig, TrainConfig,
                                                                     model_config_from_preset)
    from distributed_training_compare_jax_amd.data.synthetic import get_batch_iterator
    from distributed_training_compare_jax_amd.parallel.dist import barrier, init_distributed
    from distributed_training_compare_jax_amd.train.engine import Engine

    if "RANK" not in os.environ and args.gpus > 1:
        raise SystemExit("multi-GPU: launch with python -m torch.distributed.run --nproc-per-node N bench.py --gpus N")
    dinfo = init_distributed("cuda")
    world = dinfo.world
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    mc = model_config_from_preset(args.model)
    hybrid = args.parallel == "dp" and args.tp > 1
    if hybrid and world % args.tp:
        raise SystemExit(f"--tp {args.tp} does not divide {world} GPUs")
    if args.parallel == "dp":  # weak scaling: batch_per_gpu sequences per DP group
        global_batch, micro, scaling = args.batch_per_gpu * (world // args.tp), 1, "weak"
    elif args.parallel == "tp":
        global_batch, micro, scaling = args.batch_per_gpu, 1, "strong"
    else:
        global_batch, micro, scaling = args.batch_per_gpu, max(2, min(args.batch_per_gpu, 2 * world)), "strong"
    tc = TrainConfig(seed=0, parallel=args.parallel, batch=global_batch, steps=args.steps, log_every=10 ** 9,
                     output_dir="/tmp/bench", pp_microbatches=micro, use_graph=not args.no_graph,
                     pp_schedule=args.pp_schedule, **({"tp": args.tp} if hybrid else {}), **_overrides(args.set))
    oc = OptimConfig(lr=3e-4, weight_decay=0.1, grad_clip=1.0)
    eng = Engine(mc, tc, oc, dinfo)
    data = get_batch_iterator(global_batch, mc.max_seq_len + 1, seed=0, row0=eng.feed_row0, nrows=eng.feed_rows)

    # step 0 runs eagerly (lazy RCCL init, workspace sizing) and step 1 records the hipGraph: with
    # graphs on, at least these two run untimed whatever --warmup says (the reported "warmup" is the
    # number actually run), so graph capture never lands inside the timed steps
    warmup = max(args.warmup, 2) if eng.program.use_graph else args.warmup
    for _ in range(warmup):
        eng.set_batch(next(data))
        eng.run_step()
        eng.loss_value()

    def timed(pipelined: bool):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = float("nan")
        pending = None
        eng.stage_batch(next(data))
        for i in range(args.steps):
            eng.upload_batch()
            eng.run_step()
            handle = eng.loss_handle()
            if not pipelined:  # the reference: block on this step's loss before the next step
                # the next batch's host work (ids / labels into pinned memory, embedding sort keys) while this
                # step runs; its H2D copies are enqueued only after the loss read.  The pinned slot it fills was
                # last copied from before step i-1, whose loss was read.
                eng.stage_batch(next(data))
                loss = eng.read_loss(handle)
                continue
            if pending is not None:  # step i-1's loss, read with step i already enqueued
                loss = eng.read_loss(pending)
            pending = handle
            eng.stage_batch(next(data))  # after step i-1's read: its pinned slot's copy has landed
        if pending is not None:
            loss = eng.read_loss(pending)
        eng.flush_optimizer()  # a deferred last AdamW lands inside the timed region
        torch.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0, loss

    dt_pipe, _ = timed(True)
    dt, loss = timed(False)
    healthy = 1.0
    try:  # device-side wait timeouts (P2P flags, fused LayerNorm statistics): the timed steps computed NaN
        eng.check_health()
    except RuntimeError as exc:
        healthy = 0.0
        print(f"[rank {dinfo.rank}] ERROR: {exc}", file=sys.stderr, flush=True)
    if world > 1:
        t = torch.tensor([dt, dt_pipe, -healthy], device=dinfo.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dt_pipe, healthy = float(t[0].item()), float(t[1].item()), -float(t[2].item())
    if not (loss == loss):
        healthy = 0.0
    ms = 1e3 * dt / args.steps
    tokens = global_batch * mc.max_seq_len
    value = tokens / (ms / 1e3)
    out = None
    if dinfo.rank == 0:
        base = BASELINE_TOKENS_PER_S.get(args.parallel)
        par = {"dp": f"dp{world}", "tp": f"tp{world}", "pp": f"pp{world}"}[args.parallel]
        if hybrid:
            par = f"dp{world // args.tp}xtp{args.tp}"
        metric = METRIC if args.model == "gpt2-small" else METRIC.replace("GPT-2-small", mc.name)
        tp_path = None
        if eng.mesh.tp > 1:
            tp_path = "p2p-xgmi" if eng.p2p is not None else dinfo.backend
        try:
            rccl = ".".join(str(v) for v in torch.cuda.nccl.version()) if dinfo.backend == "nccl" else None
        except Exception:
            rccl = None
        out = {
            "metric": metric, "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": scaling,
            "ms_per_step_pipelined": round(1e3 * dt_pipe / args.steps, 4), "timed_span": "blocking per-step loss read",
            "vs_baseline": round(value / base, 3) if base else None, "dtype": tc.dtype,
            "data": "synthetic (FineWeb-shaped token stream, random-init weights)",
            "healthy": bool(healthy),
            "config": {"model": f"{mc.name} (d{mc.d_model} L{mc.n_layers} H{mc.n_heads} F{mc.d_ff} "
                                f"T{mc.max_seq_len} V{mc.vocab_size})",
                       "global_batch": global_batch, "seq_len": mc.max_seq_len, "parallelism": par,
                       "pp_microbatches": micro if args.parallel == "pp" else None,
                       "pp_schedule": args.pp_schedule if args.parallel == "pp" else None,
                       "pp_head_split": eng.pp_head_split if args.parallel == "pp" else None,
                       "capture_comms": eng.program.capture_comms,
                       "hipgraph": eng.program.use_graph, "final_loss": round(loss, 4),
                       "tflops_per_gpu": round(mc.flops_per_token() * tokens / (ms / 1e3) / world / 1e12, 1),
                       "flops_count": "causal attention (useful work)",
                       "backend": dinfo.backend, "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                       "tp_comm": tp_path, "rccl_version": rccl,
                       "graph_segments": eng.program.n_graphs, "eager_collectives": eng.program.n_comms,
                       "baseline_comparator": (f"reference 89.6M model, fp32, {args.parallel.upper()} "
                                               f"{BASELINE_TOKENS_PER_S.get(args.parallel):,.0f} tok/s (BASELINE.md)")},
        }
    # the like-for-like point: the reference's own model and precision (fp32) on this GPU, timed after the
    # headline engine is released
    del eng, data
    gc.collect()
    torch.cuda.empty_cache()
    if args.ref32 == "on" or (args.ref32 == "auto" and world == 1 and args.model != "ref"):
        ref32 = _ref_fp32_point(dinfo)
    else:
        ref32 = None
    if dinfo.rank == 0:
        out["ref_fp32"] = ref32
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not healthy:
        sys.exit(3)


if __name__ == "__main__":
    main()
