"""Training driver: warmup, timed loop, console log and ``outputs/<strategy>/log.csv``.

Mirrors ``train/train.py:22-233`` (``train_dp_tp`` / ``train_pp``):

* 5 untimed warmup steps (configurable), printed ``Warmup`` / ``Start measuring``;
* each timed step = next batch → H2D → step → BLOCKING loss read (the reference's span,
  ``train.py:75-85``), elapsed time cumulative since "Start measuring";
* every ``log_every`` steps: ``Step: {s} | Avg loss: {mean:.4f} | Average step time: {t:.4f}``;
* ``Total time: ...`` then ``End``; CSV columns ``step,elapsed_time,loss`` (0-based step).

Extra (not in the reference): the next batch is generated while the GPU runs the current
step (same work, overlapped), and a ``metrics.json`` sidecar records tokens/s, the mesh
and device-time statistics.
"""

from __future__ import annotations

import json
import os
import time
from typing import Optional

import numpy as np
import torch

from ..config.schema import ModelConfig, OptimConfig, TrainConfig
from ..data import synthetic
from ..parallel.dist import DistInfo, barrier
from .engine import Engine


def make_data_iter(eng: Engine, tcfg: TrainConfig, mcfg: ModelConfig, start_step: int = 0):
    if tcfg.data == "fineweb":
        from ..data import fineweb

        return fineweb.get_batch_iterator(eng.global_batch, mcfg.max_seq_len + 1, row0=eng.feed_row0,
                                          nrows=eng.feed_rows)
    return synthetic.get_batch_iterator(eng.global_batch, mcfg.max_seq_len + 1, seed=tcfg.seed, row0=eng.feed_row0,
                                        nrows=eng.feed_rows, start_step=start_step,
                                        vocab=min(synthetic.BPE_VOCAB, mcfg.vocab_size - 1))


def train(train_config: TrainConfig, model_config: ModelConfig, opt_config: OptimConfig, dinfo: DistInfo,
          quiet: bool = False, write_csv: bool = True) -> dict:
    eng = Engine(model_config, train_config, opt_config, dinfo)
    is_main = dinfo.rank == 0
    say = (lambda *a: print(*a, flush=True)) if (is_main and not quiet) else (lambda *a: None)
    data = make_data_iter(eng, train_config, model_config)

    from ..utils.checkpoint import maybe_resume, maybe_save

    start = maybe_resume(eng, train_config)
    if start:
        data = make_data_iter(eng, train_config, model_config, start_step=start)

    from ..utils.trace import Tracer
    from ..utils.watchdog import Watchdog

    tr = Tracer(train_config.profile, train_config.output_dir, dinfo.rank, eng.device)
    dog = Watchdog(dinfo.rank, train_config.watchdog_s).start()
    say("Warmup")
    for i in range(train_config.warmup_steps):
        with tr.span("data"):
            eng.set_batch(next(data))
        with tr.device_step(-train_config.warmup_steps + i):
            eng.run_step()
        with tr.span("loss sync"):
            eng.loss_value()
        dog.beat(-train_config.warmup_steps + i)

    barrier()
    say("Start measuring")
    eng.program.time_comms = True  # metrics.json comm_ms (events around the collectives)
    comm_ms, comm_calls = [], []
    running, history, elapsed = [], [], []
    batch = next(data)
    t0 = time.perf_counter()
    # Host pipelining: step s+1 is enqueued before step s's loss is read (Engine.loss_handle), so
    # the GPU does not idle on the host between steps.  Every step's loss is still read and
    # logged, and its elapsed time is stamped when that read returns (as the reference's
    # blocking float(loss), train/train.py:82-85).  A step that ends on a checkpoint is drained
    # before the next one is enqueued, so the checkpoint holds exactly that step's state.
    pending = None

    def finish(s, handle):
        nonlocal running
        with tr.span("loss sync"):
            loss = eng.read_loss(handle)
        comm_ms.append(eng.program.take_comm_ms())
        dog.beat(s)
        tr.collect()
        running.append(loss)
        history.append(loss)
        now = time.perf_counter()
        elapsed.append(now - t0)
        if s % train_config.log_every == 0:
            say(f"Step: {s} | Avg loss: {np.mean(running):.4f} | Average step time: {(now - t0) / s:.4f}")
            running = []

    for step in range(1, train_config.steps + 1):
        eng.set_batch(batch)
        with tr.device_step(step):
            eng.run_step()
        comm_calls.append(eng.program.step_comms)
        handle = eng.loss_handle()
        if step < train_config.steps:
            with tr.span("data"):
                batch = next(data)  # host data for the next step overlaps this step's GPU work
        if pending is not None:
            finish(*pending)
        pending = (step, handle)
        gstep = start + train_config.warmup_steps + step
        if train_config.ckpt_every and gstep % train_config.ckpt_every == 0:
            finish(*pending)
            pending = None
            with tr.span("checkpoint"):
                maybe_save(eng, train_config, gstep)
    if pending is not None:
        finish(*pending)
    eng.flush_optimizer()  # complete the last step's deferred update (timed)
    t1 = time.perf_counter()
    dog.stop()
    say(f"Total time: {t1 - t0}")
    say("End")
    total = t1 - t0
    result = dict(steps=train_config.steps, total_s=total, avg_step_ms=1e3 * total / max(1, train_config.steps),
                  tokens_per_s=eng.tokens_per_step * train_config.steps / max(total, 1e-9),
                  last_loss=history[-1] if history else float("nan"),
                  mean_last50=float(np.mean(history[-50:])) if history else float("nan"),
                  mesh=dict(dp=eng.mesh.dp, tp=eng.mesh.tp, pp=eng.mesh.pp),
                  model=model_config.name, global_batch=eng.global_batch, seq_len=eng.T,
                  dtype=str(eng.act_dtype).replace("torch.", ""), n_graphs=eng.program.n_graphs,
                  n_comms=eng.program.n_comms,
                  # collective calls issued per step (graph replay or eager) and their exposed time
                  comm_calls_per_step=int(np.max(comm_calls)) if comm_calls else 0,
                  comm_ms_mean=float(np.mean(comm_ms)) if comm_ms else 0.0,
                  # model FLOPs (fwd+bwd matmuls + attention, ModelConfig.flops_per_token) / step time
                  tflops=model_config.flops_per_token() * eng.tokens_per_step * train_config.steps / max(total, 1e-9) / 1e12,
                  world_size=dinfo.world)
    result["tflops_per_gpu"] = result["tflops"] / max(1, dinfo.world)
    if tr.enabled:
        path = tr.write()
        n_warm = train_config.warmup_steps
        dev = tr.device_ms[n_warm:] if len(tr.device_ms) > n_warm else tr.device_ms
        result.update(device_step_ms=dev, device_step_ms_mean=float(np.mean(dev)) if dev else None, trace=path)
    if is_main and write_csv:
        os.makedirs(train_config.output_dir, exist_ok=True)
        _write_csv(os.path.join(train_config.output_dir, "log.csv"), elapsed, history)
        with open(os.path.join(train_config.output_dir, "metrics.json"), "w") as f:
            json.dump(result, f, indent=2)
    result["history"] = history
    result["engine"] = eng
    return result


def _write_csv(path: str, elapsed, losses):
    with open(path, "w") as f:
        f.write("step,elapsed_time,loss\n")
        for i, (e, l) in enumerate(zip(elapsed, losses)):
            f.write(f"{i},{e},{l}\n")


_ = Optional, torch
