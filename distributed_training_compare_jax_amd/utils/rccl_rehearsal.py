"""One-GPU RCCL rehearsal of the data-parallel step's collective sequence.

The pool's GPU boxes have one MI355X, and RCCL refuses two ranks on one device, so the multi-rank GPU
tests run over gloo (``tests/test_dist_gpu.py``).  This module closes the remaining gap: it creates a
ONE-rank RCCL communicator (``DTC_WORLD1_PG=1``) and runs the engine with
``TrainConfig.dp_comm_rehearsal``, i.e. the DP code path of a dp > 1 run -- the same graph segments,
the same comm-safe GEMM plans, the same calls in the same order:

* bucketed async ``all_reduce`` of the flat fp32 grads (``parallel/dp.py``), issued between hipGraph
  segments while the next backward segment replays;
* ``all_gather_into_tensor`` of the embedding-output grads (the DP embedding gather);
* the bf16 payload chain ``all_to_all_single`` → fp32 shard sum → ``all_gather_into_tensor``
  (``dp_grad_dtype: bf16``);
* ZeRO-1's ``reduce_scatter_tensor`` / ``all_gather_into_tensor`` (``zero_stage: 1``);
* the async loss ``all_reduce``;

plus, standalone, ``batch_isend_irecv`` to self (the PP transport of ``parallel/pp.py``).  On a
one-member group every collective is an identity, so each configuration must reproduce a reference
run BIT FOR BIT: the same rehearsal over gloo (host-staged collectives, identical math) and, for the
collective-free parts, direct checks.  ``capture_comms`` additionally records the whole step --
collectives included -- as one hipGraph (reference analog: every collective inside the one jitted
program, ``train/create_train_step.py:28-50``).

    DTC_WORLD1_PG=1 WORLD_SIZE=1 RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=<p> \\
        python -m distributed_training_compare_jax_amd.utils.rccl_rehearsal <out.pt> [case ...]
"""

from __future__ import annotations

import os
import sys

import torch

CASES = {
    # name: TrainConfig overrides (every case: dp1 + dp_comm_rehearsal unless "plain"); the cut-graph cases
    # set capture_comms=False explicitly (the RCCL default captures)
    "plain": dict(dp_comm_rehearsal=False),
    "fp32": dict(capture_comms=False),
    "fp32_captured": dict(capture_comms=True),
    "no_gather": dict(dp_embed_gather=False, capture_comms=False),
    "bf16": dict(dp_grad_dtype="bf16", capture_comms=False),
    "bf16_captured": dict(dp_grad_dtype="bf16", capture_comms=True),
    "zero1": dict(zero_stage=1, capture_comms=False),
    "zero1_captured": dict(zero_stage=1, capture_comms=True),
    # bench-only variants of the captured fp32 DP path: weight gradients in groups of 4 / 6 layers (default 2)
    "fp32_captured_wg4": dict(capture_comms=True, wgrad_group=4),
    "fp32_captured_wg6": dict(capture_comms=True, wgrad_group=6),
}
STEPS = 5


def _model():
    from ..config.schema import model_config_from_preset

    return model_config_from_preset("tiny", vocab_size=1000, n_layers=4)


def run_case(name: str, dinfo) -> dict:
    from ..config.schema import OptimConfig, TrainConfig
    from ..train.loop import train

    kw = dict(dp_comm_rehearsal=True)
    kw.update(CASES[name])
    tc = TrainConfig(seed=0, parallel="dp", batch=4, steps=STEPS, log_every=1000, output_dir="/tmp/unused",
                     device="cuda", warmup_steps=2, **kw)
    oc = OptimConfig(lr=3e-3, weight_decay=0.1, grad_clip=1.0)
    r = train(tc, _model(), oc, dinfo, quiet=True, write_csv=False)
    eng = r["engine"]
    eng.flush_optimizer()
    torch.cuda.synchronize()
    return {"losses": list(r["history"]), "params": eng.flat.params.detach().cpu().clone(),
            "graphs": eng.program.n_graphs, "comms": eng.program.n_comms, "dp_comm": bool(eng.dp_comm),
            "zero": bool(eng.zero), "embed_gather": bool(eng.embed_gather)}


def bench_case(name: str, dinfo, model: str = "gpt2-small", steps: int = 20, warmup: int = 4, hog_cus: int = 0) -> dict:
    """ms/step of one case on a real model (bench.py's timing: graph replays back to back, one loss
    read per step one step late): ``plain`` vs the rehearsals measures what the DP code path costs at
    dp1 before any communication (comm-safe GEMM plans, grouped weight gradients of 2 layers, the
    embedding gather, the graph cuts) and what capturing the collectives saves.

    ``hog_cus`` > 0: a probe kernel holds that many CUs for the whole timed loop (``dtc_cu_hog`` on a side
    stream; the time is taken with events on the step's stream) -- the CU-steal proxy of a DP step whose
    RCCL kernels occupy CUs while the backward runs: which GEMM plans (one-round / comm-safe) cope better."""
    import time

    from ..config.schema import OptimConfig, TrainConfig, model_config_from_preset
    from ..data.synthetic import get_batch_iterator
    from ..parallel.dist import barrier
    from ..train.engine import Engine

    kw = dict(dp_comm_rehearsal=True)
    kw.update(CASES[name])
    mc = model_config_from_preset(model)
    tc = TrainConfig(seed=0, parallel="dp", batch=8, steps=steps, log_every=10 ** 9, output_dir="/tmp/unused",
                     device="cuda", **kw)
    eng = Engine(mc, tc, OptimConfig(lr=3e-4, weight_decay=0.1, grad_clip=1.0), dinfo)
    data = get_batch_iterator(8, mc.max_seq_len + 1, seed=0, row0=eng.feed_row0, nrows=eng.feed_rows)
    for _ in range(max(warmup, 2)):
        eng.set_batch(next(data))
        eng.run_step()
        eng.loss_value()
    barrier()
    torch.cuda.synchronize()
    hog = None
    if hog_cus > 0:
        from ..ops import _native as N

        hs = torch.cuda.Stream(priority=-1)  # its own hardware queue (a shared one would serialise it)
        sink = torch.zeros(4, dtype=torch.int32, pin_memory=True)  # host-mapped: polled without a stream op
        ticks = int(steps * 0.025 * 1e8)  # 25 ms per step of the 100 MHz clock: outlasts the loop
        with torch.cuda.stream(hs):
            N.check(N.lib().dtc_cu_hog(hog_cus, ticks, 160 * 1024 - 1024, sink.data_ptr(), N.stream_ptr(dinfo.device)),
                    "dtc_cu_hog")
        hog = (hs, sink)
        t_w = time.perf_counter()
        while int(sink[1]) < hog_cus and time.perf_counter() - t_w < 0.2:
            time.sleep(0.0005)
        if int(sink[1]) < hog_cus:
            raise RuntimeError(f"CU probe: only {int(sink[1])} of {hog_cus} workgroups resident")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    t0 = time.perf_counter()
    pending = None
    for _ in range(steps):
        eng.set_batch(next(data))
        eng.run_step()
        h = eng.loss_handle()
        if pending is not None:
            eng.read_loss(pending)
        pending = h
    loss = eng.read_loss(pending)
    ev1.record()
    ev1.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    if hog is not None:
        ms = ev0.elapsed_time(ev1) / steps
        hog[0].synchronize()
    torch.cuda.synchronize()
    out = {"ms_per_step": ms, "graphs": eng.program.n_graphs, "comms": eng.program.n_comms, "loss": loss,
           "hog_cus": hog_cus}
    del eng
    torch.cuda.empty_cache()
    return out


def primitive_checks(dev) -> dict:
    """Every collective primitive the engine uses, on the one-rank group: results must equal the
    inputs exactly (identity reductions), eager and replayed from a captured hipGraph."""
    import torch.distributed as dist

    g = torch.Generator().manual_seed(1)
    x = torch.randn(4096 * 3, generator=g).to(dev)
    out = {}
    t = x.clone()
    dist.all_reduce(t)
    out["all_reduce"] = bool(torch.equal(t, x))
    h = x.clone()
    w = dist.all_reduce(h, async_op=True)
    w.wait()
    out["all_reduce_async"] = bool(torch.equal(h, x))
    o = torch.empty_like(x)
    dist.all_gather_into_tensor(o, x)
    out["all_gather_into_tensor"] = bool(torch.equal(o, x))
    o2 = torch.empty_like(x)
    dist.reduce_scatter_tensor(o2, x)
    out["reduce_scatter_tensor"] = bool(torch.equal(o2, x))
    xb = x.to(torch.bfloat16)
    ob = torch.empty_like(xb)
    dist.all_to_all_single(ob, xb)
    out["all_to_all_single_bf16"] = bool(torch.equal(ob, xb))
    r = torch.empty_like(x)
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, r, 0)])
    for q in reqs:
        q.wait()
    out["batch_isend_irecv_self"] = bool(torch.equal(r, x))
    # captured: an all-reduce + all-gather inside one graph, replayed on new inputs
    src = torch.zeros_like(x)
    dst = torch.empty_like(x)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        gr.capture_begin()
        dist.all_reduce(src)
        dist.all_gather_into_tensor(dst, src)
        gr.capture_end()
    torch.cuda.current_stream(dev).wait_stream(s)
    ok = True
    for k in range(3):
        src.copy_(x * float(k + 1))
        gr.replay()
        torch.cuda.synchronize(dev)
        ok = ok and bool(torch.equal(dst, x * float(k + 1)))
    out["captured_replay"] = ok
    return out


def main(argv):
    from ..parallel.dist import destroy, init_distributed

    bench = argv[0] == "--bench"
    if bench:
        argv = argv[1:]
    hogs = [0]
    if argv and argv[0].startswith("--hog="):  # CU-steal proxy: --hog=0,16,32
        hogs = [int(x) for x in argv[0].split("=", 1)[1].split(",")]
        argv = argv[1:]
    path = argv[0]
    cases = argv[1:] or list(CASES)
    d = init_distributed("cuda", single_rank_pg=True)
    import torch.distributed as dist

    res = {"backend": dist.get_backend(), "cases": {}}
    if dist.get_backend() == "nccl":
        res["primitives"] = primitive_checks(d.device)
        try:
            res["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:
            res["rccl_version"] = None
    if bench:
        res["bench"] = {}
        for rnd in range(2):  # interleaved rounds (box clock drift)
            for c in cases:
                for hc in hogs:
                    # suffixes: _unsafe = comm-safe plans off; _nor8 = comm-safe plans with gemm8r off too (the
                    # round-5 scope, DTC_COMM_SAFE_R8=0); none = the engine's defaults
                    safe = not c.endswith("_unsafe")
                    os.environ["DTC_COMM_SAFE_GEMMS"] = "1" if safe else "0"
                    if c.endswith("_nor8"):
                        os.environ["DTC_COMM_SAFE_R8"] = "0"
                    else:
                        os.environ.pop("DTC_COMM_SAFE_R8", None)
                    r = bench_case(c.replace("_unsafe", "").replace("_nor8", ""), d, hog_cus=hc)
                    res["bench"].setdefault(f"{c} hog{hc}", []).append(r)
                    print(f"[bench] round {rnd} {c} hog {hc} CUs: {r['ms_per_step']:.3f} ms/step ({r['graphs']} graph "
                          f"segments, {r['comms']} eager collectives)", flush=True)
            os.environ["DTC_COMM_SAFE_GEMMS"] = "1"
            os.environ.pop("DTC_COMM_SAFE_R8", None)
        torch.save(res, path)
        destroy()
        return
    for c in cases:
        res["cases"][c] = run_case(c, d)
        print(f"[rehearsal] {c}: {res['cases'][c]['graphs']} graph segments, {res['cases'][c]['comms']} eager "
              f"collectives, last loss {res['cases'][c]['losses'][-1]:.5f}", flush=True)
    torch.save(res, path)
    destroy()


if __name__ == "__main__":
    main(sys.argv[1:])
