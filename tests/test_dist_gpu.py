"""Multi-rank GPU code paths on ONE GPU: 2-4 processes share cuda:0 over gloo (RCCL refuses two
ranks on one device).  Exercises the real GPU step programs — hipGraph segments cut at every
collective, bucketed DP all-reduce, TP all-reduces/all-gather (RCCL path and the IPC P2P kernels),
PP send/recv programs (host-staged) — and compares the loss curve AND the final parameters
(reassembled from shards / stages) with a single-process GPU run of the same global batch."""

import os
import tempfile

import pytest
import torch

from distributed_training_compare_jax_amd.parallel.dist import spawn

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
STEPS = 6


def _worker(parallel, kw, out_dir):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    kw = dict(kw)
    if "ce_fused" in kw:  # read when models.gpt is first imported (a fresh spawned rank)
        os.environ["DTC_CE_FUSED"] = kw.pop("ce_fused")
    from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed
    from distributed_training_compare_jax_amd.train.loop import train

    kw = dict(kw)
    mc = _model_cfg(kw.pop("model", None))
    tc = TrainConfig(seed=0, parallel=parallel, batch=kw.pop("batch", 4), steps=STEPS, log_every=1000, output_dir="/tmp/unused",
                     device="cuda", warmup_steps=2, **kw)
    oc = OptimConfig(lr=3e-3, weight_decay=0.1, grad_clip=1.0)
    d = init_distributed("cuda")
    r = train(tc, mc, oc, d, quiet=True, write_csv=False)
    eng = r["engine"]
    torch.save({"losses": r["history"], "graphs": r["n_graphs"], "comms": r["n_comms"], "sp": eng.stage.sp, "head_part": eng.stage.layout.head_part,
                "head_staged": eng.stage.head_dgrad_staged,
                "params": eng.flat.params.cpu(),
                "named": {n: eng.flat.p(n).detach().float().cpu().clone() for n in eng.flat.slots},
                "tp_idx": eng.mesh.tp_idx, "dp_idx": eng.mesh.dp_idx},
               os.path.join(out_dir, f"rank{d.rank}.pt"))
    destroy()


def _model_cfg(model=None):
    from distributed_training_compare_jax_amd.config.schema import model_config_from_preset

    return model_config_from_preset("tiny", vocab_size=1000, **dict({"n_layers": 4}, **(model or {})))


def _full_params(results, model=None):
    """Reassemble the full model from TP shards / PP stages (DP replica 0)."""
    from distributed_training_compare_jax_amd.models.params import all_param_specs, unshard

    specs = {s.name: s for s in all_param_specs(_model_cfg(model))}
    pieces = {}
    for r in results:
        if r["dp_idx"] != 0:
            continue
        for n, t in r["named"].items():
            # lm_head of a head split over two pipeline stages: (vocab part, tp shard)
            part = r.get("head_part", (0, 1))[0] if n.startswith("lm_head") else 0
            pieces.setdefault(n, {})[(part, r["tp_idx"])] = t
    out = {}
    for n, p in pieces.items():
        parts = sorted({k[0] for k in p})
        out[n] = torch.cat([unshard(specs[n], [p[k] for k in sorted(p) if k[0] == v]) for v in parts], 0)
    return out


@pytest.fixture(scope="module")
def init_params(cuda):
    """The canonical initial parameters (the same full model under every layout)."""
    from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig
    from distributed_training_compare_jax_amd.parallel.dist import DistInfo
    from distributed_training_compare_jax_amd.train.engine import Engine

    tc = TrainConfig(seed=0, parallel="dp", batch=4, steps=1, log_every=1000, output_dir="/tmp/unused", device="cuda")
    eng = Engine(_model_cfg(), tc, OptimConfig(lr=3e-3, weight_decay=0.1, grad_clip=1.0), DistInfo(0, 1, 0, cuda, "nccl"))
    out = {n: eng.flat.p(n).detach().float().cpu().clone() for n in eng.flat.slots}
    del eng
    return out


def _run(parallel, world, **kw):
    with tempfile.TemporaryDirectory() as td:
        if world == 1:
            for k in ("WORLD_SIZE", "RANK"):
                os.environ.pop(k, None)
            _worker(parallel, kw, td)
        else:
            spawn(_worker, world, args=(parallel, kw, td))
        return [torch.load(os.path.join(td, f"rank{r}.pt")) for r in range(world)]


@pytest.fixture(scope="module")
def single(cuda):
    return _run("dp", 1)


@pytest.mark.parametrize("parallel,world,kw", [
    ("dp", 2, {}),
    ("dp", 2, {"dp_embed_gather": False}),
    ("dp", 2, {"zero_stage": 1}),
    ("dp", 2, {"dp_grad_dtype": "bf16"}),  # bf16 bucket payload + bf16 embedding-gradient gather
    ("tp", 2, {"tp_sequence_parallel": False, "tp_comm_dtype": "fp32"}),  # the RCCL (here gloo) all-reduce path
    ("tp", 2, {"tp_comm": "p2p", "tp_sequence_parallel": False}),
    ("pp", 2, {"pp_microbatches": 2, "pp_clip": "global"}),
    ("pp", 2, {"pp_microbatches": 2, "pp_clip": "global", "pp_schedule": "1f1b"}),
    ("pp", 4, {"pp_microbatches": 4, "pp_clip": "global", "pp_schedule": "1f1b"}),
    ("pp", 4, {"pp_microbatches": 4, "pp_clip": "global", "pp_schedule": "zb"}),  # B/W split, W in the bubbles
    # lm_head + CE vocab-split over the last two stages (row-statistics exchange, partial dgrad message)
    ("pp", 4, {"pp_microbatches": 4, "pp_clip": "global", "pp_schedule": "zb", "pp_head_split": True}),
    ("dp", 4, {"tp": 2, "tp_comm": "p2p"}),
    ("tp", 2, {"tp_comm": "p2p", "tp_sequence_parallel": True, "tp_comm_dtype": "fp32"}),  # RS / AG P2P kernels
    ("tp", 2, {"tp_comm": "p2p", "tp_sequence_parallel": True, "tp_comm_dtype": "bf16"}),
])
def test_two_ranks_match_single_gpu(single, init_params, parallel, world, kw):
    res = _run(parallel, world, **kw)
    assert "tp_sequence_parallel" not in kw or all(r["sp"] == kw["tp_sequence_parallel"] for r in res)
    ref = single[0]["losses"]
    got = res[0]["losses"]
    assert got == pytest.approx(ref, rel=2e-2, abs=2e-2), (parallel, got, ref)
    # final parameters: the 6 updates (p - p0) of every tensor point the same way as the single-GPU
    # run's (bf16 compute: reduction order and rounding differ, the optimizer trajectory must not)
    full, one = _full_params(res), _full_params(single)
    assert set(full) == set(one)
    for n in one:
        a, b, p0 = full[n], one[n], init_params[n]
        if n.endswith("qkv.b"):  # key bias: analytically zero gradient, Adam normalises its noise
            a, b, p0 = (x.view(3, -1)[[0, 2]] for x in (a, b, p0))
        da, db = a - p0, b - p0
        err = ((da - db).norm() / (db.norm() + 1e-12)).item()
        assert err < 0.15, f"{parallel} {kw} {n}: update differs from the single-GPU run by {err:.3f} (relative)"
    if parallel == "tp" and kw.get("tp_comm") == "p2p":
        # every TP collective (activation all-reduces, CE row-stat gather, label logits, grad-norm
        # partial) is an in-graph P2P kernel: the whole step is ONE hipGraph, no RCCL call
        assert res[0]["graphs"] == 1 and res[0]["comms"] == 0, (res[0]["graphs"], res[0]["comms"])
    else:
        assert res[0]["graphs"] >= 2  # step was captured and cut at the collectives
    if parallel == "dp" and "tp" not in kw:  # replicas stay bit-identical (deterministic local embedding grads)
        assert torch.equal(res[0]["params"], res[1]["params"])


# GPT-2 small's 12 heads (head_dim 32 here, a size the attention kernels take) on 8 TP ranks: whole
# heads 2,2,2,2,1,1,1,1 (models/params.py head_split) -- BASELINE.json config 3's layout
HEADS12 = {"d_model": 384, "n_heads": 12, "d_ff": 512, "n_layers": 2}


@pytest.mark.parametrize("world,kw", [
    (8, {"parallel": "tp", "tp_comm": "p2p", "tp_comm_dtype": "fp32"}),
    (4, {"parallel": "dp", "tp": 2, "tp_comm": "p2p"}),  # dp2 x tp2 at the box's default HW queue count (SP auto)
    (2, {"parallel": "tp", "tp_comm": "p2p", "tp_comm_dtype": "bf16", "tp_sequence_parallel": False}),  # bf16 AR
    (4, {"parallel": "tp", "tp_comm": "p2p", "tp_comm_dtype": "bf16", "tp_sequence_parallel": False}),  # two-shot, W 4
    # sequence parallel at TP=8: one sequence of the residual stream per rank, bf16 partials
    # (unfused CE backward: the lm_head input-gradient partial goes out as bf16, as at GPT-2 small size)
    (8, {"parallel": "tp", "tp_comm": "p2p", "tp_comm_dtype": "bf16", "tp_sequence_parallel": True, "batch": 8,
         "ce_fused": "0"}),
])
def test_uneven_heads_and_hybrid_one_gpu(world, kw):
    """TP=8 with 12 heads and dp2 x tp2, 8 / 4 processes on one GPU through the P2P all-reduce kernels,
    against a single-process GPU run of the same model (losses + parameter updates, bf16 tolerances)."""
    kw = dict(kw)
    parallel = kw.pop("parallel")
    single = _run("dp", 1, model=HEADS12, batch=kw.get("batch", 4))
    res = _run(parallel, world, model=HEADS12, **kw)
    assert res[0]["losses"] == pytest.approx(single[0]["losses"], rel=2e-2, abs=2e-2)
    if kw.get("tp_comm_dtype") == "bf16" and kw.get("tp_sequence_parallel"):
        # the lm_head input-gradient shard sum travelled as a bf16 partial (GPTStage._head_dgrad; the
        # non-SP layouts here are small enough for the fused CE + dgrad kernel, whose fp32 output is summed)
        assert all(r["head_staged"] > 0 for r in res), [r["head_staged"] for r in res]
    from distributed_training_compare_jax_amd.models.params import all_param_specs, init_full

    p0 = {sp.name: init_full(sp, 0) for sp in all_param_specs(_model_cfg(HEADS12))}  # canonical init (seed 0)
    full, one = _full_params(res, HEADS12), _full_params(single, HEADS12)
    assert set(full) == set(one)
    for n in one:
        a, b, q = full[n], one[n], p0[n]
        if n.endswith("qkv.b"):
            a, b, q = (x.view(3, -1)[[0, 2]] for x in (a, b, q))
        err = (((a - q) - (b - q)).norm() / ((b - q).norm() + 1e-12)).item()
        assert err < 0.15, f"{n}: update differs from the single-GPU run by {err:.3f} (relative)"


def _p2p_worker(out_dir):
    os.environ["DTC_DIST_BACKEND"] = "gloo"
    import torch.distributed as dist

    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed
    from distributed_training_compare_jax_amd.parallel.p2p import P2PAllReduce

    d = init_distributed("cuda")
    ar = P2PAllReduce(dist.group.WORLD, d.rank, d.world, d.device, 1 << 20)
    res = {}
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(d.world, 4096 * k, generator=g) for k in (1, 3, 64)]
    for k, x in enumerate(xs):  # eager, several sizes (alternating buffer halves)
        t = x[d.rank].to(d.device).clone()
        ar.all_reduce_(t)
        res[f"eager{k}"] = t.cpu()
    ar.end_step()  # 3 calls: padded to an even count (as every engine step ends)
    # captured in a hipGraph and replayed: the device epoch counter keeps ranks in step
    t = torch.zeros(4096 * 2, device=d.device)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        gr.capture_begin(capture_error_mode="thread_local")
        ar.all_reduce_(t)
        ar.end_step()
        gr.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    outs = []
    for it in range(3):
        t.copy_(torch.full((4096 * 2,), float(d.rank + 1 + it)))
        dist.barrier()
        gr.replay()
        torch.cuda.synchronize()
        outs.append(t.cpu().clone())
    res["graph"] = outs
    # bf16 payload with the fused residual + bias: forced two-shot (1) and one-shot (2), 3 x 256 rows x 64
    xb = torch.randn(d.world, 3 * 256, 64, generator=g).to(torch.bfloat16)
    rs, bs = torch.randn(3 * 256, 64, generator=g), torch.randn(64, generator=g)
    for mode in (1, 2):
        out = torch.empty(3 * 256, 64, device=d.device)
        ar.all_reduce_bf16(xb[d.rank].to(d.device).contiguous(), out, rs.to(d.device), bs.to(d.device), mode=mode)
        res[f"bf16_{mode}"] = out.cpu()
    # staged payload (tp_comm_dtype: bf16 in the model): a GEMM writes the partial straight into this
    # rank's buffer half of the next call (identity weight here: the partial is x), then the payload-free
    # all-reduce; eager once, then captured with end_step's padding and replayed with new inputs
    from distributed_training_compare_jax_amd.ops.gemm import linear_into

    eye = torch.eye(64, dtype=torch.bfloat16, device=d.device)
    xin = torch.empty(3 * 256, 64, dtype=torch.bfloat16, device=d.device)
    rsd, bsd = rs.to(d.device), bs.to(d.device)
    out = torch.empty(3 * 256, 64, device=d.device)

    def staged():
        linear_into(xin, eye, ar.staged_out(xin.numel()))
        ar.all_reduce_bf16(None, out, rsd, bsd)

    xin.copy_(xb[d.rank])
    staged()
    ar.end_step()
    res["staged_eager"] = out.cpu()
    gr2 = torch.cuda.CUDAGraph()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gr2.capture_begin(capture_error_mode="thread_local")
        staged()
        ar.end_step()
        gr2.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    outs = []
    for it in range(3):
        xin.copy_(xb[d.rank] * float(it + 1))
        dist.barrier()
        gr2.replay()
        torch.cuda.synchronize()
        outs.append(out.cpu().clone())
    res["staged_graph"] = outs
    # sequence-parallel primitives: reduce-scatter of a [W * 128, 64] partial (bf16 / fp32) + own residual
    # rows + bias, and the all-gather of 128 own rows
    g5 = torch.Generator().manual_seed(5)
    parts = torch.randn(d.world, d.world * 128, 64, generator=g5)
    resid = torch.randn(d.world * 128, 64, generator=g5)
    bias = torch.randn(64, generator=g5)
    for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        out = torch.empty(128, 64, device=d.device)
        ar.reduce_scatter(parts[d.rank].to(dt).to(d.device), d.world * 128, 64, dt, out,
                          resid[d.rank * 128:(d.rank + 1) * 128].to(d.device), bias.to(d.device))
        res[f"rs_{name}"] = out.cpu()
    xg = torch.randn(d.world, 128, 64, generator=g5).to(torch.bfloat16)
    og = torch.empty(d.world * 128, 64, dtype=torch.bfloat16, device=d.device)
    ar.all_gather(xg[d.rank].to(d.device), og)
    res["ag"] = og.cpu()
    ar.end_step()
    ar.check()
    torch.save(res, os.path.join(out_dir, f"p2p{d.rank}.pt"))
    ar.close()
    destroy()


def test_p2p_allreduce_two_ranks_one_gpu():
    """IPC-mapped two-shot all-reduce, 2 processes on one GPU: exact sum, identical on both ranks,
    eager and replayed from a captured hipGraph; bf16 payloads (staged copy and written in place by a
    GEMM, with end_step's even-call padding across replays)."""
    world = 2
    with tempfile.TemporaryDirectory() as td:
        spawn(_p2p_worker, world, args=(td,))
        r = [torch.load(os.path.join(td, f"p2p{i}.pt")) for i in range(world)]
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(world, 4096 * k, generator=g) for k in (1, 3, 64)]
    for k, x in enumerate(xs):
        ref = x[0] + x[1]
        assert torch.equal(r[0][f"eager{k}"], r[1][f"eager{k}"])
        assert torch.allclose(r[0][f"eager{k}"], ref, atol=1e-6), k
    for it in range(3):
        exp = float(1 + it) + float(2 + it)
        for i in range(world):
            assert torch.all(r[i]["graph"][it] == exp), (i, it)
    xb = torch.randn(world, 3 * 256, 64, generator=g).to(torch.bfloat16)
    rs, bs = torch.randn(3 * 256, 64, generator=g), torch.randn(64, generator=g)
    exp = rs + bs + xb.float().sum(0)
    for mode in (1, 2):  # fp32 sum of the bf16 payload (two-shot rounds the reduced slice to bf16 once)
        for i in range(world):
            tol = 2e-2 if mode == 1 else 1e-5
            assert torch.allclose(r[i][f"bf16_{mode}"], exp, atol=tol, rtol=tol), (mode, i)
        assert torch.equal(r[0][f"bf16_{mode}"], r[1][f"bf16_{mode}"])
    # staged (one-shot at W = 2): exact fp32 sums of the bf16 partials, eager and every graph replay
    for i in range(world):
        assert torch.allclose(r[i]["staged_eager"], exp, atol=1e-5, rtol=1e-5), i
        for it in range(3):
            e_it = rs + bs + (xb.float() * float(it + 1)).to(torch.bfloat16).float().sum(0)
            assert torch.allclose(r[i]["staged_graph"][it], e_it, atol=1e-4, rtol=1e-5), (i, it)
    g5 = torch.Generator().manual_seed(5)
    parts = torch.randn(world, world * 128, 64, generator=g5)
    resid = torch.randn(world * 128, 64, generator=g5)
    bias = torch.randn(64, generator=g5)
    xg = torch.randn(world, 128, 64, generator=g5).to(torch.bfloat16)
    for i in range(world):
        rows = slice(i * 128, (i + 1) * 128)
        for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
            exp = resid[rows] + bias + parts.to(dt).float().sum(0)[rows]
            assert torch.allclose(r[i][f"rs_{name}"], exp, atol=1e-5, rtol=1e-5), (name, i)
        assert torch.equal(r[i]["ag"], xg.reshape(world * 128, 64)), i


@pytest.mark.parametrize("parallel,world,kw", [
    ("dp", 2, {}),
    ("tp", 2, {"tp_comm": "p2p", "tp_sequence_parallel": False}),
    ("pp", 2, {"pp_microbatches": 2, "pp_clip": "global", "pp_schedule": "1f1b"}),
    ("pp", 2, {"pp_microbatches": 2, "pp_clip": "global", "pp_schedule": "zb"}),
    ("pp", 2, {"pp_microbatches": 2, "pp_clip": "global", "pp_schedule": "1f1b", "pp_head_split": True}),
    ("dp", 4, {"tp": 2, "tp_comm": "p2p"}),
    ("tp", 2, {"tp_comm": "p2p", "tp_sequence_parallel": True}),
])
def test_fp32_layouts_match_single_gpu(parallel, world, kw):
    """The same layouts with the exact-fp32 kernels (dtype fp32: f32-input MFMA GEMMs and attention):
    the multi-rank composition of the HIP kernels (P2P all-reduces, PP send/recv programs, bucketed DP
    all-reduce) pinned at fp32 reduction-order tolerance instead of the bf16 runs' 2e-2 / 15 %."""
    single = _run("dp", 1, dtype="fp32")
    res = _run(parallel, world, dtype="fp32", **kw)
    assert res[0]["losses"] == pytest.approx(single[0]["losses"], rel=1e-4, abs=1e-4), (res[0]["losses"],
                                                                                         single[0]["losses"])
    from distributed_training_compare_jax_amd.models.params import all_param_specs, init_full

    p0 = {sp.name: init_full(sp, 0) for sp in all_param_specs(_model_cfg())}
    full, one = _full_params(res), _full_params(single)
    assert set(full) == set(one)
    for n in one:
        a, b, q = full[n], one[n], p0[n]
        if n.endswith("qkv.b"):
            a, b, q = (x.view(3, -1)[[0, 2]] for x in (a, b, q))
        err = (((a - q) - (b - q)).norm() / ((b - q).norm() + 1e-12)).item()
        assert err < 1e-3, f"{parallel} {kw} {n}: fp32 update differs from the single-GPU run by {err:.2e}"
