"""Checkpoint / resume / re-shard (the reference has none; SURVEY §5 plan)."""

import os
import tempfile

import pytest
import torch

from distributed_training_compare_jax_amd.config.schema import OptimConfig, TrainConfig, model_config_from_preset
from distributed_training_compare_jax_amd.parallel.dist import DistInfo, spawn
from distributed_training_compare_jax_amd.train.loop import train
from distributed_training_compare_jax_amd.utils import checkpoint as C

MC = model_config_from_preset("tiny", vocab_size=1000)
OC = OptimConfig(lr=3e-3, weight_decay=0.1, grad_clip=1.0)
CPU = DistInfo(0, 1, 0, torch.device("cpu"), "gloo")


def _tc(out, steps, **kw):
    return TrainConfig(seed=0, parallel="dp", batch=4, steps=steps, log_every=1000, output_dir=out, device="cpu",
                       warmup_steps=0, **kw)


def test_resume_reproduces_uninterrupted_run(tmp_path):
    full = train(_tc(str(tmp_path / "a"), 6), MC, OC, CPU, quiet=True)["history"]
    part1 = train(_tc(str(tmp_path / "b"), 3, ckpt_every=3), MC, OC, CPU, quiet=True)["history"]
    assert C.latest_step(str(tmp_path / "b")) == 3
    part2 = train(_tc(str(tmp_path / "b"), 3, resume=True), MC, OC, CPU, quiet=True)["history"]
    assert part1 + part2 == pytest.approx(full, rel=1e-6, abs=1e-6)


def _tp_worker(out, parallel="tp", kw=None):
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed

    d = init_distributed("cpu")
    train(TrainConfig(seed=0, parallel=parallel, batch=4, steps=2, log_every=1000, output_dir=out, device="cpu",
                      warmup_steps=0, ckpt_every=2, **(kw or {})), MC, OC, d, quiet=True)
    destroy()


@pytest.mark.slow
@pytest.mark.parametrize("parallel,kw", [
    ("tp", {}),
    # lm_head vocab-split over the two pipeline stages: consolidate joins the halves
    ("pp", {"pp_microbatches": 2, "pp_clip": "global", "pp_schedule": "1f1b", "pp_head_split": True}),
])
def test_consolidate_tp_checkpoint_equals_single_process(tmp_path, parallel, kw):
    out_tp = str(tmp_path / "tp")
    spawn(_tp_worker, 2, args=(out_tp, parallel, kw))
    full = C.consolidate(out_tp, 2)
    # vocab-indexed tensors come back at the canonical vocab whatever the writer's TP padding
    assert full["lm_head.w"].shape[0] == MC.vocab_size and full["lm_head.b"].shape[0] == MC.vocab_size
    assert C.pad_vocab(full, MC.padded_vocab)["lm_head.w"].shape[0] == MC.padded_vocab
    r = train(_tc(str(tmp_path / "dp"), 2), MC, OC, CPU, quiet=True)
    eng = r["engine"]
    for n in eng.flat.slots:
        a, b = full[n], eng.flat.p(n)[: full[n].shape[0]]
        if n.endswith("qkv.b"):  # zero-gradient key bias: Adam amplifies rounding noise (see parallel tests)
            a, b = a.view(3, -1)[[0, 2]], b.view(3, -1)[[0, 2]]
        # Adam's first steps turn near-zero gradients into +-lr updates, so compare in norm
        assert ((a - b).norm() / b.norm()).item() < 2e-3, n


def _zero_worker(out, steps, ckpt_every, resume, res_dir):
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed

    torch.set_num_threads(1)
    d = init_distributed("cpu")
    r = train(TrainConfig(seed=0, parallel="dp", batch=4, steps=steps, log_every=1000, output_dir=out, device="cpu",
                          warmup_steps=0, ckpt_every=ckpt_every, resume=resume, zero_stage=1), MC, OC, d, quiet=True)
    eng = r["engine"]
    # ZeRO-1: each rank holds its shard of the Adam state, not the whole buffer
    assert eng.flat.exp_avg.numel() < eng.flat.numel
    if d.rank == 0:
        torch.save(r["history"], os.path.join(res_dir, "hist.pt"))
    destroy()


@pytest.mark.slow
def test_zero1_resume_reproduces_uninterrupted_run(tmp_path):
    def run(out, steps, ckpt_every=0, resume=False):
        spawn(_zero_worker, 2, args=(str(tmp_path / out), steps, ckpt_every, resume, str(tmp_path)))
        return torch.load(str(tmp_path / "hist.pt"))

    full = run("a", 6)
    part1 = run("b", 3, ckpt_every=3)
    part2 = run("b", 3, resume=True)
    assert part1 + part2 == pytest.approx(full, rel=1e-6, abs=1e-6)


def _edit_meta(out, step, **kw):
    import json

    d = os.path.join(out, "ckpt", f"step_{step}")
    for x in os.listdir(d):
        if x.startswith("meta_rank"):
            p = os.path.join(d, x)
            m = json.load(open(p))
            m.update(kw)
            json.dump(m, open(p, "w"))


@pytest.mark.parametrize("edit,msg", [(dict(zero_stage=1, dp=2), "zero_stage"), (dict(tp=2), "tp=2"),
                                      (dict(model="gpt2-medium"), "model"),
                                      # same element count, different layer range (a changed PP split)
                                      (dict(layers=[1, 3]), "layer split"),
                                      (dict(slots={}), "partition map")])
def test_resume_layout_mismatch_fails_before_touching_buffers(tmp_path, edit, msg):
    out = str(tmp_path / "c")
    train(_tc(out, 2, ckpt_every=2), MC, OC, CPU, quiet=True)
    _edit_meta(out, 2, **edit)
    eng = train(_tc(str(tmp_path / "fresh"), 0), MC, OC, CPU, quiet=True)["engine"]
    before = eng.flat.params.clone()
    with pytest.raises(ValueError, match=msg):
        C.load_into(eng, out, 2)
    assert torch.equal(eng.flat.params, before)


def test_resume_missing_checkpoint_is_a_clear_error(tmp_path):
    eng = train(_tc(str(tmp_path / "fresh"), 0), MC, OC, CPU, quiet=True)["engine"]
    with pytest.raises(FileNotFoundError, match="no checkpoint"):
        C.load_into(eng, str(tmp_path / "nothing"), 5)


def test_zero_stage_validation():
    from distributed_training_compare_jax_amd.train.engine import Engine

    with pytest.raises(ValueError, match="zero_stage=2"):
        Engine(MC, _tc("/tmp/unused", 1, zero_stage=2), OC, CPU)
    with pytest.warns(UserWarning, match="dp == 1"):
        Engine(MC, _tc("/tmp/unused", 1, zero_stage=1), OC, CPU)


def _dp_resume_worker(out, res_dir):
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed

    torch.set_num_threads(1)
    d = init_distributed("cpu")
    r = train(TrainConfig(seed=0, parallel="dp", batch=4, steps=3, log_every=1000, output_dir=out, device="cpu",
                          warmup_steps=0, resume=True), MC, OC, d, quiet=True)
    if d.rank == 0:
        torch.save(r["history"], os.path.join(res_dir, "hist_dp2.pt"))
    destroy()


@pytest.mark.slow
def test_replicated_checkpoint_resumes_at_larger_dp(tmp_path):
    """dp1 checkpoint -> dp2 resume: rank 1 has no file of its own and reads the dp_idx 0 replica."""
    full = train(_tc(str(tmp_path / "a"), 6), MC, OC, CPU, quiet=True)["history"]
    out = str(tmp_path / "b")
    train(_tc(out, 3, ckpt_every=3), MC, OC, CPU, quiet=True)
    spawn(_dp_resume_worker, 2, args=(out, str(tmp_path)))
    part2 = torch.load(str(tmp_path / "hist_dp2.pt"))
    assert part2 == pytest.approx(full[3:], rel=1e-4, abs=1e-4)


def _corrupt_worker(out, res_dir):
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed

    torch.set_num_threads(1)
    d = init_distributed("cpu")
    eng = train(TrainConfig(seed=0, parallel="dp", batch=4, steps=0, log_every=1000, output_dir=out + "_fresh",
                            device="cpu", warmup_steps=0, zero_stage=1), MC, OC, d, quiet=True)["engine"]
    try:
        C.load_into(eng, out, 2)
        msg = "loaded"
    except Exception as e:  # noqa: BLE001
        msg = f"{type(e).__name__}: {e}"
    with open(os.path.join(res_dir, f"r{d.rank}.txt"), "w") as fh:
        fh.write(msg)
    destroy()


def _ckpt_worker(out):
    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed

    torch.set_num_threads(1)
    d = init_distributed("cpu")
    train(TrainConfig(seed=0, parallel="dp", batch=4, steps=2, log_every=1000, output_dir=out, device="cpu",
                      warmup_steps=0, ckpt_every=2, zero_stage=1), MC, OC, d, quiet=True)
    destroy()


@pytest.mark.slow
def test_truncated_rank_file_fails_on_every_rank(tmp_path):
    """One rank's file is a truncated zip (torch.load raises a RuntimeError, not a ValueError): that rank must
    still reach the failure agreement, so both ranks raise instead of one blocking in the all-reduce."""
    out = str(tmp_path / "z")
    spawn(_ckpt_worker, 2, args=(out,))
    p = os.path.join(out, "ckpt", "step_2", "rank1.pt")
    data = open(p, "rb").read()
    with open(p, "wb") as fh:
        fh.write(data[: len(data) // 3])
    spawn(_corrupt_worker, 2, args=(out, str(tmp_path)))
    r0 = open(tmp_path / "r0.txt").read()
    r1 = open(tmp_path / "r1.txt").read()
    assert "another rank" in r0, r0
    assert r1 != "loaded" and "another rank" not in r1, r1
