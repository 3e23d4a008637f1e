"""Checkpoint / resume (absent in the reference: params are discarded at exit,
``train/train.py:98-102``; SURVEY §5 plan).

Layout: ``<output_dir>/ckpt/step_<N>/rank<r>.pt`` (flat fp32 params, Adam m and v, the
device step counter) + ``meta.json`` (mesh, per-rank partition map: every parameter's
name, flat offset, local shape and TP rule).  The partition map lets
:func:`consolidate` rebuild the full unsharded model from any DP/TP/PP layout, so a run
can be converted between strategies.  Files are loaded with ``weights_only=True``.
"""

from __future__ import annotations

import json
import os
from typing import Dict

import torch

from ..models.params import unshard


def _dir(output_dir: str, step: int) -> str:
    return os.path.join(output_dir, "ckpt", f"step_{step}")


def save(eng, output_dir: str, step: int):
    if hasattr(eng, "flush_optimizer"):
        eng.flush_optimizer()  # a deferred AdamW must land before params are read
    d = _dir(output_dir, step)
    os.makedirs(d, exist_ok=True)
    f = eng.flat
    m = eng.mesh
    torch.save({"params": f.params.cpu(), "exp_avg": f.exp_avg.cpu(), "exp_avg_sq": f.exp_avg_sq.cpu(),
                "step_t": eng.opt.step_t.cpu(), "step": step}, os.path.join(d, f"rank{m.rank}.pt"))
    slots = {n: dict(offset=s.offset, shape=list(s.shape), tp=s.spec.tp, full=list(s.spec.shape))
             for n, s in f.slots.items()}
    meta = dict(step=step, dp=m.dp, tp=m.tp, pp=m.pp, rank=m.rank, dp_idx=m.dp_idx, tp_idx=m.tp_idx,
                pp_idx=m.pp_idx, slots=slots, model=eng.mcfg.name,
                zero_stage=int(getattr(eng, "zero", False)))
    with open(os.path.join(d, f"meta_rank{m.rank}.json"), "w") as fh:
        json.dump(meta, fh)


def _read_metas(d: str) -> Dict[int, dict]:
    if not os.path.isdir(d):
        raise FileNotFoundError(f"no checkpoint directory {d}")
    metas = {}
    for x in sorted(os.listdir(d)):
        if x.startswith("meta_rank") and x.endswith(".json"):
            with open(os.path.join(d, x)) as fh:
                m = json.load(fh)
            metas[int(m["rank"])] = m
    if not metas:
        raise FileNotFoundError(f"checkpoint {d} has no meta_rank*.json")
    return metas


def source_rank(eng, metas: Dict[int, dict]) -> int:
    """The checkpoint rank file this rank resumes from, after checking the layouts are compatible.

    Every check runs on the metadata alone, before any buffer is touched.  TP/PP degrees and
    ``zero_stage`` must match (flat buffers are laid out per TP/PP shard; ZeRO-1 Adam state per DP
    rank).  Without ZeRO the DP replicas hold identical state, so the DP degree may change: a rank
    whose own (dp, tp, pp) index has no file reads the dp_idx 0 replica of its shard."""
    mesh = eng.mesh
    m0 = metas[min(metas)]
    zero_now = int(bool(getattr(eng, "zero", False)))
    zero_ck = int(m0.get("zero_stage", 0))
    if m0.get("model") not in (None, eng.mcfg.name):
        raise ValueError(f"checkpoint is of model {m0.get('model')!r}, this run trains {eng.mcfg.name!r}")
    if (m0["tp"], m0["pp"]) != (mesh.tp, mesh.pp):
        raise ValueError(f"checkpoint layout tp={m0['tp']} pp={m0['pp']} differs from this run's tp={mesh.tp} "
                         f"pp={mesh.pp}: resume needs the same TP/PP split (use consolidate() to re-shard)")
    if zero_ck != zero_now:
        raise ValueError(f"checkpoint zero_stage={zero_ck} (dp={m0['dp']}) but this run has zero_stage={zero_now} "
                         f"(dp={mesh.dp}): Adam state is stored per layout")
    if zero_now and m0["dp"] != mesh.dp:
        raise ValueError(f"zero_stage=1 checkpoint was written at dp={m0['dp']}, this run has dp={mesh.dp}: "
                         "each rank's Adam shard resumes only at the same dp")
    want = (mesh.dp_idx, mesh.tp_idx, mesh.pp_idx)
    for r, m in metas.items():
        if (m["dp_idx"], m["tp_idx"], m["pp_idx"]) == want:
            return r
    if not zero_now:
        for r, m in metas.items():
            if (m["dp_idx"], m["tp_idx"], m["pp_idx"]) == (0, mesh.tp_idx, mesh.pp_idx):
                return r
    raise ValueError(f"checkpoint (world {len(metas)}) has no rank file for dp/tp/pp index {want}")


def load_into(eng, output_dir: str, step: int):
    d = _dir(output_dir, step)
    src = source_rank(eng, _read_metas(d))
    st = torch.load(os.path.join(d, f"rank{src}.pt"), map_location="cpu", weights_only=True)
    f = eng.flat
    for k, have in (("params", f.params), ("exp_avg", f.exp_avg), ("exp_avg_sq", f.exp_avg_sq)):
        if st[k].shape != have.shape:
            raise ValueError(f"checkpoint {k} has {st[k].numel()} elements, this rank holds {have.numel()}")
    f.params.copy_(st["params"].to(f.device))
    f.exp_avg.copy_(st["exp_avg"].to(f.device))
    f.exp_avg_sq.copy_(st["exp_avg_sq"].to(f.device))
    eng.opt.step_t.copy_(st["step_t"].to(f.device))
    f.refresh_mirror()
    return int(st["step"])


def latest_step(output_dir: str) -> int:
    root = os.path.join(output_dir, "ckpt")
    if not os.path.isdir(root):
        return 0
    steps = [int(x.split("_")[1]) for x in os.listdir(root) if x.startswith("step_")]
    return max(steps) if steps else 0


def maybe_resume(eng, tcfg) -> int:
    if not tcfg.resume:
        return 0
    s = latest_step(tcfg.output_dir)
    return load_into(eng, tcfg.output_dir, s) if s else 0


def maybe_save(eng, tcfg, step: int):
    if tcfg.ckpt_every and step % tcfg.ckpt_every == 0:
        save(eng, tcfg.output_dir, step)


def consolidate(output_dir: str, step: int) -> Dict[str, torch.Tensor]:
    """Full (unsharded) fp32 parameters from every rank file of a checkpoint."""
    from ..models.params import ParamSpec

    d = _dir(output_dir, step)
    metas = [json.load(open(os.path.join(d, x))) for x in sorted(os.listdir(d)) if x.startswith("meta_rank")]
    pieces: Dict[str, Dict[int, torch.Tensor]] = {}
    tp_rule: Dict[str, str] = {}
    full_shape: Dict[str, tuple] = {}
    for meta in metas:
        if meta["dp_idx"] != 0:
            continue
        st = torch.load(os.path.join(d, f"rank{meta['rank']}.pt"), map_location="cpu", weights_only=True)
        for n, s in meta["slots"].items():
            numel = 1
            for x in s["shape"]:
                numel *= x
            t = st["params"][s["offset"]: s["offset"] + numel].view(s["shape"]).clone()
            pieces.setdefault(n, {})[meta["tp_idx"]] = t
            tp_rule[n] = s["tp"]
            full_shape[n] = tuple(s["full"])
    out = {}
    for n, parts in pieces.items():
        spec = ParamSpec(n, full_shape[n], "zeros", 1, tp_rule[n], 0, False)
        out[n] = unshard(spec, [parts[k] for k in sorted(parts)])
    return out
