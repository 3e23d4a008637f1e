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


def load_into(eng, output_dir: str, step: int):
    d = _dir(output_dir, step)
    st = torch.load(os.path.join(d, f"rank{eng.mesh.rank}.pt"), map_location="cpu", weights_only=True)
    f = eng.flat
    f.params.copy_(st["params"].to(f.device))
    if st["exp_avg"].shape != f.exp_avg.shape:
        raise ValueError(f"checkpoint Adam state has {st['exp_avg'].numel()} elements, this rank holds "
                         f"{f.exp_avg.numel()}: a zero_stage=1 checkpoint resumes only at the same dp and zero_stage")
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
