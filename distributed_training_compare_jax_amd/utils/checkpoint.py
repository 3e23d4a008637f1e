"""Checkpoint / resume (absent in the reference: params are discarded at exit,
``train/train.py:98-102``; SURVEY §5 plan).

Layout: ``<output_dir>/ckpt/step_<N>/rank<r>.pt`` (flat fp32 params, Adam m and v, the
device step counter) + ``meta_rank<r>.json`` (mesh, this rank's layer range, the padded and
canonical vocab, and the partition map: every parameter's name, flat offset, local shape and TP
rule).  The partition map lets :func:`consolidate` rebuild the full unsharded model from any
DP/TP/PP layout (vocab rows trimmed to the canonical ``vocab_size``, whatever TP padding wrote
them), so a run can be converted between strategies.  Resume compares the map with this rank's
flat-buffer slots before touching any buffer, and every rank fails together when one rank's check
fails.  Files are loaded with ``weights_only=True``.
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
    slots = {n: dict(offset=s.offset, shape=list(s.shape), tp=s.spec.tp, full=list(s.spec.shape),
                     vpart=list(s.spec.vpart))
             for n, s in f.slots.items()}
    lr = getattr(eng, "layout", None)
    meta = dict(step=step, dp=m.dp, tp=m.tp, pp=m.pp, rank=m.rank, dp_idx=m.dp_idx, tp_idx=m.tp_idx,
                pp_idx=m.pp_idx, slots=slots, model=eng.mcfg.name,
                zero_stage=int(getattr(eng, "zero", False)),
                layers=[lr.layers.start, lr.layers.stop] if lr is not None else None,
                vocab_size=int(eng.mcfg.vocab_size), padded_vocab=int(eng.mcfg.padded_vocab))
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
    src = None
    for r, m in metas.items():
        if (m["dp_idx"], m["tp_idx"], m["pp_idx"]) == want:
            src = r
            break
    if src is None and not zero_now:
        for r, m in metas.items():
            if (m["dp_idx"], m["tp_idx"], m["pp_idx"]) == (0, mesh.tp_idx, mesh.pp_idx):
                src = r
                break
    if src is None:
        raise ValueError(f"checkpoint (world {len(metas)}) has no rank file for dp/tp/pp index {want}")
    _check_slots(eng, metas[src])
    return src


def _check_slots(eng, meta: dict):
    """The source rank's partition map must equal this rank's flat-buffer layout slot by slot (name,
    offset, local shape).  Equal element counts are not enough: two PP splits can give a stage the same
    number of identically shaped layers starting at a different index (``pp_split``/``pp_head_cost``
    changed), and those weights would load into the wrong layers without any size error."""
    mine = eng.flat.slots
    theirs = meta.get("slots", {})
    lay = meta.get("layers")
    layout = getattr(eng, "layout", None)
    if lay is not None and layout is not None and list(lay) != [layout.layers.start, layout.layers.stop]:
        raise ValueError(f"checkpoint stage {meta['pp_idx']} holds layers [{lay[0]}, {lay[1]}) but this run's stage "
                         f"holds [{layout.layers.start}, {layout.layers.stop}): the PP layer split differs "
                         "(pp_split / pp_head_cost); resume with the split that wrote it, or consolidate() and re-shard")
    if list(theirs) != list(mine):
        extra = sorted(set(theirs) - set(mine))[:3]
        missing = sorted(set(mine) - set(theirs))[:3]
        raise ValueError(f"checkpoint partition map differs from this rank's parameters (only in the checkpoint: "
                         f"{extra}, only in this run: {missing}): the layer split or model differs")
    for n, s in mine.items():
        t = theirs[n]
        if int(t["offset"]) != s.offset or list(t["shape"]) != list(s.shape):
            raise ValueError(f"checkpoint slot {n!r} is at offset {t['offset']} shape {t['shape']}, this run has "
                             f"offset {s.offset} shape {list(s.shape)} (vocab padding or layout differs)")


def _agree(ok: bool, err, device):
    """All ranks learn whether any rank's checkpoint check failed (so no rank walks into the next
    collective alone); raise here on every rank if one did."""
    import torch.distributed as dist

    failed = not ok
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([1.0 if failed else 0.0], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if float(t.item()) > 0 and ok:
            raise ValueError("checkpoint resume failed on another rank (see its error); nothing was loaded")
    if failed:
        raise err


def load_into(eng, output_dir: str, step: int):
    d = _dir(output_dir, step)
    f = eng.flat
    st, err = None, None
    try:
        src = source_rank(eng, _read_metas(d))
        st = torch.load(os.path.join(d, f"rank{src}.pt"), map_location="cpu", weights_only=True)
        for k, have in (("params", f.params), ("exp_avg", f.exp_avg), ("exp_avg_sq", f.exp_avg_sq)):
            if st[k].shape != have.shape:
                raise ValueError(f"checkpoint {k} has {st[k].numel()} elements, this rank holds {have.numel()}")
    except Exception as e:  # noqa: BLE001 -- any failure (corrupt / truncated zip, unpickling refused,
        err = e             # permission) must still reach the agreement collective on this rank
    _agree(err is None, err, f.device)
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


_VOCAB_ROWS = ("wte", "lm_head.w", "lm_head.b")  # params whose leading dim is the (padded) vocab


def consolidate(output_dir: str, step: int, vocab_size: int = None) -> Dict[str, torch.Tensor]:
    """Full (unsharded) fp32 parameters from every rank file of a checkpoint.

    Vocab-indexed tensors (wte rows, lm_head rows and bias) come back with exactly ``vocab_size`` rows
    (default: the canonical vocab recorded in the checkpoint) whatever padding the writing layout used
    (TP >= 4 pads to a multiple of 64·tp), so checkpoints of different strategies consolidate to the same
    shapes; :func:`pad_vocab` re-pads for a target layout."""
    from ..models.params import ParamSpec

    d = _dir(output_dir, step)
    metas = [json.load(open(os.path.join(d, x))) for x in sorted(os.listdir(d)) if x.startswith("meta_rank")]
    pieces: Dict[str, Dict[tuple, torch.Tensor]] = {}
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
            vp = tuple(s.get("vpart", (0, 1)))  # lm_head vocab slice of a head split over PP stages
            pieces.setdefault(n, {})[(vp[0], meta["tp_idx"])] = t
            tp_rule[n] = s["tp"]
            full_shape[n] = tuple(s["full"])
    if vocab_size is None:
        vocab_size = next((int(m["vocab_size"]) for m in metas if "vocab_size" in m), None)
    out = {}
    for n, parts in pieces.items():
        spec = ParamSpec(n, full_shape[n], "zeros", 1, tp_rule[n], 0, False)
        vparts = sorted({k[0] for k in parts})
        t = torch.cat([unshard(spec, [parts[k] for k in sorted(parts) if k[0] == v]) for v in vparts], 0) \
            if len(vparts) > 1 else unshard(spec, [parts[k] for k in sorted(parts)])
        if vocab_size is not None and n in _VOCAB_ROWS and t.shape[0] > vocab_size:
            t = t[:vocab_size].clone()
        out[n] = t
    return out


def pad_vocab(full: Dict[str, torch.Tensor], padded_vocab: int) -> Dict[str, torch.Tensor]:
    """Re-pad consolidated vocab-indexed tensors with zero rows to ``padded_vocab`` (a target layout's
    ``ModelConfig.padded_vocab``); pad rows are zero and masked in every layout."""
    out = dict(full)
    for n in _VOCAB_ROWS:
        if n in out and out[n].shape[0] < padded_vocab:
            t = out[n]
            pad = torch.zeros((padded_vocab - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype)
            out[n] = torch.cat([t, pad])
    return out
