"""DP × TP × PP process mesh.

The reference has a single 1-D device axis ``"data"`` used by both DP and TP
(``train/train.py:29``) and a separate ``pmap`` axis ``"pipe"`` for PP
(``create_train_step.py:70``).  Here the three axes are explicit process groups:

    rank = (pp_idx · dp + dp_idx) · tp + tp_idx

TP is innermost so a TP group is a block of adjacent GPUs (on an 8×MI355X xGMI mesh every
pair is one hop, but adjacency keeps a TP group inside one socket on multi-node
layouts), DP next, PP outermost.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch.distributed as dist


@dataclass
class Mesh:
    dp: int
    tp: int
    pp: int
    rank: int
    dp_idx: int
    tp_idx: int
    pp_idx: int
    dp_group: Optional[object] = None
    tp_group: Optional[object] = None
    pp_group: Optional[object] = None
    # ranks of neighbours inside the pp group (global ranks)
    pp_prev: Optional[int] = None
    pp_next: Optional[int] = None

    @property
    def world(self) -> int:
        return self.dp * self.tp * self.pp

    def rank_of(self, dp_idx: int, tp_idx: int, pp_idx: int) -> int:
        return (pp_idx * self.dp + dp_idx) * self.tp + tp_idx


def resolve_degrees(parallel: str, world: int, dp: Optional[int], tp: Optional[int], pp: Optional[int]):
    """Map the reference's single ``parallel`` string (+ optional explicit degrees) onto (dp, tp, pp)."""
    if dp or tp or pp:
        dp, tp, pp = dp or 1, tp or 1, pp or 1
        if dp * tp * pp != world:
            # fill the unspecified axis implied by the strategy
            rest = world // (dp * tp * pp) if world % (dp * tp * pp) == 0 else None
            if rest is None:
                raise ValueError(f"dp*tp*pp = {dp * tp * pp} does not divide world size {world}")
            if parallel == "tp":
                tp *= rest
            elif parallel == "pp":
                pp *= rest
            else:
                dp *= rest
        return dp, tp, pp
    if parallel == "dp":
        return world, 1, 1
    if parallel == "tp":
        return 1, world, 1
    if parallel == "pp":
        return 1, 1, world
    if parallel in ("none", "single"):
        if world != 1:
            raise ValueError("parallel=none needs world size 1")
        return 1, 1, 1
    raise ValueError(f"Unsupported strategy `{parallel}`")


def build_mesh(rank: int, world: int, dp: int, tp: int, pp: int, dp_group_always: bool = False) -> Mesh:
    """``dp_group_always``: give a dp == 1 rank a one-member DP group anyway (the DP collective rehearsal
    of ``TrainConfig.dp_comm_rehearsal``; needs an initialised process group)."""
    assert dp * tp * pp == world, (dp, tp, pp, world)
    tp_idx = rank % tp
    dp_idx = (rank // tp) % dp
    pp_idx = rank // (tp * dp)
    m = Mesh(dp, tp, pp, rank, dp_idx, tp_idx, pp_idx)
    if (world > 1 or dp_group_always) and dist.is_initialized():
        # every rank must create every group, in the same order
        for p in range(pp):
            for d in range(dp):
                ranks = [m.rank_of(d, t, p) for t in range(tp)]
                g = dist.new_group(ranks) if tp > 1 else None
                if p == pp_idx and d == dp_idx:
                    m.tp_group = g
        for p in range(pp):
            for t in range(tp):
                ranks = [m.rank_of(d, t, p) for d in range(dp)]
                g = dist.new_group(ranks) if (dp > 1 or dp_group_always) else None
                if p == pp_idx and t == tp_idx:
                    m.dp_group = g
        for d in range(dp):
            for t in range(tp):
                ranks = [m.rank_of(d, t, p) for p in range(pp)]
                g = dist.new_group(ranks) if pp > 1 else None
                if d == dp_idx and t == tp_idx:
                    m.pp_group = g
    if pp_idx > 0:
        m.pp_prev = m.rank_of(dp_idx, tp_idx, pp_idx - 1)
    if pp_idx < pp - 1:
        m.pp_next = m.rank_of(dp_idx, tp_idx, pp_idx + 1)
    return m


def head_cost_blocks(cfg, head_speedup: float = 1.7) -> float:
    """Cost of lm_head + cross-entropy (forward + backward) in units of one transformer block, from
    FLOPs: per token the head is 6·D·V against a block's 6·(4·D² + 2·D·F) + causal attention
    6·T·D, divided by ``head_speedup`` -- the head's large GEMMs run at ~1.7x the MFMA rate of a block's
    mix (layer GEMMs + attention + LayerNorm passes).  GPT-2 small: 4.9 by FLOPs, 2.9 by this model;
    measured 2.8 in the round-3 kernel table (profiles/r3_gpt2_small_profile_final.md: lm_head
    fwd 713 + dgrad 657 + wgrad 569 + CE 306 us against ~0.8 ms per block)."""
    D, F, V, T = cfg.d_model, cfg.d_ff, cfg.padded_vocab, cfg.max_seq_len
    block = 6.0 * (4 * D * D + 2 * D * F) + 6.0 * T * D
    return 6.0 * D * V / block / head_speedup


def split_layers(n_layers: int, pp: int, weights=None, head_stages: int = 1):
    """Contiguous layer ranges per stage.  Fixes the reference quirk ``layers_per_stage =
    n_layers // N`` (``train/train.py:118``) that silently drops layers when N ∤ L.

    ``weights=None``: an even split, the remainder to the EARLIEST stages (the last stage also
    carries lm_head+CE).  ``weights=(first, last)``: extra cost (in blocks) of the first stage
    (embedding) and the last (lm_head + CE, :func:`head_cost_blocks`): the contiguous split that
    minimises the most expensive stage, then the spread (sum of squared stage costs); every stage but
    the last keeps at least one layer, the last may hold the head alone.

    ``head_stages=2`` (``pp_head_split``): lm_head + CE split by vocab over the last two stages, each
    carrying half of ``last``; the last stage holds no layers, the one before may hold the head half alone."""
    if weights is None:
        base, rem = divmod(n_layers, pp)
        out, start = [], 0
        for s in range(pp):
            n = base + (1 if s < rem else 0)
            out.append(range(start, start + n))
            start += n
        return out
    first, last = (float(w) for w in weights)
    if n_layers < pp - 1:  # not enough layers for one per non-last stage
        return split_layers(n_layers, pp)
    extra = [0.0] * pp
    extra[0] += first
    if head_stages == 2 and pp >= 2:
        extra[-1] += last / 2
        extra[-2] += last / 2
    else:
        extra[-1] += last
    # DP over (stage, layers placed): minimise (max stage cost, sum of squared stage costs); every stage
    # but the last holds >= 1 layer (an empty middle stage would only relay activations)
    INF = (float("inf"), float("inf"))
    best = [[INF] * (n_layers + 1) for _ in range(pp + 1)]
    arg = [[0] * (n_layers + 1) for _ in range(pp + 1)]
    best[0][0] = (0.0, 0.0)
    for s_ in range(pp):
        lo_k = 0 if s_ == pp - 1 or (head_stages == 2 and s_ == pp - 2) else 1
        hi_k = 0 if (head_stages == 2 and s_ == pp - 1) else n_layers
        for used in range(n_layers + 1):
            if best[s_][used] == INF:
                continue
            mx, sq = best[s_][used]
            for k in range(lo_k, min(hi_k, n_layers - used) + 1):
                c = k + extra[s_]
                cand = (max(mx, c), sq + c * c)
                if cand < best[s_ + 1][used + k]:
                    best[s_ + 1][used + k] = cand
                    arg[s_ + 1][used + k] = k
    counts, used = [], n_layers
    for s_ in range(pp, 0, -1):
        k = arg[s_][used]
        counts.append(k)
        used -= k
    counts.reverse()
    out, start = [], 0
    for k in counts:
        out.append(range(start, start + k))
        start += k
    return out


def stage_costs(ranges, weights, head_stages: int = 1):
    """Per-stage cost (blocks) of a split under ``weights=(first, last)`` (``head_stages=2``: the head
    halved over the last two stages)."""
    first, last = weights
    c = [float(len(r)) for r in ranges]
    c[0] += first
    if head_stages == 2 and len(c) >= 2:
        c[-1] += last / 2
        c[-2] += last / 2
    else:
        c[-1] += last
    return c
