"""GPT decoder with explicit forward/backward (no autograd on the hot path).

Same architecture as the reference ``model/GPTModel.py`` (pre-LN blocks of
``TransformerBlock.py:13-26``: ``x += out(attn(LN1 x))``, ``x += fc2(gelu(fc1(LN2 x)))``;
learned absolute positions; untied ``lm_head`` with bias) and the same three callable
partitions the reference exposes for pipelining (``embed_forward`` / ``stage_forward`` /
``head_forward``, ``GPTModel.py:24-74``).

Why explicit backward instead of autograd: every backward op is a fused HIP kernel that
writes its gradient straight into the flat fp32 grad buffer (``parallel/buffers.py``),
activations are kept exactly as the kernels need them (bf16 GEMM operands, fp32
residual stream, LN mean/rstd, attention LSE), TP collectives sit at exactly the four
points per block Megatron-style TP needs, and the whole step is a static sequence of
kernel launches that can be captured into hipGraphs.  Numerical equivalence to the
autograd oracle (``models/reference.py``) is tested in ``tests/test_model.py``.

Dtypes: residual stream fp32; GEMM operands in the compute dtype (bf16 on MI355X, fp32
on the CPU oracle path); all accumulation fp32; grads fp32.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from ..config.schema import ModelConfig
from ..ops import attention as A
from ..ops import embedding as E
from ..ops import gemm as G
from ..ops import layernorm as LN
from ..ops import ln_fused as LF
from ..ops import xent as X
from ..ops.reduce import GradReducer
from .params import head_split
from ..parallel.buffers import FlatParams


import os as _os

# ops/xent.py ce_dgrad_fused: "1" / "0", or "auto" (default) = fused for lm_head dgrads of at most
# 4096 x 512 outputs (the reference model: 382 -> 341 us, profiles/r2_ab_ce_fused_dgrad.log); at GPT-2
# small (8192 x 768: 96 tiles x split 2 = 192 blocks on 256 CUs) the separate CE pass + the DMA-staged
# 256^2 split-K dgrad measured faster (13.50 vs 13.57 ms, profiles/r3_ab_knobs2.log)
_CE_FUSED_MODE = _os.environ.get("DTC_CE_FUSED", "auto")


def _ce_fused(tokens: int, d: int) -> bool:
    if _CE_FUSED_MODE == "auto":
        return tokens * d <= 4096 * 512
    return _CE_FUSED_MODE == "1"
# Vocab-chunked lm_head + cross-entropy (DTC_CE_CHUNK = vocab columns per chunk, a multiple of 256; 0 =
# off): the forward keeps only each chunk's per-row (max, sum exp) and label logit (logits of one chunk
# at a time), the backward recomputes a chunk's logits, turns them into dlogits in place and runs that
# chunk's dgrad (accumulated into dX) and weight / bias gradients.  Peak lm_head memory is one
# tokens x chunk bf16 buffer instead of the full tokens x vocab logits (GPT-2 small: 134 MB at 8192
# columns vs 824 MB) held from the forward to the backward -- for memory-bound configurations
# (SURVEY K10 "never materialize full logits"); it costs one extra lm_head GEMM (the recompute).
_CE_CHUNK = int(_os.environ.get("DTC_CE_CHUNK", "0"))
# residual adds of out_proj / fc2 done by the LayerNorm pass that follows (tp == 1): the GEMM epilogue
# stores a·Wᵀ + b without reading the fp32 residual (DTC_ADD_LN=0: the fused residual epilogue)
_ADD_LN = _os.environ.get("DTC_ADD_LN", "1") == "1"
# out_proj / fc2 forwards (tp == 1, DTC_ADD_LN, bf16 compute) store a·Wᵀ + b as bf16, the LayerNorm pass
# adds it to the fp32 residual (autocast-style bf16 GEMM outputs; the residual stream stays fp32)
_FWD_BF16 = _os.environ.get("DTC_FWD_BF16", "0") == "1"
# deferred weight gradients: the layers' LayerNorm / bias partial reductions wait for the group's flush (one
# batched reduce launch per 48 tasks for the whole group) instead of one reduce launch per layer: GPT-2 small
# 10.90 vs 10.97 ms/step (profiles/r4_ab_red_batch.log)
_RED_BATCH_LAYERS = _os.environ.get("DTC_RED_BATCH_LAYERS", "1") == "1"
if _CE_CHUNK < 0 or _CE_CHUNK % 256:
    # chunk offsets feed 16-byte vector loads of w[c0:], wt[:, c0:] and gw[c0:]: a ragged offset would
    # surface as an opaque native error deep in the backward
    raise ValueError(f"DTC_CE_CHUNK={_CE_CHUNK}: must be 0 (off) or a positive multiple of 256 vocab columns")



# lm_head input-gradient partial as bf16 into the P2P buffer below this shard width (GPTStage._head_dgrad)
_HEAD_BF16_MAXK = 16384


class _Staged:
    """A TP input-gradient partial a dgrad GEMM wrote into the P2P buffer (``TPComm.partial_out``)."""

    __slots__ = ("rows", "cols", "device")

    def __init__(self, rows: int, cols: int, device):
        self.rows, self.cols, self.device = rows, cols, device

class NoComm:
    """TP communicator stub for tp_size == 1."""

    size = 1
    rank = 0

    def all_reduce_(self, t):
        return t

    def all_gather_stack(self, t):
        return t.unsqueeze(0)


@dataclass
class StageLayout:
    layers: range
    has_embed: bool
    has_head: bool
    # (part, parts): lm_head + CE split by vocab over the last `parts` pipeline stages (pp_head_split);
    # part 0 also holds the final LayerNorm
    head_part: Tuple[int, int] = (0, 1)


class GPTStage:
    """The slice of the GPT owned by one rank (all of it, a TP shard, or a PP stage)."""

    def __init__(self, cfg: ModelConfig, flat: FlatParams, layout: StageLayout, tp=None,
                 dropout_seed: int = 0, act_dtype: torch.dtype = torch.bfloat16):
        self.cfg = cfg
        # one-stream GPU backward: every off-critical-path reduction of a layer (split-K weight gradient
        # slabs, LN dgamma/dbeta partials, bias column partials, grad-norm chunks) goes into ONE batched
        # launch per layer (ops/reduce.py).  (A second stream for the weight gradients measured slower on
        # one GPU -- 6.00 vs 5.44 ms, round 2 -- and was removed: the grouped launches fill the chip instead.)
        dev = torch.device(flat.device)
        # 512 MB window: a layer's split-K weight-gradient slabs (GPT-2 medium: 4 x ~67 MB) + LN partials
        self.red = GradReducer(dev, arena_mb=512) if dev.type == "cuda" else None
        self._bias_fused = set()  # layers whose fc2.b grad an upstream LN backward already produced
        # deferred optimizer (train/engine.py): params of layer l / "head" become valid when this
        # event fires; the forward waits on it right before first use
        self.param_ready: Dict = {}
        self.flat = flat
        self.layout = layout
        self.tp = tp if tp is not None else NoComm()
        self.seed = int(dropout_seed)
        self.act_dtype = act_dtype
        D, H = cfg.d_model, cfg.n_heads
        # tp_comm_dtype: bf16 -> row-parallel partials and input-gradient partials travel as bf16
        # (TPComm.reduce_to; residual + bias added after the fp32 sum), set by the engine
        self.tp_bf16 = False
        self.head_dgrad_staged = 0  # lm_head input-gradient partials sent as bf16 (_head_dgrad)
        assert D % H == 0
        # whole heads per TP rank, uneven when tp does not divide H (models/params.py head_split)
        self.heads_local = head_split(H, self.tp.size)[self.tp.rank][1]
        part, parts = layout.head_part
        self.v_local = cfg.padded_vocab // parts // self.tp.size
        self.v_start = part * (cfg.padded_vocab // parts) + self.tp.rank * self.v_local
        self.v_valid = max(0, min(self.v_local, cfg.vocab_size - self.v_start))
        self.eps = cfg.layernorm_eps
        # Deferred weight gradients (set_wgrad_group): the dgrad chain runs alone and every (dY, X, dW, db)
        # of wgrad_group consecutive layers (0 = the whole stage, + the lm_head) goes out as ONE grouped
        # launch of whole 256^2 tiles (ops/gemm.py wgrad_group)
        self.wg_group = -1  # -1 = off
        self.wg_queue = []
        # grad-norm partials from the grouped launch (engine: dp == 1 and one launch per step): the first
        # flush records its problems (wg_seen), the engine then hands back the partial slots (wg_sq)
        self.wg_record = False
        self.wg_seen = None
        self.wg_sq: Optional[torch.Tensor] = None
        # the embedding backward's Σ dwte² + Σ dwpe² partial slots (FusedAdamW fused partials), or None
        self.emb_sq: Optional[torch.Tensor] = None
        # the previous embedding backward's sort keys (its rows are the only nonzero ones of the wte grad), or
        # None: full-table zeroing every step (set by the engine where one local backward writes the table)
        self.emb_prev: Optional[torch.Tensor] = None
        self._emb_prev_valid = False
        self._wg_keys = None
        # LayerNorm fused into the layer GEMMs (ops/ln_fused.py), set up by enable_ln_fusion
        self.ln_sync: Optional[LF.LnSync] = None
        self._fuse_fwd = self._fuse_bwd = False
        # sequence parallelism (enable_sequence_parallel): residual stream / LayerNorms / embedding output on
        # rows/tp rows per rank; the LN and row-parallel-bias grads are then per-rank partials (_sp_sum)
        self.sp = False
        self._sp_idx: Dict = {}

    def set_wgrad_group(self, layers: int):
        """Defer weight gradients to grouped launches of ``layers`` consecutive layers (0 = all layers of
        the stage in one launch, with the lm_head's; -1 = off: each Dense's weight gradient right after
        its dgrad)."""
        self.wg_group = int(layers)
        return self.wg_group

    @property
    def _defer_wg(self) -> bool:
        return self.wg_group >= 0

    def _wg(self, dy, x, dense: str, bias: bool = False):
        """Queue (or run now) the weight gradient of Dense ``dense`` (+ its bias gradient)."""
        f = self.flat
        db = f.g(dense + ".b") if bias else None
        if self._defer_wg:
            self.wg_queue.append((dy, x, f.g(dense + ".w"), db))
        else:
            G.wgrad(dy, x, f.g(dense + ".w"), self._beta, red=self.red, db=db)

    def flush_wgrads(self, beta: float):
        """Launch every queued weight gradient (one grouped launch), then the reducer's batched launch."""
        if self.wg_queue:
            q, self.wg_queue = self.wg_queue, []
            if self.wg_record and self.wg_seen is None:
                self.wg_seen = [(dw, dy.shape[1], x.shape[1]) for dy, x, dw, _ in q]
            sq = None
            if self.wg_sq is not None:
                keys = sorted(dw.data_ptr() for _, _, dw, _ in q)
                if keys != self._wg_keys:
                    raise RuntimeError("grouped weight gradients: the problems differ from the ones whose grad-norm "
                                       "partials were registered (one grouped launch per step expected)")
                sq = self.wg_sq
            G.wgrad_group(q, beta, red=self.red, sq=sq)

    def use_wgrad_sumsq(self, sq: torch.Tensor):
        """From now on the grouped launch writes its tiles' Σ dW² into ``sq`` (FusedAdamW.set_fused_sumsq)."""
        self.wg_sq = sq
        self._wg_keys = sorted(dw.data_ptr() for dw, _, _ in self.wg_seen)

    def enable_ln_fusion(self, tokens: int, step: torch.Tensor, fwd: bool, bwd: bool) -> bool:
        """Fuse the LayerNorms into the GEMMs that produce their input (forward) and their output
        gradient (backward).  Needs tp = 1 (no all-reduce between the GEMM and the LayerNorm), one
        call per site and step (no pipeline microbatches) and the transposed weight mirror for the
        NT dgrads; ``tokens`` = rows of every call.  Returns whether anything was enabled."""
        D, L = self.cfg.d_model, len(self.layout.layers)
        if self.tp.size != 1 or not L or not LF.supported(tokens, D, 64) or not (fwd or bwd):
            return False
        self.ln_sync = LF.LnSync(self.flat.device, tokens, D, nsites=4 * L, step=step)
        self._fuse_fwd, self._fuse_bwd = bool(fwd), bool(bwd)
        return True

    def enable_sequence_parallel(self, batch: int) -> bool:
        """Megatron-style sequence parallelism over the TP group (``TrainConfig.tp_sequence_parallel``):
        each rank holds ``batch / tp`` whole sequences of the residual stream.  Forward per block: LN1 on
        the own rows → all-gather → qkv / attention / out_proj (full rows, local heads) → reduce-scatter
        (+ residual + bias) → LN2 → all-gather → fc1 / fc2 → reduce-scatter; the backward mirrors it.
        Same xGMI bytes as the four all-reduces (an all-reduce IS a reduce-scatter + an all-gather), while
        the LayerNorms, the residual adds and the embedding run on 1/tp of the rows.  Needs tp > 1,
        ``batch % tp == 0`` and a single pipeline stage."""
        tp = self.tp.size
        if tp == 1 or batch % tp or not (self.layout.has_embed and self.layout.has_head):
            return False
        self.sp = True
        dev = self.flat.grads.device
        for key, names in self._sp_groups().items():
            self._sp_idx[(key,)] = self._sp_index(names, dev)
        return True

    def _sp_groups(self) -> Dict:
        """Per layer (and "head"): the grads that are per-rank partial sums under sequence parallelism --
        the LayerNorm params and the row-parallel biases (out_proj, fc2), replicated over TP but produced
        from the own rows only."""
        out = {l: [f"h.{l}.{n}" for n in ("ln1.g", "ln1.b", "ln2.g", "ln2.b", "out.b", "fc2.b")]
               for l in self.layout.layers}
        out["head"] = ["lnf.g", "lnf.b"]
        return out

    def _sp_index(self, names, dev) -> torch.Tensor:
        sl = self.flat.slots
        return torch.cat([torch.arange(sl[n].offset, sl[n].offset + sl[n].numel, dtype=torch.int64)
                          for n in names]).to(dev)

    def _sp_sum(self, keys):
        """Sum the partial grads of layers / "head" ``keys`` over the TP group: one gather, one all-reduce
        (in-graph on the P2P path), one scatter back."""
        if not self.sp or not keys:
            return
        k = tuple(keys)
        idx = self._sp_idx.get(k)
        if idx is None:
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"sequence parallel: grad index of group {k} first built during graph capture")
            idx = torch.cat([self._sp_idx[(kk,)] for kk in k])
            self._sp_idx[k] = idx
        g = self.flat.grads
        buf = g.index_select(0, idx)
        self.tp.all_reduce_(buf)
        g.index_copy_(0, idx, buf)

    def _ln_site(self, l: int, k: int, backward: bool) -> int:
        """Execution-order index of a fused LayerNorm call: forward k = 0 (out_proj → ln2) / 1 (fc2 →
        the next ln1 or lnf) of layer l; backward k = 0 (ln2) / 1 (ln1), layers in reverse."""
        L = len(self.layout.layers)
        li = l - self.layout.layers[0]
        return 2 * L + 2 * (L - 1 - li) + k if backward else 2 * li + k

    # ------------------------------------------------------------------ embed
    def embed_forward(self, ids: torch.Tensor, step: torch.Tensor, row0: int, ctx: Dict,
                      want_keys: bool = True, keys: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ids int32 [b, T] → h fp32 [b*T, D]  (wte gather + wpe + dropout, GPTModel.py:30-38).

        ``keys``: the backward's sort keys, already computed on the host (``E.embed_sort_keys_host``);
        otherwise (``want_keys``) they are sorted on the device."""
        f = self.flat
        if self.sp:  # this rank's sequences only (the backward gathers the output grads of all of them)
            bl = ids.shape[0] // self.tp.size
            r0 = self.tp.rank * bl
            h = E.embed_fwd(ids[r0:r0 + bl], f.p("wte"), f.p("wpe"), self.cfg.dropout, self.seed, step, row0 + r0)
        else:
            h = E.embed_fwd(ids, f.p("wte"), f.p("wpe"), self.cfg.dropout, self.seed, step, row0)
        if keys is not None:
            ctx["embed"] = (ids, row0, (keys, None))
        else:
            ctx["embed"] = (ids, row0, self.embed_keys(ids) if want_keys else None)
        return h

    def embed_keys(self, ids: torch.Tensor):
        """Sort keys for the deterministic embedding backward (they depend only on the ids); the engine
        normally builds them on the host instead (``E.embed_sort_keys_host``)."""
        if not ids.is_cuda or ids.numel() > E.SORT_MAX:
            return None  # CPU path / chunked backward sorts per chunk
        keys = torch.empty(ids.numel(), dtype=torch.int32, device=ids.device)
        E.embed_sort_keys(ids, self.flat.p("wte").shape[0], out=keys)
        return keys, None

    def embed_backward(self, ctx: Dict, dh: torch.Tensor, step: torch.Tensor, beta: float, gathered=None):
        """``gathered`` = (ids, row0, keys) of a DP-gathered batch whose ``dh`` rows were all-gathered
        (every DP rank then builds the identical wte/wpe grads locally, no all-reduce)."""
        ids, row0, keys = ctx.pop("embed")
        if gathered is not None:
            ids, row0, keys = gathered
        if keys is not None:
            keys, _ = keys
        if self.sp and gathered is None:
            dh = self.tp.all_gather_rows(dh)  # every rank builds the identical wte / wpe grads
        f = self.flat
        sq = self.emb_sq
        if sq is not None and (beta != 0.0 or gathered is not None or self.sp):
            raise RuntimeError("fused embedding Σg² partials need one local embedding backward per step (beta 0)")
        prev = self.emb_prev
        if prev is not None and (beta != 0.0 or gathered is not None or self.sp):
            raise RuntimeError("sparse wte zeroing needs one local embedding backward per step (beta 0)")
        E.embed_bwd(ids, dh, f.g("wte"), f.g("wpe"), self.cfg.dropout, self.seed, step, row0, beta, keys=keys, sq=sq,
                    prev_keys=prev, prev_valid=self._emb_prev_valid)
        if prev is not None:
            self._emb_prev_valid = True  # from the next call on only the rows written here are zeroed

    # ------------------------------------------------------------------ block
    def _await_params(self, key):
        ev = self.param_ready.pop(key, None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    @property
    def _branch_dtype(self) -> torch.dtype:
        """dtype of the out_proj / fc2 outputs the LayerNorm pass adds to the residual (DTC_FWD_BF16)."""
        return torch.bfloat16 if _FWD_BF16 and self.act_dtype == torch.bfloat16 else torch.float32

    def block_forward(self, l: int, x: torch.Tensor, batch: int, ctx: Dict) -> torch.Tensor:
        if self.sp:
            return self._block_forward_sp(l, x, batch, ctx)
        self._await_params(l)
        f, p = self.flat, f"h.{l}."
        tp = self.tp
        lead = tp.rank == 0  # row-parallel bias + residual are added by exactly one TP rank
        T = x.shape[0] // batch
        pre = ctx.pop(("ln1", l), None)  # LN1 already produced by the previous layer's fc2 GEMM
        if pre is None:
            pre = LN.layernorm_fwd(x, f.p(p + "ln1.g"), f.p(p + "ln1.b"), self.eps, self.act_dtype)
        y1, mu1, rs1 = pre
        qkv = G.linear(y1, f.w(p + "qkv.w"), f.p(p + "qkv.b"))
        o, lse = A.attn_fwd(qkv.view(batch, T, -1), self.heads_local)
        o = o.view(batch * T, -1)
        if self._fuse_fwd:
            x2, (y2, mu2, rs2) = LF.linear_resid_ln(o, f.w(p + "out.w"), f.p(p + "out.b"), x, f.p(p + "ln2.g"),
                                                    f.p(p + "ln2.b"), self.eps, self.ln_sync, self._ln_site(l, 0, False))
        elif self.tp_bf16:
            x2 = self._row_parallel(o, p + "out.w", resid=x, bias=f.p(p + "out.b"))
            y2, mu2, rs2 = LN.layernorm_fwd(x2, f.p(p + "ln2.g"), f.p(p + "ln2.b"), self.eps, self.act_dtype)
        elif tp.size == 1 and _ADD_LN:
            # residual add in the LayerNorm pass (the GEMM stores o·Wᵀ + b; its epilogue skips the fp32
            # residual read) -- same fp32 arithmetic, (acc + b) + x
            x2, (y2, mu2, rs2) = LN.add_layernorm_fwd(G.linear(o, f.w(p + "out.w"), f.p(p + "out.b"),
                                                               out_dtype=self._branch_dtype), x,
                                                      f.p(p + "ln2.g"), f.p(p + "ln2.b"), self.eps, self.act_dtype)
        else:
            x2 = G.linear_resid(o, f.w(p + "out.w"), f.p(p + "out.b") if lead else None, x if lead else None)
            tp.all_reduce_(x2)
            y2, mu2, rs2 = LN.layernorm_fwd(x2, f.p(p + "ln2.g"), f.p(p + "ln2.b"), self.eps, self.act_dtype)
        u, gact = G.linear_gelu(y2, f.w(p + "fc1.w"), f.p(p + "fc1.b"))  # u = gelu'(pre-activation)
        # the LayerNorm that reads x3: the next layer's ln1, or the final one after the last layer
        nxt = f"h.{l + 1}.ln1" if (l + 1) in self.layout.layers else ("lnf" if self.layout.has_head else None)
        if self._fuse_fwd and nxt is not None:
            x3, pre_next = LF.linear_resid_ln(gact, f.w(p + "fc2.w"), f.p(p + "fc2.b"), x2, f.p(nxt + ".g"),
                                              f.p(nxt + ".b"), self.eps, self.ln_sync, self._ln_site(l, 1, False))
            ctx[("ln1", l + 1) if nxt != "lnf" else "lnf_pre"] = pre_next
        elif tp.size == 1 and _ADD_LN and nxt is not None and not self.tp_bf16:
            x3, pre_next = LN.add_layernorm_fwd(G.linear(gact, f.w(p + "fc2.w"), f.p(p + "fc2.b"),
                                                         out_dtype=self._branch_dtype), x2,
                                                f.p(nxt + ".g"), f.p(nxt + ".b"), self.eps, self.act_dtype)
            ctx[("ln1", l + 1) if nxt != "lnf" else "lnf_pre"] = pre_next
        elif self.tp_bf16:
            x3 = self._row_parallel(gact, p + "fc2.w", resid=x2, bias=f.p(p + "fc2.b"))
        else:
            x3 = G.linear_resid(gact, f.w(p + "fc2.w"), f.p(p + "fc2.b") if lead else None, x2 if lead else None)
            tp.all_reduce_(x3)
        ctx[l] = (x, y1, mu1, rs1, qkv, o, lse, x2, y2, mu2, rs2, u, gact, batch)
        return x3

    def block_backward(self, l: int, ctx: Dict, dx3: torch.Tensor, dx3_c: torch.Tensor, beta: float, dx_hook=None):
        """dx3 fp32 (and its compute-dtype copy) → (dx, dx_c) wrt the block input.  ``dx_hook(dx, dx_c)``
        (optional) is called as soon as dx is final, before the layer's remaining weight-gradient
        work (the DP embedding gather starts there, under that work)."""
        if self.sp:
            return self._block_backward_sp(l, ctx, dx3, dx3_c, beta, dx_hook)
        f, p = self.flat, f"h.{l}."
        x, y1, mu1, rs1, qkv, o, lse, x2, y2, mu2, rs2, u, gact, batch = ctx.pop(l)
        T = x.shape[0] // batch
        red = self.red
        # fc2.b's gradient = Σ_rows dx3 was already emitted by the LayerNorm backward that produced
        # dx3 (lnf or the next block's ln1) unless dx3 arrived from another pipeline stage
        fc2b_fused = l in self._bias_fused
        self._bias_fused.discard(l)
        self._beta = beta
        if self._defer_wg:
            # deferred weight gradients: the dgrad chain alone, (dY, X) pairs queued for the grouped launch
            wt2 = f.wt(p + "fc2.w")
            du = (G.matmul_nt_dgelu(dx3_c, wt2, u) if wt2 is not None
                  else G.matmul_nn_dgelu(dx3_c, f.w(p + "fc2.w"), u))
            self._wg(dx3_c, gact, p + "fc2")
            if not fc2b_fused:
                G.colsum(dx3, f.g(p + "fc2.b"), beta, red=red)
        else:
            # each Dense's dgrad and weight gradient share one launch (G.linear_backward), weight-gradient
            # reductions go to the layer's batched launch; with a transposed fc2 weight the paired dgrad
            # runs NT (+ GELU backward), both operands K-major
            du = G.linear_backward(dx3_c, f.w(p + "fc2.w"), gact, f.g(p + "fc2.w"), beta, red=red, dgelu_u=u,
                                   wt=f.wt(p + "fc2.w"))
            if not fc2b_fused:
                G.colsum(dx3, f.g(p + "fc2.b"), beta, red=red)
        # paired launches measured per Dense (in-step, us): fc2 44.1 vs 46.8 and qkv 35.6 vs 38.1
        # separate; fc1 48.7 vs 48.1 and out_proj 22.4 vs 21.7 -> those two stay separate
        wt1 = f.wt(p + "fc1.w")
        if self._fuse_bwd and wt1 is not None:
            # fc1 dgrad with the LN2 backward in its epilogue (+ out_proj.b's gradient), then fc1's
            # weight gradient
            dx2, dx2_c = LF.dgrad_ln_bwd(du, wt1, x2, f.p(p + "ln2.g"), mu2, rs2, dx3, f.g(p + "ln2.g"),
                                         f.g(p + "ln2.b"), beta, dbias=f.g(p + "out.b"), red=red,
                                         sync=self.ln_sync, site=self._ln_site(l, 0, True))
            self._wg(du, y2, p + "fc1", bias=True)
        else:
            dy2 = self._tp_reduce(self._dgrad_wgrad(du, p + "fc1", y2, beta, red, pair=False))
            dx2, dx2_c = self._ln_bwd(dy2, x2, p + "ln2", mu2, rs2, dx3, beta, bias_grad=p + "out.b")
        wto = f.wt(p + "out.w")
        if wto is not None:  # NT dgrad on the transposed weight, then the weight gradient
            do = G.linear(dx2_c, wto)
            self._wg(dx2_c, o, p + "out")
        elif self._defer_wg:
            do = G.matmul_nn(dx2_c, f.w(p + "out.w"), out_dtype=self.act_dtype)
            self._wg(dx2_c, o, p + "out")
        else:
            do = G.linear_backward(dx2_c, f.w(p + "out.w"), o, f.g(p + "out.w"), beta, red=red,
                                   out_dtype=self.act_dtype, pair=False)
        dqkv = A.attn_bwd(qkv.view(batch, T, -1), o.view(batch, T, -1), lse, do.view(batch, T, -1),
                          self.heads_local).view(batch * T, -1)
        wtq = f.wt(p + "qkv.w")
        if self._fuse_bwd and wtq is not None:
            bg = self._prev_fc2b(l)
            out = LF.dgrad_ln_bwd(dqkv, wtq, x, f.p(p + "ln1.g"), mu1, rs1, dx2, f.g(p + "ln1.g"), f.g(p + "ln1.b"),
                                  beta, dbias=None if bg is None else f.g(bg), red=red, sync=self.ln_sync,
                                  site=self._ln_site(l, 1, True))
            if dx_hook is not None:
                dx_hook(*out)
            self._wg(dqkv, y1, p + "qkv", bias=True)
            return out
        dy1 = self._tp_reduce(self._dgrad_wgrad(dqkv, p + "qkv", y1, beta, red, pair=True))
        out = self._ln_bwd(dy1, x, p + "ln1", mu1, rs1, dx2, beta, bias_grad=self._prev_fc2b(l))
        if dx_hook is not None:
            dx_hook(*out)
        return out

    # ------------------------------------------------------------------ sequence-parallel block
    def _row_parallel_sp(self, a, wname: str, resid, bias):
        """resid + bias + Σ_tp a·Wᵀ on this rank's rows (reduce-scatter); the partial is bf16 under
        ``tp_bf16``, else fp32, written by the GEMM straight into the P2P buffer when that path takes it."""
        w = self.flat.w(wname)
        rows, cols = a.shape[0], w.shape[0]
        dt = torch.bfloat16 if self.tp_bf16 else torch.float32
        dst = self.tp.partial_out_rows(rows, cols, dt, bias) if a.is_cuda else None
        if dst is not None:
            G.linear_into(a, w, dst)
            return self.tp.reduce_scatter_staged(rows, cols, dt, resid=resid, bias=bias, device=a.device)
        return self.tp.reduce_scatter_rows(G.linear(a, w, None, out_dtype=dt), resid=resid, bias=bias)

    def _tp_rs(self, d):
        """Reduce-scatter an input-gradient partial (the output of :meth:`_dgrad_wgrad`) to this rank's rows."""
        if isinstance(d, _Staged):
            return self.tp.reduce_scatter_staged(d.rows, d.cols, torch.bfloat16, device=d.device)
        return self.tp.reduce_scatter_rows(d)

    def _block_forward_sp(self, l: int, x: torch.Tensor, batch: int, ctx: Dict) -> torch.Tensor:
        self._await_params(l)
        f, p, tp = self.flat, f"h.{l}.", self.tp
        rows = x.shape[0] * tp.size
        T = rows // batch
        y1l, mu1, rs1 = LN.layernorm_fwd(x, f.p(p + "ln1.g"), f.p(p + "ln1.b"), self.eps, self.act_dtype)
        y1 = tp.all_gather_rows(y1l)
        qkv = G.linear(y1, f.w(p + "qkv.w"), f.p(p + "qkv.b"))
        o, lse = A.attn_fwd(qkv.view(batch, T, -1), self.heads_local)
        o = o.view(rows, -1)
        x2 = self._row_parallel_sp(o, p + "out.w", resid=x, bias=f.p(p + "out.b"))
        y2l, mu2, rs2 = LN.layernorm_fwd(x2, f.p(p + "ln2.g"), f.p(p + "ln2.b"), self.eps, self.act_dtype)
        y2 = tp.all_gather_rows(y2l)
        u, gact = G.linear_gelu(y2, f.w(p + "fc1.w"), f.p(p + "fc1.b"))
        x3 = self._row_parallel_sp(gact, p + "fc2.w", resid=x2, bias=f.p(p + "fc2.b"))
        ctx[l] = (x, y1, mu1, rs1, qkv, o, lse, x2, y2, mu2, rs2, u, gact, batch)
        return x3

    def _block_backward_sp(self, l: int, ctx: Dict, dx3: torch.Tensor, dx3_c: torch.Tensor, beta: float,
                           dx_hook=None):
        """dx3 (fp32, own rows) → (dx, dx_c) on the own rows.  The residual gradient is all-gathered in the
        compute dtype for the GEMMs, their input-gradient partials are reduce-scattered; the LayerNorm and
        row-parallel-bias grads come out as partials over the own rows (summed by :meth:`_sp_sum`)."""
        f, p, tp = self.flat, f"h.{l}.", self.tp
        x, y1, mu1, rs1, qkv, o, lse, x2, y2, mu2, rs2, u, gact, batch = ctx.pop(l)
        rows = y1.shape[0]
        T = rows // batch
        red = self.red
        fc2b_fused = l in self._bias_fused
        self._bias_fused.discard(l)
        self._beta = beta
        g3 = tp.all_gather_rows(dx3_c)
        if self._defer_wg:
            wt2 = f.wt(p + "fc2.w")
            du = (G.matmul_nt_dgelu(g3, wt2, u) if wt2 is not None
                  else G.matmul_nn_dgelu(g3, f.w(p + "fc2.w"), u))
            self._wg(g3, gact, p + "fc2")
        else:
            du = G.linear_backward(g3, f.w(p + "fc2.w"), gact, f.g(p + "fc2.w"), beta, red=red, dgelu_u=u,
                                   wt=f.wt(p + "fc2.w"))
        if not fc2b_fused:
            G.colsum(dx3, f.g(p + "fc2.b"), beta, red=red)
        dy2 = self._tp_rs(self._dgrad_wgrad(du, p + "fc1", y2, beta, red, pair=False))
        dx2, dx2_c = self._ln_bwd(dy2, x2, p + "ln2", mu2, rs2, dx3, beta, bias_grad=p + "out.b")
        g2 = tp.all_gather_rows(dx2_c)
        wto = f.wt(p + "out.w")
        if wto is not None:
            do = G.linear(g2, wto)
            self._wg(g2, o, p + "out")
        elif self._defer_wg:
            do = G.matmul_nn(g2, f.w(p + "out.w"), out_dtype=self.act_dtype)
            self._wg(g2, o, p + "out")
        else:
            do = G.linear_backward(g2, f.w(p + "out.w"), o, f.g(p + "out.w"), beta, red=red,
                                   out_dtype=self.act_dtype, pair=False)
        dqkv = A.attn_bwd(qkv.view(batch, T, -1), o.view(batch, T, -1), lse, do.view(batch, T, -1),
                          self.heads_local).view(rows, -1)
        dy1 = self._tp_rs(self._dgrad_wgrad(dqkv, p + "qkv", y1, beta, red, pair=True))
        out = self._ln_bwd(dy1, x, p + "ln1", mu1, rs1, dx2, beta, bias_grad=self._prev_fc2b(l))
        if dx_hook is not None:
            dx_hook(*out)
        return out

    def _row_parallel(self, a, wname: str, resid, bias):
        """fp32 ``resid + bias + Σ_tp a·Wᵀ`` with a bf16 partial (``tp_bf16``): the GEMM writes the partial
        straight into this rank's P2P buffer half (no stage copy) when the P2P path takes it."""
        w = self.flat.w(wname)
        dst = self.tp.partial_out(a.shape[0], w.shape[0], bias)
        if dst is not None:
            G.linear_into(a, w, dst)
            return self.tp.reduce_staged(a.shape[0], w.shape[0], resid=resid, bias=bias, device=a.device)
        return self.tp.reduce_to(G.linear(a, w, None, out_dtype=torch.bfloat16), resid=resid, bias=bias)

    def _tp_reduce(self, d):
        """All-reduce an input-gradient partial over the TP group (in place for fp32 payloads; with
        ``tp_bf16`` ``d`` is the bf16 partial -- or a ``_Staged`` marker when the dgrad wrote it into the
        P2P buffer -- and a new fp32 sum comes back)."""
        if isinstance(d, _Staged):
            return self.tp.reduce_staged(d.rows, d.cols, device=d.device)
        if self.tp.size == 1:
            return d
        if d.dtype == torch.bfloat16 and self.tp_bf16:
            return self.tp.reduce_to(d)
        return self.tp.all_reduce_(d)

    def _dgrad_wgrad(self, dy, dense: str, x, beta, red, pair: bool):
        """dX = dY·W (fp32) and dW/db of a Dense with a bias.  With the transposed weight mirror
        (``flat.wt``) the dgrad is an NT GEMM on W^T followed by the weight gradient; otherwise the
        NN dgrad (paired with the weight gradient in one launch when ``pair``)."""
        f = self.flat
        wt = f.wt(dense + ".w")
        if self._defer_wg:
            if self.tp_bf16 and self.tp.size > 1:  # bf16 partial for the bf16-payload all-reduce
                rows, cols = dy.shape[0], (wt.shape[0] if wt is not None else f.w(dense + ".w").shape[1])
                dst = self.tp.partial_out(rows, cols)
                if dst is not None:  # straight into this rank's P2P buffer half (no stage copy)
                    if wt is not None:
                        G.linear_into(dy, wt, dst)
                    else:
                        G.matmul_nn_into(dy, f.w(dense + ".w"), dst)
                    dx = _Staged(rows, cols, dy.device)
                else:
                    dx = (G.linear(dy, wt, out_dtype=torch.bfloat16) if wt is not None
                          else G.matmul_nn(dy, f.w(dense + ".w"), out_dtype=torch.bfloat16))
            else:
                dx = G.linear_resid(dy, wt, None, None) if wt is not None else G.matmul_nn(dy, f.w(dense + ".w"))
            self._wg(dy, x, dense, bias=True)
            return dx
        if wt is None:
            return G.linear_backward(dy, f.w(dense + ".w"), x, f.g(dense + ".w"), beta, red=red, db=f.g(dense + ".b"),
                                     pair=pair)
        dx = G.linear_resid(dy, wt, None, None)
        G.wgrad(dy, x, f.g(dense + ".w"), beta, red=red, db=f.g(dense + ".b"))
        return dx

    def _prev_fc2b(self, l: int):
        """fc2.b of the block feeding layer l's input, if this stage owns it (its grad = Σ_rows dx)."""
        if (l - 1) in self.layout.layers:
            self._bias_fused.add(l - 1)
            return f"h.{l - 1}.fc2.b"
        return None

    def _ln_bwd(self, dy, x, ln: str, mu, rs, dres, beta, bias_grad: Optional[str] = None):
        f = self.flat
        dx_c = None if self.act_dtype == torch.float32 else torch.empty(dy.shape, dtype=self.act_dtype,
                                                                        device=dy.device)
        dx = LN.layernorm_bwd(dy, x, f.p(ln + ".g"), mu, rs, dres, f.g(ln + ".g"), f.g(ln + ".b"), beta,
                              out_c=dx_c, dbias=None if bias_grad is None else f.g(bias_grad), red=self.red)
        return dx, (dx if dx_c is None else dx_c)

    def stage_forward(self, x: torch.Tensor, batch: int, ctx: Dict) -> torch.Tensor:
        for l in self.layout.layers:
            x = self.block_forward(l, x, batch, ctx)
        return x

    # ------------------------------------------------------------------ head
    def head_forward(self, x: torch.Tensor, labels: torch.Tensor, loss_scale: float, ctx: Dict,
                     loss_out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
        """Final LN + lm_head + CE (GPTModel.py:69-74; create_train_step.py:32-34).

        Returns a device scalar ``loss_scale · Σ_tokens CE`` (1-element fp32 tensor)."""
        self._await_params("head")
        f = self.flat
        pre = ctx.pop("lnf_pre", None)  # produced by the last layer's fc2 GEMM (fused LayerNorm)
        yf, muf, rsf = pre if pre is not None else LN.layernorm_fwd(x, f.p("lnf.g"), f.p("lnf.b"), self.eps,
                                                                     self.act_dtype)
        if self.sp:
            yf = self.tp.all_gather_rows(yf)  # the vocab-parallel lm_head reads every row
        lab = labels.reshape(-1)
        tp1 = self.tp.size == 1
        if _CE_CHUNK > 0 and self.v_local > _CE_CHUNK:
            return self._head_forward_chunked(x, yf, muf, rsf, lab, loss_scale, ctx, loss_out, accumulate)
        logits, rowstat, lab_logit = X.lmhead_logits_partials(yf, f.w("lm_head.w"), f.p("lm_head.b"), lab,
                                                              self.v_start, self.v_valid, combine=not tp1)
        if not tp1:
            rowstats = self.tp.all_gather_stack(rowstat)  # [tp, M, 2]
            self.tp.all_reduce_(lab_logit)
        else:
            rowstats = rowstat  # the GEMM's per-tile partials [P, M, 2]: combined once, in ce_finalize
        lse, loss = X.ce_finalize(rowstats, lab_logit, loss_scale, loss_out, accumulate)
        ctx["head"] = (x, yf, muf, rsf, logits, lse, lab)
        return loss

    # ------------------------------------------------------------------ head split over two pipeline stages
    def head_split_logits(self, x: torch.Tensor, labels: torch.Tensor, ctx: Dict) -> torch.Tensor:
        """``pp_head_split``: this stage's vocab half of lm_head + CE.  Part 0 normalises its stage output
        ``x`` (lnf) and sends the result to part 1 (:meth:`head_split_input`); part 1 gets that as ``x``.
        Computes the half's logits and per-row CE partials; returns them packed ``[M, 3]`` (max, Σexp,
        label logit) for the exchange with the other half."""
        self._await_params("head")
        f = self.flat
        lab = labels.reshape(-1)
        if self.layout.head_part[0] == 0:
            x, yf, muf, rsf = ctx.pop("head_yf")
        else:
            yf, muf, rsf = x, None, None
        logits, rowstat, lab_logit = X.lmhead_logits_partials(yf, f.w("lm_head.w"), f.p("lm_head.b"), lab,
                                                              self.v_start, self.v_valid, combine=True)
        stats = torch.cat([rowstat, lab_logit[:, None]], 1).contiguous()
        ctx["head"] = (x, yf, muf, rsf, logits, None, lab)
        ctx["head_stats"] = stats
        return stats

    def head_split_input(self, x: torch.Tensor, ctx: Dict) -> torch.Tensor:
        """Part 0: the final LayerNorm of the stage output -- the message to part 1 (compute dtype)."""
        f = self.flat
        self._await_params("head")
        yf, muf, rsf = LN.layernorm_fwd(x, f.p("lnf.g"), f.p("lnf.b"), self.eps, self.act_dtype)
        ctx["head_yf"] = (x, yf, muf, rsf)
        return yf

    def head_split_finalize(self, ctx: Dict, other: torch.Tensor, loss_scale: float,
                            loss_out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
        """Combine both halves' row statistics (in part order, so both stages get the identical lse and
        loss) into the loss and the lse the backward needs."""
        mine = ctx.pop("head_stats")
        a, b = (mine, other) if self.layout.head_part[0] == 0 else (other, mine)
        rowstats = torch.stack([a[:, :2], b[:, :2]]).contiguous()
        lse, loss = X.ce_finalize(rowstats, (a[:, 2] + b[:, 2]).contiguous(), loss_scale, loss_out, accumulate)
        x, yf, muf, rsf, logits, _, lab = ctx["head"]
        ctx["head"] = (x, yf, muf, rsf, logits, lse, lab)
        return loss

    def _chunks(self):
        """(column offset, columns, valid columns) of each lm_head vocab chunk of this rank's shard."""
        out = []
        for c0 in range(0, self.v_local, _CE_CHUNK):
            vc = min(_CE_CHUNK, self.v_local - c0)
            out.append((c0, vc, max(0, min(vc, self.v_valid - c0))))
        return out

    def _head_forward_chunked(self, x, yf, muf, rsf, lab, loss_scale, ctx, loss_out, accumulate):
        """Vocab-chunked lm_head + CE forward (DTC_CE_CHUNK): per chunk, the lm_head GEMM with the CE
        partials epilogue into a chunk-sized logits buffer that is dropped right away; the rows'
        (max, sum exp) of every chunk are combined like vocab-parallel shards (``ce_finalize``)."""
        f = self.flat
        w, b = f.w("lm_head.w"), f.p("lm_head.b")
        stats, lab_logit = [], None
        for c0, vc, nv in self._chunks():
            _, rs, ll = X.lmhead_logits_partials(yf, w[c0:c0 + vc], b[c0:c0 + vc], lab, self.v_start + c0, nv,
                                                 combine=True)
            stats.append(rs)
            lab_logit = ll if lab_logit is None else lab_logit + ll
        rowstat = torch.stack(stats)  # [chunks, M, 2]
        if self.tp.size > 1:
            # each rank's chunks combined first, then the shards (as the unchunked vocab-parallel path)
            lse_l, _ = X.ce_finalize(rowstat, torch.zeros_like(lab_logit), 0.0)
            one = torch.stack([lse_l, torch.ones_like(lse_l)], -1)  # (max = lse, sum exp = 1) per shard
            rowstat = self.tp.all_gather_stack(one)
            self.tp.all_reduce_(lab_logit)
        lse, loss = X.ce_finalize(rowstat.contiguous(), lab_logit, loss_scale, loss_out, accumulate)
        ctx["head"] = (x, yf, muf, rsf, None, lse, lab)
        return loss

    def _head_backward_chunked(self, x, yf, muf, rsf, lse, lab, grad_scale, beta):
        f = self.flat
        w, b = f.w("lm_head.w"), f.p("lm_head.b")
        wt = f.wt("lm_head.w")
        gw, gb = f.g("lm_head.w"), f.g("lm_head.b")
        red = self.red
        dyf = None
        for c0, vc, nv in self._chunks():
            logits, _, _ = X.lmhead_logits_partials(yf, w[c0:c0 + vc], b[c0:c0 + vc], lab, self.v_start + c0, nv,
                                                    combine=True)  # recompute (pad columns -inf)
            dl, cp = X.ce_backward_inplace(logits, lse, lab, self.v_start + c0, nv, grad_scale, colpart=True)
            if wt is not None:
                dyf = G.linear_resid(dl, wt[:, c0:c0 + vc], None, dyf, out=dyf)
            else:
                part = G.matmul_nn(dl, w[c0:c0 + vc])
                dyf = part if dyf is None else dyf.add_(part)
            G.wgrad(dl, yf, gw[c0:c0 + vc], beta, red=red)
            G.colsum(cp, gb[c0:c0 + vc], beta, red=red)
            self.flush_reductions()  # this chunk's split-K slabs: the reducer arena is reused by the next
            del logits, dl, cp
        dyf = self._head_dx(dyf)
        last = self.layout.layers[-1] + 1 if len(self.layout.layers) else None
        out = self._ln_bwd(dyf, x, "lnf", muf, rsf, None, beta,
                           bias_grad=None if last is None else self._prev_fc2b(last))
        self.flush_reductions()
        self._sp_sum(["head"])
        return out

    def _head_dx(self, dyf):
        """The lm_head input gradient summed over the vocab shards: all-reduced, or under sequence
        parallelism reduce-scattered to the own rows (``dyf`` a tensor or a :class:`_Staged` bf16 partial)."""
        if self.sp:
            return self._tp_rs(dyf)
        return self._tp_reduce(dyf)

    def _head_dgrad(self, dlogits, wt):
        """dlogits·W, the lm_head input gradient of this rank's vocab shard.  Under ``tp_bf16`` (tp > 1, no
        head split) the partial is written as bf16 straight into the P2P buffer -- the shard sum then moves
        half the bytes (GPT-2 small at tp 8: 12.6 instead of 25.2 MB per step) -- when the shard's K is short
        enough that the fp32 output would not have taken the split-K 256^2 plan anyway (K < 16384: tp >= 4
        at GPT-2 small's vocab; at tp 2 the bf16-output plan would cost more GEMM time than the bytes save)."""
        f = self.flat
        w = f.w("lm_head.w")
        rows, cols = dlogits.shape[0], (wt.shape[0] if wt is not None else w.shape[1])
        if (self.tp_bf16 and self.tp.size > 1 and dlogits.is_cuda and self.layout.head_part[1] == 1
                and dlogits.shape[1] < _HEAD_BF16_MAXK):
            dst = self.tp.partial_out(rows, cols)
            if dst is not None:
                if wt is not None:
                    G.linear_into(dlogits, wt, dst)
                else:
                    G.matmul_nn_into(dlogits, w, dst)
                self.head_dgrad_staged += 1  # (tests: the bf16 path ran)
                return _Staged(rows, cols, dlogits.device)
        return G.linear_resid(dlogits, wt, None, None) if wt is not None else G.matmul_nn(dlogits, w)

    def head_backward(self, ctx: Dict, grad_scale: float, beta: float, extra_dyf: Optional[torch.Tensor] = None):
        """lm_head + CE backward, then the final LayerNorm's.  ``pp_head_split``: part 1 returns its half's
        input-gradient partial ``(dyf, None)`` (no LayerNorm: part 0 holds it); part 0 adds the other half's
        partial ``extra_dyf`` before the LayerNorm backward."""
        f = self.flat
        x, yf, muf, rsf, logits, lse, lab = ctx.pop("head")
        if logits is None:  # vocab-chunked head (DTC_CE_CHUNK)
            return self._head_backward_chunked(x, yf, muf, rsf, lse, lab, grad_scale, beta)
        wt = f.wt("lm_head.w")  # transposed mirror: NT split-K dgrad, both operands K-major
        red = self.red
        fused = _ce_fused(x.shape[0], x.shape[1])
        if wt is not None and fused and logits.is_cuda:
            # CE backward fused into the dgrad's operand staging (no separate dlogits pass)
            dyf, dlogits, colp = X.ce_dgrad_fused(logits, lse, lab, self.v_start, self.v_valid, grad_scale, wt)
        else:
            # one pass: dlogits in place + column partials of it (the bias gradient's input)
            dlogits, colp = X.ce_backward_inplace(logits, lse, lab, self.v_start, self.v_valid, grad_scale,
                                                  colpart=True)
            # dgrad first (critical path), then the weight gradient: both lm_head GEMMs run the 256^2
            # kernel at one block per CU, so issuing them concurrently only time-slices the CUs
            dyf = self._head_dgrad(dlogits, wt)
        # the bias gradient from the CE pass's fp32 column partials
        G.colsum(colp, f.g("lm_head.b"), beta, red=red)
        if self._defer_wg:
            # the weight gradient joins the grouped launch (its 591 tiles at GPT-2 small fill the layers'
            # last round)
            self.wg_queue.append((dlogits, yf, f.g("lm_head.w"), None))
            wg = None
        else:  # after the lnf backward (off the input-gradient chain)
            wg = lambda dl=dlogits, y=yf: G.wgrad(dl, y, f.g("lm_head.w"), beta, red=red)  # noqa: E731
        del logits, dlogits
        part, parts = self.layout.head_part
        if parts > 1:
            if part == 1:  # the partial goes to part 0's stage
                if wg is not None:
                    wg()
                self.flush_reductions()
                return dyf, None
            dyf.add_(extra_dyf)
        else:
            dyf = self._head_dx(dyf)
        last = self.layout.layers[-1] + 1 if len(self.layout.layers) else None
        out = self._ln_bwd(dyf, x, "lnf", muf, rsf, None, beta,
                           bias_grad=None if last is None else self._prev_fc2b(last))
        if wg is not None:
            wg()
        self.flush_reductions()
        self._sp_sum(["head"])
        return out

    def flush_reductions(self):
        """Launch the batched reductions queued since the last flush (no-op without a reducer)."""
        if self.red is not None:
            self.red.flush()

    def take_wgrads(self):
        """Hand over the queued weight gradients (zero-bubble pipeline: the W item of a microbatch runs
        them later, :meth:`run_wgrads`); the queue is empty afterwards."""
        q, self.wg_queue = self.wg_queue, []
        return q

    def run_wgrads(self, q, beta: float):
        """The W item of a microbatch: its queued weight gradients (+ fused bias gradients) as one grouped
        launch, accumulated into the grads with ``beta`` (0 for the first W of the step)."""
        self.wg_queue = list(q)
        self.flush_wgrads(beta)
        self.flush_reductions()

    def stage_backward(self, ctx: Dict, dx: torch.Tensor, dx_c: torch.Tensor, beta: float, hook=None, dx_hook=None,
                       keep_wgrads: bool = False):
        """Backward over this stage's layers (reverse); ``hook(l)`` fires after layer l's grads exist,
        ``dx_hook(dx, dx_c)`` as soon as the stage's input gradient is final (inside the first layer).
        ``keep_wgrads`` (deferred weight gradients only): the input-gradient chain (B) alone -- the weight
        gradients stay queued for :meth:`take_wgrads` (the zero-bubble pipeline's W item)."""
        if keep_wgrads and not self._defer_wg:
            raise ValueError("keep_wgrads needs deferred weight gradients (wgrad_group >= 0)")
        first = self.layout.layers[0] if len(self.layout.layers) else None
        waiting = []  # layers whose weight gradients are still queued (deferred mode)
        for l in reversed(list(self.layout.layers)):
            dx, dx_c = self.block_backward(l, ctx, dx, dx_c, beta, dx_hook=dx_hook if l == first else None)
            if self._defer_wg:
                waiting.append(l)
                if keep_wgrads:
                    if l == first:
                        self.flush_reductions()  # the B part's LayerNorm / bias partials
                    continue
                if l == first or (self.wg_group > 0 and len(waiting) >= self.wg_group):
                    self.flush_wgrads(beta)
                    self.flush_reductions()  # the group's grads are final after these launches
                    self._sp_sum(waiting)
                    if hook is not None:
                        for ll in waiting:
                            hook(ll)
                    waiting = []
                elif not _RED_BATCH_LAYERS:
                    self.flush_reductions()  # this layer's LayerNorm / bias partials
                continue
            self.flush_reductions()  # layer l's grads are final after this launch
            self._sp_sum([l])
            if hook is not None:
                hook(l)
        if self.wg_queue and not keep_wgrads:  # a stage without layers: the lm_head's weight gradient alone
            self.flush_wgrads(beta)
            self.flush_reductions()
        return dx, dx_c


def full_forward_loss(stage: GPTStage, ids, labels, step, row0: int = 0, ctx: Optional[Dict] = None):
    """Convenience: embed → all layers → head (single-stage layout), returns (loss, ctx)."""
    ctx = {} if ctx is None else ctx
    b, T = ids.shape
    h = stage.embed_forward(ids, step, row0, ctx)
    h = stage.stage_forward(h, b, ctx)
    loss = stage.head_forward(h, labels, 1.0 / (b * T), ctx)
    return loss, ctx
