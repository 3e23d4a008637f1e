"""Training engine: one rank's model shard, flat buffers, optimizer and the step program.

Reference counterparts: the DP/TP jitted step (``train/create_train_step.py:24-52``), the
PP pmap/scan step (``:55-195``) and the state plumbing of ``train/train.py:22-233``.
One class serves every layout (DP, TP, PP and their products): the mesh decides which
layers/params this rank owns and which collectives run; the step itself is a static
sequence of HIP kernels + RCCL calls that :class:`StepProgram` captures into hipGraph
segments after the first eager warmup step.
"""

from __future__ import annotations

import math
import os
import warnings
from dataclasses import replace
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..config.schema import ModelConfig, OptimConfig, TrainConfig
from ..models.gpt import GPTStage, StageLayout
from ..models.params import stage_param_specs
from ..ops import embedding as E
from ..ops import gemm as G
from ..ops import optim as O
from ..parallel.buffers import FlatParams
from ..parallel.dist import DistInfo
from ..parallel.dp import GradBuckets
from ..parallel.mesh import Mesh, build_mesh, head_cost_blocks, resolve_degrees, split_layers
from ..parallel.program import StepProgram, csig
from ..parallel.tp import TPComm
from .optimizer import FusedAdamW, ShardedAdamW


class Engine:
    def __init__(self, model_cfg: ModelConfig, train_cfg: TrainConfig, opt_cfg: OptimConfig, dinfo: DistInfo):
        self.mcfg, self.tcfg, self.ocfg = model_cfg, train_cfg, opt_cfg
        self.dinfo = dinfo
        self.device = dinfo.device
        dp, tp, pp = resolve_degrees(train_cfg.parallel, dinfo.world, train_cfg.dp, train_cfg.tp, train_cfg.pp)
        # lm_head + CE split by vocab over the last two pipeline stages (models/gpt.py head_split_*): auto when
        # the head alone outweighs an even share of the model (GPT-2 small at pp >= 5: 2.9 blocks vs 14.9 / pp)
        hsplit = train_cfg.pp_head_split
        hc_auto = head_cost_blocks(model_cfg) if train_cfg.pp_head_cost is None else float(train_cfg.pp_head_cost)
        if hsplit is None:
            hsplit = (pp >= 4 and tp == 1 and train_cfg.pp_schedule in ("1f1b", "zb")
                      and hc_auto > (model_cfg.n_layers + hc_auto) / pp)
        if hsplit and (pp < 2 or train_cfg.pp_schedule not in ("1f1b", "zb") or tp > 1):
            raise ValueError("pp_head_split needs pp >= 2, tp == 1 and the 1f1b or zb schedule")
        self.pp_head_split = bool(hsplit)
        if self.pp_head_split and model_cfg.padded_vocab % 128:
            # each half a multiple of 64 columns
            model_cfg = replace(model_cfg, vocab_pad_multiple=math.lcm(max(1, int(model_cfg.vocab_pad_multiple)), 128))
            self.mcfg = model_cfg
        if tp > 1:
            # every TP rank's vocab shard a multiple of 64 columns (the GEMM K-steps of the lm_head dgrad and
            # the 64-wide CE tiles): pad the vocab to a multiple of 64 * tp (GPT-2 at tp = 8: 50688 instead
            # of 50304 = 8 x 6288).  Pad rows are zero and masked, and the valid rows' canonical init does not
            # depend on the padded length, so every layout still trains the same model.
            mult = math.lcm(max(1, int(model_cfg.vocab_pad_multiple)), 64 * tp)
            if mult != model_cfg.vocab_pad_multiple:
                model_cfg = replace(model_cfg, vocab_pad_multiple=mult)
                self.mcfg = model_cfg
        rehearse = bool(train_cfg.dp_comm_rehearsal and dp == 1 and dist.is_available() and dist.is_initialized())
        self.mesh: Mesh = build_mesh(dinfo.rank, dinfo.world, dp, tp, pp, dp_group_always=rehearse)
        m = self.mesh
        # the DP code path (bucketed all-reduces, embedding gather, loss all-reduce, ZeRO-1 collectives) runs
        # when there is more than one replica -- or, as a rehearsal, on a one-member DP group
        self.dp_comm = dp > 1 or (rehearse and m.dp_group is not None)
        on_gpu = self.device.type == "cuda"
        self.act_dtype = torch.bfloat16 if (on_gpu and train_cfg.dtype == "bf16") else torch.float32

        # ---- batch geometry (reference: `batch` is the global batch, train_config_*.yaml:1)
        T = model_cfg.max_seq_len
        self._D = model_cfg.d_model
        self.T = T
        self.global_batch = train_cfg.batch
        if self.global_batch % dp:
            raise ValueError(f"global batch {self.global_batch} not divisible by dp={dp}")
        self.b_local = self.global_batch // dp
        self.n_micro = max(1, train_cfg.pp_microbatches) if pp > 1 else 1
        if self.b_local % self.n_micro:
            raise ValueError(f"local batch {self.b_local} not divisible by pp_microbatches={self.n_micro}")
        self.mb_rows = self.b_local // self.n_micro
        self.row0 = m.dp_idx * self.b_local

        # ---- ownership
        if train_cfg.pp_schedule not in ("gpipe", "1f1b", "zb"):
            raise ValueError(f"pp_schedule={train_cfg.pp_schedule!r}: expected 'gpipe', '1f1b' or 'zb'")
        if train_cfg.pp_split not in ("cost", "even"):
            raise ValueError(f"pp_split={train_cfg.pp_split!r}: expected 'cost' or 'even'")
        weights = None
        if pp > 1 and train_cfg.pp_split == "cost":
            hc = train_cfg.pp_head_cost
            weights = (0.05, head_cost_blocks(model_cfg) if hc is None else float(hc))
        hstages = 2 if self.pp_head_split else 1
        if hstages == 2 and weights is None:
            weights = (0.0, 0.0)  # even split over the stages before the head halves
        layer_ranges = split_layers(model_cfg.n_layers, pp, weights, head_stages=hstages)
        self.layer_ranges = layer_ranges
        head_stage = m.pp_idx >= pp - hstages
        self.layout = StageLayout(layer_ranges[m.pp_idx], has_embed=m.pp_idx == 0, has_head=head_stage,
                                  head_part=(m.pp_idx - (pp - 2), 2) if hstages == 2 and head_stage else (0, 1))
        specs = stage_param_specs(model_cfg, self.layout.layers, self.layout.has_embed, self.layout.has_head,
                                  head_part=self.layout.head_part)
        self.flat = FlatParams(specs, m.tp_idx, tp, self.device, compute_dtype=self.act_dtype)
        if self.act_dtype == torch.bfloat16 and os.environ.get("DTC_DGRAD_NT", "1") == "1":
            # Dense / lm_head dgrads as NT GEMMs on a transposed bf16 weight copy (buffers.enable_transposed)
            # (fc2's dgrad + dGELU runs NN on the row-major weight: level with the NT form on a mirror,
            # profiles/r5_gemm8r.md, so fc2 needs no transposed copy)
            dense = ["fc1", "qkv", "out"]
            head = ["lm_head.w"] if os.environ.get("DTC_DGRAD_NT_HEAD", "1") == "1" else []
            self.flat.enable_transposed([f"h.{l}.{n}.w" for l in self.layout.layers for n in dense] + head)
        self.flat.init_canonical(train_cfg.seed)

        # ---- step program, comms, model, optimizer
        cap = train_cfg.capture_comms
        if cap is None:
            # auto: captured on a one-rank RCCL group (the rehearsal, where it was measured: -0.23 ms) and
            # wherever DTC_CAPTURE_COMMS=1 asks for it; a multi-rank step cuts its graph at each collective
            # (the eager path) until capture has run against real peers over xGMI -- an RCCL kernel that
            # misbehaves inside a capture costs the whole run, an eager one a fraction of a millisecond
            env = os.environ.get("DTC_CAPTURE_COMMS", "auto")
            cap = dinfo.backend == "nccl" and (env == "1" or (env == "auto" and dinfo.world == 1))
        self.program = StepProgram(self.device, use_graph=train_cfg.use_graph and on_gpu, capture_comms=cap)
        # gloo on GPU tensors (the one-GPU multi-rank rig): collectives complete where they are issued,
        # so no copy-back from gloo's worker thread can queue behind a later cross-process wait
        # (parallel/dist.py explains the ordering argument)
        self.program.sync_comms = bool(on_gpu and dinfo.backend == "gloo" and (dinfo.world > 1 or self.dp_comm))
        self.p2p = None
        mode = train_cfg.tp_comm
        if tp > 1 and on_gpu and (mode == "p2p" or (mode == "auto" and dinfo.backend == "nccl")):
            from ..parallel.p2p import P2PAllReduce

            rows = self.mb_rows if pp > 1 else self.b_local
            self.p2p = P2PAllReduce(m.tp_group, m.tp_idx, tp, self.device, rows * T * model_cfg.d_model * 4)
        self.tp_comm = TPComm(m.tp_group, tp, m.tp_idx, self.program, p2p=self.p2p)
        self.stage = GPTStage(model_cfg, self.flat, self.layout, self.tp_comm, dropout_seed=train_cfg.seed,
                              act_dtype=self.act_dtype)
        tcd = train_cfg.tp_comm_dtype
        if tcd not in ("fp32", "bf16", "auto"):
            raise ValueError(f"tp_comm_dtype={tcd!r}: expected 'fp32', 'bf16' or 'auto'")
        if tcd == "auto":
            tcd = "bf16" if self.act_dtype == torch.bfloat16 else "fp32"
        self.tp_comm_dtype = tcd
        self.stage.tp_bf16 = bool(tp > 1 and tcd == "bf16")
        sp = train_cfg.tp_sequence_parallel
        if sp is None:  # auto: wherever it applies
            sp = tp > 1 and pp == 1 and self.b_local % tp == 0
        if sp:
            if tp == 1:
                if dinfo.rank == 0:
                    warnings.warn("tp_sequence_parallel ignored: tp == 1")
            elif pp > 1:
                raise ValueError("tp_sequence_parallel needs pp == 1 (one stage holds the embedding and the head)")
            elif not self.stage.enable_sequence_parallel(self.b_local):
                raise ValueError(f"tp_sequence_parallel: the local batch {self.b_local} must split into whole "
                                 f"sequences over tp={tp}")
        # deferred grouped weight gradients (models/gpt.py set_wgrad_group): all layers + the lm_head in
        # one launch when no collective waits on per-layer grads (dp == 1), else groups of wgrad_group
        # layers so each group's DP buckets go out under the next group's backward
        wg = train_cfg.wgrad_group
        if wg is None:
            wg = 0 if not self.dp_comm else 2
            if wg == 0:
                wg = self._wgrad_group_for_memory(model_cfg, len(self.layout.layers))
        if pp > 1 and train_cfg.pp_schedule == "zb" and wg < 0:
            # the zero-bubble schedule runs each microbatch's weight gradients (W) apart from its
            # input-gradient chain (B): that needs the deferred grouped path.  Refused here, before any
            # collective, instead of inside the first backward (where only some ranks would raise)
            raise ValueError("pp_schedule='zb' needs deferred weight gradients: wgrad_group >= 0 (or unset)")
        self.stage.set_wgrad_group(wg)
        # DP embedding-grad gather (pp == 1): instead of all-reducing the dense wte/wpe grads
        # (103 MB fp32 for the reference vocab, issued last -> fully exposed), all-gather the
        # embedding-output grads (b_local*T*D fp32 per rank) and let every rank rebuild the
        # identical wte/wpe grads from the global batch with the deterministic sorted kernel.
        if train_cfg.zero_stage not in (0, 1):
            raise ValueError(f"zero_stage={train_cfg.zero_stage}: only 0 (replicated Adam state) and 1 (ZeRO-1) "
                             "are implemented")
        self.zero = bool(train_cfg.zero_stage == 1 and self.dp_comm)
        if self.zero and (tp > 1 or pp > 1):
            raise ValueError("zero_stage=1 is implemented for pure data parallelism (tp = pp = 1)")
        if train_cfg.zero_stage == 1 and not self.dp_comm and dinfo.rank == 0:
            warnings.warn("zero_stage=1 ignored: dp == 1 (nothing to shard); running the replicated AdamW")
        if self.zero and train_cfg.defer_optimizer and dinfo.rank == 0:
            warnings.warn("defer_optimizer ignored under zero_stage=1 (the sharded update ends the step)")
        if self.zero and train_cfg.dp_grad_dtype == "bf16" and dinfo.rank == 0:
            warnings.warn("dp_grad_dtype=bf16 ignored under zero_stage=1: ShardedAdamW reduce-scatters the fp32 grads")
        if self.stage.tp_bf16 and self.stage.wg_group < 0 and dinfo.rank == 0:
            warnings.warn("tp_comm_dtype=bf16 with wgrad_group=-1: the row-parallel "
                          "partials travel as bf16, the input-gradient partials stay fp32")
        self.embed_gather = bool(self.dp_comm and pp == 1 and train_cfg.dp_embed_gather and self.layout.has_embed
                                 and not self.zero and not self.stage.sp)
        bnd = None
        if pp == 1 and len(self.layout.layers):
            names = list(self.flat.slots)
            ends = [self.flat.range_of([n for n in names if n.startswith(f"h.{l}.")])[1] for l in self.layout.layers]
            head = [n for n in names if n.startswith("lm_head") or n.startswith("lnf")]
            bnd = ends + ([self.flat.range_of(head)[1]] if head else [])
        self.buckets = GradBuckets(self.flat, m.dp_group, dp, self.program, train_cfg.dp_bucket_mb,
                                   tail_mb=train_cfg.dp_tail_mb,
                                   local_names=("wte", "wpe") if self.embed_gather else (), boundaries=bnd,
                                   payload=train_cfg.dp_grad_dtype, active=self.dp_comm)
        if self.zero:
            self.opt = ShardedAdamW(self.flat, opt_cfg, self.program, m.dp_group, dp, m.dp_idx)
        else:
            self.opt = FusedAdamW(self.flat, opt_cfg, self.program, tp, m.tp_group, m.pp_group,
                                  pp_global_clip=(train_cfg.pp_clip == "global"))
        self.opt.reducer = self.stage.red
        if not self.zero:
            self.opt.tp_comm = self.tp_comm
        if pp == 1 and not self.zero:
            # incremental Σg²: with dp == 1 each layer's grads are final when its backward ends
            # (norm chunk per layer, in the layer's batched reduction launch); with dp > 1 only the locally
            # built embedding grads are final before the all-reduces finish
            if not self.dp_comm:
                bk = self.buckets
                cuts = [bk.head_end_offset()] + [bk.layer_end_offset(l) for l in reversed(self.layout.layers)]
                self.opt.set_chunks(sorted(set(c for c in cuts if 0 < c < self.flat.numel)) + [self.flat.numel])
                # the grouped weight-gradient launch also emits its tiles' Σ dW² (the final grads at
                # dp == 1), so the norm pass skips ~3/4 of the grads (DTC_FUSED_NORM=0: off)
                self.stage.wg_record = (on_gpu and self.stage.wg_group == 0 and self.act_dtype == torch.bfloat16
                                        and os.environ.get("DTC_FUSED_NORM", "1") == "1")
            elif self.embed_gather:
                self.opt.set_chunks([self.buckets.reduce_end, self.flat.numel])
        if on_gpu and pp == 1 and self._emb_fused_norm():
            # one local embedding backward per step writes the wte grad: zero only the rows the previous step
            # wrote instead of the 154 MB table (GPT-2 small)
            self.stage.emb_prev = torch.zeros(self.b_local * self.T, dtype=torch.int32, device=self.device)

        # ---- static device-side inputs/outputs (graph replay reads/writes these)
        D = model_cfg.d_model
        if self.embed_gather:
            self.ids_all = torch.zeros(self.global_batch, T, dtype=torch.int32, device=self.device)
            self.ids = self.ids_all[self.row0:self.row0 + self.b_local]  # contiguous row view
            self.dh_all = torch.zeros(self.global_batch * T, D, dtype=torch.float32, device=self.device)
            # dp_grad_dtype: bf16 -> the gather moves the bf16 copy the LayerNorm backward already wrote (half the
            # bytes: 100 MB instead of 201 MB per step at dp8, GPT-2 small), widened once before the backward
            self.dh_all_bf = (torch.zeros(self.global_batch * T, D, dtype=torch.bfloat16, device=self.device)
                              if train_cfg.dp_grad_dtype == "bf16" and self.act_dtype == torch.bfloat16 else None)
            self.feed_row0, self.feed_rows = 0, self.global_batch
        else:
            self.ids = torch.zeros(self.b_local, T, dtype=torch.int32, device=self.device)
            self.feed_row0, self.feed_rows = self.row0, self.b_local
        self.labels = torch.zeros(self.b_local, T, dtype=torch.int32, device=self.device)
        pin = on_gpu
        self._host = [torch.zeros(2, self.feed_rows, T, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._host_i = 0
        self._staged_slot = None  # pinned slot holding the batch stage_batch prepared, until upload_batch
        # the embedding backward's sort keys of the fed ids, sorted on the host while the GPU runs the
        # previous step (a one-block device sort would sit serially in the step: ~48 us)
        self.host_keys = bool(on_gpu and pp == 1 and self.feed_rows * T <= E.SORT_MAX)
        if self.host_keys:
            self._host_keys = [torch.zeros(self.feed_rows * T, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
            self.keys = torch.zeros(self.feed_rows * T, dtype=torch.int32, device=self.device)
        # one host->device copy per step instead of three (ids, labels and sort keys packed in one
        # pinned buffer: each copy is a ~5 us serial node at the head of the step)
        self._packed_in = bool(self.host_keys and not self.embed_gather)
        if self._packed_in:
            self._dev_in = torch.zeros(3, self.feed_rows, T, dtype=torch.int32, device=self.device)
            self.ids, self.labels, self.keys = self._dev_in[0], self._dev_in[1], self._dev_in[2].view(-1)
            self._host = [torch.zeros(3, self.feed_rows, T, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        if pp > 1:
            self.recv_x = [torch.zeros(self.mb_rows * T, D, dtype=torch.float32, device=self.device)
                           for _ in range(self.n_micro)]
            self.recv_dx = [torch.zeros(self.mb_rows * T, D, dtype=torch.float32, device=self.device)
                            for _ in range(self.n_micro)]
            self.recv_dx_c = [torch.zeros(self.mb_rows * T, D, dtype=self.act_dtype, device=self.device)
                              for _ in range(self.n_micro)] if self.act_dtype != torch.float32 else self.recv_dx
            # pp_comm_dtype=bf16: stage messages travel as bf16 (send images cast after the producing compute,
            # received images cast back to the fp32 residual stream before the consuming compute)
            pcd = train_cfg.pp_comm_dtype
            if pcd not in ("fp32", "bf16", "auto"):
                raise ValueError(f"pp_comm_dtype={pcd!r}: expected 'fp32', 'bf16' or 'auto'")
            self.pp_bf16 = pcd == "bf16" or (pcd == "auto" and self.act_dtype == torch.bfloat16)
            if self.pp_head_split and m.pp_idx >= pp - 2:
                # the final LayerNorm output (A -> B, compute dtype) and the halves' packed row statistics
                self.recv_yf = [torch.zeros(self.mb_rows * T, D, dtype=self.act_dtype, device=self.device)
                                for _ in range(self.n_micro)]
                self.recv_s = [torch.zeros(self.mb_rows * T, 3, dtype=torch.float32, device=self.device)
                               for _ in range(self.n_micro)]
            if self.pp_bf16:
                mk = lambda: [torch.zeros(self.mb_rows * T, D, dtype=torch.bfloat16, device=self.device)
                              for _ in range(self.n_micro)]
                self.send_x_bf, self.send_dx_bf, self.recv_x_bf, self.recv_dx_bf = mk(), mk(), mk(), mk()
        self.steps_done = 0
        # Deferred optimizer (pp == 1, GPU): the step ends with the global norm and the AdamW of
        # the embedding tables only; the rest of the update runs at the START of the next step
        # on a second stream, in forward order and in a few layer groups, each group signalling
        # an event the forward waits on before its first layer.  The HBM-bound AdamW (~2.2 GB of
        # traffic) then overlaps the compute-bound forward instead of idling the MFMAs at the
        # end of the step.  Semantics are unchanged (same norm, same update, before each use);
        # :meth:`flush_optimizer` completes a pending update (checkpoint, end of run, bench).
        self.defer_opt = bool(on_gpu and pp == 1 and not self.zero and train_cfg.defer_optimizer)
        if self.defer_opt:
            # its own stream: the capped-grid AdamW passes share the CUs with the forward GEMMs instead of
            # queueing ahead of them
            self.opt_stream = torch.cuda.Stream(self.device)
            self._defer_blocks = int(os.environ.get("DTC_DEFER_BLOCKS", "256"))
            self.program.before_comm.append(self._join_opt)
            # device-side "an update is pending" switch: the graph always contains the deferred
            # launch, the kernels skip when nothing is pending (first step, after a flush)
            self._pending_dev = torch.zeros(1, dtype=torch.float32, device=self.device)
            L = list(self.layout.layers)
            bk = self.buckets
            lo_emb = self.flat.range_of([n for n in ("wte", "wpe") if n in self.flat.slots])[0] \
                if self.layout.has_embed else self.flat.numel
            self._emb_range = (lo_emb, self.flat.numel)
            ng = max(1, min(train_cfg.defer_groups, len(L)))
            per = (len(L) + ng - 1) // ng
            self._opt_groups = []  # (first layer, [(lo, hi), ...]) in forward order
            for gi in range(0, len(L), per):
                ls = L[gi:gi + per]
                lo = min(self.flat.range_of([n for n in self.flat.slots if n.startswith(f"h.{l}.")])[0] for l in ls)
                hi = max(bk.layer_end_offset(l) for l in ls)
                self._opt_groups.append((ls[0], [(lo, hi)]))
            if self.layout.has_head:
                self._opt_groups.append(("head", [(0, bk.head_end_offset())]))
        # LayerNorms fused into the layer GEMMs (ops/ln_fused.py).  DTC_LN_FUSE bits: 1 forward
        # (out_proj / fc2 emit the next LayerNorm's output), 2 backward (the fc1 / qkv NT dgrads finish
        # the LayerNorm backward).  Needs tp = pp = 1 (no all-reduce between GEMM and LayerNorm, one call
        # per site and step), a single stream (the row-statistics exchange wants the whole chip for the
        # launch) and, for the backward, the transposed weight mirror.
        lnf = int(os.environ.get("DTC_LN_FUSE", "2"))
        # dp == 1 too: under DP the bucket all-reduces (RCCL kernels on other CUs) run during the
        # backward, and the in-launch row-statistics exchange needs all of its blocks co-resident.
        if (lnf and on_gpu and self.act_dtype == torch.bfloat16 and tp == 1 and pp == 1 and not self.dp_comm
                and not self.defer_opt):
            has_wt = len(self.layout.layers) > 0 and self.flat.wt(f"h.{self.layout.layers[0]}.fc1.w") is not None
            self.stage.enable_ln_fusion(self.b_local * T, self.opt.step_t, fwd=bool(lnf & 1),
                                        bwd=bool(lnf & 2) and has_wt)
        if on_gpu:
            self._reserve_workspaces()

    # ------------------------------------------------------------------ helpers
    def _wgrad_group_for_memory(self, mc: ModelConfig, n_layers: int) -> int:
        """Auto ``wgrad_group`` at dp == 1: one grouped launch for the whole stage (0) keeps every layer's
        weight-gradient operands alive until the end of the backward -- per layer the bf16 dY tensors
        (dx3, du, dx2, dqkv) and the X operands that would otherwise be freed after its backward (y1, o,
        y2, gelu(u)), (8·D + 2·F)·tokens·2 bytes (GPT-2 small at 8k tokens: 201 MB/layer, 2.4 GB in all).
        When the whole stage's share exceeds the budget (``DTC_WGRAD_MEM_MB``, default 10 % of the
        device's memory, 1 GiB on CPU) the groups shrink to what fits (at least one layer)."""
        if n_layers == 0:
            return 0
        tokens = self.b_local * self.T
        esize = 2 if self.act_dtype == torch.bfloat16 else 4
        D, F = mc.d_model, mc.d_ff
        per_layer = (8 * D + 2 * F) * tokens * esize
        env = os.environ.get("DTC_WGRAD_MEM_MB")
        if env is not None:
            budget = float(env) * (1 << 20)
        elif self.device.type == "cuda":
            budget = 0.10 * torch.cuda.get_device_properties(self.device).total_memory
        else:
            budget = float(1 << 30)
        if per_layer * n_layers <= budget:
            return 0
        return max(1, int(budget // per_layer))

    def pp_item_costs(self):
        """Per-stage F / B / W costs of one microbatch for the zero-bubble placement (``parallel/pp.py``):
        the stage sizes of the layer split (layers + the head's block-equivalents, ``mesh.stage_costs``).
        Identical on every rank (the programs of all stages must agree)."""
        from ..parallel.mesh import stage_costs
        from ..parallel.pp import stage_item_costs

        hc = self.tcfg.pp_head_cost
        w = (0.05, head_cost_blocks(self.mcfg) if hc is None else float(hc))
        hs = 2 if self.pp_head_split else 1
        return stage_item_costs(self.mesh.pp, stage_costs(self.layer_ranges, w, head_stages=hs),
                                head_half=w[1] / 2 if hs == 2 else 0.0)

    def pp_comm_costs(self):
        """Transfer time of the stage messages in the units of :meth:`pp_item_costs` (one block's F + B + W
        for one microbatch), for the zero-bubble placement: bytes over one xGMI link (assumed 50 GB/s per
        direction) against the block's FLOPs at an assumed 600 TF/s (GPT-2 small: 63 us vs 80 us per
        one-sequence microbatch -- the messages are NOT negligible).  Deterministic, identical on every rank."""
        mc, T, rows = self.mcfg, self.T, self.mb_rows
        D, F = mc.d_model, mc.d_ff
        block_s = 6.0 * (4 * D * D + 2 * D * F + T * D) * rows * T / 600e12
        esz = 2 if getattr(self, "pp_bf16", False) else 4
        fb = rows * T * D * esz / 50e9 / block_s
        return {"f": fb, "b": fb, "s": 1e-5 / block_s}

    def _reserve_workspaces(self):
        from ..ops.gemm import reserve_workspace

        # split-K slabs: the lm_head dgrad (fused CE, split 8 at the reference size) needs 67 MB
        reserve_workspace(self.device, 96 << 20)

    @property
    def tokens_per_step(self) -> int:
        return self.global_batch * self.T

    def set_batch(self, batch_np: np.ndarray):
        """batch_np int32 [feed_rows, T+1] (global rows [feed_row0, feed_row0+feed_rows): this rank's
        rows, or the whole global batch under the DP embedding gather) → static device ids/labels."""
        self.stage_batch(batch_np)
        self.upload_batch()

    def stage_batch(self, batch_np: np.ndarray):
        """The host half of :meth:`set_batch`: the token ids / labels into the next pinned host slot and the
        embedding backward's sort keys computed on the host.  A caller that blocks on every step's loss (the
        reference's timed loop, ``bench.py``) stages step t+1's batch while step t still runs on the GPU, so
        only :meth:`upload_batch` (the H2D enqueue) sits between the loss read and the next launch."""
        assert batch_np.shape[0] == self.feed_rows, (batch_np.shape, self.feed_rows)
        i = self._host_i
        h = self._host[i]
        if self._packed_in:
            h[0].copy_(torch.from_numpy(batch_np[:, :-1]))
            h[1].copy_(torch.from_numpy(batch_np[:, 1:]))
            E.embed_sort_keys_host(batch_np[:, :-1], out=h[2].view(-1).numpy())
        else:
            if self.host_keys:
                E.embed_sort_keys_host(batch_np[:, :-1], out=self._host_keys[i].numpy())
            h[0].copy_(torch.from_numpy(batch_np[:, :-1]))
            h[1].copy_(torch.from_numpy(batch_np[:, 1:]))
        self._staged_slot = i
        self._host_i ^= 1

    def upload_batch(self):
        """Enqueue the H2D copies of the batch :meth:`stage_batch` prepared (a two-slot pinned ring: the slot
        is rewritten two batches later, after a loss read has ordered its copy)."""
        i = self._staged_slot
        assert i is not None, "upload_batch without stage_batch"
        self._staged_slot = None
        h = self._host[i]
        if self._packed_in:
            self._dev_in.copy_(h, non_blocking=True)
            return
        if self.host_keys:
            self.keys.copy_(self._host_keys[i], non_blocking=True)
        if self.embed_gather:
            lo = self.row0 - self.feed_row0
            self.ids_all.copy_(h[0], non_blocking=True)
            self.labels.copy_(h[1][lo:lo + self.b_local], non_blocking=True)
        else:
            self.ids.copy_(h[0], non_blocking=True)
            self.labels.copy_(h[1], non_blocking=True)

    # ------------------------------------------------------------------ step bodies
    def _launch_deferred_update(self):
        """Queue the pending AdamW (all but the embedding tables) on the optimizer stream, group by
        group in forward order; each group's event gates the first forward use of its params."""
        if not self.defer_opt:
            return
        st, flag, s = self.stage, self._pending_dev, self.opt_stream
        s.wait_stream(torch.cuda.current_stream())
        for key, ranges in self._opt_groups:
            with torch.cuda.stream(s):
                for lo, hi in ranges:
                    self.opt.update_range(lo, hi, enable=flag, max_blocks=self._defer_blocks)
                ev = torch.cuda.Event()
                ev.record(s)
            st.param_ready[key] = ev

    def _join_opt(self):
        if self.defer_opt:
            torch.cuda.current_stream().wait_stream(self.opt_stream)

    def _finish_optimizer(self):
        if self.defer_opt:
            self.opt.norm()
            self.opt.update_range(*self._emb_range)
            O.fill_(self._pending_dev, 1.0)
        else:
            self.opt.step()

    def flush_optimizer(self):
        """Complete a deferred update now (before reading/saving params or ending a run); the
        next step's in-graph launch then finds nothing pending."""
        if self.defer_opt:
            for _, ranges in self._opt_groups:
                for lo, hi in ranges:
                    self.opt.update_range(lo, hi, enable=self._pending_dev)
            O.fill_(self._pending_dev, 0.0)
            self.stage.param_ready.clear()

    class _CommSafeGemms:
        """GEMM plans for code that runs UNDER asynchronous RCCL collectives (the DP bucket all-reduces
        during the backward, PP send/recv).  RCCL's kernels hold CUs (and LDS) for the whole transfer;
        a GEMM built as exactly one round of one-block-per-CU tiles with all 160 KB of LDS (gemm8n) or
        one ~256-block round of 128 KB-LDS blocks (split-K 256^2 weight gradients) cannot place its last
        blocks until the collective's CUs free up, and would run about twice as long.  Inside this
        context those problems take the many-block 128^2 / 256^2 plans that rebalance over the CUs left (the
        gemm8r plans already have more blocks than CUs and stay).
        No-op on CPU, with a single rank, or with DTC_COMM_SAFE_GEMMS=0."""

        def __init__(self, on: bool):
            self.on = on and torch.cuda.is_available() and os.environ.get("DTC_COMM_SAFE_GEMMS", "1") == "1"

        def __enter__(self):
            if self.on:
                from ..ops import _native as N

                L = N.lib()
                # gemm8r stays (DTC_COMM_SAFE_R8, default 1): 1.5 rounds of two interleaved tile widths, more
                # blocks than CUs, so a CU held by RCCL only delays the blocks it would have run.  One-rank
                # rehearsal with 32 CUs held by a probe kernel: 12.61-12.67 ms/step kept vs 12.77 (and one 20.7
                # outlier) off; with none held 10.97-11.02 vs 11.15-11.20 (profiles/r6_comm_safe_r8.md)
                keep_r8 = os.environ.get("DTC_COMM_SAFE_R8", "1") == "1"
                r8 = L.dtc_gemm_set_r8(0)
                if keep_r8:
                    L.dtc_gemm_set_r8(r8)
                self.prev = (L.dtc_gemm_set_n8(0), L.dtc_gemm_set_wgrad256(0), r8)

        def __exit__(self, *a):
            if self.on:
                from ..ops import _native as N

                L = N.lib()
                L.dtc_gemm_set_n8(self.prev[0])
                L.dtc_gemm_set_wgrad256(self.prev[1])
                L.dtc_gemm_set_r8(self.prev[2])

    def _step_fn_dp_tp(self):
        st, T, b = self.stage, self.T, self.b_local
        self._launch_deferred_update()
        dp = self.mesh.dp
        dpc = self.dp_comm
        ctx: Dict = {}
        step = self.opt.step_t
        hk = self.keys if self.host_keys else None
        h = st.embed_forward(self.ids, step, self.row0, ctx, want_keys=not self.embed_gather,
                             keys=None if self.embed_gather else hk)
        gathered = None
        if self.embed_gather:
            gathered = (self.ids_all, 0, (hk, None) if hk is not None else st.embed_keys(self.ids_all))
        h = st.stage_forward(h, b, ctx)
        st.head_forward(h, self.labels, 1.0 / (b * T), ctx, loss_out=self.loss)
        if dpc:
            # the loss is final here: its DP mean goes out now, under the whole backward, instead of
            # as an exposed collective at the end of the step (joined before the optimizer)
            self._loss_allreduce(name="loss_dp")  # (pp == 1 here)
        with self._CommSafeGemms(dpc and self.stage.flat.device.type == "cuda"):  # bucket all-reduces overlap it
            return self._backward_dp_tp(ctx, dp, step, gathered)

    def _backward_dp_tp(self, ctx, dp, step, gathered):
        st, T, b = self.stage, self.T, self.b_local
        dx, dx_c = st.head_backward(ctx, grad_scale=1.0 / (b * T * dp), beta=0.0)
        bk, opt = self.buckets, self.opt
        side = st.red  # grad-norm chunks: into the reducer's batched launches (None: computed right away)
        # deferred weight gradients: the head's grads are final only after the first grouped launch, so
        # what would follow the head backward runs at the first layer hook (which fires after it)
        head_later = [st._defer_wg]
        if not self.dp_comm:
            if not head_later[0]:
                opt.ready_upto(bk.head_end_offset(), side)

            def hook(l):
                if head_later[0]:
                    opt.ready_upto(bk.head_end_offset(), side)
                    head_later[0] = False
                opt.ready_upto(bk.layer_end_offset(l), side)
        else:
            # layer l's grads are final once its reduction launch is queued (before the hook), so its
            # bucket goes out right away; the head's bucket right after the head backward.  The first
            # layer's bucket waits for the embedding gather (that collective feeds compute; the bucket
            # only the optimizer).
            first = self.layout.layers[0]
            if not self.zero and not head_later[0]:  # (ZeRO-1: ShardedAdamW.step reduce-scatters)
                bk.ready_upto(bk.head_end_offset())

            def hook(l):
                if head_later[0]:
                    head_later[0] = False
                    if not self.zero:
                        bk.ready_upto(bk.head_end_offset())
                if self.embed_gather and l == first:
                    return
                bk.ready_upto(bk.layer_end_offset(l))
        if self.zero:
            hook = None  # grads are reduce-scattered in one call by ShardedAdamW.step
        dx_hook = None
        if self.embed_gather:
            # the embedding-output gradients go out the moment the first layer's dgrad produces them,
            # under that layer's remaining weight-gradient work
            def dx_hook(d, d_c, out=self.dh_all, g=self.mesh.dp_group):
                if self.dh_all_bf is not None and d_c.dtype == torch.bfloat16:
                    out, d = self.dh_all_bf, d_c
                self.program.comm(lambda: dist.all_gather_into_tensor(out, d, group=g),
                                  sig=csig("all_gather", g, d))
        dx, dx_c = st.stage_backward(ctx, dx, dx_c, 0.0, hook=hook, dx_hook=dx_hook)
        if self.embed_gather:
            bk.ready_all()
            if self.dh_all_bf is not None:
                from ..ops.payload import cast_bf16_to_f32

                cast_bf16_to_f32(self.dh_all_bf, self.dh_all)
            st.embed_backward(ctx, self.dh_all, step, 0.0, gathered=gathered)
            opt.chunk_ready(len(opt.chunks) - 1, side)  # local wte/wpe grads: overlaps the tail bucket
        else:
            st.embed_backward(ctx, dx, step, 0.0)
        if not self.zero:
            bk.ready_all()
            bk.wait_all()
        if self.dp_comm:
            self.program.wait("loss_dp")
        self._finish_optimizer()
        return self.loss

    def _loss_allreduce(self, name: Optional[str] = None, pp: bool = False):
        """Sum the loss over the DP group (and the PP group with ``pp``: only the last stage holds
        it).  With ``name`` the all-reduces are asynchronous: :meth:`StepProgram.wait` joins them
        later (the loss is read by the host only, nothing in the step consumes it)."""
        m = self.mesh
        groups = []
        if self.dp_comm:
            groups.append(m.dp_group)
        if m.pp > 1 and pp:
            groups.append(m.pp_group)
        if not groups:
            return []
        t = self.loss
        if name is None:
            for g in groups:
                self.program.comm(lambda g=g: dist.all_reduce(t, group=g), sig=csig("all_reduce", g, t))
            return []
        # one collective item (one graph cut): with both groups the pp sum must land before the dp
        # sum reads the tensor (separate communicators / streams), so the first is joined to the
        # issuing stream and only the last stays asynchronous
        def fn():
            for g in groups[:-1]:
                dist.all_reduce(t, group=g, async_op=True).wait()
            return dist.all_reduce(t, group=groups[-1], async_op=True)

        self.program.comm(fn, name=name, sig=[x for g in groups for x in csig("all_reduce", g, t)])
        return [name]

    def _step_fn_pp(self):
        from ..parallel.pp import run_pipeline

        with self._CommSafeGemms(self.stage.flat.device.type == "cuda"):  # send/recv overlap compute
            run_pipeline(self)
        self.buckets.ready_all()
        # the loss sum overlaps the bucket all-reduces and the optimizer; joined at the very end
        waits = self._loss_allreduce(name="loss_pp", pp=True)
        self.buckets.wait_all()
        self.opt.step()
        for n in waits:
            self.program.wait(n)
        return self.loss

    def _step_fn(self):
        out = self._step_fn_pp() if self.mesh.pp > 1 else self._step_fn_dp_tp()
        if self.p2p is not None:
            self.p2p.end_step()  # even P2P calls per step: every call site keeps its buffer half on replay
        return out

    # ------------------------------------------------------------------ public
    def run_step(self) -> torch.Tensor:
        """Enqueue one full training step on the static inputs; returns the (device) loss."""
        p = self.program
        p.begin_step()
        check = self.steps_done == 0 or (p.use_graph and not p.recorded)
        if check:
            p.collect()  # the first eager step and the recorded step prove the ranks agree
        if not p.use_graph:
            self._step_fn()
        elif not p.recorded:
            if self.steps_done == 0:
                self._step_fn()  # eager first step: lazy RCCL init, workspace sizing
            else:
                p.record(self._step_fn)
                p.verify("recorded step")
                p.replay()
        else:
            p.replay()
        if check and p.sigs is not None:
            p.verify("first step")
        self.steps_done += 1
        st = self.stage
        if st.wg_record and st.wg_sq is None and st.wg_seen is not None:  # after the first (eager) step
            ranges, tiles = [], 0
            base = self.flat.grads.data_ptr()
            for dw, m, n in st.wg_seen:
                ranges.append(((dw.data_ptr() - base) // 4, dw.numel()))
                tiles += G.wgrad_tiles(m, n)
            nwg = tiles * G.WG_SQ_SLOTS
            # the embedding tables' Σg² from the embedding backward itself (its last kernel writes the final
            # rows): no 154 MB norm pass over a table whose untouched rows are zero (GPT-2 small: -25 us/step)
            emb = 0
            if self._emb_fused_norm():
                for name in ("wte", "wpe"):
                    g = self.flat.g(name)
                    ranges.append(((g.data_ptr() - base) // 4, g.numel()))
                emb = E.embed_sq_slots(self.b_local, self.T, self._D)
            part = self.opt.set_fused_sumsq(ranges, nwg + emb)
            st.use_wgrad_sumsq(part[:nwg])
            if emb:
                st.emb_sq = part[nwg:]
        return self.loss

    def _emb_fused_norm(self) -> bool:
        """The embedding backward alone writes the wte / wpe grads, once per step, and they are final there: dp 1
        (no all-reduce or gather of them), no TP / sequence parallelism (norm weight 1), one sort window.  Then it
        may write the tables' share of Σg² itself and zero only the wte rows its previous call wrote."""
        return (self.layout.has_embed and not self.dp_comm and self.mesh.tp == 1 and not self.embed_gather
                and not self.stage.sp and self.b_local * self.T <= E.SORT_MAX)

    def loss_value(self) -> float:
        """Blocking read of the global mean loss (reference: float(np.asarray(loss)), train.py:82)."""
        v = float(self.loss.item())
        self.check_health()
        return v / self.mesh.dp

    def check_health(self):
        """Raise if a device-side wait of this rank timed out (P2P all-reduce flags, fused LayerNorm
        row statistics).  Blocking: call outside pipelined loops."""
        if self.p2p is not None:
            self.p2p.check()
        if self.stage.ln_sync is not None:
            self.stage.ln_sync.check()

    # -- host pipelining: read step t's loss while step t+1 is already queued --------------
    def _err_words(self):
        """Device error words of this rank's in-launch waits (P2P all-reduce flags, fused LayerNorm
        row statistics): nonzero = a wait timed out and that step computed NaN."""
        out = []
        if self.p2p is not None:
            out.append(("p2p", self.p2p.err))
        if self.stage.ln_sync is not None:
            out.append(("ln", self.stage.ln_sync.err))
        return out

    def loss_handle(self):
        """Queue a copy of this step's loss (and of the error words) to pinned host memory (2-slot
        ring) + an event.

        With the step replayed from a graph, the host can enqueue step t+1 (its H2D batch copy
        and graph launch) before blocking on step t's loss, so the GPU never idles on the host
        between steps; every step's loss is still read (one step later), and a timed-out device
        wait raises at that read instead of letting NaN losses through silently."""
        if self.device.type != "cuda":
            return self.loss_value()
        words = self._err_words()
        if not hasattr(self, "_loss_host"):
            self._loss_host = [torch.zeros(1, dtype=torch.float32, pin_memory=True) for _ in range(2)]
            self._err_host = [torch.zeros(max(1, len(words)), dtype=torch.int32, pin_memory=True) for _ in range(2)]
            self._loss_slot = 0
        i = self._loss_slot
        slot, eslot = self._loss_host[i], self._err_host[i]
        self._loss_slot ^= 1
        slot.copy_(self.loss, non_blocking=True)
        for j, (_, w) in enumerate(words):
            eslot[j:j + 1].copy_(w, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return slot, ev, eslot

    def read_loss(self, handle) -> float:
        if not isinstance(handle, tuple):
            return handle
        slot, ev, eslot = handle
        ev.synchronize()
        for j, (name, _) in enumerate(self._err_words()):
            e = int(eslot[j])
            if e:
                if name == "p2p":
                    raise RuntimeError(f"P2P all-reduce: rank {self.p2p.rank} timed out waiting for rank {e - 1000}")
                raise RuntimeError("fused LayerNorm: a row-statistics wait timed out (outputs were NaN)")
        return float(slot.item()) / self.mesh.dp

    def grad_norm(self) -> float:
        return self.opt.grad_norm()
