"""Loader for the in-tree HIP kernel library ``_dtc_kernels.so`` (gfx950).

The kernels are plain HIP C++ (``csrc/*.hip``) compiled by ``hipcc --offload-arch=gfx950``
into one shared object with a C ABI; Python calls it through ctypes with raw device
pointers and the current HIP stream, so every launch is stream-ordered and
hipGraph-capturable.  torch is imported first so the library binds to the same
``libamdhip64.so.7`` instance torch already loaded (same SONAME).

On a GPU tensor there is NO silent fallback: if the library is missing or fails to
load, :func:`lib` raises.  CPU tensors use the pure-torch reference implementations in
the op modules (the test oracle and the gloo plumbing path).
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch

_LIB = None
_LOCK = threading.Lock()
LIB_NAME = "_dtc_kernels.so"
PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DTC_KERNEL_LIB: alternative build of the same library (A/B of compile-time kernel variants)
LIB_PATH = os.environ.get("DTC_KERNEL_LIB") or os.path.join(PKG_DIR, LIB_NAME)

c_int = ctypes.c_int
c_long = ctypes.c_long
c_float = ctypes.c_float
c_vp = ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    """Mirror of ``struct GemmArgs`` in csrc/common.h (keep in sync)."""

    _fields_ = [
        ("layout", c_int),       # 0: C=A.B^T (nt)  1: C=A.B (nn)  2: C=A^T.B (tn)
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("A", c_vp), ("lda", c_long),
        ("B", c_vp), ("ldb", c_long),
        ("C", c_vp), ("ldc", c_long),
        ("c_f32", c_int),        # C dtype: 0 bf16, 1 fp32
        ("epi", c_int),          # epilogue id (EPI_*)
        ("bias", c_vp),          # fp32 [N] or null
        ("aux", c_vp), ("ldaux", c_long),   # epi-specific input (residual fp32 / gelu pre-act bf16)
        ("aux_out", c_vp),       # epi-specific second output (gelu output bf16)
        ("alpha", c_float), ("beta", c_float),
        ("labels", c_vp),        # int32 [M] (lm-head CE epilogue)
        ("vocab_start", c_int), ("n_valid", c_int),
        ("part", c_vp),          # float2 [nparts][M]
        ("label_out", c_vp),     # fp32 [M]
        ("workspace", c_vp), ("ws_bytes", c_long),
        ("split_k", c_int),      # 0 = auto
        ("defer_reduce", c_int),  # wgrad split-K: leave the slabs in `workspace` (ops/reduce.py)
        ("colsum", c_vp),        # wgrad: fp32 [split][M] bias-gradient partials (fused colsum)
    ]


class LnArgs(ctypes.Structure):
    """Mirror of ``struct LnArgs`` in csrc/common.h (keep in sync): a layer GEMM with its LayerNorm
    fused into the epilogue (``ops/ln_fused.py``)."""

    _fields_ = [
        ("bwd", c_int),
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("A", c_vp), ("lda", c_long),
        ("B", c_vp), ("ldb", c_long),
        ("C", c_vp),
        ("bias", c_vp), ("resid", c_vp), ("gamma", c_vp), ("beta", c_vp),
        ("y", c_vp), ("mean", c_vp), ("rstd", c_vp),
        ("x", c_vp), ("part", c_vp), ("nslab", c_int),
        ("eps", c_float),
        ("sync", c_vp), ("step", c_vp), ("site", c_int), ("nsites", c_int),
        ("err", c_vp),
    ]


class WgEntry(ctypes.Structure):
    """Mirror of ``struct WgEntry`` in csrc/common.h: one problem of a grouped weight-gradient launch."""

    _fields_ = [("A", c_vp), ("B", c_vp), ("C", c_vp), ("cs", c_vp), ("M", c_int), ("N", c_int),
                ("tile0", c_int), ("nfast", c_int)]


WG_MAX = 64  # csrc/common.h WG_MAX


class WgBatch(ctypes.Structure):
    _fields_ = [("n", c_int), ("K", c_int), ("beta", c_float), ("ntiles", c_int), ("sq", c_vp),
                ("tail_tiles", c_int), ("tail_split", c_int), ("tail_slab", c_vp), ("tail_cap", c_long),
                ("e", WgEntry * WG_MAX)]


EPI_STORE = 0       # C = alpha*acc (+bias) (+beta*C if fp32)
EPI_RESID = 1       # C(f32) = aux(f32) + acc + bias
EPI_GELU = 2        # u = acc+bias: C(bf16) = gelu_tanh'(u) ; aux_out(bf16) = gelu_tanh(u)
EPI_DGELU = 3       # C(bf16) = acc * aux   (aux = gelu_tanh'(u) from EPI_GELU)
EPI_LMHEAD = 4      # C(bf16) = acc+bias, pad cols -inf; per-row partial (max,sumexp); label logit


def _declare(lib):
    vp, i, l, f = c_vp, c_int, c_long, c_float
    sigs = {
        "dtc_version": ([], i),
        "dtc_gemm": ([ctypes.POINTER(GemmArgs), vp], i),
        "dtc_gemm_workspace_bytes": ([i, i, i, i], l),
        "dtc_lmhead_nparts": ([i, i, i], i),
        "dtc_layernorm_fwd": ([vp, vp, vp, vp, vp, vp, i, i, f, i, vp], i),
        "dtc_add_layernorm_fwd": ([vp, vp, vp, vp, vp, vp, vp, vp, i, i, f, i, vp], i),
        "dtc_add_layernorm_fwd_bf16": ([vp, vp, vp, vp, vp, vp, vp, vp, i, i, f, i, vp], i),
        "dtc_layernorm_bwd": ([vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i, i, i, vp, l, i, vp], i),
        "dtc_layernorm_bwd_workspace_bytes": ([i, i], l),
        "dtc_colsum": ([vp, i, i, i, l, vp, f, vp, l, i, vp], i),
        "dtc_gemm_wgrad_split": ([i, i, i, i], i),
        "dtc_gemm_set_n8": ([i], i),
        "dtc_gemm_set_n8_cb": ([i], i),
        "dtc_gemm_set_r8": ([i], i),
        "dtc_gemm_set_r8_ilv": ([i], i),
        "dtc_gemm_set_big_cb3": ([i], i),
        "dtc_gemm_set_n8_mink": ([i], i),
        "dtc_gemm_set_wgrad256": ([i], i),
        "dtc_wgrad_group": ([ctypes.POINTER(WgBatch), vp], i),
        "dtc_wg_entry_bytes": ([], i),
        "dtc_wg_max": ([], i),
        "dtc_wg_batch_bytes": ([], i),
        "dtc_gemm_pair": ([ctypes.POINTER(GemmArgs), ctypes.POINTER(GemmArgs), vp], i),
        "dtc_gemm_ln": ([ctypes.POINTER(LnArgs), vp], i),
        "dtc_gemm_ln_sync_words": ([i, i], l),
        "dtc_gemm_wgrad_fuses_colsum": ([i, i, i], i),
        "dtc_reduce_tasks": ([vp, vp], i),
        "dtc_red_max_tasks": ([], i),
        "dtc_red_task_bytes": ([], i),
        "dtc_colsum_workspace_bytes": ([i, i], l),
        "dtc_embed_fwd": ([vp, vp, vp, vp, i, i, i, i, f, l, vp, l, vp], i),
        "dtc_epoch_inc": ([vp, vp], i),
        "dtc_flag_set": ([vp, i, vp, vp], i),
        "dtc_flag_wait": ([vp, i, vp, vp, vp], i),
        "dtc_p2p_flag_bytes": ([], l),
        "dtc_p2p_alloc": ([l, vp, vp], i),
        "dtc_p2p_open": ([vp, vp], i),
        "dtc_p2p_close": ([vp], i),
        "dtc_device_pci_bus_id": ([i, ctypes.c_char_p, i], i),
        "dtc_device_count": ([ctypes.POINTER(c_int)], i),
        "dtc_graph_num_nodes": ([c_vp, ctypes.POINTER(ctypes.c_size_t)], i),
        "dtc_can_access_peer": ([i, i, ctypes.POINTER(c_int)], i),
        "dtc_p2p_free": ([vp], i),
        "dtc_p2p_allreduce": ([vp, vp, l, vp, i, i, l, vp, vp, i, vp], i),
        "dtc_p2p_allreduce_bf16": ([vp, vp, l, vp, i, i, l, vp, vp, i, vp, vp, i, vp], i),
        "dtc_p2p_barrier_round": ([vp, i, i, vp, vp, vp], i),
        "dtc_p2p_reduce_scatter": ([vp, i, vp, l, vp, i, i, l, vp, vp, vp, vp, i, vp], i),
        "dtc_p2p_all_gather": ([vp, vp, l, vp, i, i, l, vp, vp, vp], i),
        "dtc_cu_hog": ([i, l, i, vp, vp], i),
        "dtc_embed_sort_bits": ([i], i),
        "dtc_embed_sort": ([vp, i, i, vp, vp], i),
        "dtc_embed_bwd": ([vp, vp, vp, vp, vp, i, i, i, i, f, l, vp, l, i, vp, vp, i, vp], i),
        "dtc_embed_sq_slots": ([i, i, i], l),
        "dtc_attn_fwd": ([vp, vp, vp, i, i, i, i, l, f, vp], i),
        "dtc_attn_bwd": ([vp, vp, vp, vp, vp, i, i, i, i, i, f, vp, l, vp], i),
        "dtc_attn_bwd_workspace_bytes": ([i, i, i, i], l),
        "dtc_ce_combine": ([vp, i, i, l, l, vp, vp, vp, f, vp, i, vp], i),
        "dtc_ce_bwd": ([vp, l, vp, vp, i, i, i, i, f, vp, vp], i),
        "dtc_ce_colsum_rows": ([], i),
        "dtc_sumsq_segments": ([vp, vp, i, vp, vp, vp, l, vp], i),
        "dtc_sumsq_workspace_bytes": ([], l),
        "dtc_sumsq_partial": ([vp, vp, i, vp, i, vp], i),
        "dtc_sum_finish": ([vp, i, vp, vp, vp], i),
        "dtc_adamw": ([vp, vp, vp, vp, vp, l, l, vp, vp, f, f, f, f, f, f, vp, i, vp], i),
        "dtc_cast_f32_bf16": ([vp, vp, l, vp], i),
        "dtc_transpose_batch": ([vp, vp], i),
        "dtc_aw_max_seg": ([], i),
        "dtc_aw_max_tasks": ([], i),
        "dtc_aw_seg_bytes": ([], i),
        "dtc_aw_task_bytes": ([], i),
        "dtc_adamw_tr": ([vp, vp, vp, vp, vp, l, vp, vp, vp, vp, f, f, f, f, f, f, vp], i),
        "dtc_tr_max_tasks": ([], i),
        "dtc_tr_task_bytes": ([], i),
        "dtc_fill_f32": ([vp, f, l, vp], i),
        "dtc_shard_sum_bf16": ([vp, i, l, vp, vp], i),
        "dtc_cast_bf16_f32": ([vp, vp, l, vp], i),
        "dtc_ce_dgrad": ([vp, l, vp, vp, i, i, f, vp, l, vp, l, vp, vp, i, i, i, vp, l, vp], i),
        "dtc_ce_dgrad_workspace_bytes": ([i, i, i], l),
        "dtc_ce_dgrad_colpart_rows": ([i], i),
        # exact-fp32 parity path (csrc/gemm_f32.hip, csrc/attention_f32.hip)
        "dtc_gemm_f32": ([ctypes.POINTER(GemmArgs), vp], i),
        "dtc_gemm_f32_workspace_bytes": ([i, i, i, i], l),
        "dtc_lmhead_nparts_f32": ([i, i, i], i),
        "dtc_attn_f32_fwd": ([vp, vp, vp, i, i, i, i, f, vp], i),
        "dtc_attn_f32_bwd": ([vp, vp, vp, vp, vp, i, i, i, i, f, vp, l, vp], i),
        "dtc_attn_f32_bwd_workspace_bytes": ([i, i, i, i], l),
        "dtc_ce_bwd_f32": ([vp, l, vp, vp, i, i, i, i, f, vp, vp], i),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    """The loaded kernel library; raises (never falls back) if it is unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"HIP kernel library {LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(or python -m distributed_training_compare_jax_amd.csrc.build)")
            _LIB = _declare(ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL))
    return _LIB


def library_path(t: torch.Tensor) -> bool:
    """True when an op runs its pure-torch implementation: CPU tensors only (the fp32 oracle and
    the gloo plumbing path).  Every GPU tensor takes a HIP kernel of ``_dtc_kernels.so`` in BOTH
    precisions: bf16 (MFMA bf16, the default) and the exact-fp32 parity mode
    (``TrainConfig.dtype: fp32``: ``csrc/gemm_f32.hip`` / ``csrc/attention_f32.hip`` on
    ``v_mfma_f32_32x32x2_f32``) — no rocBLAS / hipBLASLt / torch matmul on the GPU path."""
    return not t.is_cuda


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")
