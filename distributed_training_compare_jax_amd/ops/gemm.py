"""GEMM-shaped ops: every Dense of the reference model, forward and backward.

Reference sites: q/k/v/out Dense (``model/CausalSelfAttention.py:18-20,46``), fc1/fc2
(``model/MLP.py:13,20``), lm_head (``model/GPTModel.py:72``).  Weights are stored
``[out, in]`` (the transpose of Flax's ``[in, out]`` kernel) so the forward GEMM has both
operands K-contiguous.  On GPU all three GEMM forms run on the hand-written MFMA kernel
in ``csrc/gemm.hip`` (bf16 in, fp32 accumulate) with fused epilogues:

* ``linear``         y = x·Wᵀ + b                       (bf16 out)
* ``linear_resid``   x_out = resid + x·Wᵀ + b           (fp32 residual stream)
* ``linear_gelu``    u = x·Wᵀ + b → (gelu_tanh'(u), gelu_tanh(u))  (fc1 + ``nn.gelu``, MLP.py:14;
  the derivative is what the backward needs, computed here from the shared tanh)
* ``matmul_nn``      dX = dY·W                           (dgrad, fp32 out)
* ``matmul_nn_dgelu`` dU = (dY·W) ⊙ d,  d = gelu'(u)      (fc2 dgrad fused with GELU bwd)
* ``wgrad``          dW = β·dW + dYᵀ·X                    (fp32, written straight into the flat grad buffer)
* ``colsum``         db = β·db + Σ_rows dY                (bias grads)

fp32 GPU tensors (the exact-fp32 parity mode, ``dtype: fp32`` — the reference's precision) run the
same ops on ``csrc/gemm_f32.hip`` (``v_mfma_f32_32x32x2_f32``, exact f32 products and fp32
accumulation, same layouts and epilogues).  CPU tensors take the pure-torch fp32 path below (the
oracle / gloo path).
"""

from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch

from . import _native as N

_SQRT_2_OVER_PI = math.sqrt(2.0 / math.pi)


def gelu_tanh(u: torch.Tensor) -> torch.Tensor:
    """``jax.nn.gelu(approximate=True)`` (flax ``nn.gelu`` default)."""
    return 0.5 * u * (1.0 + torch.tanh(_SQRT_2_OVER_PI * (u + 0.044715 * u * u * u)))


def gelu_tanh_grad(u: torch.Tensor) -> torch.Tensor:
    inner = _SQRT_2_OVER_PI * (u + 0.044715 * u * u * u)
    t = torch.tanh(inner)
    dinner = _SQRT_2_OVER_PI * (1.0 + 3.0 * 0.044715 * u * u)
    return 0.5 * (1.0 + t) + 0.5 * u * (1.0 - t * t) * dinner


# ----------------------------------------------------------------------------- native glue
_WS = {}


def _workspace(device, nbytes: int) -> torch.Tensor:
    """Persistent scratch (split-K slabs, reduction partials) per (device, stream role): kernels of
    one role run in stream order and reuse it; the backward side stream (role "side", set by
    :func:`workspace_role`) gets its own so concurrent kernels never share scratch.  Keyed by role,
    not stream handle, so the capture stream of a hipGraph reuses the eager step's buffers."""
    key = (device.type, device.index, _ROLE[0])
    ws = _WS.get(key)
    if ws is None or ws.numel() < nbytes:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("GEMM workspace must be reserved before graph capture (call ops.reserve_workspace)")
        ws = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = ws
    return ws


_ROLE = ["main"]


class workspace_role:
    """Context manager selecting the scratch-buffer role (``"main"`` / ``"side"``)."""

    def __init__(self, role: str):
        self.role = role

    def __enter__(self):
        self.prev = _ROLE[0]
        _ROLE[0] = self.role

    def __exit__(self, *a):
        _ROLE[0] = self.prev


def reserve_workspace(device, nbytes: int, role: str = "main"):
    with workspace_role(role):
        _workspace(torch.device(device), nbytes)


def _gemm_native(layout: int, M: int, N_: int, K: int, a, lda: int, b, ldb: int, c, ldc: int, **kw):
    args = _gemm_args(layout, M, N_, K, a, lda, b, ldb, c, ldc, **kw)
    if a.dtype == torch.float32:
        N.check(N.lib().dtc_gemm_f32(args, N.stream_ptr(c.device)), "dtc_gemm_f32")
    else:
        N.check(N.lib().dtc_gemm(args, N.stream_ptr(c.device)), "dtc_gemm")


def _gemm_args(layout: int, M: int, N_: int, K: int, a, lda: int, b, ldb: int, c, ldc: int, *,
               epi: int = N.EPI_STORE, bias=None, aux=None, ldaux: int = 0, aux_out=None,
               alpha: float = 1.0, beta: float = 0.0, labels=None, vocab_start: int = 0,
               n_valid: int = 0, part=None, label_out=None, workspace=None, defer_reduce: int = 0,
               colsum=None) -> "N.GemmArgs":
    L = N.lib()
    if workspace is not None:
        ws = workspace.view(torch.uint8) if workspace.dtype != torch.uint8 else workspace
    else:
        if a.dtype == torch.float32:
            ws_need = int(L.dtc_gemm_f32_workspace_bytes(layout, M, N_, K))
        else:
            ws_need = int(L.dtc_gemm_workspace_bytes(layout, M, N_, K))
        ws = _workspace(c.device, ws_need) if ws_need > 0 else None
    args = N.GemmArgs(
        layout=layout, M=M, N=N_, K=K,
        A=a.data_ptr(), lda=lda, B=b.data_ptr(), ldb=ldb, C=c.data_ptr(), ldc=ldc,
        c_f32=1 if c.dtype == torch.float32 else 0, epi=epi,
        bias=N.ptr(bias), aux=N.ptr(aux), ldaux=ldaux, aux_out=N.ptr(aux_out),
        alpha=alpha, beta=beta, labels=N.ptr(labels), vocab_start=vocab_start, n_valid=n_valid,
        part=N.ptr(part), label_out=N.ptr(label_out),
        workspace=N.ptr(ws), ws_bytes=0 if ws is None else ws.numel(), split_k=0, defer_reduce=defer_reduce,
        colsum=N.ptr(colsum))
    return args


def _check2d(t: torch.Tensor, name: str):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a row-major 2-D tensor, got shape {tuple(t.shape)} strides {t.stride()}")
    if t.is_cuda and t.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError(f"{name}: GPU GEMM operands are bf16 (MFMA bf16) or fp32 (exact fp32 MFMA), got {t.dtype}")


def _f32(t):
    return None if t is None else t.float()


# ----------------------------------------------------------------------------- forward
def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    M, K = x.shape
    Nn = w.shape[0]
    assert w.shape[1] == K
    out_dtype = out_dtype or x.dtype
    if N.library_path(x):
        y = _f32(x) @ _f32(w).t()
        if bias is not None:
            y = y + bias.float()
        return y.to(out_dtype)
    _check2d(x, "x"); _check2d(w, "w")
    y = torch.empty(M, Nn, dtype=out_dtype, device=x.device)
    _gemm_native(0, M, Nn, K, x, x.stride(0), w, w.stride(0), y, Nn, bias=bias)
    return y


class RawOut:
    """A GEMM output that is not a torch tensor: a raw device pointer to a row-major [M, N] buffer
    (ldc = N) -- the own half of the P2P all-reduce buffer a row-parallel GEMM writes its partial
    into (parallel/p2p.py ``staged_out``), so no copy kernel stages it."""

    __slots__ = ("ptr", "dtype", "device")

    def __init__(self, ptr: int, dtype: torch.dtype, device):
        self.ptr, self.dtype, self.device = int(ptr), dtype, torch.device(device)

    def data_ptr(self) -> int:
        return self.ptr


def linear_into(x: torch.Tensor, w: torch.Tensor, out: RawOut):
    """``out = x·Wᵀ`` (no bias) into a raw buffer (bf16 or fp32 per ``out.dtype``)."""
    M, K = x.shape
    Nn = w.shape[0]
    assert w.shape[1] == K and x.is_cuda
    _check2d(x, "x"); _check2d(w, "w")
    _gemm_native(0, M, Nn, K, x, x.stride(0), w, w.stride(0), out, Nn)


def matmul_nn_into(dy: torch.Tensor, w: torch.Tensor, out: RawOut):
    """``out = dY·W`` (W [N, K] row-major, the NN dgrad) into a raw buffer."""
    M, Nn = dy.shape
    K = w.shape[1]
    assert w.shape[0] == Nn and dy.is_cuda
    _check2d(dy, "dy"); _check2d(w, "w")
    _gemm_native(1, M, K, Nn, dy, dy.stride(0), w, w.stride(0), out, K)


def linear_resid(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor],
                 resid: Optional[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 ``out = resid + x·Wᵀ + bias`` (resid/bias optional; ``out`` may alias ``resid``)."""
    M, K = x.shape
    Nn = w.shape[0]
    if N.library_path(x):
        y = _f32(x) @ _f32(w).t()
        if bias is not None:
            y = y + bias.float()
        if resid is not None:
            y = y + resid
        if out is not None:
            out.copy_(y)
            return out
        return y
    _check2d(x, "x"); _check2d(w, "w")
    if out is None:
        out = torch.empty(M, Nn, dtype=torch.float32, device=x.device)
    if resid is not None:
        assert resid.dtype == torch.float32 and resid.is_contiguous()
        _gemm_native(0, M, Nn, K, x, x.stride(0), w, w.stride(0), out, Nn, epi=N.EPI_RESID, bias=bias,
                     aux=resid, ldaux=Nn)
    else:
        _gemm_native(0, M, Nn, K, x, x.stride(0), w, w.stride(0), out, Nn, bias=bias)
    return out


def linear_gelu(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor]):
    """Returns ``(d, g)`` for ``u = x·Wᵀ + b``: ``d = gelu_tanh'(u)`` (the dGELU factor the fc2 dgrad
    multiplies by: the backward needs no transcendental) and ``g = gelu_tanh(u)`` (activation dtype)."""
    M, K = x.shape
    Nn = w.shape[0]
    if N.library_path(x):
        u = _f32(x) @ _f32(w).t()
        if bias is not None:
            u = u + bias.float()
        return gelu_tanh_grad(u).to(x.dtype), gelu_tanh(u).to(x.dtype)
    _check2d(x, "x"); _check2d(w, "w")
    u = torch.empty(M, Nn, dtype=x.dtype, device=x.device)
    g = torch.empty_like(u)
    _gemm_native(0, M, Nn, K, x, x.stride(0), w, w.stride(0), u, Nn, epi=N.EPI_GELU, bias=bias, aux_out=g)
    return u, g


# ----------------------------------------------------------------------------- backward
def matmul_nn(dy: torch.Tensor, w: torch.Tensor, out_dtype=torch.float32) -> torch.Tensor:
    """dX[M,K] = dY[M,N]·W[N,K]."""
    M, Nn = dy.shape
    K = w.shape[1]
    assert w.shape[0] == Nn
    if N.library_path(dy):
        return (_f32(dy) @ _f32(w)).to(out_dtype)
    _check2d(dy, "dy"); _check2d(w, "w")
    dx = torch.empty(M, K, dtype=out_dtype, device=dy.device)
    _gemm_native(1, M, K, Nn, dy, dy.stride(0), w, w.stride(0), dx, K)
    return dx


def matmul_nn_dgelu(dy: torch.Tensor, w: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """dU = (dY·W) ⊙ u  with ``u = gelu_tanh'(pre-activation)`` from :func:`linear_gelu`
    (fc2 dgrad fused with the GELU backward)."""
    M, Nn = dy.shape
    K = w.shape[1]
    if N.library_path(dy):
        return ((_f32(dy) @ _f32(w)) * _f32(u)).to(u.dtype)
    _check2d(dy, "dy"); _check2d(w, "w")
    du = torch.empty(M, K, dtype=u.dtype, device=dy.device)
    _gemm_native(1, M, K, Nn, dy, dy.stride(0), w, w.stride(0), du, K, epi=N.EPI_DGELU, aux=u, ldaux=K)
    return du


def matmul_nt_dgelu(dy: torch.Tensor, wt: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """dU = (dY·W) ⊙ u with W given transposed (``wt`` = Wᵀ, [K, N]): the fc2 dgrad fused with the
    GELU backward as an NT GEMM (both operands K-major)."""
    M = dy.shape[0]
    K = wt.shape[0]
    if N.library_path(dy):
        return ((_f32(dy) @ _f32(wt).t()) * _f32(u)).to(u.dtype)
    _check2d(dy, "dy"); _check2d(wt, "wt")
    du = torch.empty(M, K, dtype=u.dtype, device=dy.device)
    _gemm_native(0, M, K, dy.shape[1], dy, dy.stride(0), wt, wt.stride(0), du, K, epi=N.EPI_DGELU, aux=u, ldaux=K)
    return du


def wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, beta: float = 0.0, red=None,
          db: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dW[N,K] = β·dW + dY[M,N]ᵀ·X[M,K]  (fp32 ``dw`` is a view into the flat grad buffer);
    with ``db``: also db[N] = β·db + Σ_m dY[m, :] (the layer's bias gradient).

    ``red`` (an ``ops.reduce.GradReducer``): a split-K GEMM leaves its fp32 slabs in the reducer's
    arena and the final sum (+β·dW) happens in the reducer's next batched launch; the bias
    gradient is then summed inside the GEMM (column sums of the dY tiles it already loads)."""
    M, Nn = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and tuple(dw.shape) == (Nn, K)
    if N.library_path(dy):
        g = _f32(dy).t() @ _f32(x)
        if beta != 0.0:
            dw.mul_(beta).add_(g)
        else:
            dw.copy_(g)
        if db is not None:
            colsum(dy, db, beta)
        return dw
    _check2d(dy, "dy"); _check2d(x, "x")
    assert dw.dtype == torch.float32 and dw.is_contiguous()
    if dy.dtype == torch.float32:  # exact-fp32 kernel: split-K + its own fixed-order reduce
        _gemm_native(2, Nn, K, M, dy, dy.stride(0), x, x.stride(0), dw, K, beta=beta)
        if db is not None:
            colsum(dy, db, beta, red=red)
        return dw
    if red is not None:
        L = N.lib()
        split = int(L.dtc_gemm_wgrad_split(Nn, K, M, 1 if db is not None else 0))
        cs = None
        if db is not None and L.dtc_gemm_wgrad_fuses_colsum(Nn, K, M):
            cs = red.alloc(split * Nn)
        elif db is not None:
            colsum(dy, db, beta, red=red)
        if split > 1:
            slab = red.alloc(split * Nn * K)
            _gemm_native(2, Nn, K, M, dy, dy.stride(0), x, x.stride(0), dw, K, beta=beta, workspace=slab,
                         defer_reduce=1, colsum=cs)
            red.add_wide(slab, dw, split, beta)
        else:
            _gemm_native(2, Nn, K, M, dy, dy.stride(0), x, x.stride(0), dw, K, beta=beta, colsum=cs)
        if cs is not None:
            red.add_wide(cs, db, split, beta)
        return dw
    _gemm_native(2, Nn, K, M, dy, dy.stride(0), x, x.stride(0), dw, K, beta=beta)
    if db is not None:
        colsum(dy, db, beta)
    return dw


_WG_CHECKED = [False]


WG_SQ_SLOTS = 8  # grad-norm partial slots per 256² tile (one per wave of gemm8p_group_kernel)


def wgrad_tiles(m: int, n: int) -> int:
    """256² tiles of one grouped weight-gradient problem dW[m, n] (WG_SQ_SLOTS grad-norm slots each)."""
    return ((m + 255) // 256) * ((n + 255) // 256)


# DTC_WG_TAIL_SPLIT: the grouped launch's last, partly filled round of whole tiles runs as K-pieces of those
# tiles (0 off, 1 auto = CUs // tail pieces, clamped to 2..4; >= 2 forced), finished by wg_tail_reduce.
# Default 1: GPT-2 small 1887 tiles = 7 rounds + 95 -> 7 rounds + 190 half tiles, step -0.07 ms
# (profiles/r4_ab_wg_tail.log)
_WG_TAIL = int(__import__("os").environ.get("DTC_WG_TAIL_SPLIT", "1"))
_CUS = {}


def _cu_count(device) -> int:
    n = _CUS.get(device.index)
    if n is None:
        n = _CUS[device.index] = torch.cuda.get_device_properties(device).multi_processor_count
    return n


def wgrad_group(items, beta: float = 0.0, red=None, sq: Optional[torch.Tensor] = None):
    """Weight gradients of several Dense layers that share the token dimension, in ONE launch:
    for every ``(dy, x, dw, db)``: dW = β·dW + dYᵀ·X and (``db`` not None) db = β·db + Σ_rows dY.

    GPU bf16: ``gemm8p_group_kernel`` (csrc/gemm.hip) runs whole 256² tiles of every problem — no
    split-K slabs and no reduction pass, the bias gradients summed by the tiles' MFMAs.  Problems it
    cannot take (fp32 operands, a width not a multiple of 8, tokens not a multiple of 64) go through
    :func:`wgrad` one by one (``red``: its batched reducer), as do CPU tensors.

    ``sq`` (fp32, >= WG_SQ_SLOTS · Σ :func:`wgrad_tiles` slots): every tile's waves also write the sums of
    squares of their final dW values there (the global grad norm's partials, so the norm pass skips these grads); then every
    item must take the grouped kernel."""
    if not items:
        return
    dy0 = items[0][0]
    K = dy0.shape[0]
    ok = (dy0.is_cuda and dy0.dtype == torch.bfloat16 and K % 64 == 0)
    fast, slow = [], []
    for it in items:
        dy, x, dw, db = it
        good = (ok and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.shape[0] == K
                and x.shape[0] == K and dy.is_contiguous() and x.is_contiguous() and dw.is_contiguous()
                and dw.dtype == torch.float32 and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0
                and tuple(dw.shape) == (dy.shape[1], x.shape[1]) and dw.data_ptr() % 16 == 0
                and (db is None or (db.is_contiguous() and db.dtype == torch.float32)))
        (fast if good else slow).append(it)
    if sq is not None and slow:
        raise ValueError("wgrad_group(sq=...): every problem must take the grouped kernel "
                         f"({len(slow)} of {len(items)} cannot)")
    for dy, x, dw, db in slow:
        wgrad(dy, x, dw, beta, red=red, db=db)
    if not fast:
        return
    L = N.lib()
    if not _WG_CHECKED[0]:
        assert L.dtc_wg_entry_bytes() == ctypes.sizeof(N.WgEntry) and L.dtc_wg_max() == N.WG_MAX
        assert L.dtc_wg_batch_bytes() == ctypes.sizeof(N.WgBatch)
        _WG_CHECKED[0] = True
    # largest problems first: their tiles start in the first rounds, the small ones fill the tail.  With
    # the tail split the bias-free problems (the lm_head's) go last: the split tail tiles carry no bias sums
    if _WG_TAIL:
        fast.sort(key=lambda it: (it[3] is None, -(it[0].shape[1] * it[1].shape[1])))
    else:
        fast.sort(key=lambda it: -(it[0].shape[1] * it[1].shape[1]))
    if sq is not None:
        assert sq.dtype == torch.float32 and sq.is_contiguous() and sq.is_cuda
        assert sq.numel() >= WG_SQ_SLOTS * sum(wgrad_tiles(it[0].shape[1], it[1].shape[1]) for it in fast), "sq"
    off = 0
    for i0 in range(0, len(fast), N.WG_MAX):
        chunk = fast[i0:i0 + N.WG_MAX]
        b = N.WgBatch()
        b.n, b.K, b.beta, b.ntiles = len(chunk), K, float(beta), 0
        b.sq = None if sq is None else sq.data_ptr() + 4 * WG_SQ_SLOTS * off
        if _WG_TAIL:  # fp32 tile slabs of the split tail (the kernel re-derives tail and split, checks the cap)
            t = sum(wgrad_tiles(it[0].shape[1], it[1].shape[1]) for it in chunk)
            cus = _cu_count(dy0.device)
            tail = t % cus if t > cus else 0
            split = _WG_TAIL if _WG_TAIL > 1 else max(2, min(4, cus // tail)) if tail else 0
            nbytes = tail * split * 256 * 256 * 4
            if nbytes:
                b.tail_split, b.tail_slab, b.tail_cap = _WG_TAIL, _workspace(dy0.device, nbytes).data_ptr(), nbytes // 4
        for j, (dy, x, dw, db) in enumerate(chunk):
            b.e[j] = N.WgEntry(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), N.ptr(db), dy.shape[1], x.shape[1], 0, 0)
            off += wgrad_tiles(dy.shape[1], x.shape[1])
        N.check(L.dtc_wgrad_group(ctypes.byref(b), N.stream_ptr(dy0.device)), "dtc_wgrad_group")


_PAIR = __import__("os").environ.get("DTC_GEMM_PAIR", "1") == "1"  # A/B knob for the paired launch


def linear_backward(dy: torch.Tensor, w: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, beta: float = 0.0,
                    red=None, db: Optional[torch.Tensor] = None, dgelu_u: Optional[torch.Tensor] = None,
                    out_dtype=torch.float32, pair: bool = True, wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Both backward GEMMs of a Dense ``y = x·Wᵀ (+b)``: returns dX = dY·W (⊙ gelu'(u) when
    ``dgelu_u`` is given — the fc2 dgrad fused with the GELU backward) and accumulates
    dW = β·dW + dYᵀ·X (+ db = β·db + Σ_rows dY).

    On the GPU with a batched reducer both GEMMs go out as ONE launch (``dtc_gemm_pair``: they
    read the same dY, the weight gradient's blocks fill the CUs the dgrad's last wave leaves
    idle, one dependent kernel boundary less); otherwise two calls.  ``wt``: the transposed weight
    ``[in, out]`` (``FlatParams.wt``) — the dgrad then runs as an NT GEMM (both operands K-major)."""
    if N.library_path(dy) or red is None or not (_PAIR and pair) or dy.dtype == torch.float32:
        if wt is not None and not N.library_path(dy):
            dx = matmul_nt_dgelu(dy, wt, dgelu_u) if dgelu_u is not None else linear(dy, wt, out_dtype=out_dtype)
        else:
            dx = matmul_nn_dgelu(dy, w, dgelu_u) if dgelu_u is not None else matmul_nn(dy, w, out_dtype=out_dtype)
        wgrad(dy, x, dw, beta, red=red, db=db)
        return dx
    _check2d(dy, "dy"); _check2d(w, "w"); _check2d(x, "x")
    assert dw.dtype == torch.float32 and dw.is_contiguous()
    L = N.lib()
    M, Nn = dy.shape
    K = w.shape[1]
    Kx = x.shape[1]
    assert w.shape[0] == Nn and x.shape[0] == M and tuple(dw.shape) == (Nn, Kx)
    lay, bw = (0, wt) if wt is not None else (1, w)
    if wt is not None:
        assert tuple(wt.shape) == (K, Nn)
    if dgelu_u is not None:
        dx = torch.empty(M, K, dtype=torch.bfloat16, device=dy.device)
        a1 = _gemm_args(lay, M, K, Nn, dy, dy.stride(0), bw, bw.stride(0), dx, K, epi=N.EPI_DGELU, aux=dgelu_u, ldaux=K)
    else:
        dx = torch.empty(M, K, dtype=out_dtype, device=dy.device)
        a1 = _gemm_args(lay, M, K, Nn, dy, dy.stride(0), bw, bw.stride(0), dx, K)
    split = int(L.dtc_gemm_wgrad_split(Nn, Kx, M, 1 if db is not None else 0))
    fuse_cs = db is not None and bool(L.dtc_gemm_wgrad_fuses_colsum(Nn, Kx, M))
    mark = red.off
    cs = red.alloc(split * Nn) if fuse_cs else None
    slab = red.alloc(split * Nn * Kx) if split > 1 else None
    a2 = _gemm_args(2, Nn, Kx, M, dy, dy.stride(0), x, x.stride(0), dw, Kx, beta=beta, workspace=slab,
                    defer_reduce=1 if split > 1 else 0, colsum=cs)
    rc = L.dtc_gemm_pair(a1, a2, N.stream_ptr(dy.device))
    if rc == 1100:  # not pairable (tile plans): two launches
        red.off = mark
        N.check(L.dtc_gemm(a1, N.stream_ptr(dy.device)), "dtc_gemm")
        wgrad(dy, x, dw, beta, red=red, db=db)
        return dx
    N.check(rc, "dtc_gemm_pair")
    if slab is not None:
        red.add_wide(slab, dw, split, beta)
    if cs is not None:
        red.add_wide(cs, db, split, beta)
    elif db is not None:
        colsum(dy, db, beta, red=red)
    return dx


def colsum(dy: torch.Tensor, db: torch.Tensor, beta: float = 0.0, red=None) -> torch.Tensor:
    """db[N] = β·db + Σ_m dY[m, :]  (deterministic two-stage reduction on GPU; with ``red`` the
    second stage is a task of the reducer's next batched launch)."""
    M, Nn = dy.shape
    if not dy.is_cuda:
        s = _f32(dy).sum(0)
        if beta != 0.0:
            db.mul_(beta).add_(s)
        else:
            db.copy_(s)
        return db
    L = N.lib()
    nbytes = int(L.dtc_colsum_workspace_bytes(M, Nn))
    ws = _workspace(dy.device, nbytes) if red is None else red.alloc(nbytes // 4)
    is_f32 = 1 if dy.dtype == torch.float32 else 0
    N.check(L.dtc_colsum(dy.data_ptr(), is_f32, M, Nn, dy.stride(0), db.data_ptr(), beta,
                         ws.data_ptr(), nbytes if red is not None else ws.numel(), 1 if red is not None else 0,
                         N.stream_ptr(dy.device)), "dtc_colsum")
    if red is not None:
        red.add_tall(ws.data_ptr(), Nn, nbytes // 4 // Nn, db, beta)
    return db
