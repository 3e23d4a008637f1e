"""Token + position embedding with fused dropout (reference ``model/GPTModel.py:30-38``).

``h = dropout(wte[ids] + wpe[t])`` with inverted scaling ``1/(1-p)`` — the only dropout in
the reference model.  The mask comes from a counter-based Philox4x32-10 stream keyed on
``(seed, step)`` and indexed by the GLOBAL element index ``((row0 + b)·T + t)·D + d``, so
the mask is identical whatever the DP/TP/PP split (the reference draws one global mask
that GSPMD shards, ``train/create_train_step.py:31``).  The backward regenerates the mask
(nothing stored).  ``step`` is a device-resident int64 counter so the whole step can be
replayed from a hipGraph.

GPU path: ``csrc/elementwise.hip``.  The CPU path below reproduces the kernel's Philox bits
exactly (tested).
"""

from __future__ import annotations

import numpy as np
import torch

from . import _native as N

PHILOX_M0 = 0xD2511F53
PHILOX_M1 = 0xCD9E8D57
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85
_U32 = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0: int, k1: int, rounds: int = 10):
    """Vectorised Philox4x32 (numpy uint64 lanes holding uint32 values)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _U32 for c in (c0, c1, c2, c3))
    k0 = np.uint64(k0 & 0xFFFFFFFF)
    k1 = np.uint64(k1 & 0xFFFFFFFF)
    for r in range(rounds):
        if r > 0:
            k0 = np.uint64((int(k0) + PHILOX_W0) & 0xFFFFFFFF)
            k1 = np.uint64((int(k1) + PHILOX_W1) & 0xFFFFFFFF)
        p0 = c0 * np.uint64(PHILOX_M0)
        p1 = c2 * np.uint64(PHILOX_M1)
        hi0, lo0 = p0 >> np.uint64(32), p0 & _U32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _U32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _U32, lo1, (hi0 ^ c3 ^ k1) & _U32, lo0
    return c0, c1, c2, c3


def dropout_keep_mask(n_tokens: int, D: int, token0: int, p: float, seed: int, step: int) -> torch.Tensor:
    """Keep-mask [n_tokens, D] (bool) for global tokens [token0, token0+n_tokens)."""
    assert D % 4 == 0
    e0 = token0 * D
    groups = np.arange(e0 // 4, (e0 + n_tokens * D) // 4, dtype=np.uint64)
    r = philox4x32(groups & _U32, groups >> np.uint64(32), 0, 0, seed, step)
    u = np.stack(r, axis=1).reshape(-1)  # element e = 4*group + lane
    thr = np.uint64(min(int(p * 4294967296.0), 0xFFFFFFFF))
    keep = u >= thr
    return torch.from_numpy(keep.reshape(n_tokens, D))


def embed_fwd(ids: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor, p: float, seed: int,
              step: torch.Tensor, row0: int) -> torch.Tensor:
    """ids int32 [B,T] → h fp32 [B*T, D]."""
    B, T = ids.shape
    D = wte.shape[1]
    if not ids.is_cuda:
        h = wte[ids.long()].float() + wpe[:T].float()[None]
        h = h.reshape(B * T, D)
        if p > 0.0:
            keep = dropout_keep_mask(B * T, D, row0 * T, p, seed, int(step.item()))
            h = torch.where(keep, h / (1.0 - p), torch.zeros_like(h))
        return h
    assert ids.dtype == torch.int32 and ids.is_contiguous() and wte.dtype == torch.float32
    h = torch.empty(B * T, D, dtype=torch.float32, device=ids.device)
    N.check(N.lib().dtc_embed_fwd(ids.data_ptr(), wte.data_ptr(), wpe.data_ptr(), h.data_ptr(), B, T, D,
                                  wte.shape[0], p, seed, step.data_ptr(), row0, N.stream_ptr(ids.device)),
            "dtc_embed_fwd")
    return h


def embed_sq_slots(B: int, T: int, D: int) -> int:
    """Partial slots :func:`embed_bwd` writes into ``sq`` (``dtc_embed_sq_slots``)."""
    return int(N.lib().dtc_embed_sq_slots(B, T, D))


def embed_bwd(ids: torch.Tensor, dh: torch.Tensor, dwte: torch.Tensor, dwpe: torch.Tensor, p: float, seed: int,
              step: torch.Tensor, row0: int, beta: float = 0.0, keys: torch.Tensor = None, sq: torch.Tensor = None,
              prev_keys: torch.Tensor = None, prev_valid: bool = False):
    """dwte (β·)+= scatter_add(ids, dropout'(dh)); dwpe (β·)+= Σ_b dropout'(dh).

    GPU path is bitwise deterministic (sorted segment sums, no float atomics; see
    ``csrc/elementwise.hip``); ``keys`` = :func:`embed_sort_keys` of ``ids`` if precomputed.
    ``sq`` (GPU, beta = 0, one sort window): :func:`embed_sq_slots` fp32 partials whose sum is Σ dwte² + Σ dwpe²
    of the new grads (the gradient norm's share of both tables without reading them again).
    ``prev_keys`` (GPU, beta = 0, one sort window): int32 [B*T] that holds the previous call's sort keys for this
    same ``dwte`` (``prev_valid``) -- only their rows are zeroed instead of the whole table -- and receives this
    call's keys."""
    B, T = ids.shape
    D = dh.shape[1]
    if not ids.is_cuda:
        g = dh.float()
        if p > 0.0:
            keep = dropout_keep_mask(B * T, D, row0 * T, p, seed, int(step.item()))
            g = torch.where(keep, g / (1.0 - p), torch.zeros_like(g))
        if beta == 0.0:
            dwte.zero_()
            dwpe.zero_()
        dwte.index_add_(0, ids.reshape(-1).long(), g)
        dwpe[:T].add_(g.view(B, T, D).sum(0))
        return
    if sq is not None:
        assert beta == 0.0 and B * T <= SORT_MAX and sq.dtype == torch.float32 and sq.is_contiguous()
        assert sq.numel() == embed_sq_slots(B, T, dh.shape[1]), (sq.numel(), B, T)
    if prev_keys is not None:
        assert beta == 0.0 and B * T <= SORT_MAX and prev_keys.numel() == B * T and prev_keys.dtype == torch.int32
    if B * T > SORT_MAX:  # sort capacity of one workgroup: accumulate row chunks in order
        rows = max(1, SORT_MAX // T)
        for r0 in range(0, B, rows):
            r1 = min(B, r0 + rows)
            embed_bwd(ids[r0:r1], dh[r0 * T:r1 * T], dwte, dwpe, p, seed, step, row0 + r0,
                      beta if r0 == 0 else 1.0)
        return
    if keys is None:
        keys = embed_sort_keys(ids, dwte.shape[0])
    assert keys.numel() == B * T and dh.shape[0] == B * T and dh.is_contiguous()
    P = torch.empty(B * T, D, dtype=torch.float32, device=dh.device)
    N.check(N.lib().dtc_embed_bwd(keys.data_ptr(), dh.data_ptr(), dwte.data_ptr(), dwpe.data_ptr(), P.data_ptr(), B,
                                  T, D, dwte.shape[0], p, seed, step.data_ptr(), row0, 1 if beta != 0.0 else 0,
                                  N.ptr(sq), N.ptr(prev_keys), 1 if prev_valid else 0, N.stream_ptr(ids.device)),
            "dtc_embed_bwd")


SORT_MAX = 32768  # keys one LDS bitonic sort handles (csrc/elementwise.hip)


def sort_bits(n: int) -> int:
    """Token-index bits of a sort key (``dtc_embed_sort_bits``)."""
    nb = 1
    while (1 << nb) < n:
        nb += 1
    return nb


def embed_sort_keys_host(ids: np.ndarray, out: np.ndarray = None) -> np.ndarray:
    """Host-side version of :func:`embed_sort_keys` (same keys: the sorted order of unique keys
    is unique).  The training loop computes them while the GPU runs the previous step and ships
    them with the batch, so no sort kernel sits in the step."""
    flat = np.ascontiguousarray(ids, dtype=np.int32).reshape(-1)
    n = flat.size
    keys = (flat.astype(np.uint32) << np.uint32(sort_bits(n))) | np.arange(n, dtype=np.uint32)
    keys.sort()
    if out is not None:
        out[:] = keys.view(np.int32)
        return out
    return keys.view(np.int32)


def embed_sort_keys(ids: torch.Tensor, vocab: int, out: torch.Tensor = None) -> torch.Tensor:
    """Sorted ``id << nb | token`` keys (int32 storage of uint32) for the deterministic backward.

    Depends only on the ids, so the step issues it right after the forward embedding, off the
    critical path (side stream)."""
    n = ids.numel()
    keys = out if out is not None else torch.empty(n, dtype=torch.int32, device=ids.device)
    N.check(N.lib().dtc_embed_sort(ids.data_ptr(), n, vocab, keys.data_ptr(), N.stream_ptr(ids.device)),
            "dtc_embed_sort")
    return keys
