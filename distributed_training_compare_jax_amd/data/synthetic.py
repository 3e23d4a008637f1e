"""Synthetic FineWeb-shaped token stream.

The reference streams FineWeb-edu through the GPT-2 tokenizer and yields non-overlapping
``int32 [batch, seq_len]`` chunks (``data/fineweb_edu.py:15-39``); the driver asks for
``seq_len = max_seq_len + 1`` and splits ``x = [:, :-1]``, ``y = [:, 1:]``
(``train/train.py:55,66-67``).  There is no network here, so this module produces a
deterministic stream of the same shape and vocabulary (50257 BPE ids; the added
``<pad>`` id 50257 never occurs, exactly as in the reference data).

Design (host side; native C++ sampler ``csrc/host_data.cpp`` when built, else vectorised
numpy — bit-identical token streams either way):

* Every token is a pure function of ``(seed, global token position)`` through a
  splitmix64 counter hash, so any rank can generate exactly its own rows of the global
  batch — the stream is identical whatever the DP/TP/PP layout (layout-invariant data,
  like the reference's single shared iterator).
* Marginals are Zipf-like (natural-text-shaped unigram histogram), and half of the
  tokens follow a fixed random bigram map ``succ[prev]`` so the loss actually falls
  (a learnable signal, floor well below the unigram entropy).
"""

from __future__ import annotations

import ctypes
import os
from typing import Iterator, Optional

import numpy as np

from ..config.schema import REFERENCE_VOCAB_SIZE

BPE_VOCAB = REFERENCE_VOCAB_SIZE - 1  # ids the data can contain (pad id excluded)

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def _key(seed: int, stream: int) -> int:
    return (seed * 0x632BE59BD9B4E019 + stream * 0x8CB92BA72F3D8DD7) & 0xFFFFFFFFFFFFFFFF


def _uniform(seed: int, stream: int, pos: np.ndarray) -> np.ndarray:
    key = np.uint64(_key(seed, stream))
    with np.errstate(over="ignore"):
        h = _splitmix64(pos.astype(np.uint64) ^ key)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


_HOST_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_dtc_host.so")
_host = None


def host_lib():
    """The native host runtime (``csrc/host_data.cpp`` -> ``_dtc_host.so``), or None if not built
    (then the vectorised numpy path runs; both produce the same tokens bit for bit).
    ``DTC_NATIVE_DATA=0`` forces the numpy path."""
    global _host
    if _host is None:
        _host = False
        if os.environ.get("DTC_NATIVE_DATA", "1") != "0" and os.path.exists(_HOST_LIB):
            lib = ctypes.CDLL(_HOST_LIB)
            f = lib.dtc_synth_tokens
            u64, i64, vp = ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p
            f.argtypes = [u64, u64, vp, ctypes.c_int, vp, ctypes.c_int, vp, vp, ctypes.c_double, i64, i64, vp]
            f.restype = ctypes.c_int
            _host = lib
    return _host or None


class SyntheticTokenStream:
    """Row-addressable deterministic token source with FineWeb-like statistics."""

    GUIDE_BITS = 16  # u-buckets of the native sampler's guide table

    def __init__(self, vocab: int = BPE_VOCAB, seed: int = 0, zipf_s: float = 1.1, p_bigram: float = 0.5,
                 native: Optional[bool] = None):
        self.vocab = int(vocab)
        self.seed = int(seed)
        self.p_bigram = float(p_bigram)
        ranks = np.arange(1, self.vocab + 1, dtype=np.float64)
        w = ranks ** (-zipf_s)
        self.cdf = np.cumsum(w / w.sum())
        self.cdf[-1] = 1.0
        rng = np.random.default_rng(self.seed + 12345)
        # frequency rank -> token id, and a fixed successor map (the learnable structure)
        self.rank_to_id = rng.permutation(self.vocab).astype(np.int64)
        self.succ = rng.permutation(self.vocab).astype(np.int64)
        self._lib = host_lib() if native is None or native else None
        if native and self._lib is None:
            raise RuntimeError(f"native data pipeline requested but {_HOST_LIB} is not built")
        if self._lib is not None:
            g = 1 << self.GUIDE_BITS
            self._guide = np.searchsorted(self.cdf, np.arange(g + 1, dtype=np.float64) / g,
                                          side="right").astype(np.int32)

    def tokens(self, start: int, count: int) -> np.ndarray:
        """Tokens at global positions [start, start+count) as int32."""
        if self._lib is not None:
            out = np.empty(count, dtype=np.int32)
            rc = self._lib.dtc_synth_tokens(_key(self.seed, 1), _key(self.seed, 2), self.cdf.ctypes.data, self.vocab,
                                            self._guide.ctypes.data, self.GUIDE_BITS, self.rank_to_id.ctypes.data,
                                            self.succ.ctypes.data, self.p_bigram, start, count, out.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"dtc_synth_tokens failed ({rc})")
            return out
        return self.tokens_numpy(start, count)

    def tokens_numpy(self, start: int, count: int) -> np.ndarray:
        """Vectorised numpy path (fallback and test oracle of the native sampler)."""
        pos = np.arange(start - 1, start + count, dtype=np.int64)
        z = self.rank_to_id[np.searchsorted(self.cdf, _uniform(self.seed, 1, pos), side="right").clip(0, self.vocab - 1)]
        follow = _uniform(self.seed, 2, pos[1:]) < self.p_bigram
        out = np.where(follow, self.succ[z[:-1]], z[1:])
        return out.astype(np.int32)

    def rows(self, step: int, row0: int, nrows: int, batch: int, seq_len: int) -> np.ndarray:
        """Rows [row0, row0+nrows) of global batch ``step`` (each row = seq_len tokens)."""
        base = (step * batch + row0) * seq_len
        return self.tokens(base, nrows * seq_len).reshape(nrows, seq_len)


def get_tokenizer():
    """Reference ``get_tokenizer`` (GPT-2 + <pad>, len 50258).

    Tries the HF GPT-2 tokenizer (needs a local cache: there is no network); otherwise
    returns a stub whose ``len()`` is the reference vocab size, which is all main.py uses.
    """
    try:  # pragma: no cover - only with a cached tokenizer
        from transformers import AutoTokenizer

        tok = AutoTokenizer.from_pretrained("gpt2", local_files_only=True)
        tok.add_special_tokens({"pad_token": "<pad>"})
        return tok
    except Exception:
        class _Stub:
            pad_token_id = BPE_VOCAB

            def __len__(self):
                return REFERENCE_VOCAB_SIZE

        return _Stub()


def get_batch_iterator(batch_size: int, seq_len: int, seed: int = 0, row0: int = 0,
                       nrows: Optional[int] = None, start_step: int = 0,
                       vocab: int = BPE_VOCAB) -> Iterator[np.ndarray]:
    """Same contract as reference ``get_batch_iterator``: yields ``int32 [nrows, seq_len]``.

    ``batch_size`` is the GLOBAL batch; a rank passes ``row0``/``nrows`` to receive only
    its slice (DP), which is bit-identical to slicing the global batch.
    """
    stream = SyntheticTokenStream(vocab=vocab, seed=seed)
    n = batch_size if nrows is None else nrows
    step = start_step
    while True:
        yield stream.rows(step, row0, n, batch_size, seq_len)
        step += 1
