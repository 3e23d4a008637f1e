"""Synthetic FineWeb-shaped token stream.

The reference streams FineWeb-edu through the GPT-2 tokenizer and yields non-overlapping
``int32 [batch, seq_len]`` chunks (``data/fineweb_edu.py:15-39``); the driver asks for
``seq_len = max_seq_len + 1`` and splits ``x = [:, :-1]``, ``y = [:, 1:]``
(``train/train.py:55,66-67``).  There is no network here, so this module produces a
deterministic stream of the same shape and vocabulary (50257 BPE ids; the added
``<pad>`` id 50257 never occurs, exactly as in the reference data).

Design (host side, vectorised numpy, no Python per-token loop):

* Every token is a pure function of ``(seed, global token position)`` through a
  splitmix64 counter hash, so any rank can generate exactly its own rows of the global
  batch — the stream is identical whatever the DP/TP/PP layout (layout-invariant data,
  like the reference's single shared iterator).
* Marginals are Zipf-like (natural-text-shaped unigram histogram), and half of the
  tokens follow a fixed random bigram map ``succ[prev]`` so the loss actually falls
  (a learnable signal, floor well below the unigram entropy).
"""

from __future__ import annotations

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


def _uniform(seed: int, stream: int, pos: np.ndarray) -> np.ndarray:
    key = np.uint64((seed * 0x632BE59BD9B4E019 + stream * 0x8CB92BA72F3D8DD7) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        h = _splitmix64(pos.astype(np.uint64) ^ key)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


class SyntheticTokenStream:
    """Row-addressable deterministic token source with FineWeb-like statistics."""

    def __init__(self, vocab: int = BPE_VOCAB, seed: int = 0, zipf_s: float = 1.1, p_bigram: float = 0.5):
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

    def tokens(self, start: int, count: int) -> np.ndarray:
        """Tokens at global positions [start, start+count) as int32."""
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
