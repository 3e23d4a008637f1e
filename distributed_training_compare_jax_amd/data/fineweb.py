"""Optional real FineWeb-edu stream (reference ``data/fineweb_edu.py:15-39``).

Needs the HF ``datasets`` + ``transformers`` caches and network access, neither of which
exists on the build or GPU boxes, so it is gated: selecting ``data: fineweb`` without
them raises a clear error instead of silently falling back.
"""

from __future__ import annotations

from typing import Iterator

import numpy as np


def get_batch_iterator(batch_size: int, seq_len: int, row0: int = 0, nrows: int | None = None) -> Iterator[np.ndarray]:
    try:
        from datasets import load_dataset
        from transformers import AutoTokenizer
    except Exception as e:  # pragma: no cover
        raise RuntimeError("data=fineweb needs `datasets` and `transformers`") from e
    try:
        tok = AutoTokenizer.from_pretrained("gpt2")
        tok.add_special_tokens({"pad_token": "<pad>"})
        ds = load_dataset("HuggingFaceFW/fineweb-edu", split="train", streaming=True)
    except Exception as e:  # pragma: no cover
        raise RuntimeError("FineWeb-edu / GPT-2 tokenizer not reachable (offline box); use data: synthetic") from e
    n = batch_size if nrows is None else nrows
    chunk = batch_size * seq_len
    buf: list[int] = []
    for item in ds:  # pragma: no cover
        buf.extend(tok.encode(item["text"]))
        while len(buf) >= chunk:
            batch = np.asarray(buf[:chunk], dtype=np.int32).reshape(batch_size, seq_len)
            del buf[:chunk]
            yield batch[row0:row0 + n]
