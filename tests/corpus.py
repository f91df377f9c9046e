"""Seeded synthetic corpora (Zipf rank-frequency), as SURVEY.md §8(d) plans."""
from __future__ import annotations

import numpy as np


def zipf_ids(n_tokens: int, vmax: int, s: float = 1.0, seed: int = 0) -> np.ndarray:
    """Token ranks 0..vmax-1 drawn with p(r) ∝ (r+1)^-s."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, vmax + 1, dtype=np.float64) ** s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return np.searchsorted(cdf, rng.random(n_tokens), side="right").astype(np.int64).clip(0, vmax - 1)


def zipf_sentences(n_sent: int, sent_len: int, vmax: int, seed: int = 0, ragged: bool = False):
    """List of sentences of string tokens 'w<rank>'."""
    rng = np.random.default_rng(seed + 1)
    lens = rng.integers(1, sent_len + 1, n_sent) if ragged else np.full(n_sent, sent_len)
    ids = zipf_ids(int(lens.sum()), vmax, seed=seed)
    out, k = [], 0
    for L in lens:
        out.append([f"w{r}" for r in ids[k:k + L]])
        k += L
    return out
