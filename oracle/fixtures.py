"""TEST INFRASTRUCTURE: seeded random CSR operands with the edge cases the tests need."""
from __future__ import annotations

import numpy as np


def random_csr(M: int, K: int, lens, rng: np.random.Generator, full_extra: int = 3):
    """CSR with the given per-row lengths (clipped to K), ascending unique columns.

    Returns (fullrowptr, rowptr, col int32, normfact float32)."""
    lens = np.minimum(np.asarray(lens, dtype=np.int64), K)
    rowptr = np.zeros(M + 1, np.int32)
    rowptr[1:] = np.cumsum(lens)
    cols = [np.sort(rng.choice(K, int(l), replace=False)) for l in lens]
    col = (np.concatenate(cols) if cols else np.zeros(0)).astype(np.int32)
    full = np.zeros(M + 1, np.int32)
    full[1:] = np.cumsum(lens + rng.integers(0, full_extra + 1, M) + (lens == 0))
    normfact = rng.uniform(0.25, 8.0, K).astype(np.float32)
    return full, rowptr, col, normfact


def powerlaw_lens(M: int, mean: float, sigma: float, rng: np.random.Generator, max_len: int):
    l = rng.lognormal(np.log(max(mean, 1.0)) - sigma * sigma / 2, sigma, M).astype(np.int64)
    return np.clip(l, 0, max_len)
