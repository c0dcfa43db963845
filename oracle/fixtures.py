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


def duplicate_columns_case():
    """A sampled layer whose row 1 names column 3 twice (out of column order) and row 4 column 0 twice (the
    reference's samplers never make one; its .coalesce() sums them, cuda_spmm.cu:825)."""
    M, K = 6, 5
    lens = np.array([2, 4, 0, 1, 3, 2])
    rowptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.array([1, 4, 3, 0, 3, 2, 2, 0, 4, 0, 0, 1], np.int64)
    full = np.concatenate([[0], np.cumsum(lens + np.array([3, 1, 2, 0, 5, 1]))]).astype(np.int32)
    nf = np.linspace(0.25, 2.0, K).astype(np.float32)
    return M, K, full, rowptr, col, nf


def coalesced_reference(M, K, full, rowptr, col, nf):
    """The reference's create_coo_tensor on the host: cuda_spmm.cu:800's values, then .coalesce()."""
    import torch

    rows = np.repeat(np.arange(M), np.diff(rowptr))
    deg = np.diff(full).astype(np.float64)
    val = ((1.0 / deg)[rows] * nf.astype(np.float64)[col]).astype(np.float32)
    return torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, col])), torch.from_numpy(val), (M, K)).coalesce()

