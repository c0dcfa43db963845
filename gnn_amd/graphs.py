"""Synthetic graph datasets with the shapes of the reference's benchmark graphs.

The reference loads GraphSAINT / OGB files (preprocess.py:17-143); none exist offline, so
the benchmarks and tests use seeded Chung-Lu graphs with a lognormal expected-degree
sequence. Feature rows are N(0,1) fp32, mirroring the StandardScaler
normalisation of preprocess.py:27-31; labels are one class per node (Reddit, products).

The returned tuple follows load_graphsaint_data (preprocess.py:52):
    (adj_full CSR float32, class_arr CSR, feat_data torch.FloatTensor, num_classes,
     train_nodes, valid_nodes, test_nodes)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import torch


@dataclass(frozen=True)
class GraphSpec:
    name: str
    num_nodes: int
    num_edge_samples: int  # endpoint pairs drawn before symmetrisation / dedup
    num_feats: int
    num_classes: int
    train_frac: float
    valid_frac: float
    sigma: float = 1.3


# Reddit (GraphSAINT): 232,965 nodes, 602 features, 41 classes, 153,431 train nodes.
REDDIT = GraphSpec("reddit", 232_965, 11_606_919, 602, 41, 153_431 / 232_965, 23_831 / 232_965)
# ogbn-products: 2,449,029 nodes, 100 features, 47 classes (public OGB statistics).
PRODUCTS = GraphSpec("ogbn-products", 2_449_029, 61_859_140, 100, 47, 0.08, 0.016)
# ogbn-papers100M per-batch geometry on a graph scaled to fit the box (128 feats, 172 classes).
PAPERS_SCALED = GraphSpec("ogbn-papers100M-scaled", 4_000_000, 60_000_000, 128, 172, 0.011, 0.001)
TINY = GraphSpec("tiny", 3_000, 15_000, 602, 41, 0.66, 0.1)
# Per-batch geometry of configs 3-5 at a size the GPU parity tests build in seconds: the same
# expected degree (edge samples per node) and feature / class widths on 500 k nodes, so a
# LADIES / FastGCN batch (samp 8192, batch 512) has the full-size layer shapes.
PRODUCTS_TEST = GraphSpec("ogbn-products-test", 500_000, 500_000 * 61_859_140 // 2_449_029, 100, 47, 0.08, 0.016)
PAPERS_TEST = GraphSpec("ogbn-papers100M-test", 500_000, 500_000 * 60_000_000 // 4_000_000, 128, 172, 0.011, 0.001)


def chung_lu(num_nodes: int, num_edge_samples: int, sigma: float, rng: np.random.Generator) -> sp.csr_matrix:
    """Undirected Chung-Lu graph, binary weights, no self loops, sorted CSR (float32)."""
    w = rng.lognormal(0.0, sigma, num_nodes)
    w /= w.sum()
    u = rng.choice(num_nodes, num_edge_samples, p=w)
    v = rng.choice(num_nodes, num_edge_samples, p=w)
    A = sp.csr_matrix((np.ones(num_edge_samples, np.float32), (u, v)), shape=(num_nodes, num_nodes))
    A = A + A.T
    A.data[:] = 1
    A.setdiag(0)
    A.eliminate_zeros()
    A.sort_indices()
    return A.astype(np.float32)


def make_dataset(spec: GraphSpec, seed: int = 0, with_features: bool = True):
    rng = np.random.default_rng(seed)
    A = chung_lu(spec.num_nodes, spec.num_edge_samples, spec.sigma, rng)
    N = spec.num_nodes
    cls = rng.integers(0, spec.num_classes, N)
    labels = sp.csr_matrix((np.ones(N, np.int32), (np.arange(N), cls)), shape=(N, spec.num_classes))
    if with_features:
        g = torch.Generator().manual_seed(seed)
        feats = torch.randn(N, spec.num_feats, generator=g, dtype=torch.float32)
    else:
        feats = None
    n_train = int(round(spec.train_frac * N))
    n_valid = int(round(spec.valid_frac * N))
    train = np.arange(0, n_train)
    valid = np.arange(n_train, n_train + n_valid)
    test = np.arange(n_train + n_valid, N)
    return A, labels, feats, spec.num_classes, train, valid, test


def row_normalize(mx: sp.spmatrix) -> sp.csr_matrix:
    """utils.py:56-64: D^-1 A (rows with zero sum stay zero)."""
    rowsum = np.array(mx.sum(1))
    with np.errstate(divide="ignore"):
        r_inv = np.power(rowsum, -1).flatten()
    r_inv[np.isinf(r_inv)] = 0.0
    return sp.diags(r_inv).dot(mx).tocsr()


def lap_matrix(A: sp.spmatrix, model: str) -> sp.csr_matrix:
    """main.py:267-270: row_normalize(A) for GraphSAGE, row_normalize(A + I) for GCN
    (canonical CSR: duplicates summed, indices sorted)."""
    if model == "gcn":
        A = A + sp.eye(A.shape[0], dtype=A.dtype, format="csr")
    lap = row_normalize(A)
    lap.sum_duplicates()
    return lap
