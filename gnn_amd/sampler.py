"""LADIES layer-wise importance sampler and the batch scheduler (host side).

Restates sampler.py:90-160 (``ladies_sampler``) and sampler.py:164-193 (``prepare_data``)
of the reference with the same numpy call sequence, so a given seed yields the same
sampled nodes, sub-graph CSR and masks (pinned by tests/golden). The split is:

  * ``ladies_sample_host`` — pure numpy/scipy; returns a ``HostBatch`` (CSR pieces per
    layer, feature-placement indices, labels). Runs in sampler worker processes: no GPU.
  * ``HostBatch.to_device`` — H2D of the index arrays and the GPU operand build
    (``custom_sparse_ops.build_operand``, the create_coo_tensor kernel).
  * ``ladies_sampler`` — the reference's signature and return tuple, both steps in one.

Deviation (documented, values unchanged): column ids travel as int32 instead of int16
(sampler.py:136), lifting the 32,767-column cap; the values are identical whenever the
reference's int16 would not have overflowed.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import scipy.sparse as sp
import torch


@dataclass
class HostLayer:
    fullrowptr: np.ndarray  # int32 [M+1]: indptr of U = lap[previous, :]
    rowptr: np.ndarray      # int32 [M+1]: indptr of U[:, after]
    colidx: np.ndarray      # int32 [nnz]
    normfact: np.ndarray    # float32 [K]: 1 / float32(clip(s_num * p[after], 1e-10, 1))
    shape: tuple            # (M, K)


@dataclass
class HostBatch:
    layers: List[Optional[HostLayer]]          # bottom-up (layer 0 first), as adjs
    sampled_nodes: List[np.ndarray]            # bottom-up
    input_nodes: np.ndarray                    # ids of the layer-0 input rows (sorted)
    input_nodes_mask_on_devices: List[np.ndarray]
    input_nodes_mask_on_cpu: np.ndarray
    nodes_idx_on_devices: List[np.ndarray]
    nodes_idx_on_cpu: np.ndarray
    batch_nodes: np.ndarray
    labels: np.ndarray                         # dense float32 [batch, classes]
    seed: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def num_input_nodes(self) -> int:
        return int(len(self.input_nodes))

    def nnz(self) -> int:
        return int(sum(l.colidx.size for l in self.layers if l is not None))

    def to_device(self, device, with_coo: bool = True, build: bool = True):
        """Materialise on the GPU (H2D of the CSR pieces, labels, sampled_nodes) and, unless
        build=False, run the operand builder. Returns a DeviceBatch."""
        dev = torch.device(device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(dev, non_blocking=True)
        raw = [None if L is None else (t(L.fullrowptr), t(L.rowptr), t(L.colidx), t(L.normfact), L.shape)
               for L in self.layers]
        sampled = [torch.from_numpy(np.asarray(s, dtype=np.int64)).to(dev, non_blocking=True) for s in self.sampled_nodes]
        labels = torch.from_numpy(self.labels).to(dev, non_blocking=True)
        db = DeviceBatch(self, raw, None, sampled, labels)
        if build:
            db.build_operands(with_coo=with_coo)
        return db


@dataclass
class DeviceBatch:
    host: HostBatch
    raw: list            # per layer: device (fullrowptr, rowptr, colidx, normfact, shape) or None
    adjs: Optional[list]
    sampled_nodes: list
    labels: torch.Tensor

    def build_operands(self, with_coo: bool = False) -> list:
        """create_coo_tensor for every layer (stream-ordered on the current stream)."""
        from . import custom_sparse_ops as cso

        adjs = []
        for r in self.raw:
            if r is None:
                adjs.append(None)
                continue
            fr, rp, ci, nf, shape = r
            op, coo = cso.build_operand(fr, rp, ci, nf, shape[0], shape[1], with_coo=with_coo)
            if with_coo:
                a = torch.sparse_coo_tensor(coo, op.val, shape, is_coalesced=True)
                a._gnn_csr = op
                adjs.append(a)
            else:
                adjs.append(op)
        self.adjs = adjs
        return adjs


def column_nnz_counts(U: sp.csr_matrix, num_nodes: int) -> np.ndarray:
    """sp.linalg.norm(U, ord=0, axis=0) (sampler.py:117): nonzeros per column, int64."""
    idx = U.indices if U.data.size == 0 or np.all(U.data != 0) else U.indices[U.data != 0]
    return np.bincount(idx, minlength=num_nodes).astype(np.int64)


def ladies_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix: sp.csr_matrix, labels_full,
                       orders: Sequence[int], device_id_of_nodes, idx_of_nodes_on_device,
                       skewed_sampling_nodes=None, scale_factor: float = 1.0, devices=(0,)) -> HostBatch:
    """sampler.py:90-160 without the device work."""
    np.random.seed(seed)
    batch_nodes = np.asarray(batch_nodes)
    previous_nodes = batch_nodes
    layers: List[Optional[HostLayer]] = []
    sampled_nodes: List[np.ndarray] = []
    orders1 = list(orders)[::-1]
    for d in range(len(orders1)):
        if orders1[d] == 0:
            layers.append(None)
            sampled_nodes.append(np.zeros(0, dtype=np.int64))
            continue
        U = lap_matrix[previous_nodes, :]
        # The reference's sp.linalg.norm(U, ord=0) canonicalises U in place (sorted,
        # duplicate-free indices) before U[:, after] is taken, so its sub-graph columns
        # come out ascending even when lap_matrix is unsorted (row_normalize's product).
        U.sum_duplicates()
        pi = column_nnz_counts(U, num_nodes)
        if scale_factor > 1:
            # int64 counts scaled in place: the product is truncated on assignment, as in
            # the reference (sampler.py:119-121; never reached there since scale_factor=1).
            nodes_on_this_gpu = skewed_sampling_nodes[len(orders1) - d - 1]
            pi[nodes_on_this_gpu] = pi[nodes_on_this_gpu] * scale_factor
        p = pi / np.sum(pi)
        samp_num_d = samp_num_list[d]
        s_num = np.min([np.sum(p > 0), samp_num_d])
        after_nodes = np.random.choice(num_nodes, s_num, p=p, replace=False)
        after_nodes = np.unique(np.concatenate((after_nodes, previous_nodes)))
        adj = U[:, after_nodes]
        layers.append(HostLayer(
            fullrowptr=U.indptr.astype(np.int32),
            rowptr=adj.indptr.astype(np.int32),
            colidx=adj.indices.astype(np.int32),
            # sampler.py:137 casts the clipped value to float32 BEFORE the reciprocal, so the
            # division is a float32 one: keep that precedence.
            normfact=1 / np.clip(s_num * p[after_nodes], 1e-10, 1).astype(np.float32),
            shape=(int(adj.shape[0]), int(adj.shape[1])),
        ))
        sampled_nodes.append(np.where(np.isin(after_nodes, previous_nodes))[0])
        previous_nodes = after_nodes
    layers.reverse()
    sampled_nodes.reverse()

    input_nodes_devices = device_id_of_nodes[previous_nodes]
    input_nodes_mask_on_cpu = input_nodes_devices == -1
    nodes_idx_on_cpu = previous_nodes[input_nodes_mask_on_cpu]
    masks, idxs = [], []
    for dv in devices:
        m = input_nodes_devices == dv
        masks.append(m)
        idxs.append(idx_of_nodes_on_device[previous_nodes[m]].copy())
    labels = np.asarray(labels_full[batch_nodes].todense(), dtype=np.float32)
    return HostBatch(layers=layers, sampled_nodes=sampled_nodes, input_nodes=previous_nodes,
                     input_nodes_mask_on_devices=masks, input_nodes_mask_on_cpu=input_nodes_mask_on_cpu,
                     nodes_idx_on_devices=idxs, nodes_idx_on_cpu=nodes_idx_on_cpu, batch_nodes=batch_nodes,
                     labels=labels, seed=int(seed))


def ladies_sampler(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                   device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, rank, devices):
    """Reference signature and return tuple (sampler.py:90, :160)."""
    hb = ladies_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                            device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, devices)
    dev = devices[rank]
    db = hb.to_device(torch.device("cuda", dev) if isinstance(dev, int) else dev)
    return (db.adjs, hb.input_nodes_mask_on_devices, hb.input_nodes_mask_on_cpu, hb.nodes_idx_on_devices,
            hb.nodes_idx_on_cpu, hb.num_input_nodes, db.labels, hb.sampled_nodes)


def rank_batches(target_nodes, batch_size: int, rank: int, world_size: int, iter_num: int,
                 local_shuffle: bool = False):
    """Batch node lists of one epoch for one rank (sampler.py:168-189): a torch.manual_seed
    permutation, a contiguous per-rank chunk of ceil(n/world) positions, batch_size slices."""
    n = len(target_nodes)
    chunk_size = n // world_size + (1 if n % world_size else 0)
    chunk_start = rank * chunk_size
    chunk_end = min((rank + 1) * chunk_size, n)
    num_batches = (chunk_end - chunk_start) // batch_size
    if (chunk_end - chunk_start) % batch_size:
        num_batches += 1
    if not local_shuffle:
        g = torch.Generator().manual_seed(iter_num)
        idxs = torch.randperm(n, generator=g).numpy()
    else:
        g = torch.Generator().manual_seed(iter_num)
        idxs = np.empty(n, dtype=np.int64)
        idxs[chunk_start:chunk_end] = torch.randperm(chunk_end - chunk_start, generator=g).numpy() + chunk_start
    out = []
    for j in range(num_batches):
        sl = idxs[chunk_start + j * batch_size: min(chunk_start + (j + 1) * batch_size, chunk_end)]
        out.append(np.asarray(target_nodes)[sl])
    return out
