"""Feature-cache placement across GPUs ("ours", the reference's default).

Restates create_buffer's default branch (preprocess.py:311-407, branch :343-347,:354-386):

  1. sample_prob = 1ᵀ · L[train, :] · L^(layers-1) — expected touches of every node.
  2. buffered = argsort(-sample_prob)[: k·ndev] (the hottest k·ndev nodes).
  3. Every GPU starts with the same hottest k; then, walking the next candidates in order,
     (ndev-1) GPUs per round (ordered by least accumulated probability) replace their tail
     slots with the candidate, while the GPU with the most accumulated probability keeps the
     replaced node. Result per rank: device_id_of_nodes (N, -1 = host), the shared
     idx_of_nodes_on_device (N) and the per-GPU buffer node lists.

Also get_skewed_sampled_nodes (preprocess.py:414-423) for --locality_sampling, which the
reference computes but whose effect is disabled (scale_factor fixed at 1.0, main.py:256).
The on-disk pickle cache of the reference (preprocess.py:317,386-395) is replaced by an
optional .npz cache written by this process (no unpickling).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import scipy.sparse as sp


@dataclass
class Placement:
    device_id_of_nodes_group: List[np.ndarray]   # per rank: (N,) device id or -1
    idx_of_nodes_on_device_group: List[np.ndarray]  # per rank view of one shared (N,) array
    gpu_buffer_group: List[np.ndarray]           # per rank: node ids held, in slot order
    change_num: int
    p_accum: np.ndarray


def sample_probability(lap_matrix: sp.csr_matrix, train_nodes, num_conv_layers: int) -> np.ndarray:
    sample_prob = np.ones(len(train_nodes)) * lap_matrix[train_nodes, :]
    for _ in range(num_conv_layers - 1):
        sample_prob *= lap_matrix
    return np.asarray(sample_prob).ravel()


def create_buffer_ours(lap_matrix: sp.csr_matrix, train_nodes, num_nodes_per_dev: int, devices: Sequence[int],
                       num_conv_layers: int, alpha: float = 1.0) -> Placement:
    num_devs = len(devices)
    N = lap_matrix.shape[1]
    sample_prob = sample_probability(lap_matrix, train_nodes, num_conv_layers)
    buffer_size = num_nodes_per_dev * num_devs
    buffered_nodes = np.argsort(-1 * sample_prob)[:buffer_size]

    gpu_buffer_group: List[np.ndarray] = []
    device_id_of_nodes_group: List[np.ndarray] = []
    idx_of_nodes_on_device = np.arange(N)
    for i in range(num_devs):
        device_id_of_nodes = np.array([-1] * N)
        gpu_buffer_group.append(buffered_nodes[:num_nodes_per_dev].copy())
        on_dev = buffered_nodes[:num_nodes_per_dev]
        device_id_of_nodes[on_dev] = devices[i]
        device_id_of_nodes_group.append(device_id_of_nodes.copy())
        idx_of_nodes_on_device[on_dev] = np.arange(len(on_dev))
    idx_of_nodes_on_device_group = [idx_of_nodes_on_device] * num_devs

    p_accum = np.array([0.0] * num_devs)
    change_num = num_devs - 1  # the reference reads the leftover loop variable when no swap runs
    device_order = None
    for i in range(len(buffered_nodes) - num_nodes_per_dev):
        if i % (num_devs - 1) == 0:
            device_order = np.argsort(p_accum)
        candidate_node = buffered_nodes[num_nodes_per_dev + i]
        new_node_idx = num_nodes_per_dev - 1 - i // (num_devs - 1)
        node_to_be_replaced = buffered_nodes[new_node_idx]
        if sample_prob[candidate_node] >= alpha * sample_prob[node_to_be_replaced]:
            current_dev = device_order[i % (num_devs - 1)]
            p_accum[current_dev] += sample_prob[candidate_node]
            for j in range(num_devs):
                device_id_of_nodes_group[j][candidate_node] = devices[current_dev]
                idx_of_nodes_on_device_group[j][candidate_node] = new_node_idx
            device_id_of_nodes_group[current_dev][node_to_be_replaced] = devices[device_order[-1]]
            gpu_buffer_group[current_dev][new_node_idx] = candidate_node
        else:
            change_num = i
            break
        change_num = i
    return Placement(device_id_of_nodes_group, idx_of_nodes_on_device_group, gpu_buffer_group, change_num, p_accum)


def create_buffer(lap_matrix, train_nodes, num_nodes_per_dev: int, devices: Sequence[int], num_conv_layers: int,
                  alpha: float = 1.0, cache_path: Optional[str] = None) -> Placement:
    """create_buffer (default branch) with an optional .npz cache keyed by the caller."""
    if cache_path and os.path.exists(cache_path):
        z = np.load(cache_path, allow_pickle=False)
        nd = len(devices)
        idx = z["idx"]
        return Placement([z[f"dev{i}"] for i in range(nd)], [idx] * nd, [z[f"buf{i}"] for i in range(nd)],
                         int(z["change_num"]), z["p_accum"])
    pl = create_buffer_ours(lap_matrix, train_nodes, num_nodes_per_dev, devices, num_conv_layers, alpha)
    if cache_path:
        arrs = {f"dev{i}": a for i, a in enumerate(pl.device_id_of_nodes_group)}
        arrs.update({f"buf{i}": a for i, a in enumerate(pl.gpu_buffer_group)})
        np.savez(cache_path, idx=pl.idx_of_nodes_on_device_group[0], change_num=pl.change_num,
                 p_accum=pl.p_accum, **arrs)
    return pl


def get_skewed_sampled_nodes(adj_matrix: sp.spmatrix, gpu_buffers_group, orders: Sequence[int]):
    """preprocess.py:414-423: per-layer top-8192 nodes by propagated buffer indicator."""
    neighboring_nodes = [np.unique(np.concatenate(gpu_buffers_group))]
    v = np.array([0] * adj_matrix.shape[1])
    v[neighboring_nodes[0]] = 1
    for _ in range(1, len(orders)):
        v = v * adj_matrix
        neighboring_nodes.append(np.argsort(-1 * v)[:8192])
    return neighboring_nodes
