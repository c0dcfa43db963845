"""Mini-batch producer: LADIES sampling + host-side feature staging in worker threads.

Reference: ``prepare_data`` (sampler.py:163-210) submits ``ladies_sampler`` calls to a
ThreadPoolExecutor (main.py:77, ``--pool_num`` 4) in groups of 32 and yields the futures;
each call re-seeds numpy's GLOBAL RNG (sampler.py:96) while the driver draws the next seeds
from that same global RNG, so concurrent threads race on it.

Here the worker threads run the native sampler (libgnn_sampler.so: bit-identical to the
numpy path, its own MT19937 per call, GIL released) and the host half of the X0 staging
(native row gather into a pinned buffer), so sampling scales with threads and the training
thread only issues asynchronous copies. Seeds come from the loader's own RandomState, so a
run is reproducible whatever the thread timing.
"""
from __future__ import annotations

import collections
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, Optional, Sequence

import numpy as np

from . import sampler as smp
from . import staging


def prepare_data(pool, sampler_fn, target_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                 batch_size, rank, world_size, device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes,
                 device, devices, scale_factor=1.0, local_shuffle=False, mode="train", iter_num=1, rng=None):
    """Reference signature (sampler.py:163): yields futures of ``sampler_fn`` calls.

    ``iter_num`` replaces the reference's module-global epoch counter (torch.manual_seed of
    the train permutation); ``rng`` (default: numpy's global RNG, as the reference) supplies
    the per-batch seeds."""
    rng = np.random if rng is None else rng
    target_nodes = np.asarray(target_nodes)

    def submit(nodes):
        return pool.submit(sampler_fn, int(rng.randint(2**32 - 1)), nodes, samp_num_list, num_nodes, lap_matrix,
                           labels_full, orders, device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes,
                           scale_factor, rank, devices)

    if mode == "train":
        for chunk in smp.rank_batches(target_nodes, batch_size, rank, world_size, iter_num, local_shuffle):
            yield submit(chunk)
    elif mode == "val":
        import torch

        idx = torch.randperm(len(target_nodes))[:batch_size].numpy()
        yield submit(target_nodes[idx])
    elif mode == "test":
        # sampler.py:199-201: num_batches = len // bs, +1 when (num_batches % bs) != 0 (sic)
        num_batches = len(target_nodes) // batch_size
        if num_batches % batch_size:
            num_batches += 1
        for j in range(num_batches):
            chunk = target_nodes[batch_size * j: min((j + 1) * batch_size, len(target_nodes))]
            if len(chunk):
                yield submit(chunk)
    else:
        raise ValueError(f"unknown mode {mode!r}")


@dataclass
class LoadedBatch:
    host: smp.HostBatch
    plan: Optional[staging.StagePlan]


class BatchLoader:
    """Ordered, bounded-prefetch stream of sampled + host-staged training batches of one rank.

    ``workers`` threads each run: native LADIES sampling -> pinned copies of the batch's
    index arrays -> (with a FeatureStore) the pinned host-row gather of its X0 plan. The
    iterator hands batches out in submission order, keeping ``prefetch`` in flight."""

    def __init__(self, lap, labels_full, train_nodes, samp_num: int, batch_size: int, orders: Sequence[int],
                 device_id_of_nodes, idx_of_nodes_on_device, rank: int = 0, world_size: int = 1,
                 store: Optional[staging.FeatureStore] = None, workers: int = 8, prefetch: int = 0,
                 seed: int = 0, devices=None, kind: str = "ladies", device_extract: bool = False):
        fns = {"ladies": smp.ladies_sample_host, "subgraph": smp.subgraph_sample_host,
               "fastgcn": smp.fastgcn_sample_host}
        if kind not in fns:
            raise ValueError("sampler configuration is wrong")  # main.py:88
        self.sample_fn = fns[kind]
        # LADIES: leave the layers below the top one to the GPU extraction (to_device), so the
        # worker threads only draw (sampler.ladies_sample_host(device_extract=True))
        self.kw = {"device_extract": True} if device_extract and kind == "ladies" else {}
        self.graph = smp.native_graph(lap)
        self.labels = labels_full
        self.train = np.asarray(train_nodes)
        self.samp = np.array([samp_num] * 5)
        self.batch_size = batch_size
        self.orders = list(orders)
        self.dev_of = device_id_of_nodes
        self.idx_on = idx_of_nodes_on_device
        self.rank = rank
        self.world = world_size
        self.devices = list(range(world_size)) if devices is None else list(devices)
        self.store = store
        self.workers = max(1, int(workers))
        self.prefetch = prefetch if prefetch > 0 else 2 * self.workers
        self.rng = np.random.RandomState(seed + 7919 * rank)
        self.pool = ThreadPoolExecutor(max_workers=self.workers, thread_name_prefix="gnn-sampler")

    def _produce(self, seed: int, nodes: np.ndarray) -> LoadedBatch:
        hb = self.sample_fn(seed, nodes, self.samp, self.graph.num_nodes, self.graph, self.labels, self.orders,
                            self.dev_of, self.idx_on, None, 1.0, self.devices, **self.kw)
        hb.pin()
        plan = staging.make_plan(hb, self.store, self.rank, self.world, self.devices) if self.store else None
        return LoadedBatch(hb, plan)

    def epoch(self, iter_num: int) -> Iterator[LoadedBatch]:
        chunks = smp.rank_batches(self.train, self.batch_size, self.rank, self.world, iter_num)
        return self._stream(chunks)

    def forever(self, first_epoch: int = 1) -> Iterator[LoadedBatch]:
        def chunks():
            e = first_epoch
            while True:
                yield from smp.rank_batches(self.train, self.batch_size, self.rank, self.world, e)
                e += 1
        return self._stream(chunks())

    def _stream(self, chunks) -> Iterator[LoadedBatch]:
        q = collections.deque()
        it = iter(chunks)
        done = False
        while True:
            while not done and len(q) < self.prefetch:
                try:
                    nodes = next(it)
                except StopIteration:
                    done = True
                    break
                q.append(self.pool.submit(self._produce, int(self.rng.randint(2**32 - 1)), nodes))
            if not q:
                return
            yield q.popleft().result()

    def close(self):
        self.pool.shutdown(wait=True, cancel_futures=True)
