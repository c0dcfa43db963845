"""CPU: the threaded batch producer returns, in order, exactly the batches a sequential
sampler produces from the same seeds; prepare_data keeps the reference's batching."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import scipy.sparse as sp
import torch

from gnn_amd import loader, placement, sampler, staging
from gnn_amd.graphs import chung_lu, row_normalize


def _setup(N=5000, avg=16, seed=3):
    A = chung_lu(N, N * avg // 2, 1.3, np.random.default_rng(seed))
    lap = row_normalize(A)
    lap.sum_duplicates()
    labels = sp.csr_matrix((np.ones(N, np.float32), (np.arange(N), np.arange(N) % 5)), shape=(N, 5))
    train = np.arange(0, N, 2)
    return lap, labels, train


def test_batch_loader_matches_sequential():
    lap, labels, train = _setup()
    N = lap.shape[0]
    pl = placement.create_buffer_ours(lap, train, 300, [0, 1], 3, alpha=0)
    feats = torch.randn(N, 10)
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], "cpu", 0)
    ld = loader.BatchLoader(lap, labels, train, 400, 64, [1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], rank=0, world_size=2, store=store, workers=4,
                            seed=11)
    got = list(ld.epoch(1))
    ld.close()
    chunks = sampler.rank_batches(train, 64, 0, 2, 1)
    assert len(got) == len(chunks)
    rs = np.random.RandomState(11)
    for lb, nodes in zip(got, chunks):
        seed = int(rs.randint(2**32 - 1))
        ref = sampler.ladies_sample_host(seed, nodes, np.array([400] * 5), N, lap, labels, [1, 1],
                                         pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0], None,
                                         1.0, [0, 1], native=False)
        assert np.array_equal(lb.host.batch_nodes, nodes)
        for a, b in zip(lb.host.layers, ref.layers):
            assert np.array_equal(a.colidx, b.colidx) and np.array_equal(a.normfact, b.normfact)
        assert np.array_equal(lb.host.input_nodes, ref.input_nodes)
        # host rows staged for X0: exactly the non-buffered input nodes' features, zero padded
        rows = lb.plan.host_rows.numpy()
        assert np.array_equal(rows[:, :10], feats.numpy()[ref.nodes_idx_on_cpu])
        assert np.all(rows[:, 10:] == 0)


def test_prepare_data_reference_batching():
    lap, labels, train = _setup(N=3000)
    N = lap.shape[0]
    calls = []

    def fake_sampler(seed, nodes, *rest):
        calls.append((seed, np.asarray(nodes)))
        return len(nodes)

    with ThreadPoolExecutor(2) as pool:
        sizes = [f.result() for f in loader.prepare_data(pool, fake_sampler, train, [10] * 3, N, lap, labels,
                                                          [1, 1, 1], 100, 1, 3, None, None, None, "cpu", [0],
                                                          iter_num=4, rng=np.random.RandomState(0))]
    # rank 1 of 3 over 1500 train nodes: chunk 500 -> 5 batches of 100
    assert sizes == [100] * 5
    perm = torch.randperm(len(train), generator=torch.Generator().manual_seed(4)).numpy()
    got = np.sort(np.concatenate([c[1] for c in calls]))
    assert np.array_equal(got, np.sort(train[perm[500:1000]]))


def test_wait_event_polls_until_complete(monkeypatch):
    """staging.wait_event: with a sleep interval it polls the event (never HIP's spinning wait)
    until it completes; with 0 it calls synchronize()."""

    class Ev:
        def __init__(self, ready_after):
            self.n, self.ready_after, self.synced = 0, ready_after, False

        def query(self):
            self.n += 1
            return self.n > self.ready_after

        def synchronize(self):
            self.synced = True

    monkeypatch.setattr(staging, "_WAIT_SLEEP_S", 1e-6)
    ev = Ev(5)
    staging.wait_event(ev)
    assert ev.n == 6 and not ev.synced
    monkeypatch.setattr(staging, "_WAIT_SLEEP_S", 0.0)
    ev = Ev(5)
    staging.wait_event(ev)
    assert ev.synced and ev.n == 0
