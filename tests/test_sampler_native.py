"""CPU: the native LADIES sampler (libgnn_sampler.so) against the numpy restatement and
numpy's own RNG stream, bit for bit (the reference goldens are in test_sampler_placement)."""
from concurrent.futures import ThreadPoolExecutor

import ctypes

import numpy as np
import pytest
import scipy.sparse as sp

from gnn_amd import _lib, sampler
from gnn_amd.graphs import chung_lu, row_normalize


@pytest.mark.parametrize("seed", [0, 1, 12345, 2**31 - 2, 2**32 - 1])
def test_mt19937_stream_matches_numpy(seed):
    out = np.empty(5000, np.float64)
    _lib.check_sampler(_lib.sampler_lib().gnn_mt19937_random_sample(seed, out.size, out.ctypes.data), "rng")
    assert np.array_equal(out, np.random.RandomState(seed).random_sample(out.size))


def _lap(N, avg, seed, sigma=1.3):
    A = chung_lu(N, N * avg // 2, sigma, np.random.default_rng(seed))
    lap = row_normalize(A)
    lap.sum_duplicates()
    return lap


def _labels(N, C=7):
    return sp.csr_matrix((np.ones(N, np.float32), (np.arange(N), np.arange(N) % C)), shape=(N, C))


def _same(a, b):
    assert len(a.layers) == len(b.layers)
    for La, Lb in zip(a.layers, b.layers):
        if La is None or Lb is None:
            assert La is None and Lb is None
            continue
        assert La.shape == Lb.shape
        assert np.array_equal(La.fullrowptr, Lb.fullrowptr)
        assert np.array_equal(La.rowptr, Lb.rowptr)
        assert np.array_equal(La.colidx, Lb.colidx)
        assert np.array_equal(La.normfact.view(np.uint32), Lb.normfact.view(np.uint32))
    for x, y in zip(a.sampled_nodes, b.sampled_nodes):
        assert np.array_equal(np.asarray(x, np.int64), np.asarray(y, np.int64))
    assert np.array_equal(a.input_nodes, b.input_nodes)
    assert np.array_equal(a.input_nodes_mask_on_cpu, b.input_nodes_mask_on_cpu)
    for x, y in zip(a.nodes_idx_on_devices, b.nodes_idx_on_devices):
        assert np.array_equal(x, y)
    assert np.array_equal(a.labels, b.labels)


def _both(lap, N, batch, samp, orders, seed, ndev=2, kind="ladies"):
    dev_of = np.where(np.arange(N) % 3 == 0, -1, np.arange(N) % ndev)
    idx_on = np.arange(N) // 3
    args = (seed, batch, np.array(samp), N, lap, _labels(N), orders, dev_of, idx_on, None, 1.0, list(range(ndev)))
    fn = {"ladies": sampler.ladies_sample_host, "subgraph": sampler.subgraph_sample_host,
          "fastgcn": sampler.fastgcn_sample_host}[kind]
    return fn(*args, native=True), fn(*args, native=False)


@pytest.mark.parametrize("kind", ["ladies", "subgraph", "fastgcn"])
@pytest.mark.parametrize("samp,bs,seed", [(64, 16, 3), (512, 128, 11), (2048, 256, 99), (5000, 300, 7)])
def test_native_matches_numpy(samp, bs, seed, kind):
    N = 6000
    lap = _lap(N, 20, seed)
    batch = np.random.default_rng(seed).permutation(N)[:bs]
    a, b = _both(lap, N, batch, [samp] * 3, [1, 1, 1], seed, kind=kind)
    _same(a, b)


@pytest.mark.parametrize("orders", [[0, 1, 1], [1, 0, 1], [0, 0, 1], [0, 0, 0]])
def test_subgraph_orders(orders):
    N = 2000
    lap = _lap(N, 10, 8)
    a, b = _both(lap, N, np.arange(100, 164), [300] * 3, orders, 21, kind="subgraph")
    _same(a, b)


def test_native_csc_matches_scipy():
    """Layers >= 1 carry their CSC (the backward operand's structure): scipy's tocsc of the
    layer, exactly; layer 0 (input = features, no gradient) carries none."""
    N = 5000
    lap = _lap(N, 18, 6)
    batch = np.random.default_rng(1).permutation(N)[:128]
    a, _ = _both(lap, N, batch, [700] * 3, [1, 1, 1], 9)
    assert a.layers[0].csc_colptr is None
    for L in a.layers[1:]:
        M, K = L.shape
        csc = sp.csr_matrix((np.ones(L.colidx.size), L.colidx, L.rowptr), shape=(M, K)).tocsc()
        assert np.array_equal(L.csc_colptr, csc.indptr)
        assert np.array_equal(L.csc_rows, csc.indices)


def test_native_exhausts_support():
    """samp_num above the number of reachable columns: s_num = #(p > 0), every one taken."""
    N = 3000
    lap = _lap(N, 3, 5, sigma=0.5)
    batch = np.arange(0, 40)
    a, b = _both(lap, N, batch, [100000] * 3, [1, 1, 1], 5)
    _same(a, b)


@pytest.mark.parametrize("orders", [[1, 1, 1], [1, 1, 0], [1, 0, 1]])
def test_native_repeated_batch_nodes(orders):
    """A batch with repeated nodes repeats rows of U (their columns counted twice), so the
    column counts cannot carry over into the next layer there; later layers' rows are unique."""
    N = 4000
    lap = _lap(N, 12, 4)
    batch = np.concatenate([np.arange(200, 260), np.arange(230, 250), [777, 777]])
    a, b = _both(lap, N, batch, [600, 400, 300], orders, 13)
    _same(a, b)


def test_native_orders_with_zero_layers():
    N = 2000
    lap = _lap(N, 10, 8)
    batch = np.arange(100, 164)
    a, b = _both(lap, N, batch, [300, 200, 100], [1, 0, 1], 21)
    _same(a, b)
    assert a.layers[1] is None


def test_native_explicit_zeros_and_unsorted_rows():
    """Explicit zeros stay in the structure but are not counted (ord-0 norm); a lap with
    unsorted rows is canonicalised first, as sp.linalg.norm does to U."""
    N = 1500
    lap = _lap(N, 12, 4)
    rng = np.random.default_rng(0)
    lap.data[rng.random(lap.data.size) < 0.1] = 0.0
    perm_rows = []
    for r in range(N):  # shuffle each row's entries
        b, e = lap.indptr[r], lap.indptr[r + 1]
        perm_rows.append(b + rng.permutation(e - b))
    order = np.concatenate(perm_rows)
    shuffled = sp.csr_matrix((lap.data[order], lap.indices[order], lap.indptr.copy()), shape=lap.shape)
    assert not shuffled.has_sorted_indices
    batch = np.arange(0, 50)
    a, b = _both(shuffled, N, batch, [400] * 3, [1, 1, 1], 77)
    _same(a, b)


def test_native_threads_match_sequential():
    N = 8000
    lap = _lap(N, 25, 2)
    batches = [np.random.default_rng(i).permutation(N)[:200] for i in range(8)]
    dev_of = np.full(N, -1)
    idx_on = np.zeros(N, np.int64)

    def one(i):
        return sampler.ladies_sample_host(1000 + i, batches[i], np.array([1000] * 3), N, lap, _labels(N), [1, 1, 1],
                                          dev_of, idx_on, None, 1.0, [0])

    seq = [one(i) for i in range(8)]
    with ThreadPoolExecutor(4) as ex:
        par = list(ex.map(one, range(8)))
    for a, b in zip(seq, par):
        _same(a, b)


def test_native_scratch_reuse_across_graphs_and_kinds():
    """The per-thread scratch is reset from what the previous call touched (not refilled), and
    FastGCN's candidate list / base cdf is cached per p array: alternating two graphs of the
    same size and all three samplers on one thread must still match numpy call for call."""
    N = 4000
    laps = [_lap(N, 15, 31), _lap(N, 9, 32, sigma=0.5)]
    for it in range(3):
        for gi, lap in enumerate(laps):
            for kind in ("ladies", "fastgcn", "subgraph"):
                batch = np.random.default_rng(10 * it + gi).permutation(N)[:150]
                a, b = _both(lap, N, batch, [900] * 3, [1, 1, 1], 100 * it + gi, kind=kind)
                _same(a, b)


def test_native_isolated_batch_raises_like_numpy():
    """A layer whose rows have no entries: p = 0/0 and numpy's choice raises; so does native."""
    N = 50
    lap = sp.csr_matrix((N, N), dtype=np.float32)
    for native in (True, False):
        with pytest.raises((ValueError, RuntimeError), match="NaN"):
            sampler.ladies_sample_host(0, np.arange(4), np.array([8] * 3), N, lap, _labels(N), [1, 1, 1],
                                       np.full(N, -1), np.zeros(N, np.int64), None, 1.0, [0], native=native)


def test_fastgcn_sampling_law():
    """FastGCN (parity unpinned: not in the reference): drawn nodes follow the global
    importance p ∝ column sums of lap∘lap — chi-square-style check of inclusion frequencies
    on the top-probability nodes, and the operand convention (normfact from p)."""
    N = 3000
    lap = _lap(N, 12, 13)
    p = sampler.fastgcn_probability(lap)
    assert abs(p.sum() - 1) < 1e-12
    dense = lap.toarray().astype(np.float64)
    np.testing.assert_allclose(p, (dense ** 2).sum(0) / (dense ** 2).sum(), rtol=1e-12)
    s = 40
    hits = np.zeros(N)
    trials = 400
    dev_of = np.full(N, -1)
    for t in range(trials):
        hb = sampler.fastgcn_sample_host(t, np.arange(10), np.array([s] * 3), N, lap, _labels(N), [1],
                                         dev_of, np.zeros(N, np.int64), None, 1.0, [0])
        hits[hb.input_nodes] += 1
        L = hb.layers[0]
        q = np.clip(s * p[hb.input_nodes], 1e-10, 1).astype(np.float32)
        assert np.array_equal(L.normfact, 1 / q)
    # without replacement, inclusion prob ~ s*p for small p: compare on the mid-probability nodes
    mid = np.argsort(p)[-200:-20]
    expect = trials * s * p[mid]
    assert abs(hits[mid].sum() / expect.sum() - 1) < 0.1


def test_fastgcn_cache_invalidated_by_p_changed():
    """The native FastGCN draw caches the candidate list of the p array it last saw per thread;
    an in-place rewrite of p announced through gnn_fastgcn_p_changed() must not reuse it: the
    next draw equals the numpy restatement on the rewritten p."""
    N = 2000
    lap = _lap(N, 10, 21)
    g = sampler.native_graph(lap)
    p = np.array(g.fastgcn_p, copy=True)  # a writable array the test owns
    assert not g.fastgcn_p.flags.writeable
    g._fastgcn_p = p
    args = (5, np.arange(16), np.array([60] * 2), N, lap, _labels(N), [1, 1], np.full(N, -1),
            np.zeros(N, np.int64), None, 1.0, [0])
    with ThreadPoolExecutor(1) as pool:  # one thread: its cache sees both calls
        a = pool.submit(sampler.fastgcn_sample_host, *args).result()
        # rewrite p in place: same address and length, and the 64 values the cache key samples
        # ((k * (N - 1)) // 63) untouched — only the generation tells the change apart
        keyed = np.zeros(N, bool)
        keyed[(np.arange(64) * (N - 1)) // 63] = True
        free = np.flatnonzero(~keyed)
        p[free] = np.roll(p[free], 997)
        _lib.sampler_lib().gnn_fastgcn_p_changed()
        b = pool.submit(sampler.fastgcn_sample_host, *args).result()
    ref = sampler.fastgcn_sample_host(*args, native=False)
    assert np.array_equal(b.input_nodes, ref.input_nodes)
    assert not np.array_equal(a.input_nodes, b.input_nodes)
    for x, y in zip(b.layers, ref.layers):
        assert np.array_equal(x.colidx, y.colidx) and np.array_equal(x.normfact, y.normfact)


def test_native_errors():
    L = _lib.sampler_lib()
    h = ctypes.c_void_p()
    indptr = np.zeros(3, np.int64)
    indices = np.zeros(0, np.int32)
    bad = np.array([5], np.int64)
    sn = np.array([1], np.int64)
    od = np.array([1], np.int32)
    rc = L.gnn_ladies_sample(indptr.ctypes.data, indices.ctypes.data, None, 2, bad.ctypes.data, 1, sn.ctypes.data,
                             od.ctypes.data, 1, 0, ctypes.byref(h))
    assert rc != 0 and b"out of range" in L.gnn_sampler_last_error()
