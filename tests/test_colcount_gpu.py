"""U's column counts for the LADIES draw on the GPU (gnn_colcount_*, include/gnn_extract.h;
gnn_ladies_sample_cc / gnn_loader_set_colcount, include/gnn_sampler.h).

The device counts replace only the host's column counting (reference sampler.py:116-122,
pi = norm(U, ord=0, axis=0)); the draw stays on the host. So the checks are exact: the raw API
returns numpy's column counts of lap[rows, :] (bitmap of the non-zero columns + their counts in
ascending column order, repeats counted again, counts carried over between calls until reset),
and a sampler using it yields batches identical to the host-counting sampler — itself pinned to
the reference's ladies_sampler by tests/golden — on symmetric and directed graphs, with repeated
batch nodes (the non-nested first layer), with and without the GPU layer extraction, and through
the C++ batch producer.
"""
import ctypes

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from gnn_amd import _lib, graphs, loader, placement, sampler, staging

pytestmark = pytest.mark.gpu

_G = {}


def _graph(name):
    if not _G:
        rng = np.random.default_rng(7)
        A = graphs.chung_lu(20_000, 150_000, 1.3, rng)
        _G["symmetric"] = graphs.lap_matrix(A, "graphsage")
        n = 12_000
        u = rng.integers(0, n, 90_000)
        v = (u + rng.integers(1, 300, u.size)) % n
        D = sp.csr_matrix((np.ones(u.size, np.float32), (u, v)), shape=(n, n))
        D.data[:] = 1
        D.sort_indices()
        _G["directed"] = graphs.lap_matrix(D, "gcn")
        _G["wide"] = graphs.lap_matrix(graphs.chung_lu(150_003, 600_000, 1.3, rng), "graphsage")  # 19 buckets
    return _G[name]


def _labels(N):
    return sp.csr_matrix((np.ones(N, np.int32), (np.arange(N), np.zeros(N, np.int64))), shape=(N, 1))


def _add(cc, rows, N):
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    nlive = ctypes.c_int64()
    bits, counts = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(_lib.lib().gnn_colcount_add(cc.ctx, rows.ctypes.data, rows.size, ctypes.byref(nlive),
                                           ctypes.byref(bits), ctypes.byref(counts)), "gnn_colcount_add")
    W = (N + 63) // 64
    b = np.ctypeslib.as_array(ctypes.cast(bits, ctypes.POINTER(ctypes.c_uint64)), shape=(W,)).copy()
    c = (np.ctypeslib.as_array(ctypes.cast(counts, ctypes.POINTER(ctypes.c_int32)), shape=(nlive.value,)).copy()
         if nlive.value else np.zeros(0, np.int32))
    live = np.nonzero(np.unpackbits(b.view(np.uint8), bitorder="little")[:N])[0]
    return live, c


# the histogram's forms (colcount.hip): partitioned (default), one atomic per entry, and the
# partitioned form whose offsets buffer is too small for the first calls (the atomic kernel runs,
# then the buffer grows)
_FORMS = {"part": {}, "atomic": {"GNN_CC_HIST": "atomic"}, "part-grow": {"GNN_CC_KEYS": "100"}}


@pytest.mark.parametrize("form", list(_FORMS))
@pytest.mark.parametrize("gname", ["symmetric", "directed", "wide"])
def test_colcount_api_matches_numpy(dev, gname, form, monkeypatch):
    for k, v in _FORMS[form].items():
        monkeypatch.setenv(k, v)
    lap = _graph(gname)
    N = lap.shape[0]
    cc = sampler.ColumnCounter(lap, dev)
    try:
        rng = np.random.default_rng(1)
        acc = np.zeros(N, np.int64)
        for step in range(4):  # counts carry over between calls
            rows = rng.integers(0, N, 500 * (step + 1))  # repeats count again
            acc += np.bincount(lap[rows].indices, minlength=N)
            live, counts = _add(cc, rows, N)
            assert np.array_equal(live, np.nonzero(acc)[0])
            assert np.array_equal(counts, acc[live])
        _lib.check(_lib.lib().gnn_colcount_reset(cc.ctx), "gnn_colcount_reset")
        live, counts = _add(cc, np.zeros(0, np.int64), N)
        assert live.size == 0 and counts.size == 0
        rows = np.array([3, 3, 17])
        live, counts = _add(cc, rows, N)
        ref = np.bincount(lap[rows].indices, minlength=N)
        assert np.array_equal(live, np.nonzero(ref)[0]) and np.array_equal(counts, ref[live])
    finally:
        cc.close()


def _same(a, b):
    assert np.array_equal(a.input_nodes, b.input_nodes)
    for x, y in zip(a.sampled_nodes, b.sampled_nodes):
        assert np.array_equal(np.asarray(x, np.int64), np.asarray(y, np.int64))
    for La, Lb in zip(a.layers, b.layers):
        assert (La is None) == (Lb is None)
        if La is None:
            continue
        assert La.shape == Lb.shape and La.on_device == Lb.on_device and La.nnz == Lb.nnz
        for k in ("fullrowptr", "rowptr", "colidx", "normfact", "csc_colptr", "csc_rows", "rows", "cols", "colseg"):
            va, vb = getattr(La, k, None), getattr(Lb, k, None)
            assert (va is None) == (vb is None), k
            if va is not None:
                assert np.array_equal(np.asarray(va).view(np.uint8), np.asarray(vb).view(np.uint8)), k


@pytest.mark.parametrize("gname,orders,samp,bs,dx,dup", [
    ("symmetric", [1, 1, 1], 2000, 256, True, False), ("symmetric", [1, 1, 1], 300, 64, False, False),
    ("symmetric", [1, 0, 1], 800, 128, True, True), ("directed", [1, 1, 1], 600, 128, True, False),
    ("directed", [1, 1], 3000, 400, False, True)])
def test_sampler_with_device_counts_equals_host(dev, gname, orders, samp, bs, dx, dup):
    lap = _graph(gname)
    N = lap.shape[0]
    cc = sampler.ColumnCounter(lap, dev)
    try:
        for seed in range(3):
            batch = np.random.default_rng(seed).choice(N, bs, replace=False)
            if dup:  # repeated batch nodes: U repeats rows, the first layer's counts do not carry over
                batch = np.concatenate([batch, batch[: bs // 4]])
            args = (seed + 5, batch, np.array([samp] * 5), N, lap, _labels(N), orders, np.full(N, -1),
                    np.zeros(N, np.int64), None, 1.0, [0])
            host = sampler.ladies_sample_host(*args, device_extract=dx)
            devc = sampler.ladies_sample_host(*args, device_extract=dx, colcount=cc)
            _same(host, devc)
    finally:
        cc.close()


@pytest.mark.parametrize("cc_workers", [None, 1, 2])
def test_native_loader_with_device_counts(dev, cc_workers):
    """The native producer with U's column counts on the GPU — in every worker, or (cc_workers)
    in the first k of 3 workers with the rest counting on the host, the device contexts on
    CU-masked streams of their own (bench.py's `mixed`) — yields the host-counting batches."""
    lap = _graph("symmetric")
    N = lap.shape[0]
    rng = np.random.default_rng(3)
    cls = rng.integers(0, 5, N)
    labels = sp.csr_matrix((np.ones(N, np.int32), (np.arange(N), cls)), shape=(N, 5))
    train = np.arange(0, 9000)
    pl = placement.create_buffer(lap, train, 2000, [0], 2, alpha=0)
    dev_of, idx_on = pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0]
    feats = torch.randn(N, 24, generator=torch.Generator().manual_seed(0))
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], "cpu", 0)
    kw = dict(store=store, workers=3, seed=4, device_extract=True)
    a = loader.NativeLoader(lap, labels, train, 1500, 128, [1, 1, 1], dev_of, idx_on, **kw)
    b = loader.NativeLoader(lap, labels, train, 1500, 128, [1, 1, 1], dev_of, idx_on, device_count=dev,
                            device_count_workers=cc_workers, **kw)
    assert b.device_count and b.device_count_workers == (cc_workers or 0)
    try:
        for n, (pa, pb) in enumerate(zip(a.epoch(1), b.epoch(1))):
            _same(pa.host, pb.host)
            if n == 12:
                break
    finally:
        a.close()
        b.close()
        _lib.lib().gnn_colcount_set_cus(0)  # process-wide: later tests get plain streams again
