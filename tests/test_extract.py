"""LADIES layer extraction on the GPU (gnn_ladies_extract_f32, include/gnn_extract.h).

The host sampler in device-extraction mode (gnn_ladies_sample_dev) keeps the draw and leaves
adj = lap[rows, :][:, after] of every layer below the top one to the GPU. CPU tests: the draw is
bit-identical to the host-extracting sampler (which tests/golden pins to the reference's
ladies_sampler) and the host-side nnz / CSC column pointer it derives from the column counts equal
those of the host-extracted sub-graph. GPU tests: the device-extracted operands and their
transposes are bit-identical to the host-extracted path's (gnn_build_operand_f32 on the host
pieces, gnn_build_operand_t_f32 on the host CSC — both pinned to the C oracle elsewhere), on a
symmetric graph (lapᵀ aliases lap) and on a directed one (lapᵀ stored separately).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from gnn_amd import graphs, sampler


def _graphs():
    rng = np.random.default_rng(5)
    A = graphs.chung_lu(20_000, 150_000, 1.3, rng)
    sym = graphs.lap_matrix(A, "graphsage")
    n = 15_000
    u = rng.integers(0, n, 120_000)
    v = (u + rng.integers(1, 400, u.size)) % n  # directed, no self loops
    D = sp.csr_matrix((np.ones(u.size, np.float32), (u, v)), shape=(n, n))
    D.data[:] = 1
    D.sort_indices()
    directed = graphs.lap_matrix(D, "gcn")  # + I: every row non-empty
    return {"symmetric": sym, "directed": directed}


_G = {}


def _graph(name):
    if not _G:
        _G.update(_graphs())
    return _G[name]


CASES = [("symmetric", [1, 1, 1], 300, 64, 0), ("symmetric", [1, 1, 1], 2000, 256, 1),
         ("symmetric", [1, 0, 1], 300, 64, 2), ("directed", [1, 1, 1], 500, 128, 3),
         ("directed", [1, 1], 4000, 512, 4)]


def _pair(gname, orders, samp, bs, seed):
    lap = _graph(gname)
    N = lap.shape[0]
    dev_of = np.full(N, -1, np.int64)
    idx_on = np.zeros(N, np.int64)
    batch = np.random.default_rng(seed).choice(N, bs, replace=False)
    sn = np.array([samp] * 5)
    args = (seed + 11, batch, sn, N, lap, None, orders, dev_of, idx_on, None, 1.0, [0])
    hb = sampler.ladies_sample_host(*args[:5], _labels(N), *args[6:])
    hd = sampler.ladies_sample_host(*args[:5], _labels(N), *args[6:], device_extract=True)
    return hb, hd


def _labels(N):
    return sp.csr_matrix((np.ones(N, np.int32), (np.arange(N), np.zeros(N, np.int64))), shape=(N, 1))


@pytest.mark.parametrize("case", CASES)
def test_device_draw_equals_host_draw(case):
    hb, hd = _pair(*case)
    assert np.array_equal(hb.input_nodes, hd.input_nodes)
    for a, b in zip(hb.sampled_nodes, hd.sampled_nodes):
        assert np.array_equal(a, b)
    present = [li for li, L in enumerate(hb.layers) if L is not None]
    assert present == [li for li, L in enumerate(hd.layers) if L is not None]
    top = present[-1]
    cols_below = hb.input_nodes
    for li in present:
        L, D = hb.layers[li], hd.layers[li]
        assert L.shape == D.shape and np.array_equal(L.normfact, D.normfact)
        if li == top:  # the batch's layer stays host-extracted
            assert not D.on_device
            for k in ("fullrowptr", "rowptr", "colidx"):
                assert np.array_equal(getattr(L, k), getattr(D, k))
            continue
        assert D.on_device and D.colidx is None
        assert D.nnz == L.colidx.size
        assert np.array_equal(D.fullrowptr, L.fullrowptr), "rowseg = U's row pointer"
        lt = sp.csr_matrix(_graph(case[0]).T)
        degt = np.diff(lt.indptr)[D.cols]
        assert np.array_equal(D.colseg, np.concatenate([[0], np.cumsum(degt)]).astype(np.int32))
        K = L.shape[1]
        colptr = np.concatenate([[0], np.cumsum(np.bincount(L.colidx, minlength=K))]).astype(np.int32)
        assert np.array_equal(D.csc_colptr, colptr)
        assert np.all(np.diff(D.rows) > 0), "rows below the top layer are unique and ascending"
        assert np.all(np.diff(D.cols) > 0)
        if li == present[0]:
            assert np.array_equal(D.cols, cols_below)
    # rows of a layer = columns (after_nodes) of the layer above
    for lo, hi in zip(present[:-1], present[1:]):
        if hd.layers[hi].on_device:
            assert np.array_equal(hd.layers[lo].rows, hd.layers[hi].cols)
    assert hd.nnz() == hb.nnz()


def test_stored_zeros_keep_host_extraction():
    lap = _graph("symmetric").copy()
    lap.data[::7] = 0.0  # stored zeros: the column counts are no longer the structural counts
    N = lap.shape[0]
    batch = np.arange(64)
    hd = sampler.ladies_sample_host(3, batch, np.array([300] * 3), N, lap, _labels(N), [1, 1, 1],
                                    np.full(N, -1), np.zeros(N, np.int64), None, 1.0, [0], device_extract=True)
    assert all(not L.on_device for L in hd.layers if L is not None)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_extraction_bitexact(dev, case):
    hb, hd = _pair(*case)
    db = hb.to_device(dev, with_coo=False)
    dd = hd.to_device(dev, with_coo=False)
    torch.cuda.synchronize()
    for li, (a, b) in enumerate(zip(db.adjs, dd.adjs)):
        if a is None:
            assert b is None
            continue
        assert a.shape == b.shape and a.nnz == b.nnz
        for k in ("rowptr", "col", "val"):
            assert torch.equal(getattr(a, k), getattr(b, k)), f"layer {li} {k}"
        if li >= 1:
            at, bt = a.transpose(), b.transpose()
            for k in ("rowptr", "col", "val"):
                assert torch.equal(getattr(at, k), getattr(bt, k)), f"layer {li} transpose {k}"
            # and the canonical GPU transpose of the device-extracted operand agrees
            b._t = None
            bt2 = b.transpose()
            for k in ("rowptr", "col", "val"):
                assert torch.equal(getattr(at, k), getattr(bt2, k)), f"layer {li} gpu transpose {k}"
    dd.graph.check()
    assert dd.graph.symmetric == (case[0] == "symmetric")


@pytest.mark.gpu
def test_gpu_extraction_empty_and_count_mismatch(dev):
    """M = 0 / K = 0 calls are no-ops with a valid rowptr; a wrong host nnz raises the flag
    without writing outside the outputs."""
    from gnn_amd import custom_sparse_ops as cso

    lap = _graph("symmetric")
    ip = lap.indptr.astype(np.int64)
    g = sampler.device_graph(lap, dev)
    i32 = lambda a: torch.tensor(np.asarray(a, np.int64), dtype=torch.int32, device=dev)
    seg = lambda nodes: i32(np.concatenate([[0], np.cumsum(ip[np.asarray(nodes, np.int64) + 1] - ip[np.asarray(nodes, np.int64)])]))
    op = cso.extract_operand(g, i32([]), i32([1, 2]), torch.ones(2, device=dev), 0, seg([]), seg([1, 2]),
                             i32([0, 0, 0]))
    assert op.rowptr.tolist() == [0] and op.nnz == 0
    assert op.transpose().rowptr.tolist() == [0, 0, 0]
    op = cso.extract_operand(g, i32([3, 4]), i32([]), torch.ones(0, device=dev), 0, seg([3, 4]))
    assert op.rowptr.tolist() == [0, 0, 0]
    g.check()
    nb = np.asarray(lap[[5, 6]].indices)
    cols = np.unique(nb)[:5].astype(np.int32)
    true_nnz = int(np.isin(lap[[5, 6]].indices, cols).sum())
    op = cso.extract_operand(g, i32([5, 6]), torch.from_numpy(cols).to(dev), torch.ones(cols.size, device=dev),
                             true_nnz, seg([5, 6]))
    torch.cuda.synchronize()
    g.check()
    assert op.rowptr[-1].item() == true_nnz
    op = cso.extract_operand(g, i32([5, 6]), torch.from_numpy(cols).to(dev), torch.ones(cols.size, device=dev),
                             true_nnz + 1, seg([5, 6]))
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="disagree"):
        g.check()
    g.err.zero_()


def test_extract_layer_mask():
    """device_extract as bottom-up layer indices: only those layers go to the GPU; the others
    keep the host extraction (and CSC) of the plain sampler, the draw is unchanged."""
    lap = _graph("symmetric")
    N = lap.shape[0]
    batch = np.random.default_rng(7).choice(N, 128, replace=False)
    args = (13, batch, np.array([500] * 3), N, lap, _labels(N), [1, 1, 1], np.full(N, -1), np.zeros(N, np.int64),
            None, 1.0, [0])
    hb = sampler.ladies_sample_host(*args)
    for mask, on in (([0], [True, False, False]), ([1], [False, True, False]), ([], [False, False, False])):
        hd = sampler.ladies_sample_host(*args, device_extract=mask)
        assert [L.on_device for L in hd.layers] == on
        for L, D in zip(hb.layers, hd.layers):
            assert np.array_equal(L.normfact, D.normfact) and L.nnz == D.nnz
            if not D.on_device:
                assert np.array_equal(L.colidx, D.colidx) and np.array_equal(L.rowptr, D.rowptr)


@pytest.mark.gpu
def test_gpu_extraction_layer_mask(dev):
    lap = _graph("symmetric")
    N = lap.shape[0]
    batch = np.random.default_rng(8).choice(N, 128, replace=False)
    args = (17, batch, np.array([500] * 3), N, lap, _labels(N), [1, 1, 1], np.full(N, -1), np.zeros(N, np.int64),
            None, 1.0, [0])
    db = sampler.ladies_sample_host(*args).to_device(dev, with_coo=False)
    dd = sampler.ladies_sample_host(*args, device_extract=[0]).to_device(dev, with_coo=False)
    for li, (a, b) in enumerate(zip(db.adjs, dd.adjs)):
        for k in ("rowptr", "col", "val"):
            assert torch.equal(getattr(a, k), getattr(b, k)), (li, k)
        if li >= 1:
            for k in ("rowptr", "col", "val"):
                assert torch.equal(getattr(a.transpose(), k), getattr(b.transpose(), k)), (li, "t", k)
    dd.graph.check()


def _hub_graph():
    """Two hub nodes adjacent to every node (rows of 30 k entries: segments spanning ~60 chunks
    of the walk) on top of a sparse random graph, symmetric."""
    rng = np.random.default_rng(21)
    n = 30_000
    u = rng.integers(0, n, 90_000)
    v = rng.integers(0, n, 90_000)
    hubs = np.array([0, 17])
    hu = np.repeat(hubs, n)
    hv = np.tile(np.arange(n), hubs.size)
    r = np.concatenate([u, v, hu, hv])
    c = np.concatenate([v, u, hv, hu])
    keep = r != c
    A = sp.csr_matrix((np.ones(keep.sum(), np.float32), (r[keep], c[keep])), shape=(n, n))
    A.data[:] = 1
    A.sort_indices()
    return graphs.lap_matrix(A, "graphsage")


@pytest.mark.gpu
def test_gpu_extraction_hub_rows(dev):
    """Rows far longer than a walk chunk (the hubs' 30 k-entry rows, in U and in lapᵀ): the
    device-extracted operands and transposes equal the host path's, bit for bit."""
    lap = _hub_graph()
    N = lap.shape[0]
    batch = np.concatenate([[0, 17], np.random.default_rng(4).choice(np.arange(18, N), 254, replace=False)])
    args = (29, batch, np.array([3000] * 5), N, lap, _labels(N), [1, 1, 1], np.full(N, -1), np.zeros(N, np.int64),
            None, 1.0, [0])
    hb = sampler.ladies_sample_host(*args)
    hd = sampler.ladies_sample_host(*args, device_extract=True)
    assert any(L is not None and L.on_device for L in hd.layers)
    db = hb.to_device(dev, with_coo=False)
    dd = hd.to_device(dev, with_coo=False)
    torch.cuda.synchronize()
    for li, (a, b) in enumerate(zip(db.adjs, dd.adjs)):
        for k in ("rowptr", "col", "val"):
            assert torch.equal(getattr(a, k), getattr(b, k)), (li, k)
        if li >= 1:
            for k in ("rowptr", "col", "val"):
                assert torch.equal(getattr(a.transpose(), k), getattr(b.transpose(), k)), (li, "t", k)
    dd.graph.check()


@pytest.mark.gpu
def test_count_mismatch_raises_before_the_step(dev):
    """A GPU-extracted layer whose device count disagrees with the host's raises when the staged
    batch is handed to its step (StagedX0.wait, before any kernel of the step is issued), not at
    the end of the run: the flag is copied to pinned memory on the staging stream right after the
    batch's extractions."""
    from gnn_amd import staging

    hb, hd = _pair("symmetric", [1, 1, 1], 300, 64, 7)
    dd = hd.to_device(dev, with_coo=False)
    ev = torch.cuda.Event()
    ev.record()
    x0 = torch.zeros(4, 8, device=dev)
    assert dd.err_host is not None
    staging.StagedX0(x0, ev, (), 8, dd).wait()  # a consistent batch passes
    li = next(i for i, L in enumerate(hd.layers) if L is not None and L.on_device)
    hd.layers[li].dev_nnz += 1  # the host's count now disagrees with the device's
    bad = hd.to_device(dev, with_coo=False)
    ev = torch.cuda.Event()
    ev.record()
    try:
        with pytest.raises(RuntimeError, match="disagree"):
            staging.StagedX0(x0, ev, (), 8, bad).wait()
    finally:
        torch.cuda.synchronize()
        bad.graph.err.zero_()
