"""Native batch producer (libgnn_sampler.so gnn_loader_*, gnn_amd.loader.NativeLoader).

CPU: for the same seed schedule the C++ workers produce exactly what the Python BatchLoader
produces (whose sampler and placement are pinned to the reference by tests/golden): every layer
array, the CSC of host-extracted layers, sampled nodes and residual row maps, dense labels, the
placement split of the layer-0 inputs (own buffer / host / each peer), and the gathered host
feature rows — for LADIES (host and device extraction), subgraph and FastGCN, at world sizes 1
and 2. GPU: a NativeBatch uploads as one blob and its DeviceBatch / staged X0 equal the Python
path's, operands bit-exact.
"""
import numpy as np
import pytest
import torch

from gnn_amd import graphs, loader, placement, sampler, staging


def _setup(world=1):
    rng = np.random.default_rng(2)
    A = graphs.chung_lu(12_000, 90_000, 1.3, rng)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]

    cls = rng.integers(0, 7, N)
    import scipy.sparse as sp
    labels = sp.csr_matrix((np.ones(N, np.int32), (np.arange(N), cls)), shape=(N, 7))
    feats = torch.randn(N, 37, generator=torch.Generator().manual_seed(0))
    train = np.arange(0, 8000)
    pl = placement.create_buffer(lap, train, 1500, list(range(world)), 2, alpha=0)
    return lap, labels, feats, train, pl


def _loaders(kind, world, rank, dx, samp=400, bs=96):
    lap, labels, feats, train, pl = _setup(world)
    dev_of, idx_on = pl.device_id_of_nodes_group[rank], pl.idx_of_nodes_on_device_group[rank]
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[rank], "cpu", rank)
    kw = dict(rank=rank, world_size=world, store=store, workers=3, seed=9, kind=kind, device_extract=dx)
    a = loader.BatchLoader(lap, labels, train, samp, bs, [1, 1, 1], dev_of, idx_on, **kw)
    b = loader.NativeLoader(lap, labels, train, samp, bs, [1, 1, 1], dev_of, idx_on, **kw)
    return a, b, store


def _eq(x, y, what):
    x = x.numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
    y = y.numpy() if isinstance(y, torch.Tensor) else np.asarray(y)
    assert x.shape == y.shape and np.array_equal(x, y), what


@pytest.mark.parametrize("kind,world,rank,dx", [("ladies", 1, 0, False), ("ladies", 1, 0, True),
                                                ("ladies", 2, 1, True), ("subgraph", 1, 0, False),
                                                ("fastgcn", 2, 0, False)])
def test_native_loader_equals_python_loader(kind, world, rank, dx):
    a, b, store = _loaders(kind, world, rank, dx)
    try:
        for pa, pb in zip(a.epoch(1), b.epoch(1)):
            ha, hb = pa.host, pb.host
            assert ha.seed == hb.seed
            _eq(ha.input_nodes, hb.input_nodes, "input nodes")
            _eq(ha.labels, hb.labels, "labels")
            assert ha.nnz() == hb.nnz()
            for li, (La, Lb) in enumerate(zip(ha.layers, hb.layers)):
                assert (La is None) == (Lb is None)
                if La is None:
                    continue
                assert La.shape == Lb.shape and La.on_device == Lb.on_device and La.nnz == Lb.nnz
                for k in ("fullrowptr", "rowptr", "colidx", "normfact", "csc_colptr", "csc_rows", "rows", "cols"):
                    va, vb = getattr(La, k), getattr(Lb, k)
                    assert (va is None) == (vb is None), (li, k)
                    if va is not None:
                        _eq(va, vb, f"layer {li} {k}")
            for li, (sa, sb) in enumerate(zip(ha.sampled_nodes, hb.sampled_nodes)):
                _eq(np.asarray(sa, np.int64), sb, f"sampled {li}")
            rmaps = ha.pin().extra["rmaps"]
            for li in range(len(ha.layers)):
                base = loader.BLOB_HEADER + li * loader.BLOB_LAYER_SLOTS
                if rmaps[li] is not None:
                    _eq(rmaps[li], hb._h(base + loader.L_RMAP, np.dtype(np.int32)), f"rmap {li}")
            qa, qb = pa.plan, pb.plan
            for k in ("own_pos", "own_src", "host_pos"):
                _eq(getattr(qa, k), getattr(qb, k), k)
            for j in range(world):
                _eq(qa.peer_pos[j], qb.peer_pos[j], f"peer_pos {j}")
                _eq(qa.peer_src[j], qb.peer_src[j], f"peer_src {j}")
            bb = hb._bb
            rows = hb._h(bb + loader.B_HOST_ROWS, np.dtype(np.float32)).reshape(-1, store.ld)
            _eq(qa.host_rows, rows, "host rows")
    finally:
        a.close()
        b.close()


def test_native_loader_bad_batch_raises():
    lap, labels, feats, train, pl = _setup()
    b = loader.NativeLoader(lap, labels, train, 100, 16, [1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], workers=2)
    try:
        with pytest.raises(RuntimeError, match="out of range"):
            b._submit(np.array([0, lap.shape[0] + 5]))
    finally:
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dx", [False, True])
def test_native_batch_on_device(dev, dx):
    lap, labels, feats, train, pl = _setup()
    dev_of, idx_on = pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0]
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    kw = dict(store=store, workers=2, seed=3, device_extract=dx)
    a = loader.BatchLoader(lap, labels, train, 400, 96, [1, 1, 1], dev_of, idx_on, **kw)
    b = loader.NativeLoader(lap, labels, train, 400, 96, [1, 1, 1], dev_of, idx_on, **kw)
    stager = staging.Stager(store)
    try:
        for n, (pa, pb) in enumerate(zip(a.epoch(1), b.epoch(1))):
            sa = stager.issue(pa.plan, lambda: pa.host.to_device(dev, with_coo=False))
            sb = stager.issue(pb.plan, lambda: pb.host.to_device(dev, with_coo=False))
            xa, xb = sa.wait(), sb.wait()
            torch.cuda.synchronize()
            assert torch.equal(xa, xb)
            ref = feats[torch.from_numpy(np.asarray(pa.host.input_nodes, np.int64))].to(dev)
            assert torch.equal(xb, ref), "X0 rows = the feature table's rows"
            da, db = sa.batch, sb.batch
            assert torch.equal(da.labels, db.labels)
            for x, y in zip(da.sampled_nodes, db.sampled_nodes):
                assert torch.equal(x, y)
                ra, rb = getattr(x, "_gnn_rmap", None), getattr(y, "_gnn_rmap", None)
                assert (ra is None) == (rb is None) and (ra is None or torch.equal(ra, rb))
            for li, (oa, ob) in enumerate(zip(sa.adjs, sb.adjs)):
                for k in ("rowptr", "col", "val"):
                    assert torch.equal(getattr(oa, k), getattr(ob, k)), (li, k)
                if li >= 1:
                    ta, tb = oa.transpose(), ob.transpose()
                    for k in ("rowptr", "col", "val"):
                        assert torch.equal(getattr(ta, k), getattr(tb, k)), (li, "t", k)
            if n == 3:
                break
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_blob_dropped_right_after_upload(dev):
    """A NativeBatch dropped while its upload is still queued: the pinned blob must not go back
    to the loader's pool (where a worker refills it for the next batch) before the H2D has read
    it. The upload is held behind a GPU spin on its stream, the batch is dropped at once, and the
    workers keep producing; the device copy must equal the blob as it was at upload time."""
    import gc

    lap, labels, feats, train, pl = _setup()
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    b = loader.NativeLoader(lap, labels, train, 400, 96, [1, 1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], store=store, workers=3, seed=4, prefetch=2)
    side = torch.cuda.Stream(dev)
    try:
        it = b.epoch(1)
        for _ in range(6):
            lb = next(it)
            want = torch.from_numpy(lb.host.blob.copy())
            with torch.cuda.stream(side):
                torch.cuda._sleep(20_000_000)  # the H2D below waits behind this spin
                d = lb.host.device_blob(dev)
            del lb  # the blob's finaliser runs here
            gc.collect()
            next_lb = next(it)  # workers refill pooled blobs meanwhile
            torch.cuda.synchronize()
            assert torch.equal(d.cpu(), want), "the uploaded blob was overwritten before its copy ran"
            del next_lb
    finally:
        b.close()


def test_locality_sampling_leaves_the_draw_unchanged_at_scale_1():
    """--locality_sampling (main.py:284-287): the skewed node sets (preprocess.py:414-423) reach
    every sampler call; at the reference's scale_factor 1.0 (main.py:256) they do not change the
    draw (sampler.py:119-121) — the native producer with the flag yields the same batches, bit for
    bit, as without it. With scale_factor > 1 the numpy branch boosts the skewed nodes (the draw
    then differs), and the native producer refuses it."""
    import scipy.sparse as sp

    lap, labels, feats, train, pl = _setup(world=2)
    A = (lap != 0).astype(np.float32).tocsr()
    skew = placement.get_skewed_sampled_nodes(A + sp.eye(A.shape[0], dtype=np.float32, format="csr"),
                                              pl.gpu_buffer_group, [1, 1, 1])
    assert len(skew) == 3 and all(len(s) > 0 for s in skew)
    dev_of, idx_on = pl.device_id_of_nodes_group[1], pl.idx_of_nodes_on_device_group[1]
    kw = dict(rank=1, world_size=2, workers=2, seed=5, kind="ladies", device_extract=True)
    plain = loader.NativeLoader(lap, labels, train, 300, 64, [1, 1, 1], dev_of, idx_on, **kw)
    flag = loader.NativeLoader(lap, labels, train, 300, 64, [1, 1, 1], dev_of, idx_on, **kw,
                               skewed_sampling_nodes=skew, scale_factor=1.0)
    py = loader.BatchLoader(lap, labels, train, 300, 64, [1, 1, 1], dev_of, idx_on, **kw,
                            skewed_sampling_nodes=skew, scale_factor=1.0)
    try:
        n = 0
        for a, b, c in zip(plain.epoch(1), flag.epoch(1), py.epoch(1)):
            for other in (b.host, c.host):
                _eq(a.host.input_nodes, other.input_nodes, "input nodes")
                for La, Lb in zip(a.host.layers, other.layers):
                    assert La.nnz == Lb.nnz
                    for k in ("fullrowptr", "rowptr", "colidx", "normfact", "rows", "cols"):
                        va, vb = getattr(La, k), getattr(Lb, k)
                        assert (va is None) == (vb is None)
                        if va is not None:
                            _eq(va, vb, k)
            n += 1
            if n == 4:
                break
    finally:
        plain.close()
        flag.close()
        py.close()
    with pytest.raises(ValueError, match="scale_factor"):
        loader.NativeLoader(lap, labels, train, 300, 64, [1, 1, 1], dev_of, idx_on, **kw,
                            skewed_sampling_nodes=skew, scale_factor=2.0)
    # scale_factor > 1 (numpy branch): the boosted nodes change the draw
    batch = sampler.rank_batches(train, 64, 1, 2, 1)[0]
    args = (3, batch, np.array([300] * 5), lap.shape[0], lap, labels, [1, 1, 1], dev_of, idx_on)
    h1 = sampler.ladies_sample_host(*args, skew, 1.0, [0, 1], native=False)
    h4 = sampler.ladies_sample_host(*args, skew, 4.0, [0, 1], native=False)
    assert not np.array_equal(h1.input_nodes, h4.input_nodes)
    hn = sampler.ladies_sample_host(*args, skew, 1.0, [0, 1])
    _eq(h1.input_nodes, hn.input_nodes, "numpy == native at scale 1")


def _compare_staging(a, b, store, dev, nbatches, gate=True):
    """Batches of two NativeLoaders with the same seeds: a's through the Python sequence of staging
    calls, b's through the one native call; everything the step reads must be bit-identical."""
    stager = staging.Stager(store)
    gate_stream = torch.cuda.Stream(device=dev)
    stager.gate = torch.cuda.Event() if gate else None
    built = []
    for n, (pa, pb) in enumerate(zip(a.epoch(1), b.epoch(1))):
        if gate:
            with torch.cuda.stream(gate_stream):
                torch.cuda._sleep(2_000_000)  # the staging must wait for the gate, not run past it
                stager.gate.record(gate_stream)
        sa = stager.issue(pa.plan, lambda: pa.host.to_device(dev, with_coo=False))
        sb = stager.issue(pb.plan, loader.ToDevice(pb.host, dev, on_built=built.append))
        assert sb.batch.raw is None and built[-1] is sb.batch, "the native path ran"
        xa, xb = sa.wait(), sb.wait()
        torch.cuda.synchronize()
        assert torch.equal(xa, xb)
        da, db = sa.batch, sb.batch
        assert torch.equal(da.labels, db.labels)
        assert (da.err_host is None) == (db.err_host is None)
        if db.err_host is not None:
            assert int(db.err_host[0]) == 0
        for x, y in zip(da.sampled_nodes, db.sampled_nodes):
            assert torch.equal(x, y)
            ra, rb = getattr(x, "_gnn_rmap", None), getattr(y, "_gnn_rmap", None)
            assert (ra is None) == (rb is None) and (ra is None or torch.equal(ra, rb))
        for li, (oa, ob) in enumerate(zip(sa.adjs, sb.adjs)):
            assert oa.shape == ob.shape and oa.nnz == ob.nnz
            for k in ("rowptr", "col", "val"):
                assert torch.equal(getattr(oa, k), getattr(ob, k)), (li, k)
            assert (oa._t is None) == (ob._t is None), li
            if oa._t is not None:
                for k in ("rowptr", "col", "val"):
                    assert torch.equal(getattr(oa._t, k), getattr(ob._t, k)), (li, "t", k)
        with pytest.raises(RuntimeError, match="staged natively"):
            db.build_operands()
        if n + 1 == nbatches:
            break


@pytest.mark.gpu
@pytest.mark.parametrize("dx", [False, True, [1]])
def test_native_stage_equals_python_staging(dev, dx):
    """Stager.issue with a loader.ToDevice batch_fn stages the batch through ONE native call
    (gnn_stage_batch_f32: blob upload, X0 gather, every layer's operand, the error flag) — X0,
    every operand and transpose, sampled nodes, row maps and labels bit-identical to the Python
    sequence of calls on the same batch (two loaders with the same seeds: both upload). dx=[1]:
    layer 1 extracted on the GPU, the others built from the blob's CSR / CSC. A gate event that
    the stream must wait for is recorded on another stream behind a delay first."""
    lap, labels, feats, train, pl = _setup()
    dev_of, idx_on = pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0]
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    kw = dict(store=store, workers=2, seed=5, device_extract=dx)
    a = loader.NativeLoader(lap, labels, train, 400, 96, [1, 1, 1], dev_of, idx_on, **kw)
    b = loader.NativeLoader(lap, labels, train, 400, 96, [1, 1, 1], dev_of, idx_on, **kw)
    try:
        _compare_staging(a, b, store, dev, 4)
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_native_stage_config2(dev):
    """The same comparison at BASELINE config 2 (Reddit-shaped graph, samp 8192, batch 512, buffer
    0.1 of the nodes, every layer extracted on the GPU, 602 features in 608-float X0 rows)."""
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    dev_of, idx_on = pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0]
    kw = dict(store=store, workers=2, seed=11, device_extract=True)
    a = loader.NativeLoader(lap, labels, train, 8192, 512, [1, 1, 1], dev_of, idx_on, **kw)
    b = loader.NativeLoader(lap, labels, train, 8192, 512, [1, 1, 1], dev_of, idx_on, **kw)
    try:
        _compare_staging(a, b, store, dev, 2)
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("dx", [False, True, [1]])
def test_stage_plan_layout(dx):
    """gnn_stage_plan (host-only code of include/gnn_stage.h) on real native-loader batches: every
    array the staging call writes gets a 256-byte-aligned, non-overlapping arena range of its
    size; GPU-extracted layers get their row pointer (and from layer 1 their transpose's rows and
    values), host-built layers only col / val (+ the transpose's values: the blob holds its CSC);
    the extraction workspace exists iff a layer is extracted and is large enough for each; a
    descriptor of another blob version is refused with a message."""
    from gnn_amd import _lib

    lap, labels, feats, train, pl = _setup()
    dev_of, idx_on = pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0]
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], "cpu", 0)
    b = loader.NativeLoader(lap, labels, train, 400, 96, [1, 1, 1], dev_of, idx_on, store=store, workers=2, seed=4,
                            device_extract=dx)
    L = _lib.lib()
    try:
        lb = next(iter(b.epoch(1)))
        nb = lb.host
        a = np.zeros(loader.STAGE_SLOTS, np.int64)
        a[loader.ST_DESC], a[loader.ST_HOST_BLOB] = nb.desc.ctypes.data, nb.ptr
        a[loader.ST_NUM_NODES], a[loader.ST_CSC_FROM] = lap.shape[0], 1
        out = np.full(loader.BLOB_MAX_LAYERS * loader.STAGE_OUT_SLOTS, -7, np.int64)
        nbytes = L.gnn_stage_plan(a.ctypes.data, out.ctypes.data)
        assert nbytes > 0 and nbytes % 256 == 0
        ranges = []
        any_dev = False
        for li in range(nb.num_layers):
            base = nb._lb(li)
            o = out[li * loader.STAGE_OUT_SLOTS:(li + 1) * loader.STAGE_OUT_SLOTS]
            M, K, nnz = (int(nb.desc[base + s]) for s in (loader.L_M, loader.L_K, loader.L_NNZ))
            on_dev = bool(nb.desc[base + loader.L_ON_DEVICE])
            sizes = {loader.SO_COL: 4 * nnz, loader.SO_VAL: 4 * nnz}
            if on_dev:
                any_dev = True
                sizes[loader.SO_ROWPTR] = 4 * (M + 1)
                if li >= 1:
                    sizes[loader.SO_ROWS_T] = sizes[loader.SO_VAL_T] = 4 * nnz
                else:
                    assert o[loader.SO_ROWS_T] == -1 and o[loader.SO_VAL_T] == -1
                rt = int(nb._h(base + loader.L_FULLROWPTR, np.dtype(np.int32))[M])
                ct = int(nb._h(base + loader.L_COLSEG, np.dtype(np.int32))[K]) if li >= 1 else 0
                ws = L.gnn_ladies_extract_workspace_bytes(lap.shape[0], M, K, int(li >= 1), rt, ct)
                assert out[5] >= 0 and out[5] + ws <= nbytes
            else:
                assert o[loader.SO_ROWPTR] == -1 and o[loader.SO_ROWS_T] == -1
                if nb._count(base + loader.L_CSC_COLPTR) > 0:
                    sizes[loader.SO_VAL_T] = 4 * nnz
            for k, sz in sizes.items():
                off = int(o[k])
                assert off >= 0 and off % 256 == 0 and off + sz <= nbytes, (li, k, off, sz)
                ranges.append((off, off + max(sz, 1)))
        if any_dev:
            ranges.append((int(out[5]), nbytes))
        else:
            assert out[5] == -1
        ranges.sort()
        assert all(e0 <= s1 for (_, e0), (s1, _) in zip(ranges, ranges[1:])), "arena ranges overlap"
        d2 = nb.desc.copy()
        d2[loader.H_VERSION] = 99
        a[loader.ST_DESC] = d2.ctypes.data
        assert L.gnn_stage_plan(a.ctypes.data, out.ctypes.data) == 0
        assert b"version" in L.gnn_last_error()
    finally:
        b.close()


def test_set_colcount_workers_contract():
    """gnn_loader_set_colcount_workers: a negative count is refused, and so is any call once a
    batch has been submitted (the workers read it per batch)."""
    from gnn_amd import _lib

    lap, labels, feats, train, pl = _setup()
    b = loader.NativeLoader(lap, labels, train, 100, 16, [1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], workers=2)
    L = _lib.sampler_lib()
    try:
        assert L.gnn_loader_set_colcount_workers(b.handle, -1) != 0
        assert L.gnn_loader_set_colcount_workers(b.handle, 1) == 0
        next(iter(b.epoch(1)))
        assert L.gnn_loader_set_colcount_workers(b.handle, 1) != 0
        assert b"already submitted" in L.gnn_sampler_last_error()
    finally:
        b.close()
