"""CPU: host sampler and placement restatements vs the reference's goldens (bit-exact)."""
import numpy as np
import pytest
import scipy.sparse as sp

from gnn_amd import placement, sampler
from gnn_amd.graphs import row_normalize


def _graph(golden):
    g = golden("graph_tiny.npz")
    N = int(g["N"])
    A = sp.csr_matrix((np.ones(len(g["A_indices"]), np.float32), g["A_indices"], g["A_indptr"]), shape=(N, N))
    lap = sp.csr_matrix((g["lap_data"], g["lap_indices"], g["lap_indptr"]), shape=(N, N))
    ncls = int(g["num_classes"])
    labels = sp.csr_matrix((np.ones(N, np.int32), (np.arange(N), g["labels_cls"])), shape=(N, ncls))
    train = np.arange(int(g["n_train"]))
    return A, lap, labels, train, N


def test_row_normalize_matches_reference(golden):
    A, lap, _, _, _ = _graph(golden)
    mine = row_normalize(A)
    assert np.array_equal(mine.indptr, lap.indptr)
    assert np.array_equal(mine.indices, lap.indices)
    assert np.array_equal(mine.data.astype(np.float32), lap.data)


def test_placement_matches_reference(golden):
    A, lap, _, train, N = _graph(golden)
    pl = golden("placement_tiny.npz")
    k = int(pl["k"])
    for ndev in (1, 2, 4, 8):
        mine = placement.create_buffer_ours(lap, train, k, list(range(ndev)), 3, alpha=0)
        for i in range(ndev):
            assert np.array_equal(mine.device_id_of_nodes_group[i], pl[f"n{ndev}_dev{i}"]), (ndev, i)
            assert np.array_equal(np.asarray(mine.gpu_buffer_group[i]), pl[f"n{ndev}_buf{i}"]), (ndev, i)
        assert np.array_equal(mine.idx_of_nodes_on_device_group[0], pl[f"n{ndev}_idx"])
    skew = placement.get_skewed_sampled_nodes(A + sp.eye(N), [pl["n2_buf0"], pl["n2_buf1"]], [1, 1, 1])
    for i, s in enumerate(skew):
        assert np.array_equal(np.asarray(s), pl[f"skew{i}"])


def test_placement_cache_roundtrip(golden, tmp_path):
    _, lap, _, train, _ = _graph(golden)
    path = str(tmp_path / "p.npz")
    a = placement.create_buffer(lap, train, 100, [0, 1, 2], 3, alpha=0, cache_path=path)
    b = placement.create_buffer(lap, train, 100, [0, 1, 2], 3, alpha=0, cache_path=path)
    for x, y in zip(a.device_id_of_nodes_group, b.device_id_of_nodes_group):
        assert np.array_equal(x, y)
    assert np.array_equal(a.idx_of_nodes_on_device_group[0], b.idx_of_nodes_on_device_group[0])


@pytest.mark.parametrize("native", [True, False])
def test_ladies_matches_reference(golden, native):
    _, lap, labels, _, N = _graph(golden)
    z = golden("ladies_tiny.npz")
    pl = golden("placement_tiny.npz")
    for c in range(4):
        samp, bs, seed, ndev = (int(v) for v in z[f"c{c}_cfg"])
        hb = sampler.ladies_sample_host(seed, z[f"c{c}_batch"], np.array([samp] * 5), N, lap, labels, [1, 1, 1],
                                        pl[f"n{ndev}_dev0"], pl[f"n{ndev}_idx"], None, 1.0, list(range(ndev)),
                                        native=native)
        for li in range(3):  # recorded top-down; hb.layers bottom-up
            L = hb.layers[2 - li]
            p = f"c{c}_call{li}_"
            assert np.array_equal(L.fullrowptr, z[p + "fullrowptr"])
            assert np.array_equal(L.rowptr, z[p + "rowptr"])
            assert np.array_equal(L.colidx, z[p + "colidx"].astype(np.int32))
            assert np.array_equal(L.normfact, z[p + "normfact"])
            assert tuple(L.shape) == tuple(z[p + "shape"])
        for li in range(3):
            assert np.array_equal(hb.sampled_nodes[li], z[f"c{c}_sampled{li}"])
        for i in range(ndev):
            assert np.array_equal(hb.input_nodes_mask_on_devices[i], z[f"c{c}_mask{i}"])
            assert np.array_equal(hb.nodes_idx_on_devices[i], z[f"c{c}_idxdev{i}"])
        assert np.array_equal(hb.input_nodes_mask_on_cpu, z[f"c{c}_cpumask"])
        assert np.array_equal(hb.nodes_idx_on_cpu, z[f"c{c}_idxcpu"])
        assert hb.num_input_nodes == int(z[f"c{c}_nin"])
        assert np.array_equal(hb.labels, z[f"c{c}_labels"])


def test_rank_batches_partition():
    nodes = np.arange(1000, 2003)
    seen = []
    for rank in range(3):
        bs = sampler.rank_batches(nodes, 64, rank, 3, iter_num=5)
        assert all(len(b) <= 64 for b in bs)
        seen.extend(np.concatenate(bs).tolist())
    assert sorted(seen) == nodes.tolist()


def _rows_as_sets_equal(rowptr, a, b):
    for r in range(len(rowptr) - 1):
        s, e = rowptr[r], rowptr[r + 1]
        if not np.array_equal(np.sort(a[s:e]), np.sort(b[s:e])):
            return False
    return True


@pytest.mark.parametrize("native", [True, False])
def test_subgraph_sampler_matches_reference(golden, native):
    """subgraph_sampler (sampler.py:7-88) vs the reference's own outputs. Below the first
    layer the reference slices the (unsorted) lap without canonicalising it, so its recorded
    colidx rows are permutations of ours: rows compared as sets, and the operand the GPU
    builds (the coalesced COO) compared exactly."""
    _, lap, labels, _, N = _graph(golden)
    z = golden("subgraph_tiny.npz")
    pl = golden("placement_tiny.npz")
    for c in range(4):
        samp, bs, seed, ndev = (int(v) for v in z[f"c{c}_cfg"])
        orders = [int(v) for v in z[f"c{c}_orders"]]
        hb = sampler.subgraph_sample_host(seed, z[f"c{c}_batch"], np.array([samp] * 5), N, lap, labels, orders,
                                          pl[f"n{ndev}_dev0"], pl[f"n{ndev}_idx"], None, 1.0, list(range(ndev)),
                                          native=native)
        nl = len(orders)
        present = [li for li in range(nl) if bool(z[f"c{c}_present{li}"])]
        assert [li for li in range(nl) if hb.layers[li] is not None] == present
        assert int(z[f"c{c}_ncalls"]) == len(present)
        for k, li in enumerate(sorted(present, reverse=True)):  # calls recorded top-down
            L = hb.layers[li]
            p = f"c{c}_call{k}_"
            assert np.array_equal(L.fullrowptr, z[p + "fullrowptr"])
            assert np.array_equal(L.rowptr, z[p + "rowptr"])
            assert _rows_as_sets_equal(L.rowptr, L.colidx, z[p + "colidx"].astype(np.int32))
            assert np.array_equal(L.normfact, z[p + "normfact"])
            assert tuple(L.shape) == tuple(z[p + "shape"])
            # the operand as the reference's create_coo_tensor + coalesce sees it
            rows = np.repeat(np.arange(L.shape[0]), np.diff(L.rowptr))
            deg = np.diff(L.fullrowptr).astype(np.float64)
            vals = ((1.0 / deg[rows]) * L.normfact[L.colidx].astype(np.float64)).astype(np.float32)
            order = np.lexsort((L.colidx, rows))
            assert np.array_equal(np.stack([rows[order], L.colidx[order]]), z[f"c{c}_adj{li}_indices"])
            assert np.array_equal(vals[order], z[f"c{c}_adj{li}_values"])
        for li in range(nl):
            assert np.array_equal(np.asarray(hb.sampled_nodes[li], np.int64), z[f"c{c}_sampled{li}"])
        for i in range(ndev):
            assert np.array_equal(hb.input_nodes_mask_on_devices[i], z[f"c{c}_mask{i}"])
            assert np.array_equal(hb.nodes_idx_on_devices[i], z[f"c{c}_idxdev{i}"])
        assert np.array_equal(hb.input_nodes_mask_on_cpu, z[f"c{c}_cpumask"])
        assert np.array_equal(hb.nodes_idx_on_cpu, z[f"c{c}_idxcpu"])
        assert hb.num_input_nodes == int(z[f"c{c}_nin"])
        assert np.array_equal(hb.labels, z[f"c{c}_labels"])
