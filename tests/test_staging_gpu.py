"""GPU: batch staging on the side stream — X0 assembly plus the batch's H2D copies and
operand builds (Stager.issue(plan, batch_fn)) — gives the compute stream exactly the inputs
a build on the compute stream gives: X0 rows bit-identical to the feature table, operands
bit-identical, and the same training-step loss."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from gnn_amd import loader, placement, staging
from gnn_amd.graphs import chung_lu, row_normalize
from gnn_amd.models import build_model
from gnn_amd.train import Trainer

pytestmark = pytest.mark.gpu


def _setup(N=6000, avg=16, seed=5):
    A = chung_lu(N, N * avg // 2, 1.3, np.random.default_rng(seed))
    lap = row_normalize(A)
    lap.sum_duplicates()
    labels = sp.csr_matrix((np.ones(N, np.float32), (np.arange(N), np.arange(N) % 7)), shape=(N, 7))
    train = np.arange(0, N, 2)
    return lap, labels, train


def test_side_stream_batch_matches_compute_stream(dev):
    lap, labels, train = _setup()
    N = lap.shape[0]
    pl = placement.create_buffer_ours(lap, train, 500, [0], 3, alpha=0)
    feats = torch.randn(N, 30)
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    ld = loader.BatchLoader(lap, labels, train, 800, 128, [1, 1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], rank=0, world_size=1, store=store, workers=2,
                            seed=21)
    lbs = list(ld.epoch(1))[:3]
    ld.close()
    stager = staging.Stager(store)
    torch.manual_seed(0)
    m1 = build_model("graphsage", 30, 16, [1, 1, 1], 7, dropout=0.0, fused=True).to(dev)
    torch.manual_seed(0)
    m2 = build_model("graphsage", 30, 16, [1, 1, 1], 7, dropout=0.0, fused=True).to(dev)
    t1, t2 = Trainer(m1, 0.01, dev), Trainer(m2, 0.01, dev)
    for lb in lbs:
        # side stream: X0 + H2D + operand builds, issued before anything else touches them
        staged = stager.issue(lb.plan, lambda: lb.host.to_device(dev, with_coo=False))
        x0 = staged.wait()
        db = staged.batch
        # reference: everything on the compute stream
        ref = lb.host.to_device(dev, with_coo=False)
        assert torch.equal(x0.cpu(), feats[torch.from_numpy(lb.host.input_nodes)])
        for a, b in zip(staged.adjs, ref.adjs):
            assert torch.equal(a.rowptr, b.rowptr) and torch.equal(a.col, b.col) and torch.equal(a.val, b.val)
            ta, tb = a.transpose(), b.transpose()
            assert torch.equal(ta.rowptr, tb.rowptr) and torch.equal(ta.col, tb.col) and torch.equal(ta.val, tb.val)
        l1 = t1.step(x0, staged.adjs, db.sampled_nodes, db.labels)
        x0r = x0.clone()
        l2 = t2.step(x0r, ref.adjs, ref.sampled_nodes, ref.labels)
        assert float(l1) == float(l2)
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1, p2)


def test_zero_copy_host_rows_match_copy_path(dev):
    """FeatureStore(zero_copy=True): the GPU reads the non-buffered rows from the pinned,
    device-mapped host table (gnn_gather_rows_host_f32); X0 must be bit-identical to the
    feature table rows and to the pinned-copy path's X0, pads zero."""
    lap, labels, train = _setup()
    N = lap.shape[0]
    pl = placement.create_buffer_ours(lap, train, 500, [0], 3, alpha=0)
    feats = torch.randn(N, 37)  # odd width: 8-byte vectors, 64-float padded rows
    zc = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0, zero_copy=True)
    cp = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    ld = loader.BatchLoader(lap, labels, train, 800, 128, [1, 1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], rank=0, world_size=1, store=zc, workers=2, seed=3)
    lbs = list(ld.epoch(1))[:3]
    ld.close()
    s_zc, s_cp = staging.Stager(zc), staging.Stager(cp)
    for lb in lbs:
        assert lb.plan.host_rows is None and len(lb.plan.host_pos) > 0
        plan_cp = staging.make_plan(lb.host, cp, 0, 1)
        x_zc = s_zc.issue(lb.plan).wait()
        x_cp = s_cp.issue(plan_cp).wait()
        torch.cuda.synchronize()
        want = feats[torch.from_numpy(lb.host.input_nodes)]
        assert torch.equal(x_zc.cpu(), want)
        assert torch.equal(x_zc.cpu(), x_cp.cpu())
        full = x_zc.as_strided((x_zc.shape[0], zc.ld), (zc.ld, 1))
        assert torch.all(full[:, 37:].cpu() == 0)


def test_zero_copy_gather_rejects_unregistered_memory(dev):
    from gnn_amd import custom_sparse_ops as cso

    host = torch.randn(16, 8)  # plain pageable memory, never registered
    idx = torch.arange(4, device=dev)
    dst = torch.empty(4, 8, device=dev)
    with pytest.raises(RuntimeError, match="hipHostGetDevicePointer"):
        cso.gather_rows_host(host, idx, dst, None)


def test_retirement_pipeline_on_priority_stream_matches(dev):
    # bench.py's pipeline: batch i+1 staged on the side stream before batch i's step, the step
    # on a high-priority stream, staged buffers kept alive by one retirement event per step
    # (depth 1: the host waits for the GPU every step, so freed blocks are reused at once)
    # instead of record_stream — same losses and weights as the record_stream path.
    lap, labels, train = _setup(seed=7)
    N = lap.shape[0]
    pl = placement.create_buffer_ours(lap, train, 500, [0], 3, alpha=0)
    feats = torch.randn(N, 30)
    store = staging.FeatureStore(feats, pl.gpu_buffer_group[0], dev, 0)
    ld = loader.BatchLoader(lap, labels, train, 800, 128, [1, 1, 1], pl.device_id_of_nodes_group[0],
                            pl.idx_of_nodes_on_device_group[0], rank=0, world_size=1, store=store, workers=2,
                            seed=3)
    lbs = list(ld.epoch(1))[:6]
    ld.close()

    def run(retire, stream):
        torch.manual_seed(0)
        m = build_model("graphsage", 30, 16, [1, 1, 1], 7, dropout=0.0, fused=True).to(dev)
        tr = Trainer(m, 0.01, dev)
        stager = staging.Stager(store)
        losses = []
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            it = iter(lbs)
            nxt = lambda lb: stager.issue(lb.plan, lambda: lb.host.to_device(dev, with_coo=False))
            staged = nxt(next(it))
            for i in range(len(lbs)):
                staged_next = nxt(next(it)) if i + 1 < len(lbs) else None
                x0 = staged.wait(retire)
                db = staged.batch
                losses.append(tr.step(x0, staged.adjs, db.sampled_nodes, db.labels))
                if retire is not None:
                    retire.retire(staged)
                staged = staged_next
        torch.cuda.synchronize()
        return [float(l) for l in losses], [p.detach().clone() for p in m.parameters()]

    lo, hi = torch.cuda.Stream.priority_range()
    ref_l, ref_p = run(None, torch.cuda.Stream(device=dev))
    got_l, got_p = run(staging.Retirement(depth=1), torch.cuda.Stream(device=dev, priority=hi))
    assert got_l == ref_l
    for a, b in zip(got_p, ref_p):
        assert torch.equal(a, b)


@pytest.mark.parametrize("F,ld0,ld1,ldd", [(602, 608, 608, 608), (602, 602, 608, 602), (100, 100, 100, 100),
                                           (1024, 1024, 1024, 1024), (3000, 3000, 3000, 3000)])
@pytest.mark.parametrize("n0,n1", [(900, 1300), (0, 17), (33, 0)])
def test_gather_rows2_matches_indexing(dev, F, ld0, ld1, ldd, n0, n1):
    """gnn_gather_rows2_f32 (X0's own-buffer and host rows in one launch) against torch indexing,
    bit for bit; padded and unpadded strides, one empty source, rows too wide for one pass."""
    from gnn_amd import custom_sparse_ops as cso

    g = torch.Generator().manual_seed(F + n0 + n1)
    src0 = torch.randn(2000, ld0, generator=g).to(dev)
    src1 = torch.randn(max(n1, 1), ld1, generator=g).to(dev)
    perm = torch.randperm(n0 + n1, generator=g)
    pos0, pos1 = perm[:n0].to(dev), perm[n0:].to(dev)
    idx0 = torch.randint(0, 2000, (n0,), generator=g).to(dev)
    dst = torch.full((n0 + n1, ldd), float("nan"), device=dev)
    cso.gather_rows2(src0[:, :F], idx0, pos0, n0, src1[:, :F], None, pos1, n1, dst[:, :F])
    torch.cuda.synchronize()
    ref = torch.empty(n0 + n1, F, device=dev)
    ref[pos0] = src0[idx0, :F]
    if n1:
        ref[pos1] = src1[:n1, :F]
    assert torch.equal(dst[:, :F], ref)
