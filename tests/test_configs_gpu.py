"""GPU parity at the per-batch geometry of BASELINE configs 3, 4 and 5.

* config 3 — ogbn-products-shaped GraphSAGE / LADIES (F = 100 input, hidden 2·512 = 1024);
* config 4 — ogbn-papers100M-shaped GraphSAGE / LADIES (F = 128, 172 classes);
* config 5 — ogbn-products-shaped GCN / FastGCN (F = 100 → 512; lap = row_normalize(A + I),
  main.py:267-270).
Each builds a synthetic graph with the config's expected degree and feature / class widths on
500 k nodes (graphs.PRODUCTS_TEST / PAPERS_TEST) and samples ONE batch (samp 8192, batch 512)
with the product's native sampler — the layer shapes of a full-size batch. Checked:
  * the native sampler equals its numpy restatement on this batch (LADIES: the restatement
    is pinned to the reference by tests/golden; FastGCN is absent from the reference, so its
    sampler is "parity unpinned" — only the aggregation and model on its operands are checked);
  * every operand (create_coo_tensor values, columns) and every transposed operand (from the
    sampler's CSC) bit-exact against the C oracle;
  * every aggregation call of a training step — 3 forwards, 2 backwards (GraphSAGE: with the
    fused x[sampled] residual) — against the oracle, allclose(rtol=1e-5, atol=1e-5);
  * one whole training step (fused HIP encoder + head on the GPU, eval mode) against the
    reference's CPU path on the same inputs (torch.sparse.mm + the same modules): logits and
    loss rtol 1e-4, every parameter gradient within 1e-4 of the reference in relative L2 norm
    (a norm-wise bound: elementwise rtol is meaningless for gradient entries near zero).
"""
import numpy as np
import pytest
import torch

import oracle as O
from gnn_amd import custom_sparse_ops as cso
from gnn_amd import graphs, sampler, staging
from gnn_amd.models import build_model

pytestmark = pytest.mark.gpu
RTOL = 1e-5
ATOL = 1e-5

CONFIGS = {
    "c3_products_graphsage_ladies": (graphs.PRODUCTS_TEST, "graphsage", "ladies"),
    "c4_papers_graphsage_ladies": (graphs.PAPERS_TEST, "graphsage", "ladies"),
    "c5_products_gcn_fastgcn": (graphs.PRODUCTS_TEST, "gcn", "fastgcn"),
}
_cache = {}


def _setup(name):
    if name in _cache:
        return _cache[name]
    spec, model, kind = CONFIGS[name]
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(spec, seed=3)
    lap = graphs.lap_matrix(A, model)
    N = A.shape[0]
    dev_of = np.full(N, -1, np.int64)  # one GPU, no buffer: every row from the host table
    idx_on = np.zeros(N, np.int64)
    fn = {"ladies": sampler.ladies_sample_host, "fastgcn": sampler.fastgcn_sample_host}[kind]
    batch = sampler.rank_batches(train, 512, 0, 1, 5)[0]
    samp = np.array([8192] * 5)
    hb = fn(77, batch, samp, N, lap, labels, [1, 1, 1], dev_of, idx_on, None, 1.0, [0])
    hb_np = fn(77, batch, samp, N, lap, labels, [1, 1, 1], dev_of, idx_on, None, 1.0, [0], native=False)
    _cache.clear()  # one graph alive at a time
    _cache[name] = (spec, model, kind, feats, ncls, hb, hb_np)
    return _cache[name]


@pytest.mark.parametrize("name", list(CONFIGS))
def test_sampler_native_equals_restatement(name):
    spec, model, kind, feats, ncls, hb, hb_np = _setup(name)
    assert hb.nnz() > 100_000  # a full-size batch, not a toy
    for L, Ln in zip(hb.layers, hb_np.layers):
        assert L.shape == Ln.shape
        for k in ("fullrowptr", "rowptr", "colidx", "normfact"):
            assert np.array_equal(getattr(L, k), getattr(Ln, k)), k
    for a, b in zip(hb.sampled_nodes, hb_np.sampled_nodes):
        assert np.array_equal(a, b)
    assert np.array_equal(hb.input_nodes, hb_np.input_nodes)


def _x0(feats, hb, dev):
    """X0 as staging lays it out: padded 128-byte rows, the (n x F) view."""
    F = feats.shape[1]
    ld = staging.padded_ld(F)
    x = torch.zeros((hb.num_input_nodes, ld), dtype=torch.float32)
    x[:, :F] = feats[torch.from_numpy(np.asarray(hb.input_nodes, np.int64))]
    return x.to(dev)[:, :F], x[:, :F].numpy().copy()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_operands_and_aggregations(dev, name):
    spec, model, kind, feats, ncls, hb, _ = _setup(name)
    db = hb.to_device(dev, with_coo=False)
    H = 1024 if model == "graphsage" else 512  # width of the layer-1/2 inputs
    rng = np.random.default_rng(11)
    x0_d, x0_h = _x0(feats, hb, dev)
    for li, (L, op) in enumerate(zip(hb.layers, db.adjs)):
        M, K = L.shape
        ocol, oval = O.build_operand(L.fullrowptr, L.rowptr, L.colidx, L.normfact)
        assert np.array_equal(op.col.cpu().numpy(), ocol), f"layer {li} columns"
        assert np.array_equal(op.val.cpu().numpy(), oval), f"layer {li} values (bit-exact)"
        # forward
        if li == 0:
            Xd, Xh = x0_d, x0_h
        else:
            Xh = rng.standard_normal((K, H)).astype(np.float32)
            Xd = torch.from_numpy(Xh).to(dev)
        Y = cso.spmm_csr(op, Xd)
        np.testing.assert_allclose(Y.cpu().numpy(), O.spmm_f32(L.rowptr, ocol, oval, Xh), rtol=RTOL, atol=ATOL,
                                   err_msg=f"layer {li} forward")
        if li == 0:
            continue  # layer 0's input (the features) needs no gradient
        # backward: the transposed operand from the sampler's CSC, bit-exact canonical transpose
        trp, trc, trv = O.csr_transpose(L.rowptr, ocol, oval, K)
        t = op.transpose()
        assert np.array_equal(t.rowptr.cpu().numpy(), trp) and np.array_equal(t.col.cpu().numpy(), trc)
        assert np.array_equal(t.val.cpu().numpy(), trv), f"layer {li} transposed values"
        Gh = rng.standard_normal((M, H if li < 2 else H)).astype(np.float32)
        ref = O.spmm_f32(trp, trc, trv, Gh)
        if model == "graphsage":  # d(x) = Aᵀ·G + scatter(d(x[sampled])): the fused residual
            sn = np.asarray(hb.sampled_nodes[li], np.int64)
            Rh = rng.standard_normal((len(sn), H)).astype(np.float32)
            rmap = np.full(K, -1, np.int32)
            rmap[sn] = np.arange(len(sn), dtype=np.int32)
            got = cso.spmm_csr(t, torch.from_numpy(Gh).to(dev), residual=torch.from_numpy(Rh).to(dev),
                               rmap=torch.from_numpy(rmap).to(dev))
            ref[sn] += Rh
        else:
            got = cso.spmm_csr(t, torch.from_numpy(Gh).to(dev))
        np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=RTOL, atol=ATOL, err_msg=f"layer {li} backward")


@pytest.mark.parametrize("name", list(CONFIGS))
def test_training_step_matches_cpu_reference(dev, name):
    from oracle.cpu_reference import cpu_inputs, torch_spmm

    spec, model, kind, feats, ncls, hb, _ = _setup(name)
    adjs_c, x0_c, sampled_c, y_c = cpu_inputs(hb, feats)
    torch.manual_seed(0)
    ref = build_model(model, feats.shape[1], 512, [1, 1, 1], ncls, 0.1, spmm_fn=torch_spmm)
    torch.manual_seed(0)
    net = build_model(model, feats.shape[1], 512, [1, 1, 1], ncls, 0.1, fused=True).to(dev)
    ref.eval()
    net.eval()
    from gnn_amd.models import loss as loss_fn

    out_r = ref(x0_c, adjs_c, sampled_c)
    lo_r = loss_fn(out_r, y_c, True, "cpu")
    lo_r.backward()
    db = hb.to_device(dev, with_coo=False)
    x0_d, _ = _x0(feats, hb, dev)
    lo, out = net.forward_loss(x0_d, db.adjs, db.sampled_nodes, db.labels, True)
    lo.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_r.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(lo.detach()), float(lo_r.detach()), rtol=1e-4)
    for (pn, p), (_, pr) in zip(net.named_parameters(), ref.named_parameters()):
        g, gr = p.grad.detach().cpu().double(), pr.grad.detach().double()
        rel = float((g - gr).norm() / max(float(gr.norm()), 1e-30))
        assert rel < 1e-4, f"{name} {pn}: relative gradient error {rel:.2e}"


def test_operand_build_and_aggregation_graph_capture(dev):
    """The ABI's graph-capturable promise: create_coo_tensor's builder (with its unsorted-row
    check, whose flag lives in the caller's workspace) and the aggregation captured in one
    HIP graph replay to the eager results, bit for bit."""
    from oracle.fixtures import random_csr

    rng = np.random.default_rng(3)
    M, K, F = 700, 900, 256
    lens = rng.integers(0, 300, M)
    full, rowptr, col, nf = random_csr(M, K, lens, rng)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ins = (t(full), t(rowptr), t(col), t(nf))
    X = torch.randn(K, F, device=dev)
    op_e, _ = cso.build_operand(*ins, M, K, with_coo=False)
    Y_e = cso.spmm_csr(op_e, X)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        cso.build_operand(*ins, M, K, with_coo=False)  # warm the allocator pools outside capture
        with torch.cuda.graph(g, stream=s):
            op_g, _ = cso.build_operand(*ins, M, K, with_coo=False)
            Y_g = cso.spmm_csr(op_g, X)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(op_g.val, op_e.val) and torch.equal(op_g.col, op_e.col)
    assert torch.equal(Y_g, Y_e)
