"""Generate the golden fixtures in tests/golden/ from the reference's own Python.

Runs ONLY in the build container (it imports /root/reference, which never reaches the GPU
box). The committed .npz files are data: inputs and the outputs the reference produced.

How the reference is driven:
  * ``custom_sparse_ops`` (which JIT-builds CUDA at import, custom_sparse_ops.py:8) is
    replaced by a stub: spmm = torch.sparse.mm autograd op (the reference's own commented
    CPU path, custom_sparse_ops.py:25,36) and a create_coo_tensor that RECORDS its inputs
    and returns the COO computed by the formula of cuda_spmm.cu:800 in double precision.
  * ``ogb``/``torch_geometric`` (imported at preprocess.py:8-9, unused here) are empty
    stub modules.
  * ``torch.Tensor.to(<int>)`` is a no-op so integer device ids work on a CPU-only host.
What is pinned by executing the reference: LADIES sampling (RNG sequence, sub-graph CSR,
normfact, sampled_nodes, placement masks), create_buffer placement maps, torch.sparse.mm
SpMM outputs, and a GraphSAGE/GCN forward/backward/Adam step with the reference modules.

Usage: python tests/golden/make_golden.py [--subgraph | --spmm-wide]   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from gnn_amd.graphs import TINY, make_dataset  # noqa: E402  (generator only; data stored below)

# ---------------------------------------------------------------- stubs
RECORD = []


def _create_coo_stub(fullrowptr, rowptr, colidx, normfact, nrows, ncols):
    fr = fullrowptr.numpy().astype(np.int64)
    rp = rowptr.numpy().astype(np.int64)
    ci = colidx.numpy()
    nf = normfact.numpy()
    RECORD.append(dict(fullrowptr=fullrowptr.numpy().copy(), rowptr=rowptr.numpy().copy(), colidx=ci.copy(),
                       colidx_dtype=str(ci.dtype), normfact=nf.copy(), shape=(int(nrows), int(ncols))))
    rows = np.repeat(np.arange(nrows, dtype=np.int64), np.diff(rp))
    deg = (fr[1:] - fr[:-1]).astype(np.float64)
    vals = ((1.0 / deg[rows]) * nf[ci.astype(np.int64)].astype(np.float64)).astype(np.float32)
    idx = torch.from_numpy(np.stack([rows, ci.astype(np.int64)]))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(vals), (int(nrows), int(ncols))).coalesce()


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a)
        return torch.sparse.mm(a, b)

    @staticmethod
    def backward(ctx, g):
        (a,) = ctx.saved_tensors
        return None, torch.sparse.mm(a.t().coalesce(), g.contiguous())


def install_stubs():
    cso = types.ModuleType("custom_sparse_ops")
    cso.spmm = _SpMM.apply
    cso.create_coo_tensor = _create_coo_stub
    cso.spmm_forward_time = 0.0
    cso.spmm_backward_time = 0.0
    sys.modules["custom_sparse_ops"] = cso
    for name in ["ogb", "ogb.nodeproppred", "torch_geometric", "torch_geometric.utils"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["ogb.nodeproppred"].PygNodePropPredDataset = None
    sys.modules["torch_geometric.utils"].to_undirected = None
    sys.modules["torch_geometric.utils"].dropout_adj = None
    orig_to = torch.Tensor.to

    def to(self, *a, **k):
        if a and isinstance(a[0], int):
            return self
        return orig_to(self, *a, **k)

    torch.Tensor.to = to
    sys.path.insert(0, REF)


class _FakeFeat:
    def __getitem__(self, i):
        return types.SimpleNamespace(to=lambda d: None)


def main():
    install_stubs()
    import models as ref_models  # noqa: E402
    import preprocess as ref_pre  # noqa: E402
    import sampler as ref_sampler  # noqa: E402
    import utils as ref_utils  # noqa: E402

    A, labels, _, ncls, train, valid, test = make_dataset(TINY, seed=1, with_features=False)
    N = A.shape[0]
    lap = ref_utils.row_normalize(A).tocsr()
    lap_gcn = ref_utils.row_normalize(A + sp.eye(N)).tocsr()
    out = dict(A_indptr=A.indptr.astype(np.int64), A_indices=A.indices.astype(np.int64),
               labels_cls=np.asarray(labels.argmax(axis=1)).ravel().astype(np.int64), num_classes=ncls,
               n_train=len(train), n_valid=len(valid), N=N,
               lap_data=lap.data.astype(np.float32), lap_indptr=lap.indptr.astype(np.int64),
               lap_indices=lap.indices.astype(np.int64))
    np.savez_compressed(os.path.join(HERE, "graph_tiny.npz"), **out)

    # ------------------------------------------------------------ placement (create_buffer)
    k = int(0.1 * N)
    gd = (A, labels, _FakeFeat(), ncls, train, valid, test)
    pl = {}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        os.makedirs("save")
        try:
            for ndev in (1, 2, 4, 8):
                devs = list(range(ndev))
                dev_grp, idx_grp, _bufs, buf_grp, _ = ref_pre.create_buffer(lap, gd, k, devs, "tiny", 3, alpha=0)
                for i in range(ndev):
                    pl[f"n{ndev}_dev{i}"] = np.asarray(dev_grp[i]).astype(np.int64)
                    pl[f"n{ndev}_buf{i}"] = np.asarray(buf_grp[i]).astype(np.int64)
                pl[f"n{ndev}_idx"] = np.asarray(idx_grp[0]).astype(np.int64)
            skew = ref_pre.get_skewed_sampled_nodes(A + sp.eye(N), [pl["n2_buf0"], pl["n2_buf1"]], [1, 1, 1])
            for i, s in enumerate(skew):
                pl[f"skew{i}"] = np.asarray(s).astype(np.int64)
        finally:
            os.chdir(cwd)
    pl["k"] = k
    np.savez_compressed(os.path.join(HERE, "placement_tiny.npz"), **pl)

    # ------------------------------------------------------------ LADIES sampler
    smp = {}
    rng = np.random.default_rng(5)
    cases = [(512, 128, 1234, 1), (512, 128, 7, 2), (64, 16, 99, 1), (64, 16, 2024, 4)]
    for ci, (samp, bs, seed, ndev) in enumerate(cases):
        batch = rng.choice(train, bs, replace=False)
        devs = list(range(ndev))
        dev_of = pl[f"n{ndev}_dev0"]
        idx_on = pl[f"n{ndev}_idx"]
        RECORD.clear()
        res = ref_sampler.ladies_sampler(seed, batch, np.array([samp] * 5), N, lap, labels, [1, 1, 1], dev_of, idx_on,
                                         None, 1.0, 0, devs)
        adjs, masks, cpu_mask, idx_dev, idx_cpu, nin, ylab, sampled = res
        p = f"c{ci}_"
        smp[p + "cfg"] = np.array([samp, bs, seed, ndev])
        smp[p + "batch"] = batch.astype(np.int64)
        for li, rec in enumerate(RECORD):  # top-down order of the create_coo_tensor calls
            for key in ("fullrowptr", "rowptr", "colidx", "normfact"):
                smp[f"{p}call{li}_{key}"] = rec[key]
            smp[f"{p}call{li}_shape"] = np.array(rec["shape"])
        for li, a in enumerate(adjs):
            a = a.coalesce()
            smp[f"{p}adj{li}_indices"] = a.indices().numpy()
            smp[f"{p}adj{li}_values"] = a.values().numpy()
            smp[f"{p}adj{li}_shape"] = np.array(a.shape)
            smp[f"{p}sampled{li}"] = np.asarray(sampled[li]).astype(np.int64)
        for i in range(ndev):
            smp[f"{p}mask{i}"] = np.asarray(masks[i])
            smp[f"{p}idxdev{i}"] = np.asarray(idx_dev[i]).astype(np.int64)
        smp[p + "cpumask"] = np.asarray(cpu_mask)
        smp[p + "idxcpu"] = np.asarray(idx_cpu).astype(np.int64)
        smp[p + "nin"] = nin
        smp[p + "labels"] = ylab.numpy()
    np.savez_compressed(os.path.join(HERE, "ladies_tiny.npz"), **smp)

    # ------------------------------------------------------------ SpMM fwd/bwd (torch.sparse.mm)
    sm = {}
    z = smp
    for li in range(3):
        idx = z[f"c2_adj{li}_indices"]
        val = z[f"c2_adj{li}_values"]
        shape = tuple(z[f"c2_adj{li}_shape"])
        a = torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(val), shape).coalesce()
        for F in (1, 26, 64, 100, 602):
            g = torch.Generator().manual_seed(1000 * li + F)
            X = torch.randn(shape[1], F, generator=g)
            G = torch.randn(shape[0], F, generator=g)
            Xr = X.clone().requires_grad_(True)
            Y = _SpMM.apply(a, Xr)
            Y.backward(G)
            sm[f"l{li}_F{F}_Y"] = Y.detach().numpy()
            sm[f"l{li}_F{F}_dX"] = Xr.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "spmm_tiny.npz"), **sm)

    # ------------------------------------------------------------ model step (reference modules)
    st = {}
    for model_name in ("graphsage", "gcn"):
        torch.manual_seed(0)
        enc_cls = ref_models.GraphSage if model_name == "graphsage" else ref_models.GCN
        enc = enc_cls(nfeat=602, nhid=32, orders=[1, 1, 1], dropout=0.1)
        net = ref_models.GNN(encoder=enc, num_classes=ncls, dropout=0.1, inp=602)
        net.eval()  # dropout off: deterministic across CPU and GPU RNGs
        z = smp
        adjs = []
        for li in range(3):
            adjs.append(torch.sparse_coo_tensor(torch.from_numpy(z[f"c2_adj{li}_indices"]),
                                                torch.from_numpy(z[f"c2_adj{li}_values"]),
                                                tuple(z[f"c2_adj{li}_shape"])).coalesce())
        sampled = [z[f"c2_sampled{li}"] for li in range(3)]
        nin = int(z["c2_nin"])
        g = torch.Generator().manual_seed(77)
        x0 = torch.randn(nin, 602, generator=g)
        y = torch.from_numpy(z["c2_labels"])
        p = model_name + "_"
        for name, prm in net.named_parameters():
            st[p + "init_" + name] = prm.detach().numpy().copy()
        opt = torch.optim.Adam(net.parameters(), lr=0.01)
        opt.zero_grad()
        o = net(x0, adjs, sampled)
        lo = ref_utils.loss(o, y, True, "cpu")
        lo.backward()
        st[p + "out"] = o.detach().numpy()
        st[p + "loss"] = np.array(float(lo))
        for name, prm in net.named_parameters():
            st[p + "grad_" + name] = prm.grad.numpy().copy()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 5)
        opt.step()
        for name, prm in net.named_parameters():
            st[p + "step_" + name] = prm.detach().numpy().copy()
    np.savez_compressed(os.path.join(HERE, "model_step_tiny.npz"), **st)
    print("golden fixtures written to", HERE)


def subgraph_goldens():
    """subgraph_sampler (sampler.py:7-88) outputs -> subgraph_tiny.npz (same tiny graph and
    placement as graph_tiny.npz / placement_tiny.npz)."""
    install_stubs()
    import sampler as ref_sampler  # noqa: E402
    import utils as ref_utils  # noqa: E402

    A, labels, _, ncls, train, valid, test = make_dataset(TINY, seed=1, with_features=False)
    N = A.shape[0]
    lap = ref_utils.row_normalize(A).tocsr()
    pl = np.load(os.path.join(HERE, "placement_tiny.npz"))
    out = {}
    rng = np.random.default_rng(17)
    cases = [(512, 128, 31, 1, [1, 1, 1]), (64, 16, 5, 2, [1, 1, 1]), (256, 64, 8, 4, [0, 1, 1]),
             (128, 32, 77, 1, [1, 0, 1])]
    for ci, (samp, bs, seed, ndev, orders) in enumerate(cases):
        batch = rng.choice(train, bs, replace=False)
        devs = list(range(ndev))
        RECORD.clear()
        res = ref_sampler.subgraph_sampler(seed, batch, np.array([samp] * 5), N, lap, labels, orders,
                                           pl[f"n{ndev}_dev0"], pl[f"n{ndev}_idx"], None, 1.0, 0, devs)
        adjs, masks, cpu_mask, idx_dev, idx_cpu, nin, ylab, sampled = res
        p = f"c{ci}_"
        out[p + "cfg"] = np.array([samp, bs, seed, ndev])
        out[p + "orders"] = np.array(orders)
        out[p + "batch"] = batch.astype(np.int64)
        out[p + "ncalls"] = len(RECORD)
        for li, rec in enumerate(RECORD):  # top-down order of the create_coo_tensor calls
            for key in ("fullrowptr", "rowptr", "colidx", "normfact"):
                out[f"{p}call{li}_{key}"] = rec[key]
            out[f"{p}call{li}_shape"] = np.array(rec["shape"])
        for li, a in enumerate(adjs):
            out[f"{p}present{li}"] = a is not None
            out[f"{p}sampled{li}"] = np.asarray(sampled[li]).astype(np.int64)
            if a is not None:
                a = a.coalesce()
                out[f"{p}adj{li}_indices"] = a.indices().numpy()
                out[f"{p}adj{li}_values"] = a.values().numpy()
        for i in range(ndev):
            out[f"{p}mask{i}"] = np.asarray(masks[i])
            out[f"{p}idxdev{i}"] = np.asarray(idx_dev[i]).astype(np.int64)
        out[p + "cpumask"] = np.asarray(cpu_mask)
        out[p + "idxcpu"] = np.asarray(idx_cpu).astype(np.int64)
        out[p + "nin"] = nin
        out[p + "labels"] = ylab.numpy()
    np.savez_compressed(os.path.join(HERE, "subgraph_tiny.npz"), **out)
    print("subgraph fixtures written to", HERE)


WIDE_CASES = (("c2", (0, 1, 2)), ("c0", (2,)))  # (ladies_tiny case, layers) at the hidden width
WIDE_F = 1024


def spmm_wide_goldens():
    """torch.sparse.mm forward / Aᵀ.coalesce() backward (the reference's CPU path,
    custom_sparse_ops.py:25,36) at F = 1024, the GraphSAGE hidden width the layer-1/2
    aggregations run at, on the reference sampler's sub-graphs already in ladies_tiny.npz
    -> spmm_wide.npz. X and G are regenerated from the seed by the tests (only Y, dX stored)."""
    z = np.load(os.path.join(HERE, "ladies_tiny.npz"))
    out = {}
    for case, layers in WIDE_CASES:
        for li in layers:
            shape = tuple(int(v) for v in z[f"{case}_adj{li}_shape"])
            a = torch.sparse_coo_tensor(torch.from_numpy(z[f"{case}_adj{li}_indices"]),
                                        torch.from_numpy(z[f"{case}_adj{li}_values"]), shape).coalesce()
            g = torch.Generator().manual_seed(7000 + 100 * li + int(case[1:]))
            X = torch.randn(shape[1], WIDE_F, generator=g)
            G = torch.randn(shape[0], WIDE_F, generator=g)
            Xr = X.clone().requires_grad_(True)
            Y = _SpMM.apply(a, Xr)
            Y.backward(G)
            out[f"{case}_l{li}_Y"] = Y.detach().numpy()
            out[f"{case}_l{li}_dX"] = Xr.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "spmm_wide.npz"), **out)
    print("wide SpMM fixtures written to", HERE)


if __name__ == "__main__":
    if "--subgraph" in sys.argv:
        subgraph_goldens()
    elif "--spmm-wide" in sys.argv:
        spmm_wide_goldens()
    else:
        main()
        subgraph_goldens()
        spmm_wide_goldens()
