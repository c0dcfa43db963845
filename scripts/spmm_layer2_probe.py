"""GPU: the layer-2 aggregations of a BASELINE config-2 batch (Reddit-shaped LADIES, samp 8192,
batch 512): the unit kernel + its combine (GNN_SPMM_ROWK=0) against spmm_row_kernel with 1 / 2 /
4 / 8 waves per row. Whole calls timed with HIP events (main kernel + combine), median of 50.
  fwd_L2: Y = A2 . X2        (512 x 8.7 k, ~15 k nonzeros, F = 1024)
  bwd_L2: dX2 = A2ᵀ . G + R[rmap]   (8.7 k x 512, residual rows of x[sampled])
Usage: python scripts/spmm_layer2_probe.py [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gnn_amd import graphs, placement, sampler  # noqa: E402
from gnn_amd import custom_sparse_ops as cso  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return round(float(np.median(ts)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--batches", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    chunks = sampler.rank_batches(train, 512, 0, 1, 1)
    rs = np.random.RandomState(4242)
    out = []
    for b in range(a.batches):
        hb = sampler.ladies_sample_host(int(rs.randint(2**32 - 1)), chunks[b], np.array([8192] * 5), N, lap, labels,
                                        [1, 1, 1], pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0],
                                        None, 1.0, [0])
        db = hb.to_device(dev, with_coo=False)
        op = db.adjs[2]
        opt = op.transpose()
        M, K = op.shape
        g = torch.Generator(device=dev).manual_seed(b)
        X = torch.randn(K, 1024, device=dev, generator=g)
        G = torch.randn(M, 1024, device=dev, generator=g)
        sn = db.sampled_nodes[2]
        rmap = sn._gnn_rmap
        R = torch.randn(sn.numel(), 1024, device=dev, generator=g)
        calls = {"fwd_L2": lambda: cso.spmm_csr(op, X), "bwd_L2": lambda: cso.spmm_csr(opt, G, residual=R, rmap=rmap)}
        ent = {"shape": [M, K], "nnz": op.nnz}
        for name, fn in calls.items():
            r = {}
            os.environ["GNN_SPMM_ROWK"] = "0"
            ref = fn()
            r["unit+combine"] = timeit(fn)
            os.environ.pop("GNN_SPMM_ROWK")
            for w in ("1", "2", "4", "8"):
                os.environ["GNN_SPMM_ROWK_WPR"] = w
                y = fn()
                torch.cuda.synchronize()
                ok = bool(torch.allclose(y, ref, rtol=1e-5, atol=1e-5))
                r[f"row_wpr{w}"] = timeit(fn)
                r[f"row_wpr{w}_close"] = ok
            os.environ.pop("GNN_SPMM_ROWK_WPR")
            r["default_kernel"] = cso.spmm_config(*(op.shape[:1] if name == "fwd_L2" else opt.shape[:1]), op.nnz, 1024,
                                                  K=(K if name == "fwd_L2" else M))["kernel"]
            r["default_us"] = timeit(fn)
            ent[name] = r
            print(b, name, r, file=sys.stderr, flush=True)
        out.append(ent)
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
