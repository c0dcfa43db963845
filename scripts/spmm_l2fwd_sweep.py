"""GPU: the layer-2 forward aggregation (512 x 8.7 k, ~15 k nonzeros, F = 1024, rows up to ~480
nonzeros) over the unit kernel's lane-group widths G (GNN_SPMM_G) and unit sizes S (unit_nnz), and
the row kernel's waves per row — whole calls (main kernel + combine) timed with HIP events, median
of 50, on a BASELINE config-2 batch. Run under rocprofv3 --kernel-trace --stats for the per-kernel
split. Usage: python scripts/spmm_l2fwd_sweep.py [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    chunks = sampler.rank_batches(train, 512, 0, 1, 1)
    rs = np.random.RandomState(4242)
    hb = sampler.ladies_sample_host(int(rs.randint(2**32 - 1)), chunks[0], np.array([8192] * 5), N, lap, labels,
                                    [1, 1, 1], pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0],
                                    None, 1.0, [0])
    db = hb.to_device(dev, with_coo=False)
    op = db.adjs[2]
    M, K = op.shape
    X = torch.randn(K, 1024, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    ref = cso.spmm_csr(op, X)
    res = {"shape": [M, K], "nnz": op.nnz, "cases": []}
    for g in ("64", "32", "16"):
        for s in (0, 16, 32, 64, 128):
            os.environ["GNN_SPMM_G"], os.environ["GNN_SPMM_NJ"] = g, "1"
            fn = lambda: cso.spmm_csr(op, X, unit_nnz=s)
            y = fn()
            torch.cuda.synchronize()
            e = {"kernel": "unit", "G": int(g), "S": s or cso.spmm_config(M, op.nnz, 1024, K=K)["unit_nnz"],
                 "us": timeit(fn), "close": bool(torch.allclose(y, ref, rtol=1e-5, atol=1e-5))}
            print(e, file=sys.stderr, flush=True)
            res["cases"].append(e)
    os.environ.pop("GNN_SPMM_G")
    os.environ.pop("GNN_SPMM_NJ")
    os.environ["GNN_SPMM_ROWK"] = "1"
    for w in ("4", "8"):
        os.environ["GNN_SPMM_ROWK_WPR"] = w
        fn = lambda: cso.spmm_csr(op, X)
        y = fn()
        torch.cuda.synchronize()
        e = {"kernel": "row", "WPR": int(w), "us": timeit(fn), "close": bool(torch.allclose(y, ref, rtol=1e-5, atol=1e-5))}
        print(e, file=sys.stderr, flush=True)
        res["cases"].append(e)
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
