"""SpMM main-kernel time per call site under kernel-config variants (XCD work map, column
tile width) on one live-sampled Reddit LADIES batch (BASELINE config 2 geometry).

Variants are environment overrides read by the library at every call (GNN_SPMM_XCD,
GNN_SPMM_G / GNN_SPMM_NJ). Reports the median HIP-event time of the main kernel, the
algorithmic GB/s, and whether the output is bitwise equal to the default configuration's.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso, graphs, placement, sampler as smp  # noqa: E402


def main():
    reps = int(os.environ.get("REPS", "20"))
    variants = [v for v in os.environ.get("VARIANTS", "xcd0;xcd1;xcd1,g8;xcd0,g8").split(";") if v]
    A, labels, feats, nc, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0)
    lap = graphs.row_normalize(A)
    lap.sum_duplicates()
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    bn = np.random.RandomState(0).choice(train, 512, replace=False)
    hb = smp.ladies_sample_host(5, bn, np.array([8192] * 3), N, lap, labels, [1, 1, 1],
                                pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
    dev = torch.device("cuda", 0)
    db = hb.to_device(dev, with_coo=False)
    ops = db.adjs
    torch.manual_seed(0)
    sites = []
    x0 = torch.randn(ops[0].shape[1], 608, device=dev)[:, :602]
    sites.append(("fwd_L0", ops[0], x0))
    for li in (1, 2):
        sites.append((f"fwd_L{li}", ops[li], torch.randn(ops[li].shape[1], 1024, device=dev)))
        t = ops[li].transpose()
        sites.append((f"bwd_L{li}", t, torch.randn(t.shape[1], 1024, device=dev)))
    ref = {}
    for var in ["default"] + variants:
        for k in ("GNN_SPMM_XCD", "GNN_SPMM_G", "GNN_SPMM_NJ"):
            os.environ.pop(k, None)
        if var != "default":
            for part in var.split(","):
                if part.startswith("xcd"):
                    os.environ["GNN_SPMM_XCD"] = part[3:]
                elif part.startswith("g"):
                    os.environ["GNN_SPMM_G"] = part[1:]
                elif part.startswith("nj"):
                    os.environ["GNN_SPMM_NJ"] = part[2:]
        for tag, op, X in sites:
            F = X.shape[1]
            y = cso.spmm_csr(op, X)  # warm
            cso.take_timing_records()
            cso.enable_timing(True)
            for _ in range(reps):
                cso.spmm_csr(op, X)
            recs = cso.take_timing_records()
            cso.enable_timing(False)
            ms = float(np.median([r[1] for r in recs]))
            nbytes = recs[0][2]
            if var == "default":
                ref[tag] = y.clone()
            same = bool(torch.equal(y, ref[tag]))
            maxdiff = float((y - ref[tag]).abs().max()) if not same else 0.0
            cfg = cso.spmm_config(op.shape[0], op.nnz, F, ldx=X.stride(0), ldy=y.stride(0), K=op.shape[1])
            print(json.dumps(dict(variant=var, site=tag, M=op.shape[0], K=op.shape[1], nnz=op.nnz, F=F,
                                  us=round(ms * 1e3, 1), alg_GBps=round(nbytes / (ms * 1e-3) / 1e9, 1),
                                  kernel=recs[0][3], default_cfg=cfg, bitwise_equal_default=same,
                                  maxdiff=maxdiff)), flush=True)


if __name__ == "__main__":
    main()
