"""Standalone cost of the GPU layer extraction (gnn_ladies_extract_f32) on live-sampled Reddit
LADIES batches (samp 8192, batch 512), against the host-extraction path's operand builds
(gnn_build_operand_sorted_f32 + gnn_build_operand_t_f32) on the same batch — each timed alone
on an idle GPU with HIP events, median of REPS."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso, graphs, placement, sampler as smp  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ts])) * 1e3


VARIANTS = [v for v in os.environ.get("VARIANTS", "").split(";") if v]  # e.g. "GNN_LX_XW=16384"


def _totals(L, tr):
    """The host-known segment totals (as the training path passes them: no device read-back)."""
    return dict(rowseg_total=int(L.fullrowptr[-1]), colseg_total=int(L.colseg[-1]) if tr else None)


def main():
    reps = int(os.environ.get("REPS", "20"))
    A, labels, feats, nc, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0)
    lap = graphs.row_normalize(A)
    lap.sum_duplicates()
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    dev = torch.device("cuda", 0)
    g = smp.native_graph(lap)
    dg = smp.device_graph(g, dev)
    bn = np.random.RandomState(0).choice(train, 512, replace=False)
    args = (5, bn, np.array([8192] * 3), N, g, labels, [1, 1, 1], pl.device_id_of_nodes_group[0],
            pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
    hd = smp.ladies_sample_host(*args, device_extract=True)
    hb = smp.ladies_sample_host(*args)
    dd = hd.to_device(dev, build=False)
    db = hb.to_device(dev, build=False)
    torch.cuda.synchronize()
    for var in VARIANTS:
        for kv in var.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
        for li in (0, 1):
            fr, rp, ci, nf, shape, cp, cr, rows, cols, nnz, cs = dd.raw[li]
            L = hd.layers[li]
            us = timed(lambda: cso.extract_operand(dg, rows, cols, nf, nnz, fr, **_totals(L, False)), reps)
            ust = timed(lambda: cso.extract_operand(dg, rows, cols, nf, nnz, fr, cs, cp, **_totals(L, True)), reps)
            print(json.dumps({"variant": var, "layer": li, "extract_us": round(us, 1), "with_t_us": round(ust, 1)}),
                  flush=True)
        for kv in var.split(","):
            os.environ.pop(kv.split("=")[0], None)
        torch.cuda.synchronize()
        dg.err.zero_()  # GNN_LX_FLAGS variants produce wrong counts by design
    for li in range(3):
        r = dd.raw[li]
        L = hd.layers[li]
        row = {"layer": li, "M": L.shape[0], "K": L.shape[1], "nnz": L.nnz, "on_device": L.on_device}
        if L.on_device:
            fr, rp, ci, nf, shape, cp, cr, rows, cols, nnz, cs = r
            row["U_entries"] = int((dg.indptr[rows.long() + 1] - dg.indptr[rows.long()]).sum())
            row["T_entries"] = int(L.colseg[-1])
            row["extract_us"] = round(timed(lambda: cso.extract_operand(dg, rows, cols, nf, nnz, fr,
                                                                        **_totals(L, False)), reps), 1)
            row["extract_with_t_us"] = round(
                timed(lambda: cso.extract_operand(dg, rows, cols, nf, nnz, fr, cs, cp, **_totals(L, True)), reps), 1)
        fr, rp, ci, nf, shape, cp, cr = db.raw[li][:7]

        def build():
            op, _ = cso.build_operand(fr, rp, ci, nf, shape[0], shape[1], with_coo=False, sorted_rows=True)
            if cp is not None:
                cso.attach_transpose(op, fr, cp, cr, nf)
        row["host_path_build_us"] = round(timed(build, reps), 1)
        print(json.dumps(row), flush=True)
    dg.check()


if __name__ == "__main__":
    main()
