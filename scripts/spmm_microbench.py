"""Per-call-site SpMM kernel timing on a dumped LADIES batch (bench.py --dump-batch).

For every layer (forward A·X, and backward Aᵀ·G for layers 1-2) and a sweep of work-unit
sizes, times the aggregation main kernel with HIP events (on the launch stream) and reports
algorithmic GB/s (SURVEY.md §8d bytes). Used to tune the default unit size and to produce
the per-kernel rows of DESIGN.md.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402


def time_call(op, X, unit, reps):
    """(median main-kernel ms, bytes, median whole-call ms incl. the combine pass)."""
    cso.enable_timing(True)
    tot = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        cso.spmm_csr(op, X, unit_nnz=unit)
        e1.record()
        tot.append((e0, e1))
    torch.cuda.synchronize()
    recs = cso.take_timing_records()
    cso.enable_timing(False)
    ms = np.array([r[1] for r in recs])
    tms =np.array([a.elapsed_time(b) for a, b in tot])
    return float(np.median(ms)), recs[0][2], float(np.median(tms))  # (tag, ms, bytes, kernel)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("batch")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--units", default="0,16,32,64,128,256,512")
    ap.add_argument("--out", default="")
    ap.add_argument("--f0", default="602,600", help="layer-0 widths; F:ld reads an F-wide view of ld-wide rows")
    ap.add_argument("--layers", default="0,1,2")
    args = ap.parse_args()
    z = np.load(args.batch)
    dev = torch.device("cuda", 0)
    res = []
    for li in [int(v) for v in args.layers.split(",")]:
        shape = tuple(int(v) for v in z[f"l{li}_shape"])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        op, _ = cso.build_operand(t(z[f"l{li}_fullrowptr"]), t(z[f"l{li}_rowptr"]), t(z[f"l{li}_colidx"]),
                                  t(z[f"l{li}_normfact"]), shape[0], shape[1], with_coo=False)
        Fs = args.f0.split(",") if li == 0 else ["1024"]
        sites = [("fwd", op)] if li == 0 else [("fwd", op), ("bwd", op.transpose())]
        for tag, o in sites:
            for fs in Fs:
                F, ld = (int(v) for v in fs.split(":")) if ":" in fs else (int(fs), int(fs))
                X = torch.randn(o.shape[1], ld, device=dev)[:, :F]
                for unit in [int(u) for u in args.units.split(",")]:
                    cso.spmm_csr(o, X, unit_nnz=unit)  # warm
                    ms, nbytes, tms = time_call(o, X, unit, args.reps)
                    cfg = cso.spmm_config(o.shape[0], o.nnz, F, unit_nnz=unit, K=o.shape[1])
                    row = dict(layer=li, site=tag, M=o.shape[0], K=o.shape[1], nnz=o.nnz, F=F, unit=cfg["unit_nnz"],
                               units=cfg["units"], vw=cfg["vw"], g=cfg["g"], nj=cfg["nj"], us=round(ms * 1e3, 1),
                               GBps=round(nbytes / (ms * 1e-3) / 1e9, 1), call_us=round(tms * 1e3, 1),
                               call_GBps=round(nbytes / (tms * 1e-3) / 1e9, 1))
                    row["ld"] = ld
                    res.append(row)
                    print(json.dumps(row), flush=True)
        # operand build + transpose costs
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            op2, _ = cso.build_operand(t(z[f"l{li}_fullrowptr"]), t(z[f"l{li}_rowptr"]), t(z[f"l{li}_colidx"]),
                                       t(z[f"l{li}_normfact"]), shape[0], shape[1], with_coo=False)
        e1.record()
        torch.cuda.synchronize()
        build_us = 1e3 * e0.elapsed_time(e1) / args.reps
        e0.record()
        for _ in range(args.reps):
            op._t = None
            op.transpose()
        e1.record()
        torch.cuda.synchronize()
        tr_us = 1e3 * e0.elapsed_time(e1) / args.reps
        row = dict(layer=li, build_operand_us_incl_h2d=round(build_us, 1), transpose_us=round(tr_us, 1))
        res.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
