"""Kernel launches for the PMC traffic measurement (run under rocprofv3 --pmc by bench.py).

1. Calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for known access widths;
   "calibrate on a known byte count in your own access pattern"): gnn_gather_rows_f32 copies
   every row of a 1.2 GB table (> the 256 MiB Infinity Cache) exactly once, in random order,
   with the SAME row width / vector width as the aggregation kernel being measured, so the
   read bytes are known exactly.
2. The forward aggregations of the benchmark's batch 0, R times each, with the operands laid
   out as bench.py runs them (layer 0: X0 in padded rows, staging.padded_ld — 608 floats for 602; layers 1-2: 1024 wide),
   so the kernel instantiations — the names rocprofv3 reports — are the benchmark's.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402
from gnn_amd.staging import padded_ld  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("batch")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--hidden", type=int, default=1024, help="width of the layer-1/2 inputs ((1+order)*nhid)")
    ap.add_argument("--feat", type=int, default=602)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    F = args.feat
    ld = padded_ld(F)
    # calibration table: rows of ld floats (16-byte vectors, as the aggregation's X0 reads)
    n = int(1.2e9 // (ld * 4))
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.empty((n, ld), dtype=torch.float32, device=dev).normal_(generator=g)
    perm = torch.randperm(n, device=dev, generator=g)
    out = torch.empty((n, ld), dtype=torch.float32, device=dev)
    for _ in range(2):
        cso.gather_rows(table, perm, out, None, n=n)
    torch.cuda.synchronize()
    del table, out, perm
    z = np.load(args.batch)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    for li in range(3):
        shape = tuple(int(v) for v in z[f"l{li}_shape"])
        op, _ = cso.build_operand(t(z[f"l{li}_fullrowptr"]), t(z[f"l{li}_rowptr"]), t(z[f"l{li}_colidx"]),
                                  t(z[f"l{li}_normfact"]), shape[0], shape[1], with_coo=False)
        if li == 0:
            X = torch.zeros((shape[1], ld), device=dev)
            X[:, :F].normal_()
            X = X[:, :F]
        else:
            X = torch.randn(shape[1], args.hidden, device=dev)
        for _ in range(args.reps):
            cso.spmm_csr(op, X)
        torch.cuda.synchronize()
        print(f"layer {li}: M={shape[0]} K={shape[1]} nnz={op.nnz} F={X.shape[1]} ldx={X.stride(0)}", flush=True)
    print(f"calib_rows={n} row_bytes={ld * 4}", flush=True)


if __name__ == "__main__":
    main()
