"""Kernel launches for the PMC traffic measurement (run under rocprofv3 --pmc by bench.py).

1. Calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for known access widths;
   "calibrate on a known byte count in your own access pattern"): gnn_gather_rows_f32 copies
   every row of a 1.2 GB table (> the 256 MiB Infinity Cache) exactly once, in random order,
   with the SAME row width / vector width as the aggregation kernel being measured, so the
   read bytes are known exactly.
2. The layer-0 forward aggregation of the benchmark's batch 0 (the dominant kernel), R times.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("batch")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layer", type=int, default=0)
    ap.add_argument("--feat", type=int, default=602)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    F = args.feat
    # calibration table: rows of F floats, contiguous (same vector width as the SpMM)
    n = int(1.2e9 // (F * 4))
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.empty((n, F), dtype=torch.float32, device=dev).normal_(generator=g)
    perm = torch.randperm(n, device=dev, generator=g)
    out = torch.empty((n, F), dtype=torch.float32, device=dev)
    for _ in range(2):
        cso.gather_rows(table, perm, out, None, n=n)
    torch.cuda.synchronize()
    del table, out, perm
    z = np.load(args.batch)
    li = args.layer
    shape = tuple(int(v) for v in z[f"l{li}_shape"])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    op, _ = cso.build_operand(t(z[f"l{li}_fullrowptr"]), t(z[f"l{li}_rowptr"]), t(z[f"l{li}_colidx"]),
                              t(z[f"l{li}_normfact"]), shape[0], shape[1], with_coo=False)
    X = torch.randn(shape[1], F, device=dev)
    for _ in range(args.reps):
        cso.spmm_csr(op, X)
    torch.cuda.synchronize()
    print(f"calib_rows={n} row_bytes={F * 4} M={shape[0]} K={shape[1]} nnz={op.nnz} F={F}", flush=True)


if __name__ == "__main__":
    main()
