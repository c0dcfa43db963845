"""Kernel launches for the PMC traffic measurement (run under rocprofv3 --pmc by bench.py).

1. Calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for known access widths;
   "calibrate on a known byte count in your own access pattern"): the aggregation kernel
   itself, forced to the benchmark's layer-0 instantiation (GNN_SPMM_G/NJ: 16 lanes x 16-byte
   vectors, one chunk = 4 rows x 256 B per wave instruction, 64-column tiles), on an operand
   whose columns are a permutation of X's rows: every X row is gathered exactly once per
   column tile, and X (2.4 GB) is far larger than the 256 MiB Infinity Cache, so the bytes
   the kernel must fetch are known — X's rows in whole 128-byte lines, plus the (col, val)
   stream once per column tile and the row pointer. Y is written once.
2. The forward aggregations of the benchmark's batch 0, R times each, with the operands laid
   out as bench.py runs them (layer 0: X0 in padded rows, staging.padded_ld — 608 floats for
   602; layers 1-2: 1024 wide), so the kernel instantiations — the names rocprofv3 reports —
   are the benchmark's.
Prints one JSON line with the calibration's known byte counts.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402
from gnn_amd.staging import padded_ld  # noqa: E402


def calibration(dev, F: int, ld: int, K: int = 1 << 20, row_nnz: int = 128):
    """spmm_unit_kernel<4, 16, 1, 4, false> over a permutation operand; returns known bytes."""
    g = torch.Generator(device=dev).manual_seed(0)
    M = K // row_nnz
    perm = torch.randperm(K, device=dev, generator=g).view(M, row_nnz)
    col = torch.sort(perm, dim=1).values.reshape(-1).to(torch.int32).contiguous()
    rowptr = torch.arange(0, K + 1, row_nnz, dtype=torch.int32, device=dev)
    val = torch.rand(K, device=dev, generator=g)
    op = cso.CsrOperand(rowptr, col, val, (M, K))
    X = torch.zeros((K, ld), dtype=torch.float32, device=dev)
    X[:, :F].normal_(generator=g)
    Fk = (F + 3) // 4 * 4
    os.environ["GNN_SPMM_G"], os.environ["GNN_SPMM_NJ"] = "16", "1"  # the layer-0 instantiation
    try:
        cfg = cso.spmm_config(M, K, Fk, ldx=ld, ldy=ld, unit_nnz=0, K=K)
        for _ in range(2):
            cso.spmm_csr(op, X[:, :F])
        torch.cuda.synchronize()
    finally:
        del os.environ["GNN_SPMM_G"], os.environ["GNN_SPMM_NJ"]
    tiles = cfg["tiles"]
    lines_per_row = (Fk * 4 + 127) // 128  # the kernel clamps past-F columns onto the row's last line
    known_read = K * lines_per_row * 128 + tiles * K * 8 + (M + 1) * 4
    known_write = M * Fk * 4
    return {"calib_known_read_bytes": known_read, "calib_known_write_bytes": known_write, "calib_tiles": tiles,
            "calib_K": K, "calib_M": M, "calib_cfg": cfg}


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
    info = calibration(dev, F, ld)
    z = np.load(args.batch)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    layers = []
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
        layers.append({"M": shape[0], "K": shape[1], "nnz": op.nnz, "F": int(X.shape[1]), "ldx": int(X.stride(0))})
    info["layers"] = layers
    print("PMCPROBE " + json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
