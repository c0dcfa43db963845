"""GPU measurement: the aggregation of a real operand as (cold entries on the gather kernel) +
(a dense hot block on the matrix cores), against the gather kernel alone.

north_star: "MFMA only where a row-block is dense enough to be a real GEMM tile";
scripts/mfma_density_probe.py finds the candidates (columns by frequency, rows by their count of
hot entries). This probe takes the densest RECTANGLE of that order — the Ch most frequent columns
x the Rh rows with the most entries among them — and times, on the real BASELINE config-2 layer
operands (Reddit-shaped LADIES batch as the bench draws it):
  full     Y = A.X                              spmm_unit_kernel over every nonzero
  hybrid   T = A_hot . X[hot cols]              split3 GEMM (fp32-accurate, bf16 matrix cores),
                                                X rows read in place (row-indexed k-major B)
           Y = A_cold.X + T[rmap]               the gather kernel's residual variant adds T's
                                                rows in its row stores (one launch, no extra pass)
and checks hybrid vs full (rtol/atol 1e-5). The per-batch cost of cutting A into A_cold + A_hot
(and Aᵀ likewise for the backward) is NOT in the hybrid time: a lower bound on the hybrid's cost.

Usage (GPU box): python scripts/mfma_hybrid_probe.py [--out FILE.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gnn_amd import _lib, graphs, placement, sampler  # noqa: E402
from gnn_amd import custom_sparse_ops as cso  # noqa: E402


def timeit(fn, reps=20):
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
    return float(np.median(ts))


def csr_op(dev, A: sp.csr_matrix):
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)
    return cso.CsrOperand(t(A.indptr, np.int32), t(A.indices, np.int32), t(A.data, np.float32), A.shape)


def gemm_indexed(Ah, X, ib, Rh, F, Ch, out):
    """out (Rh x F) = Ah (Rh x Ch, m-major) . X[ib] (Ch x F, k-major rows of X by index)."""
    L = _lib.lib()
    dev = Ah.device
    wsb = L.gnn_gemm_f32_split3_workspace_bytes(Rh, F, Ch, 1)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    one = lambda p: (ctypes.c_void_p * 1)(p)
    _lib.check(L.gnn_gemm_f32_split3_indexed(0, 1, Rh, F, Ch, 1, one(Ah.data_ptr()), Ah.stride(0), None, 0,
                                             one(X.data_ptr()), X.stride(0), one(ib.data_ptr()), X.shape[0],
                                             one(out.data_ptr()), out.stride(0), ws.data_ptr(), wsb,
                                             _lib.stream_of(dev)), "gnn_gemm_f32_split3_indexed")


def probe(dev, A: sp.csr_matrix, F: int, ld: int, shapes, name):
    M, K = A.shape
    g = torch.Generator(device=dev).manual_seed(3)
    Xb = torch.randn(K, ld, device=dev, generator=g)
    X = Xb[:, :F]
    full = csr_op(dev, A)
    t_full = timeit(lambda: cso.spmm_csr(full, X))
    Yref = cso.spmm_csr(full, X)
    freq = np.bincount(A.indices, minlength=K)
    corder = np.argsort(-freq, kind="stable")
    rows = np.repeat(np.arange(M), np.diff(A.indptr))
    res = {"operand": name, "shape": [M, K], "nnz": int(A.nnz), "F": F, "full_us": round(t_full, 1), "cases": []}
    for Ch, Rh in shapes:
        hotc = np.zeros(K, bool)
        hotc[corder[:Ch]] = True
        h = np.bincount(rows[hotc[A.indices]], minlength=M)
        hot_rows = np.sort(np.argsort(-h, kind="stable")[:Rh])
        hotr = np.zeros(M, bool)
        hotr[hot_rows] = True
        inblk = hotr[rows] & hotc[A.indices]
        cold = sp.csr_matrix((A.data[~inblk], A.indices[~inblk], np.concatenate([[0], np.cumsum(
            np.bincount(rows[~inblk], minlength=M))])), shape=(M, K))
        hot_cols = np.sort(corder[:Ch])
        cpos = np.full(K, -1, np.int64)
        cpos[hot_cols] = np.arange(Ch)
        rpos = np.full(M, -1, np.int64)
        rpos[hot_rows] = np.arange(Rh)
        Ah = np.zeros((Rh, Ch), np.float32)
        Ah[rpos[rows[inblk]], cpos[A.indices[inblk]]] = A.data[inblk]
        Ah_d = torch.from_numpy(Ah).to(dev)
        ib = torch.from_numpy(hot_cols.astype(np.int64)).to(dev)
        rmap = torch.from_numpy(rpos.astype(np.int32)).to(dev)
        cold_op = csr_op(dev, cold)
        T = torch.empty(Rh, F, device=dev)
        t_gemm = timeit(lambda: gemm_indexed(Ah_d, X, ib, Rh, F, Ch, T))
        t_cold = timeit(lambda: cso.spmm_csr(cold_op, X))
        t_cold_res = timeit(lambda: cso.spmm_csr(cold_op, X, residual=T, rmap=rmap))

        def hybrid():
            gemm_indexed(Ah_d, X, ib, Rh, F, Ch, T)
            return cso.spmm_csr(cold_op, X, residual=T, rmap=rmap)

        t_h = timeit(hybrid)
        Y = hybrid()
        torch.cuda.synchronize()
        err = (Y - Yref).abs() - 1e-5 * Yref.abs()
        e = {"Ch": Ch, "Rh": Rh, "hot_nnz_share": round(float(inblk.sum()) / A.nnz, 4),
             "block_density": round(float(inblk.sum()) / (Ch * Rh), 4), "gemm_us": round(t_gemm, 1),
             "gemm_TFLOPs": round(2.0 * Rh * Ch * F / (t_gemm * 1e-6) / 1e12, 1),
             "cold_gather_us": round(t_cold, 1), "cold_gather_with_residual_us": round(t_cold_res, 1),
             "hybrid_us": round(t_h, 1), "saving_us": round(t_full - t_h, 1),
             "within_1e-5": bool((err <= 1e-5).all().item()), "max_abs_diff": float((Y - Yref).abs().max().item())}
        print(name, e, file=sys.stderr, flush=True)
        res["cases"].append(e)
    return res


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
    seed = int(np.random.RandomState(4242).randint(2**32 - 1))
    hb = sampler.ladies_sample_host(seed, chunks[0], np.array([8192] * 5), N, lap, labels, [1, 1, 1],
                                    pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
    ops = {}
    for li in (0, 1):
        L = hb.layers[li]
        # create_coo_tensor's values (cuda_spmm.cu:800): (1 / full degree of the row) * normfact[col]
        deg = np.maximum(np.diff(L.fullrowptr), 1).astype(np.float64)  # (rows without entries: unused)
        r = np.repeat(np.arange(L.shape[0]), np.diff(L.rowptr))
        val = ((1.0 / deg)[r] * L.normfact.astype(np.float64)[L.colidx]).astype(np.float32)
        ops[li] = sp.csr_matrix((val, L.colidx, L.rowptr), shape=L.shape)
    shapes = [(512, 1024), (1024, 1024), (1024, 2048), (512, 2048), (2048, 2048), (256, 512)]
    out = [probe(dev, ops[0], 602, 608, shapes, "L0_fwd"),
           probe(dev, ops[1], 1024, 1024, shapes, "L1_fwd"),
           probe(dev, ops[1].T.tocsr(), 1024, 1024, shapes, "L1_bwd_transpose")]
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
