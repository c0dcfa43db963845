"""Is any block of the real aggregation operands dense enough for the matrix cores?

north_star: "MFMA only where a row-block is dense enough to be a real GEMM tile". The kernel
being replaced is cuda_spmm.cu:163-212 (a gather per nonzero). A block of R rows x C columns of A
can instead run as a dense (R x C) . (C x F) product on MFMA; it pays when its density d (nonzeros
/ (R C)) exceeds the break-even

    d* = (cost of one dense element on MFMA) / (cost of one gathered nonzero)
       = (2 F / MFMA rate) / (4 F / gather rate) = gather rate / (2 MFMA rate)   [bytes/flop]

with the measured rates of THIS chip: the gather kernel moves 16.6 TB/s of algorithmic bytes
(bench r3bb, layer-0 forward), the split3 GEMM reaches 140-158 TF/s fp32-equivalent (DESIGN §3.5b;
417 TF/s peak), the f32-input MFMA kernel ~100 TF/s. So d* = 16.6e12 / (2 * 150e12) = 5.5 %
(split3 at its measured rate), 2.0 % (split3 at peak), 8.3 % (f32 MFMA).

Columns are ordered by descending frequency (the hot columns together), rows either in the
operand's order (sampled node ids ascending, as the kernel sees them) or, as the best case for a
dense tile, sorted by their number of hot-column entries. For tile shapes R x C (MFMA-sized
multiples) the probe reports the share of the operand's nonzeros that lie in tiles at or above
each density threshold, and the time a perfect hybrid would save at the measured rates:
   saved = nnz_in_dense_tiles * t_gather - tiles * R * C * t_dense.
Operands: the Reddit-shaped LADIES batch of BASELINE config 2 (samp 8192, batch 512) as the
bench draws it: layer 0 (F = 602), layer 1 (F = 1024), layer 1 transposed (its backward, F = 1024).

CPU only (numpy). Usage: python scripts/mfma_density_probe.py [--batches 3] [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gnn_amd import graphs, placement, sampler  # noqa: E402

GATHER_TBPS = 16.6       # bench r3bb: dominant kernel, algorithmic bytes / launch time
SPLIT3_TFLOPS = 150.0    # measured split3 layer GEMMs (140-158)
SPLIT3_PEAK = 417.0
F32_MFMA_TFLOPS = 100.0
THRESHOLDS = [0.01, 0.02, 0.055, 0.1, 0.2, 0.5]
TILES = [(32, 32), (32, 64), (64, 64), (128, 64), (128, 128), (256, 256)]


def tile_stats(A: sp.csr_matrix, F: int, row_order: str):
    M, K = A.shape
    freq = np.bincount(A.indices, minlength=K)
    corder = np.argsort(-freq, kind="stable")
    crank = np.empty(K, np.int64)
    crank[corder] = np.arange(K)
    rows = np.repeat(np.arange(M), np.diff(A.indptr))
    cr = crank[A.indices]
    if row_order == "hot_sorted":
        # rows with the most entries among the 1,024 hottest columns first
        hot = np.bincount(rows[cr < 1024], minlength=M)
        rorder = np.argsort(-hot, kind="stable")
        rrank = np.empty(M, np.int64)
        rrank[rorder] = np.arange(M)
        rr = rrank[rows]
    else:
        rr = rows
    nnz = A.nnz
    t_gather = 4.0 * F / (GATHER_TBPS * 1e12)       # s per gathered nonzero
    t_dense = 2.0 * F / (SPLIT3_TFLOPS * 1e12)     # s per dense element
    out = {}
    for R, C in TILES:
        key = (rr // R) * ((K + C - 1) // C) + (cr // C)
        cnt = np.bincount(key)
        cnt = cnt[cnt > 0]
        dens = cnt / float(R * C)
        e = {"tiles_nonempty": int(cnt.size), "max_density": round(float(dens.max()), 4)}
        for th in THRESHOLDS:
            sel = dens >= th
            e[f"nnz_share_at_{th:g}"] = round(float(cnt[sel].sum()) / nnz, 4)
        # best hybrid at the measured split3 rate: every tile that pays goes to MFMA
        pays = cnt * t_gather > R * C * t_dense
        saved = float((cnt[pays] * t_gather - R * C * t_dense).sum())
        e["tiles_that_pay"] = int(pays.sum())
        e["nnz_share_that_pays"] = round(float(cnt[pays].sum()) / nnz, 4)
        e["best_saving_us"] = round(saved * 1e6, 2)
        out[f"{R}x{C}"] = e
    top = freq[corder]
    return {"shape": [int(M), int(K)], "nnz": int(nnz), "F": F,
            "gather_us_at_measured_rate": round(nnz * t_gather * 1e6, 1),
            "hottest_columns_density": [round(float(x) / M, 4) for x in top[:8]],
            "columns_above_breakeven": int((top / M >= 0.055).sum()),
            "nnz_share_in_columns_above_breakeven": round(float(top[top / M >= 0.055].sum()) / nnz, 4),
            "nnz_share_top256_cols": round(float(top[:256].sum()) / nnz, 4),
            "nnz_share_top1024_cols": round(float(top[:1024].sum()) / nnz, 4),
            "tiles": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    t0 = time.time()
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    print(f"graph {time.time() - t0:.1f}s", file=sys.stderr)
    res = {"breakeven_density": {"split3_measured": round(GATHER_TBPS / (2 * SPLIT3_TFLOPS), 4),
                                 "split3_peak": round(GATHER_TBPS / (2 * SPLIT3_PEAK), 4),
                                 "f32_mfma": round(GATHER_TBPS / (2 * F32_MFMA_TFLOPS), 4)},
           "rates": {"gather_TBps": GATHER_TBPS, "split3_TFLOPs": SPLIT3_TFLOPS}, "batches": []}
    chunks = sampler.rank_batches(train, 512, 0, 1, 1)
    seeds = np.random.RandomState(4242)
    for b in range(a.batches):
        hb = sampler.ladies_sample_host(int(seeds.randint(2**32 - 1)), chunks[b], np.array([8192] * 5), N, lap,
                                        labels, [1, 1, 1], pl.device_id_of_nodes_group[0],
                                        pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
        ops = {}
        for li, F in ((0, 602), (1, 1024)):
            L = hb.layers[li]
            op = sp.csr_matrix((np.ones(L.colidx.size, np.float32), L.colidx, L.rowptr), shape=L.shape)
            ops[f"L{li}_fwd"] = (op, F)
        ops["L1_bwd_transpose"] = (ops["L1_fwd"][0].T.tocsr(), 1024)
        ent = {}
        for name, (op, F) in ops.items():
            ent[name] = {ro: tile_stats(op, F, ro) for ro in ("operand_order", "hot_sorted")}
            best = max(v["best_saving_us"] for ro in ent[name].values() for v in ro["tiles"].values())
            print(f"batch {b} {name}: nnz {op.nnz}, cols above break-even {ent[name]['operand_order']['columns_above_breakeven']}"
                  f", best saving {best:.1f} us of {ent[name]['operand_order']['gather_us_at_measured_rate']} us",
                  file=sys.stderr)
        res["batches"].append(ent)
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
