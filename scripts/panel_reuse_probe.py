"""Could the dominant aggregation reuse X rows below L2 (in LDS)?

VERDICT r4 item 3: the layer-0/1 aggregations (spmm_unit_kernel) serve 86 % of their
gathered bytes from L2 and run at 0.87 of their L2 access-shape ceiling; the only lever left on the
kernel would be to gather each X slice once per panel of R consecutive rows into LDS and read the
recurring ones from there (ds_read_b128) instead of L2. The reference stages only (col, val) in
shared memory, never X (cuda_spmm.cu:163-212).

For each real config-2 operand (Reddit-shaped LADIES batch, samp 8192, batch 512, as the bench draws
it: layer 0 forward F = 602, layer 1 forward F = 1024, layer 1 backward = the transpose) and panel
heights R = 8 ... 512 this reports, per panel of R rows (in the operand's own row order, which the
kernel walks):
  * recur_share — the share of nonzeros whose column occurs at least twice in the panel;
  * saved_share — (nonzeros - distinct columns) / nonzeros: the X-slice loads an LDS panel cache
    would save (each distinct column loaded once, every repeat served from LDS);
  * recurring_cols — distinct columns occurring >= 2 times per panel (mean / p95), and the LDS one
    64-float column tile of them takes (256 B each) against the 160 KB of a CU;
and the same for the rows sorted by their hot-column content (an upper bound a row reorder could
reach). The bar VERDICT set: saved_share >= 30 % at an R whose recurring slices fit LDS.

CPU only (numpy). Usage: python scripts/panel_reuse_probe.py [--batches 2] [--out FILE.json]
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

PANELS = [8, 16, 32, 64, 128, 256, 512]
TILE_BYTES = 64 * 4  # one 64-float column tile of an X row (the kernel's G = 16 lanes x 16 B)
LDS_BYTES = 160 * 1024


def panel_stats(A: sp.csr_matrix, R: int) -> dict:
    M, K = A.shape
    rows = np.repeat(np.arange(M, dtype=np.int64), np.diff(A.indptr))
    key = (rows // R) * K + A.indices.astype(np.int64)
    uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    nnz = A.nnz
    recur = cnt[inv] >= 2
    npanel = (M + R - 1) // R
    pan = uk // K
    rc = np.bincount(pan[cnt >= 2], minlength=npanel)
    dc = np.bincount(pan, minlength=npanel)
    return {"R": R, "recur_share": round(float(recur.mean()), 4),
            "saved_share": round(float((nnz - len(uk)) / nnz), 4),
            "distinct_cols_mean": round(float(dc.mean()), 1),
            "recurring_cols_mean": round(float(rc.mean()), 1), "recurring_cols_p95": int(np.percentile(rc, 95)),
            "lds_KB_recurring_p95": round(float(np.percentile(rc, 95)) * TILE_BYTES / 1024, 1),
            "fits_lds": bool(np.percentile(rc, 95) * TILE_BYTES <= LDS_BYTES)}


def hot_sorted(A: sp.csr_matrix) -> sp.csr_matrix:
    freq = np.bincount(A.indices, minlength=A.shape[1])
    hot = np.argsort(-freq, kind="stable")[:1024]
    ish = np.zeros(A.shape[1], bool)
    ish[hot] = True
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    score = np.bincount(rows[ish[A.indices]], minlength=A.shape[0])
    return A[np.argsort(-score, kind="stable")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    t0 = time.time()
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    print(f"graph {time.time() - t0:.1f}s", file=sys.stderr)
    chunks = sampler.rank_batches(train, 512, 0, 1, 1)
    seeds = np.random.RandomState(4242)
    res = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "lds_bytes": LDS_BYTES, "tile_bytes": TILE_BYTES,
           "batches": []}
    for b in range(a.batches):
        hb = sampler.ladies_sample_host(int(seeds.randint(2**32 - 1)), chunks[b], np.array([8192] * 5), N, lap,
                                        labels, [1, 1, 1], pl.device_id_of_nodes_group[0],
                                        pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
        ops = {}
        for li in (0, 1):
            L = hb.layers[li]
            ops[f"L{li}_fwd"] = sp.csr_matrix((np.ones(L.colidx.size, np.float32), L.colidx, L.rowptr), shape=L.shape)
        ops["L1_bwd_transpose"] = ops["L1_fwd"].T.tocsr()
        ent = {}
        for name, op in ops.items():
            op.sort_indices()
            ent[name] = {"shape": list(op.shape), "nnz": int(op.nnz),
                         "operand_order": [panel_stats(op, R) for R in PANELS],
                         "hot_sorted_rows": [panel_stats(hot_sorted(op), R) for R in PANELS]}
            best = max((s for s in ent[name]["operand_order"] if s["fits_lds"]), key=lambda s: s["saved_share"])
            print(f"batch {b} {name}: best fitting R={best['R']} saved {best['saved_share']:.3f} "
                  f"(recur {best['recur_share']:.3f}, {best['lds_KB_recurring_p95']} KB p95)", file=sys.stderr)
        res["batches"].append(ent)
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
