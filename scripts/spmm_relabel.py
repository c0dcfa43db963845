"""Does relabelling X0's rows by column frequency help the layer-0 aggregation? (VERDICT r2,
next-round item 4: "relabel the batch's input nodes by column frequency, so the hot rows of a tile
sit in one <= 4 MiB block".)

Cases, on the real layer-0 operand of a live-sampled Reddit LADIES batch (BASELINE config 2:
15.8 k rows x 22 k columns, 1.8 M nonzeros, F = 602 in 608-float rows), HIP events, median of
REPS launches of the production kernel (spmm_unit_kernel<4, 16, 1, 4, false>):

  orig        the operand as extracted (columns = positions in the sorted input-node list)
  freq        columns relabelled by descending frequency (hot X rows first, contiguous), rows of
              X permuted to match, each row's columns re-sorted: the same gathers, other addresses
  freq_hc<P>  freq, then cut into a hot block (the columns holding the first half of the
              nonzeros) and a cold block, one launch each, summed: the hot block's slice is small
              enough for every L2

Every case's output is checked against orig (a relabel reorders each row's sum: allclose, not
bitwise). With CASE=<name> only that case runs (REPS launches), for one rocprofv3 --pmc pass.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso, graphs, placement, sampler as smp  # noqa: E402


def timed(op, X, reps):
    y = cso.spmm_csr(op, X)
    cso.take_timing_records()
    cso.enable_timing(True)
    for _ in range(reps):
        cso.spmm_csr(op, X)
    recs = cso.take_timing_records()
    cso.enable_timing(False)
    return float(np.median([r[1] for r in recs])), recs[0][2], recs[0][3], y


def csr_of(rows, col, val, M, K, dev):
    """CSR with columns ascending per row from unordered (row, col, val) triples."""
    order = torch.argsort(rows.long() * K + col.long())
    cnt = torch.bincount(rows.long(), minlength=M)
    rp = torch.zeros(M + 1, dtype=torch.int32, device=dev)
    rp[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    return cso.CsrOperand(rp, col[order].to(torch.int32).contiguous(), val[order].contiguous(), (M, K))


def main():
    reps = int(os.environ.get("REPS", "20"))
    only = os.environ.get("CASE", "")
    dev = torch.device("cuda", 0)
    A, labels, feats, nc, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    seed = int(np.random.RandomState(4242).randint(2**32 - 1))
    bn = smp.rank_batches(train, 512, 0, 1, 1)[0]
    hb = smp.ladies_sample_host(seed, bn, np.array([8192] * 3), N, lap, labels, [1, 1, 1],
                                pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
    L0 = hb.to_device(dev, with_coo=False).adjs[0]
    M, K = L0.shape
    F, ld = 602, 608
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(K, ld, device=dev, generator=g)[:, :F]

    rows = torch.repeat_interleave(torch.arange(M, device=dev), torch.diff(L0.rowptr))
    col = L0.col.long()
    freq = torch.bincount(col, minlength=K)
    order = torch.argsort(-freq, stable=True)          # new label i = old column order[i]
    rank = torch.empty_like(order)
    rank[order] = torch.arange(K, device=dev)           # old column c -> new label rank[c]
    Lf = csr_of(rows, rank[col], L0.val, M, K, dev)
    Xf = torch.empty(K, ld, device=dev)
    Xf[:, :F] = X[order]
    Xf = Xf[:, :F]
    cum = torch.cumsum(freq[order], 0)
    hot = int(torch.searchsorted(cum, cum[-1] // 2).item()) + 1  # columns holding half the nonzeros
    newc = rank[col]
    blocks = []
    for lo, hi in ((0, hot), (hot, K)):
        m = (newc >= lo) & (newc < hi)
        blocks.append((csr_of(rows[m], newc[m] - lo, L0.val[m], M, hi - lo, dev), Xf[lo:hi], lo, hi))

    for _ in range(int(os.environ.get("WARM", "100"))):  # clocks up before any timing
        cso.spmm_csr(L0, X)
    torch.cuda.synchronize()
    ref = cso.spmm_csr(L0, X)

    def emit(**kw):
        print(json.dumps(kw), flush=True)

    def check(y):
        return bool(torch.allclose(y, ref, rtol=1e-5, atol=1e-5)), float((y - ref).abs().max().item())

    top = freq[order]
    common = dict(M=M, K=K, nnz=L0.nnz, F=F)
    if not only or only == "orig":
        ms, nb, kn, _ = timed(L0, X, reps)
        emit(case="orig", us=round(ms * 1e3, 1), alg_GBps=round(nb / (ms * 1e-3) / 1e9, 1), kernel=kn, **common)
    if not only or only == "freq":
        ms, nb, kn, y = timed(Lf, Xf, reps)
        ok, md = check(y)
        emit(case="freq", us=round(ms * 1e3, 1), alg_GBps=round(nb / (ms * 1e-3) / 1e9, 1), kernel=kn,
             allclose_vs_orig=ok, maxabs_vs_orig=md,
             nnz_share_top={str(k): round(float(top[:k].sum() / top.sum()), 3) for k in (256, 1024, 4096, 8192)},
             **common)
    if not only or only == "freq_hc2":
        parts, tot, ysum = [], 0.0, torch.zeros_like(ref)
        for op, Xb, lo, hi in blocks:
            ms, nb, kn, y = timed(op, Xb, reps)
            ysum += y
            tot += ms
            parts.append({"cols": hi - lo, "nnz": op.nnz, "us": round(ms * 1e3, 1),
                          "slice_MB": round((hi - lo) * 256 / 1e6, 2)})
        ok, md = check(ysum)
        emit(case="freq_hc2", us=round(tot * 1e3, 1), parts=parts, allclose_vs_orig=ok, maxabs_vs_orig=md, **common)


if __name__ == "__main__":
    main()
