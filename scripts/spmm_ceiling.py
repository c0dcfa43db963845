"""What bounds the aggregation kernel (spmm_unit_kernel) on MI355X: its own access shape over
tables of known size, and a K-split of the layer-0 operand.

The kernel's gather: per wave instruction 4 rows x 256 B (16 lanes x 16 B per row, VW = 4,
G = 16), 4 nonzeros in flight per lane group, 64-column tiles walked one XCD at a time (each
XCD's L2 holds one tile's slice of X: K rows x 256 B). Measured here with HIP events, median of
REPS launches, on operands with the REAL row lengths of a live-sampled Reddit LADIES batch
(BASELINE config 2: layer 0 = 15.8 k rows, 1.8 M nonzeros, F = 602 in 608-float rows):

  real_L0 / real_L1     the batch's own operands (fwd), for reference
  uniform_K<k>          same row lengths, columns uniform over K = k rows: slice per XCD
                        k x 256 B (2.8 / 4.2 / 5.7 / 11.4 MB) — the L2-capacity curve of the
                        exact access shape (slice <= 4 MiB: L2-resident)
  tiny_K512             K = 512 (slice 128 KB): every gather an L2 (mostly L1) hit — the
                        kernel's instruction-issue ceiling
  ksplit<P>_L0          the real layer-0 operand cut into P column blocks (X row ranges of
                        K / P), one launch per block, times summed: what a K-blocked kernel
                        (slice / P per XCD) would cost, minus its partial-sum traffic

Algorithmic bytes = nnz*F*4 + nnz*8 + (M+1)*4 + M*F*4 per launch.
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso, graphs, placement, sampler as smp  # noqa: E402


def timed(op, X, reps, unit=0):
    y = cso.spmm_csr(op, X, unit_nnz=unit)  # warm (and the output for checks)
    cso.take_timing_records()
    cso.enable_timing(True)
    for _ in range(reps):
        cso.spmm_csr(op, X, unit_nnz=unit)
    recs = cso.take_timing_records()
    cso.enable_timing(False)
    ms = float(np.median([r[1] for r in recs]))
    return ms, recs[0][2], recs[0][3], y


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    reps = int(os.environ.get("REPS", "20"))
    dev = torch.device("cuda", 0)
    A, labels, feats, nc, train, *_ = graphs.make_dataset(graphs.REDDIT, seed=0, with_features=False)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(0.1 * N), [0], 3, alpha=0)
    seed = int(np.random.RandomState(4242).randint(2**32 - 1))
    bn = smp.rank_batches(train, 512, 0, 1, 1)[0]
    hb = smp.ladies_sample_host(seed, bn, np.array([8192] * 3), N, lap, labels, [1, 1, 1],
                                pl.device_id_of_nodes_group[0], pl.idx_of_nodes_on_device_group[0], None, 1.0, [0])
    db = hb.to_device(dev, with_coo=False)
    L0, L1 = db.adjs[0], db.adjs[1]
    g = torch.Generator(device=dev).manual_seed(0)
    F, ld = 602, 608

    def xmat(K, width=ld):
        return torch.randn(K, width, device=dev, generator=g)[:, :F]

    # clocks up first: the first hundred-odd launches of a fresh process run slower
    Xw = xmat(L0.shape[1])
    for _ in range(int(os.environ.get("WARM", "100"))):
        cso.spmm_csr(L0, Xw)
    torch.cuda.synchronize()
    # the step's own call shapes: layer-0 forward (F = 602 in 608-float rows), layer-1 forward and
    # backward (F = 1024, the GraphSAGE hidden width); sha = checksum of the output bits (the
    # prefetching and the plain kernel must agree bit for bit)
    for tag, op, width in (("real_L0", L0, None), ("real_L1", L1, None), ("real_L1_F1024", L1, 1024),
                           ("real_L1T_F1024", L1.transpose(), 1024)):
        X = xmat(op.shape[1]) if width is None else torch.randn(op.shape[1], width, device=dev, generator=g)
        ms, nb, kn, y = timed(op, X, reps)
        sha = hashlib.md5(y.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]
        emit(case=tag, M=op.shape[0], K=op.shape[1], nnz=op.nnz, F=int(X.shape[1]), us=round(ms * 1e3, 1),
             alg_GBps=round(nb / (ms * 1e-3) / 1e9, 1), kernel=kn, slice_MB=round(op.shape[1] * 256 / 1e6, 2),
             sha=sha)
    # work-unit size sweep on the step's call shapes (UNITS="256,512,..."): each wave's start-up
    # (two row searches + the first (col, val) chunk) against its 16-64 rounds of gathers
    for unit in [int(v) for v in os.environ.get("UNITS", "").split(",") if v]:
        for tag, op, width in (("real_L0", L0, None), ("real_L1_F1024", L1, 1024),
                               ("real_L1T_F1024", L1.transpose(), 1024)):
            X = xmat(op.shape[1]) if width is None else torch.randn(op.shape[1], width, device=dev, generator=g)
            ms, nb, kn, _ = timed(op, X, reps, unit)
            emit(case=tag, unit=unit, us=round(ms * 1e3, 1), alg_GBps=round(nb / (ms * 1e-3) / 1e9, 1), kernel=kn)
    if os.environ.get("QUICK") == "1":
        return

    # the layer-0 row lengths with uniform random columns over K rows of X
    rowptr = L0.rowptr
    M, nnz = L0.shape[0], L0.nnz
    lens = torch.diff(rowptr)
    rows = torch.repeat_interleave(torch.arange(M, device=dev), lens)
    for K in (512, 11008, 16384, 22176, 44352):
        col = torch.randint(0, K, (nnz,), device=dev, generator=g, dtype=torch.int64)
        # CSR order: columns ascending within each row (as the operand builder emits them)
        key = rows * K + col
        col = (torch.sort(key).values - rows * K).to(torch.int32)
        val = torch.rand(nnz, device=dev, generator=g)
        op = cso.CsrOperand(rowptr, col, val, (M, K))
        X = xmat(K)
        ms, nb, kn, _ = timed(op, X, reps)
        emit(case=("tiny" if K == 512 else "uniform") + f"_K{K}", M=M, K=K, nnz=nnz, us=round(ms * 1e3, 1),
             alg_GBps=round(nb / (ms * 1e-3) / 1e9, 1), kernel=kn, slice_MB=round(K * 256 / 1e6, 2))

    # K-split of the real layer-0 operand: P launches over column blocks
    X0 = xmat(L0.shape[1])
    ref = cso.spmm_csr(L0, X0)
    r0 = torch.repeat_interleave(torch.arange(M, device=dev), torch.diff(L0.rowptr))
    c0 = L0.col.long()
    K0 = L0.shape[1]
    for P in (2, 3, 4):
        bounds = [K0 * p // P for p in range(P + 1)]
        tot_ms, tot_nb, parts = 0.0, 0, []
        ysum = torch.zeros_like(ref)
        for p in range(P):
            lo, hi = bounds[p], bounds[p + 1]
            m = (c0 >= lo) & (c0 < hi)
            cnt = torch.bincount(r0[m], minlength=M)
            rp = torch.zeros(M + 1, dtype=torch.int32, device=dev)
            rp[1:] = torch.cumsum(cnt, 0).to(torch.int32)
            op = cso.CsrOperand(rp, (c0[m] - lo).to(torch.int32), L0.val[m].contiguous(), (M, hi - lo))
            ms, nb, kn, y = timed(op, X0[lo:hi], reps)
            ysum += y
            tot_ms += ms
            tot_nb += nb
            parts.append(round(ms * 1e3, 1))
        full_nb = timed(L0, X0, 1)[1]
        err = float(((ysum - ref).abs().max() / ref.abs().max()).item())
        emit(case=f"ksplit{P}_L0", parts_us=parts, us=round(tot_ms * 1e3, 1),
             alg_GBps_of_unsplit=round(full_nb / (tot_ms * 1e-3) / 1e9, 1), slice_MB=round(K0 / P * 256 / 1e6, 2),
             rel_maxdiff_vs_unsplit=err)


if __name__ == "__main__":
    main()
