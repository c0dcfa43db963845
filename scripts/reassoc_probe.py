"""GPU probe: GraphSAGE layer 1 of BASELINE config 2 computed as (A·H)·Wᵀ (today) or A·(H·Wᵀ)
(reassociated: the aggregation runs on 512 instead of 1024 columns, the neighbour GEMMs on the
15.8 k input rows instead of the 8.7 k sampled rows). Times every product each form launches
(split3 GEMMs, the aggregation forward and its transpose) on config-2 shapes, so the step-level
trade can be read before building it. Usage: python scripts/reassoc_probe.py"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gnn_amd import custom_sparse_ops as cso  # noqa: E402
from gnn_amd.fused import gemm  # noqa: E402
from oracle.fixtures import powerlaw_lens  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 1)


def operand(M, K, nnz_target, rng, dev):
    lens = powerlaw_lens(M, nnz_target / M, 1.3, rng, K)
    rows = np.repeat(np.arange(M, dtype=np.int64), lens)
    w = rng.lognormal(0.0, 1.3, K)
    cols = rng.choice(K, rows.size, p=w / w.sum())
    key = np.unique(rows * K + cols)
    r, c = key // K, (key % K).astype(np.int32)
    rowptr = np.zeros(M + 1, np.int32)
    rowptr[1:] = np.cumsum(np.bincount(r, minlength=M))
    nf = rng.uniform(0.25, 8.0, K).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    op, _ = cso.build_operand(t(rowptr), t(rowptr), t(c), t(nf), M, K, with_coo=False)
    return op


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rng = np.random.default_rng(5)
    M0, M1, F, N = 15809, 8689, 1024, 512
    A1 = operand(M1, M0, 0.86e6, rng, dev)
    A1t = A1.transpose()
    H0 = torch.randn(M0, F, device=dev)
    xs = torch.randn(M1, F, device=dev)
    W = [torch.randn(N, F, device=dev) for _ in range(2)]
    agg = torch.randn(M1, F, device=dev)
    dh = [torch.randn(M1, N, device=dev) for _ in range(2)]
    Z = torch.randn(M0, N, device=dev)
    dZ = torch.randn(M0, N, device=dev)
    G1 = torch.randn(M1, F, device=dev)
    out = {}
    rounds = int(os.environ.get("ROUNDS", "3"))
    for rnd in range(rounds):
        t = {
            # today
            "spmm_fwd_F1024": timeit(lambda: cso.spmm_csr(A1, H0)),
            "spmm_bwd_F1024": timeit(lambda: cso.spmm_csr(A1t, G1)),
            "gemm_fwd_pair_M1": timeit(lambda: gemm(False, False, [xs, agg], W, M1, N, F)),
            "gemm_dx_pair_M1": timeit(lambda: gemm(False, True, dh, W, M1, F, N)),
            "gemm_dw_pair_M1": timeit(lambda: gemm(True, True, dh, [xs, agg], N, F, M1)),
            # reassociated
            "spmm_fwd_F512": timeit(lambda: cso.spmm_csr(A1, Z)),
            "spmm_bwd_F512": timeit(lambda: cso.spmm_csr(A1t, dh[1])),
            "gemm_fwd_M1": timeit(lambda: gemm(False, False, [xs], W[:1], M1, N, F)),
            "gemm_fwd_M0": timeit(lambda: gemm(False, False, [H0], W[1:], M0, N, F)),
            "gemm_dx_M1": timeit(lambda: gemm(False, True, dh[:1], W[:1], M1, F, N)),
            "gemm_dx_M0": timeit(lambda: gemm(False, True, [dZ], W[1:], M0, F, N)),
            "gemm_dw_M1": timeit(lambda: gemm(True, True, dh[:1], [xs], N, F, M1)),
            "gemm_dw_M0": timeit(lambda: gemm(True, True, [dZ], [H0], N, F, M0)),
        }
        for k, v in t.items():
            out.setdefault(k, []).append(v)
    med = {k: sorted(v)[len(v) // 2] for k, v in out.items()}
    today = sum(med[k] for k in ("spmm_fwd_F1024", "spmm_bwd_F1024", "gemm_fwd_pair_M1", "gemm_dx_pair_M1",
                                 "gemm_dw_pair_M1"))
    reassoc = sum(med[k] for k in ("spmm_fwd_F512", "spmm_bwd_F512", "gemm_fwd_M1", "gemm_fwd_M0", "gemm_dx_M1",
                                   "gemm_dx_M0", "gemm_dw_M1", "gemm_dw_M0"))
    print(json.dumps({"median_us": med, "all_us": out, "today_us": round(today, 1), "reassoc_us": round(reassoc, 1),
                      "nnz": int(A1.nnz)}, indent=1))


if __name__ == "__main__":
    main()
