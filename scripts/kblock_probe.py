"""GPU probe: does splitting the aggregation's K (X rows) into blocks make each column-tile
pass L2-resident? Times A·X against A1·X1 + A2·X2 (column halves of the same operand, built
on the host) on a dumped batch (bench.py --dump-batch)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402


def t_call(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    cso.enable_timing(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    recs = cso.take_timing_records()
    cso.enable_timing(False)
    return float(np.median([r[1] for r in recs])) * 1e3


def main():
    z = np.load(sys.argv[1])
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = {}
    for li, F, ld in ((0, 602, 604), (1, 1024, 1024)):
        M, K = (int(v) for v in z[f"l{li}_shape"])
        full, rp, ci, nf = (z[f"l{li}_{k}"] for k in ("fullrowptr", "rowptr", "colidx", "normfact"))
        X = torch.zeros(K, ld, device=dev)
        X[:, :F].normal_()
        Xv = X[:, :F]
        op, _ = cso.build_operand(t(full), t(rp), t(ci), t(nf), M, K, with_coo=False)
        base = t_call(lambda: cso.spmm_csr(op, Xv))
        res = {"base_us": round(base, 1)}
        for P in (2, 3, 4):
            bounds = [K * b // P for b in range(P + 1)]
            tot = 0.0
            for b in range(P):
                keep = (ci >= bounds[b]) & (ci < bounds[b + 1])
                rows = np.repeat(np.arange(M), np.diff(rp))
                rpb = np.zeros(M + 1, np.int32)
                np.add.at(rpb, rows[keep] + 1, 1)
                rpb = np.cumsum(rpb).astype(np.int32)
                opb, _ = cso.build_operand(t(full), t(rpb), t(ci[keep]), t(nf), M, K, with_coo=False)
                tot += t_call(lambda: cso.spmm_csr(opb, Xv))
            res[f"P{P}_sum_us"] = round(tot, 1)
        out[f"layer{li}"] = res
        print(li, res, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
