"""Layer-0 forward aggregation on a dumped LADIES batch (bench.py --dump-batch): back-to-back
launches (the bench's isolated probe condition: X0 and the operand partly cache-resident from the
previous launch) against launches that each follow a write of a 1 GiB scratch buffer (L2 and the
256 MB Infinity Cache flushed of X0) and launches that each follow a split3 GEMM of the layer-0
forward shape (what precedes the aggregation's inputs in the step). Reports the main kernel's
median µs per condition (the dispatch timestamps of the SpMM timing hook)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402
from gnn_amd.fused import gemm  # noqa: E402


def main():
    z = np.load(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    shape = tuple(int(v) for v in z["l0_shape"])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    op, _ = cso.build_operand(t(z["l0_fullrowptr"]), t(z["l0_rowptr"]), t(z["l0_colidx"]), t(z["l0_normfact"]),
                              shape[0], shape[1], with_coo=False)
    X = torch.randn(op.shape[1], 608, device=dev)[:, :602]
    scratch = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
    M = op.shape[0]
    A = [torch.randn(M, 608, device=dev)[:, :602] for _ in range(2)]
    W = [torch.randn(512, 602, device=dev) for _ in range(2)]

    def run(between):
        cso.take_timing_records()
        cso.enable_timing(True)
        for _ in range(reps):
            between()
            cso.spmm_csr(op, X)
        torch.cuda.synchronize()
        recs = cso.take_timing_records()
        cso.enable_timing(False)
        return round(float(np.median([r[1] for r in recs])) * 1e3, 1)

    for _ in range(3):
        cso.spmm_csr(op, X)
    out = {"M": M, "K": op.shape[1], "nnz": op.nnz}
    for rnd in range(2):
        out[f"back_to_back_{rnd}"] = run(lambda: None)
        out[f"after_1GiB_write_{rnd}"] = run(lambda: scratch.fill_(1.0))
        out[f"after_gemm_{rnd}"] = run(lambda: gemm(False, False, A, W, M, 512, 602))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
