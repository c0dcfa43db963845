"""The aggregation kernel alone on a cache-resident operand, for a PMC comparison with the
access-shape microbenchmark (scripts/gather_shape.hip) under rocprofv3 --pmc: rows of 128
nonzeros, columns uniform over K rows (sorted per row, as the operand builder emits them),
X of 602 floats in 608-float rows, the layer-0 instantiation forced (G = 16, one chunk)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import custom_sparse_ops as cso  # noqa: E402


def main():
    K = int(os.environ.get("K", "4096"))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, L = 16384, 128
    col = torch.randint(0, K, (M, L), device=dev, generator=g).sort(dim=1).values.reshape(-1).to(torch.int32)
    rowptr = torch.arange(0, M * L + 1, L, dtype=torch.int32, device=dev)
    op = cso.CsrOperand(rowptr, col, torch.rand(M * L, device=dev, generator=g), (M, K))
    X = torch.randn(K, 608, device=dev, generator=g)[:, :602]
    os.environ["GNN_SPMM_G"], os.environ["GNN_SPMM_NJ"] = "16", "1"
    for _ in range(10):
        cso.spmm_csr(op, X)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
