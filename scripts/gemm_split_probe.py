"""GPU microbench: forced k-splits (GNN_GEMM_SPLITS, read per call) for the forward and
input-gradient GEMM pairs of the 1024-wide GraphSAGE layer (8.7k rows), against the vendor
GEMMs torch picks. Prints one JSON object: µs and TF/s per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd.fused import gemm  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    torch.backends.cuda.preferred_blas_library("cublas")
    res = {}
    for (M, K, N) in ((8680, 1024, 512), (15768, 602, 512)):
        x = torch.randn(M, K + (-K) % 4, device=dev)[:, :K]
        W = torch.randn(N, K + (-K) % 4, device=dev)[:, :K]
        g = torch.randn(M, N, device=dev)
        fl = 4.0 * M * N * K
        res[f"{M}x{K}x{N}/fwd_pair/vendor"] = timeit(lambda: [torch.mm(x, W.t()) for _ in range(2)])
        res[f"{M}x{K}x{N}/dX_pair/vendor"] = timeit(lambda: [torch.mm(g, W) for _ in range(2)])
        for sp in ("1", "2", "3", "4"):
            os.environ["GNN_GEMM_SPLITS"] = sp
            res[f"{M}x{K}x{N}/fwd_pair/s{sp}"] = timeit(lambda: gemm(False, False, [x, x], [W, W], M, N, K))
            res[f"{M}x{K}x{N}/dX_pair/s{sp}"] = timeit(lambda: gemm(False, True, [g, g], [W, W], M, K, N))
        os.environ.pop("GNN_GEMM_SPLITS")
        for k in list(res):
            if k.startswith(f"{M}x") and not isinstance(res[k], list):
                res[k] = [round(res[k], 1), round(fl / res[k] * 1e-6, 1)]
    print(json.dumps(res, indent=0))


if __name__ == "__main__":
    main()
