"""GPU microbench: gnn_gemm_f32 split-k / stage-depth sweep for the layer shapes (env knobs
GNN_GEMM_SPLITS / GNN_GEMM_BKT are read per call)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd.fused import gemm  # noqa: E402


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
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for (M, K, N) in ((15768, 602, 512), (8680, 1024, 512)):
        x = torch.randn(M, K + (K & 1), device=dev)[:, :K]
        W = torch.randn(N, K + (K & 1), device=dev)[:, :K]
        g = torch.randn(M, N, device=dev)
        fl = 2.0 * M * N * K
        for bkt in ("16", "32"):
            os.environ["GNN_GEMM_BKT"] = bkt
            os.environ.pop("GNN_GEMM_SPLITS", None)
            for name, fn, f in (("fwd", lambda: gemm(False, False, [x], [W], M, N, K), fl),
                                ("fwd_pair", lambda: gemm(False, False, [x, x], [W, W], M, N, K), 2 * fl),
                                ("dX_pair", lambda: gemm(False, True, [g, g], [W, W], M, K, N), 2 * fl)):
                us = timeit(fn)
                res[f"{M}x{K}x{N}/{name}/bkt{bkt}"] = [round(us, 1), round(f / us * 1e-6, 1)]
            for sp in (1, 2, 4, 6, 8, 10, 12, 13, 16, 24):
                os.environ["GNN_GEMM_SPLITS"] = str(sp)
                us = timeit(lambda: gemm(True, True, [g, g], [x, x], N, K, M))
                res[f"{M}x{K}x{N}/dW_pair/bkt{bkt}/s{sp}"] = [round(us, 1), round(2 * fl / us * 1e-6, 1)]
            print(bkt, M, file=sys.stderr, flush=True)
    print(json.dumps(res, indent=0))


if __name__ == "__main__":
    main()
