"""GPU microbench: fp32 GEMM layouts for the GraphSAGE layer shapes (Reddit config 2).

Compares F.linear(x, W) (x @ Wᵀ, "NT") against x @ Wt with a pre-transposed weight ("NN"),
padded K, and rocBLAS vs hipBLASLt. Prints one JSON object.
"""
import json
import sys

import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd.fused import gemm  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = {}
    for lib in ("cublas", "cublaslt"):
        torch.backends.cuda.preferred_blas_library(lib)
        for (M, K, N) in ((15768, 602, 512), (8680, 1024, 512)):
            flops = 2.0 * M * K * N
            x = torch.randn(M, K, device=dev)
            W = torch.randn(N, K, device=dev)
            Wt = W.t().contiguous()
            g = torch.randn(M, N, device=dev)
            Kp = (K + 7) // 8 * 8
            xp = torch.zeros(M, Kp, device=dev)
            xp[:, :K] = x
            Wp = torch.zeros(N, Kp, device=dev)
            Wp[:, :K] = W
            Wpt = Wp.t().contiguous()
            cases = {
                "fwd_NT": lambda: F.linear(x, W),
                "fwd_NN": lambda: torch.mm(x, Wt),
                "fwd_NN_tr": lambda: torch.mm(x, W.t().contiguous()),
                "fwd_NT_padK": lambda: F.linear(xp, Wp),
                "fwd_NN_padK": lambda: torch.mm(xp, Wpt),
                "bwd_dX": lambda: torch.mm(g, W),
                "bwd_dW": lambda: torch.mm(g.t(), x),
                "bwd_dW_padK": lambda: torch.mm(g.t(), xp),
                "bwd_dWt": lambda: torch.mm(x.t(), g),
            }
            if lib == "cublas":  # the hand-written MFMA kernel (library-independent)
                xp4 = torch.zeros(M, (K + 3) // 4 * 4, device=dev)
                xp4[:, :K] = x
                xv = xp4[:, :K]
                cases.update({
                    "gnn_fwd": lambda: gemm(False, False, [x], [W], M, N, K),
                    "gnn_fwd_pad": lambda: gemm(False, False, [xv], [W], M, N, K),
                    "gnn_fwd_pair": lambda: gemm(False, False, [x, x], [W, W], M, N, K),
                    "gnn_dX": lambda: gemm(False, True, [g], [W], M, K, N),
                    "gnn_dW": lambda: gemm(True, True, [g], [x], N, K, M),
                    "gnn_dW_pair": lambda: gemm(True, True, [g, g], [x, x], N, K, M),
                })
            for name, fn in cases.items():
                us = timeit(fn)
                f = flops * (2 if name.endswith("_pair") else 1)
                res[f"{lib}/{M}x{K}x{N}/{name}"] = {"us": round(us, 1), "TFLOPs": round(f / us * 1e-6, 1)}
            print(f"{lib} {M}x{K}x{N} done", file=sys.stderr, flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
