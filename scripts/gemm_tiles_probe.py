"""GPU probe: split3 GEMM time against the number of 128 x 128 output tiles (the layer-1 forward
shape N = 512, K = 1024, two products, M varied), to see whether a launch's time follows its
workgroups per CU (3 slots per CU: 256 CUs) — i.e. what the layer-1 forward's 544 tiles (2.125
per CU) and the layer-1 input gradient's 1,088 (4.25) pay for their last, partial round.
Usage: python scripts/gemm_tiles_probe.py [--out FILE.json]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd.fused import gemm  # noqa: E402


def timeit(fn, reps=30):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = []
    for K, N in ((1024, 512), (512, 1024)):
        W = [torch.randn(N, K, device=dev) for _ in range(2)] if N == 512 else [torch.randn(K, N, device=dev)
                                                                                 for _ in range(2)]
        for mt in (32, 48, 64, 68, 72, 80, 96, 104, 128, 136, 144):
            M = mt * 128
            X = [torch.randn(M, K, device=dev) for _ in range(2)]
            bk = N != 512  # dX = G·W: W k-major
            us = timeit(lambda: gemm(False, bk, X, W, M, N, K))
            tiles = mt * (N // 128) * 2
            row = {"K": K, "N": N, "M": M, "tiles": tiles, "per_cu": tiles / 256, "us": round(us, 1),
                   "us_per_tile_round": round(us / max(1.0, -(-tiles // 768)), 1),
                   "TF": round(2.0 * 2 * M * N * K / us * 1e-6, 1)}
            print(json.dumps(row), flush=True)
            res.append(row)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
