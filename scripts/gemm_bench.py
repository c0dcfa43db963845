"""GPU microbench: the GraphSAGE-Reddit layer GEMM shapes (config 2) on gnn_gemm_f32 kernel
variants (env knobs read per call: VARIANTS="GNN_GEMM_PF=2,GNN_GEMM_XCD=1;..." — ';' between
variants, ',' between settings, '-' = defaults) and on the vendor GEMM (torch.matmul), with an fp64
error check of every variant: |C - C64| <= 4e-6 (|A|·|B|) as in tests/test_gemm_gpu.py."""
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


def mat(r, c, ld, dev):
    return torch.randn(r, ld, device=dev)[:, :c]


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    variants = os.environ.get("VARIANTS", "-").split(";")
    knobs = ("GNN_GEMM_PF", "GNN_GEMM_XCD", "GNN_GEMM_ALGO", "GNN_GEMM_WIDE", "GNN_GEMM_TAIL")
    res = []
    # (name, a_kmajor, b_kmajor, M, N, K, A (as stored), B (as stored)) for the pair of a layer
    M0, M1 = 15809, 8689
    x0 = [mat(M0, 602, 608, dev) for _ in range(2)]
    W0 = [torch.randn(512, 602, device=dev) for _ in range(2)]
    g0 = [torch.randn(M0, 512, device=dev) for _ in range(2)]
    x1 = [torch.randn(M1, 1024, device=dev) for _ in range(2)]
    W1 = [torch.randn(512, 1024, device=dev) for _ in range(2)]
    g1 = [torch.randn(M1, 512, device=dev) for _ in range(2)]
    cases = [
        ("L0 fwd x.Wt", False, False, M0, 512, 602, x0, W0, lambda a, b: a @ b.t()),
        ("L0 dW g^t.x", True, True, 512, 602, M0, g0, x0, lambda a, b: a.t() @ b),
        ("L1 fwd x.Wt", False, False, M1, 512, 1024, x1, W1, lambda a, b: a @ b.t()),
        ("L1 dX g.W", False, True, M1, 1024, 512, g1, W1, lambda a, b: a @ b),
        ("L1 dW g^t.x", True, True, 512, 1024, M1, g1, x1, lambda a, b: a.t() @ b),
    ]
    for name, ak, bk, M, N, K, As, Bs, ref in cases:
        fl = 2.0 * 2 * M * N * K
        row = {"case": name, "M": M, "N": N, "K": K}
        us = timeit(lambda: [ref(a, b) for a, b in zip(As, Bs)])
        row["vendor_us"] = round(us, 1)
        row["vendor_TF"] = round(fl / us * 1e-6, 1)
        C64 = [ref(a.double(), b.double()) for a, b in zip(As, Bs)]
        S64 = [ref(a.double().abs(), b.double().abs()) for a, b in zip(As, Bs)]
        times = {v: [] for v in variants}
        for rnd in range(int(os.environ.get("ROUNDS", "1"))):  # variants interleaved, ROUNDS times
            for v in variants:
                for k in knobs:
                    os.environ.pop(k, None)
                for kv in v.split(","):
                    if "=" in kv:
                        k, val = kv.split("=")
                        os.environ[k] = val
                times[v].append(timeit(lambda: gemm(ak, bk, As, Bs, M, N, K)))
                if rnd == 0:
                    Cs = gemm(ak, bk, As, Bs, M, N, K)
                    err = max(float(((c.double() - c64).abs() / (s64 + 1e-30)).max())
                              for c, c64, s64 in zip(Cs, C64, S64))
                    row[f"v{v}_relerr"] = float(f"{err:.2e}")
                    row[f"v{v}_ok"] = err <= 4e-6
        for v in variants:
            us = sorted(times[v])[len(times[v]) // 2]
            row[f"v{v}_us"] = round(us, 1)
            row[f"v{v}_min_us"] = round(min(times[v]), 1)
            row[f"v{v}_TF"] = round(fl / us * 1e-6, 1)
        res.append(row)
        print(json.dumps(row), flush=True)
    for k in knobs:
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
