"""GPU: split3 on pre-split ("p3") operands vs split3 splitting in registers, on the GraphSAGE-Reddit
layer GEMM shapes (config 2): bit-identity, kernel time (HIP events, median of 20), the packing
passes' time. Usage: python scripts/gemm_p3_probe.py [--out FILE.json]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd import _lib  # noqa: E402
from gnn_amd.fused import gemm  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return round(float(np.median(ts)), 1)


def pack(L, t, kmajor, R, K, dev):
    nb = L.gnn_gemm_p3_packed_bytes(R, K)
    out = torch.empty(nb, dtype=torch.uint8, device=dev)
    _lib.check(L.gnn_gemm_p3_pack_f32(t.data_ptr(), t.stride(0), kmajor, None, R, K, out.data_ptr(), nb,
                                      _lib.stream_of(dev)), "pack")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    torch.manual_seed(0)
    M0, M1 = 15809, 8689
    mat = lambda r, c, ld: torch.randn(r, ld, device=dev)[:, :c]
    x0 = [mat(M0, 602, 608) for _ in range(2)]
    W0 = [torch.randn(512, 602, device=dev) for _ in range(2)]
    g0 = [torch.randn(M0, 512, device=dev) for _ in range(2)]
    x1 = [torch.randn(M1, 1024, device=dev) for _ in range(2)]
    W1 = [torch.randn(512, 1024, device=dev) for _ in range(2)]
    g1 = [torch.randn(M1, 512, device=dev) for _ in range(2)]
    # (name, a_kmajor, b_kmajor, M, N, K, As, Bs): C = A·B with the layouts of gnn_gemm_f32
    cases = [("L0 fwd x.Wt", False, False, M0, 512, 602, x0, W0),
             ("L0 dW g^t.x", True, True, 512, 602, M0, g0, x0),
             ("L1 fwd x.Wt", False, False, M1, 512, 1024, x1, W1),
             ("L1 dX g.W", False, True, M1, 1024, 512, g1, W1),
             ("L1 dW g^t.x", True, True, 512, 1024, M1, g1, x1)]
    res = []
    for name, ak, bk, M, N, K, As, Bs in cases:
        ref = gemm(ak, bk, As, Bs, M, N, K, algo="split3")
        t_s3 = timeit(lambda: gemm(ak, bk, As, Bs, M, N, K, algo="split3"))
        # packed: A viewed as M rows x K (m-major unless ak), B as N rows x K (k-major source when bk:
        # B(k, n) = B[k*ld + n] -> element (n, k) at src[k*ld + n]; n-major: src[n*ld + k])
        pa = [pack(L, t, int(ak), M, K, dev) for t in As]
        pb = [pack(L, t, int(bk), N, K, dev) for t in Bs]
        t_pack = timeit(lambda: ([pack(L, t, int(ak), M, K, dev) for t in As],
                                 [pack(L, t, int(bk), N, K, dev) for t in Bs]))
        nb = len(As)
        C = [torch.empty(M, N, device=dev) for _ in range(nb)]
        wsb = L.gnn_gemm_p3_workspace_bytes(M, N, K, nb)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        arr = lambda ts: (ctypes.c_void_p * nb)(*[t.data_ptr() for t in ts])

        def run():
            _lib.check(L.gnn_gemm_p3(M, N, K, nb, arr(pa), arr(pb), arr(C), N, ws.data_ptr(), wsb,
                                     _lib.stream_of(dev)), "gnn_gemm_p3")

        run()
        torch.cuda.synchronize()
        same = all(torch.equal(c, r) for c, r in zip(C, ref))
        t_p3 = timeit(run)
        fl = 2.0 * nb * M * N * K
        e = {"case": name, "M": M, "N": N, "K": K, "split3_us": t_s3, "p3_us": t_p3, "pack_us": t_pack,
             "split3_TF": round(fl / t_s3 * 1e-6, 1), "p3_TF": round(fl / t_p3 * 1e-6, 1), "bit_identical": same}
        print(e, file=sys.stderr, flush=True)
        res.append(e)
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
