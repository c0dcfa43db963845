"""GPU probe: best vendor (rocBLAS/hipBLASLt) fp32 GEMM time per layer shape with torch's
TunableOp exhaustive search, against the default heuristic choice."""
import json
import os
import sys

import torch


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


def cases(dev):
    out = {}
    for (M, K, N) in ((15768, 602, 512), (8680, 1024, 512)):
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        g = torch.randn(M, N, device=dev)
        out[f"{M}x{K}x{N}/fwd"] = (lambda x=x, W=W: torch.nn.functional.linear(x, W), 2.0 * M * N * K)
        out[f"{M}x{K}x{N}/dX"] = (lambda g=g, W=W: torch.mm(g, W), 2.0 * M * N * K)
        out[f"{M}x{K}x{N}/dW"] = (lambda g=g, x=x: torch.mm(g.t(), x), 2.0 * M * N * K)
    return out


def main():
    dev = torch.device("cuda", 0)
    res = {}
    torch.backends.cuda.preferred_blas_library("cublas")
    for k, (fn, fl) in cases(dev).items():
        us = timeit(fn)
        res[k + "/default"] = [round(us, 1), round(fl / us * 1e-6, 1)]
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), "tunable.csv"))
    for k, (fn, fl) in cases(dev).items():
        fn()  # tunes
        torch.cuda.synchronize()
        us = timeit(fn)
        res[k + "/tuned"] = [round(us, 1), round(fl / us * 1e-6, 1)]
        print(k, res[k + "/default"], res[k + "/tuned"], file=sys.stderr, flush=True)
    print(json.dumps(res, indent=0))


if __name__ == "__main__":
    main()
