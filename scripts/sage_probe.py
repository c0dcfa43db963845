"""GPU microbench: the fused layer epilogue (gnn_sage_norm_fwd/bwd) at the Reddit config-2
layer shapes, training mode. Prints one JSON object (µs per call and effective GB/s).
Sweep the backward grid with GNN_SAGE_BWD_GRID=<workgroups>."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnn_amd.fused import sage_norm  # noqa: E402


def timeit(fn, reps=50):
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
    res = {"grid": os.environ.get("GNN_SAGE_BWD_GRID", "default")}
    for M in (15768, 8680, 512):
        hB = torch.randn(M, 512, device=dev, requires_grad=True)
        hW = torch.randn(M, 512, device=dev, requires_grad=True)
        bB = torch.randn(512, device=dev, requires_grad=True)
        bW = torch.randn(512, device=dev, requires_grad=True)
        scale = torch.ones(1024, device=dev, requires_grad=True)
        offset = torch.zeros(1024, device=dev, requires_grad=True)
        g = torch.randn(M, 1024, device=dev)
        with torch.no_grad():
            fwd = timeit(lambda: sage_norm(hB, hW, scale, offset, 0.1, True, bB, bW))
        # backward kernel pair through the C ABI with preallocated outputs (autograd's host
        # overhead would dominate otherwise)
        from gnn_amd import _lib

        L = _lib.lib()
        mean = torch.randn(M, device=dev)
        rstd = torch.rand(M, device=dev) + 0.5
        dhB, dhW = torch.empty_like(hB), torch.empty_like(hW)
        outs = [torch.empty(1024, device=dev) for _ in range(2)] + [torch.empty(512, device=dev) for _ in range(2)]
        wsb = L.gnn_sage_norm_bwd_workspace_bytes(M, 1024)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        st = _lib.stream_of(dev)
        bwd = timeit(lambda: L.gnn_sage_norm_bwd_f32(
            g.data_ptr(), 1024, hB.data_ptr(), 512, 512, hW.data_ptr(), 512, 512, bB.data_ptr(), bW.data_ptr(),
            scale.data_ptr(), mean.data_ptr(), rstd.data_ptr(), M, 0.1, 7, 1, dhB.data_ptr(), dhW.data_ptr(),
            outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), outs[3].data_ptr(), ws.data_ptr(), wsb, st))
        nb = M * 1024 * 4
        res[str(M)] = {"fwd_us": round(fwd, 1), "fwd_GBps": round(3 * nb / fwd * 1e-3, 1), "bwd_us": round(bwd, 1),
                       "bwd_GBps": round(3 * nb / bwd * 1e-3, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
