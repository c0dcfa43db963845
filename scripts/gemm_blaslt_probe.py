"""GPU probe: how fast would the layer GEMMs run as plain bf16 GEMMs on the vendor library?

split3 computes an fp32 product C = A·B as the six largest bf16 piece products
(x = h + m + l exactly) on our own MFMA kernel, at 128-180 TF/s fp32-equivalent (31-43 % of the
417 TF/s split3 peak). The same six products written as ONE bf16 GEMM with k = 6K
(A6 = [h m h l m h] . B6 = [h h m h m l] along k, fp32 accumulate and output) or as three with
prefix operands (A3 = [h | m | l] along k, C = A3[:, :3K]·[Bh;Bh;Bh] + A3[:, :2K]·[Bm;Bm] +
A3[:, :K]·Bl) run on hipBLASLt through torch.mm(..., out_dtype=float32). This probe times those
forms on the five config-2 layer shapes (the pair of each product, as the step runs them) beside
split3 and the fp32 vendor GEMM, with the fp64 error bound of tests/test_gemm_gpu.py
(|C - C64| <= 4e-6 (|A|·|B|)), and the cost of splitting an fp32 operand in torch.

Usage (GPU): python scripts/gemm_blaslt_probe.py [out.json]
"""
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


def pieces(x):
    """x = h + m + l exactly, each a bf16 tensor (truncation)."""
    xi = x.contiguous().view(torch.int32)
    mask = torch.tensor(-65536, dtype=torch.int32, device=x.device)  # 0xffff0000
    h = (xi & mask).view(torch.float32)
    r = x - h
    m = (r.view(torch.int32) & mask).view(torch.float32)
    lo = r - m
    return h.to(torch.bfloat16), m.to(torch.bfloat16), lo.to(torch.bfloat16)


def mm32(a, b):
    return torch.mm(a, b, out_dtype=torch.float32)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else ""
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M0, M1 = 15809, 8689
    # C = A (M x K) . B (K x N), A and B as row-major tensors in the orientation of the product
    cases = [("L0 fwd x.Wt", M0, 512, 602), ("L0 dW g^t.x", 512, 602, M0), ("L1 fwd x.Wt", M1, 512, 1024),
             ("L1 dX g.W", M1, 1024, 512), ("L1 dW g^t.x", 512, 1024, M1)]
    res = []
    for name, M, N, K in cases:
        kmaj = "dW" in name  # weight gradients: A = Gᵀ with G (K x M) row-major, as the step stores it
        As = [torch.randn(K, M, device=dev) if kmaj else torch.randn(M, K, device=dev) for _ in range(2)]
        A = [a.t().contiguous() if kmaj else a for a in As]
        B = [torch.randn(K, N, device=dev) * 0.05 for _ in range(2)]
        fl = 2.0 * 2 * M * N * K
        row = {"case": name, "M": M, "N": N, "K": K, "pair_GFLOP": round(fl / 1e9, 2)}
        C64 = [a.double() @ b.double() for a, b in zip(A, B)]
        S64 = [a.double().abs() @ b.double().abs() for a, b in zip(A, B)]

        def err(Cs):
            return max(float(((c.double() - c64).abs() / s64.clamp_min(1e-300)).max()) for c, c64, s64 in zip(Cs, C64, S64))

        us = timeit(lambda: [a @ b for a, b in zip(A, B)])
        row["vendor_f32_us"] = round(us, 1)
        # split3 (our kernel): the pair as one batched launch, A m-major, B k-major (row k contiguous in n)
        us = timeit(lambda: gemm(kmaj, True, As, B, M, N, K, algo="split3"))
        row["split3_us"] = round(us, 1)
        row["split3_err"] = err(gemm(kmaj, True, As, B, M, N, K, algo="split3"))
        # pieces
        us = timeit(lambda: [pieces(a) for a in A])
        row["torch_split_A_us"] = round(us, 1)
        PA = [pieces(a) for a in A]
        PB = [pieces(b) for b in B]
        # one k = 6K GEMM
        A6 = [torch.cat([p[0], p[1], p[0], p[2], p[1], p[0]], dim=1).contiguous() for p in PA]
        B6 = [torch.cat([q[0], q[0], q[1], q[0], q[1], q[2]], dim=0).contiguous() for q in PB]
        us = timeit(lambda: [mm32(a, b) for a, b in zip(A6, B6)])
        row["blaslt_k6_us"] = round(us, 1)
        row["blaslt_k6_err"] = err([mm32(a, b) for a, b in zip(A6, B6)])
        # three prefix GEMMs over A3 = [h | m | l]
        A3 = [torch.cat([p[0], p[1], p[2]], dim=1).contiguous() for p in PA]
        Bh3 = [torch.cat([q[0]] * 3, dim=0).contiguous() for q in PB]
        Bm2 = [torch.cat([q[1]] * 2, dim=0).contiguous() for q in PB]
        Bl = [q[2].contiguous() for q in PB]

        def three(a3, bh, bm, bl):
            c = mm32(a3[:, : 3 * K], bh)
            c += mm32(a3[:, : 2 * K], bm)
            c += mm32(a3[:, :K], bl)
            return c

        us = timeit(lambda: [three(*z) for z in zip(A3, Bh3, Bm2, Bl)])
        row["blaslt_3prefix_us"] = round(us, 1)
        row["blaslt_3prefix_err"] = err([three(*z) for z in zip(A3, Bh3, Bm2, Bl)])
        # plain bf16 GEMM at k = K (one piece product): the library's rate on the shape
        us = timeit(lambda: [mm32(p[0], q[0]) for p, q in zip(PA, PB)])
        row["blaslt_k1_us"] = round(us, 1)
        row["blaslt_k1_TF_bf16"] = round(fl / us * 1e-6, 1)
        for k in ("vendor_f32", "split3", "blaslt_k6", "blaslt_3prefix"):
            row[k + "_TF_f32eq"] = round(fl / row[k + "_us"] * 1e-6, 1)
        print(json.dumps(row), flush=True)
        res.append(row)
        del A, As, B, C64, S64, PA, PB, A6, B6, A3, Bh3, Bm2, Bl
        torch.cuda.empty_cache()
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
