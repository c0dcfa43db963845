"""GPU: the fp32 GEMMs (gnn_gemm_f32 on f32-input MFMA, gnn_gemm_f32_split3 on bf16 MFMA over an
exact three-way operand split) against an fp64 evaluation, every operand layout,
edge tiles, split-k and batched problems; and LinearPairFn against F.linear's autograd.

Tolerance: fp32 products summed in a different order than the fp64 reference — error
bounded by ~K·eps·Σ|a·b|: checked as |C - C64| <= 4e-6 · (|A|·|B|)(m, n) + 1e-30.
"""
import numpy as np
import pytest
import torch

from gnn_amd.fused import GEMM_ALGOS, gemm, linear_pair

pytestmark = pytest.mark.gpu


def _operand(kmajor, rows, cols, ld, g, dev):
    """Matrix (rows x cols) as the kernel reads it; stored k-major/m-major with row stride ld."""
    buf = torch.randn(rows, ld + (ld & 1), generator=g)  # the kernel needs even row strides
    return buf.to(dev)[:, :cols]


def _check(a_km, b_km, M, N, K, nb, dev, lda_pad=0, ldb_pad=0, algo=None):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + nb)
    As, Bs, A64, B64 = [], [], [], []
    for _ in range(nb):
        a = _operand(a_km, K if a_km else M, M if a_km else K, (M if a_km else K) + lda_pad, g, dev)
        b = _operand(b_km, K if b_km else N, N if b_km else K, (N if b_km else K) + ldb_pad, g, dev)
        As.append(a)
        Bs.append(b)
        A64.append((a.t() if a_km else a).double().cpu())
        B64.append((b if b_km else b.t()).double().cpu())
    Cs = gemm(a_km, b_km, As, Bs, M, N, K, algo=algo)
    torch.cuda.synchronize()
    for c, a, b in zip(Cs, A64, B64):
        ref = a @ b
        bound = 4e-6 * (a.abs() @ b.abs()) + 1e-30
        err = (c.double().cpu() - ref).abs()
        assert bool((err <= bound).all()), f"max excess {(err - bound).max().item()}"


@pytest.mark.parametrize("algo", GEMM_ALGOS)
@pytest.mark.parametrize("a_km,b_km", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 16), (300, 200, 77), (1, 5, 3), (130, 513, 602), (257, 64, 1024)])
def test_gemm_layouts(dev, a_km, b_km, M, N, K, algo):
    _check(a_km, b_km, M, N, K, 1, dev, algo=algo)


@pytest.mark.parametrize("algo", GEMM_ALGOS)
def test_gemm_split_k_and_batch(dev, algo):
    # weight-gradient shape: small output, long reduction -> split over k, two problems batched
    _check(True, True, 512, 602, 5000, 2, dev, algo=algo)
    _check(True, True, 100, 130, 3001, 3, dev, algo=algo)


@pytest.mark.parametrize("algo", GEMM_ALGOS)
def test_gemm_padded_and_even_strides(dev, algo):
    _check(False, False, 333, 512, 602, 2, dev, lda_pad=2, ldb_pad=0, algo=algo)   # 604-float rows (16-B loads)
    _check(False, True, 200, 602, 512, 1, dev, lda_pad=0, ldb_pad=0, algo=algo)    # 602-float rows (8-B loads)


def test_split3_wide_exponents(dev):
    # operands spanning 2^-40 .. 2^40 (the split is exact at every exponent; each piece
    # product is exact in fp32) against fp64, and exactly representable results stay exact
    g = torch.Generator().manual_seed(5)
    M, N, K = 160, 140, 334
    a = torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-40, 41, (M, 1), generator=g).float())
    b = torch.randn(N, K, generator=g) * torch.exp2(torch.randint(-40, 41, (1, K), generator=g).float())
    (c,) = gemm(False, False, [a.to(dev)], [b.to(dev)], M, N, K, algo="split3")
    ref = a.double() @ b.double().t()
    bound = 4e-6 * (a.double().abs() @ b.double().abs().t()) + 1e-30
    assert bool(((c.cpu().double() - ref).abs() <= bound).all())
    ai = torch.randint(-64, 65, (M, K), generator=g).float()  # small integers: every partial sum exact
    bi = torch.randint(-64, 65, (N, K), generator=g).float()
    (ci,) = gemm(False, False, [ai.to(dev)], [bi.to(dev)], M, N, K, algo="split3")
    assert torch.equal(ci.cpu(), (ai.double() @ bi.double().t()).float())


@pytest.mark.parametrize("algo", GEMM_ALGOS)
def test_gemm_k_zero(dev, algo):
    a = torch.zeros(10, 2, device=dev)[:, :0]
    b = torch.zeros(7, 2, device=dev)[:, :0]
    (c,) = gemm(False, False, [a], [b], 10, 7, 0, algo=algo)
    torch.cuda.synchronize()
    assert torch.count_nonzero(c) == 0


@pytest.mark.parametrize("n", [1, 2])
def test_linear_pair_matches_torch(dev, n):
    g = torch.Generator().manual_seed(n)
    xs = [torch.randn(777, 602, generator=g).to(dev).requires_grad_(True) for _ in range(n)]
    Ws = [torch.randn(512, 602, generator=g).to(dev).requires_grad_(True) for _ in range(n)]
    gys = [torch.randn(777, 512, generator=g).to(dev) for _ in range(n)]
    ys = linear_pair(xs, Ws)
    torch.autograd.backward(ys, gys)
    xr = [x.detach().double().requires_grad_(True) for x in xs]
    Wr = [W.detach().double().requires_grad_(True) for W in Ws]
    yr = [torch.nn.functional.linear(x, W) for x, W in zip(xr, Wr)]
    torch.autograd.backward(yr, [gy.double() for gy in gys])
    for a, b in zip(ys, yr):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=1e-4, atol=2e-4)
    for a, b in zip(xs + Ws, xr + Wr):
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.cpu().numpy(), rtol=1e-4, atol=2e-3)
