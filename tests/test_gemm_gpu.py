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


def _ptrs(ts):
    import ctypes

    arr = (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])
    return arr


@pytest.mark.parametrize("case", ["a_fwd", "b_wgrad"])
@pytest.mark.parametrize("M,N,K,R", [(4100, 512, 602, 6000), (300, 130, 77, 1000), (513, 1024, 1024, 800)])
def test_split3_row_indexed_equals_gathered(dev, case, M, N, K, R):
    """gnn_gemm_f32_split3_indexed: an m-major A (the forward's x[sampled]) or a k-major B (the
    weight gradient's x[sampled]) read through a row index (repeats allowed) gives exactly the
    split3 product of the gathered operand — same bits, batched with an unindexed product."""
    from gnn_amd import _lib
    from gnn_amd.fused import gemm

    g = torch.Generator().manual_seed(M + N + K)
    L = _lib.lib()
    if case == "a_fwd":  # C (M x N) = A[idx] (M x K) · Bᵀ, B (N x K)
        src = torch.randn(R, K + (K & 1), generator=g).to(dev)
        idx = torch.randint(0, R, (M,), generator=g).to(dev)
        other = torch.randn(M, src.shape[1], generator=g).to(dev)
        Bw = torch.randn(N, K + (K & 1), generator=g).to(dev)
        A_ref = [src[idx][:, :K], other[:, :K]]
        ref = gemm(False, False, A_ref, [Bw[:, :K], Bw[:, :K]], M, N, K, algo="split3")
        out = [torch.empty(M, N, device=dev) for _ in range(2)]
        wsb = L.gnn_gemm_f32_split3_workspace_bytes(M, N, K, 2)
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
        # the indexed source and the plain operand share the row stride
        rc = L.gnn_gemm_f32_split3_indexed(0, 0, M, N, K, 2, _ptrs([src, other]), src.stride(0),
                                           _ptrs([idx, None]), R, _ptrs([Bw, Bw]), Bw.stride(0), None, 0,
                                           _ptrs(out), N, ws.data_ptr(), wsb, _lib.stream_of(dev))
    else:  # C (N x K) = Gᵀ (G: M x N, k-major over M) · X[idx] (M x K, k-major B)
        src = torch.randn(R, K + (K & 1), generator=g).to(dev)
        idx = torch.randint(0, R, (M,), generator=g).to(dev)
        other = torch.randn(M, src.shape[1], generator=g).to(dev)
        G = torch.randn(M, N + (N & 1), generator=g).to(dev)
        ref = gemm(True, True, [G[:, :N], G[:, :N]], [src[idx][:, :K], other[:, :K]], N, K, M, algo="split3")
        out = [torch.empty(N, K, device=dev) for _ in range(2)]
        wsb = L.gnn_gemm_f32_split3_workspace_bytes(N, K, M, 2)
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
        rc = L.gnn_gemm_f32_split3_indexed(1, 1, N, K, M, 2, _ptrs([G, G]), G.stride(0), None, 0,
                                           _ptrs([src, other]), src.stride(0), _ptrs([idx, None]), R,
                                           _ptrs(out), K, ws.data_ptr(), wsb, _lib.stream_of(dev))
    assert rc == 0, L.gnn_last_error()
    torch.cuda.synchronize()
    for c, r in zip(out, ref):
        assert torch.equal(c, r)


def test_split3_indexed_rejects_bad_layouts(dev):
    from gnn_amd import _lib

    L = _lib.lib()
    a = torch.zeros(64, 64, device=dev)
    idx = torch.zeros(64, dtype=torch.int64, device=dev)
    c = torch.empty(64, 64, device=dev)
    rc = L.gnn_gemm_f32_split3_indexed(1, 0, 64, 64, 64, 1, _ptrs([a]), 64, _ptrs([idx]), 64, _ptrs([a]), 64, None, 0,
                                       _ptrs([c]), 64, None, 0, _lib.stream_of(dev))
    assert rc != 0 and b"row indices" in L.gnn_last_error()


@pytest.mark.parametrize("a_km,b_km,M,N,K,nb", [(False, False, 300, 200, 70, 2), (True, True, 130, 257, 4000, 2),
                                                (False, True, 129, 512, 33, 1), (True, False, 64, 64, 16, 1)])
def test_p3_packed_equals_split3(dev, a_km, b_km, M, N, K, nb):
    """gnn_gemm_p3 over operands packed once into their bf16 pieces (gnn_gemm_p3_pack_f32, also
    through a row index) is bit-identical to gnn_gemm_f32_split3 on the same operands (same pieces,
    k steps and MFMA order), edge tiles, k tails and split-k included."""
    import ctypes

    from gnn_amd import _lib

    L = _lib.lib()
    g = torch.Generator().manual_seed(M + N + K)
    As = [_operand(a_km, K if a_km else M, M if a_km else K, (M if a_km else K) + 2, g, dev) for _ in range(nb)]
    Bs = [_operand(b_km, K if b_km else N, N if b_km else K, (N if b_km else K) + 2, g, dev) for _ in range(nb)]
    ref = gemm(a_km, b_km, As, Bs, M, N, K, algo="split3")
    st = _lib.stream_of(dev)

    def pack(t, kmajor, R, idx=None):
        nb_ = L.gnn_gemm_p3_packed_bytes(R, K)
        out = torch.empty(nb_, dtype=torch.uint8, device=dev)
        src = t if idx is None else t
        _lib.check(L.gnn_gemm_p3_pack_f32(src.data_ptr(), src.stride(0), int(kmajor),
                                          None if idx is None else idx.data_ptr(), R, K, out.data_ptr(), nb_, st),
                   "gnn_gemm_p3_pack_f32")
        return out

    pa = [pack(a, a_km, M) for a in As]
    pb = [pack(b, b_km, N) for b in Bs]
    C = [torch.full((M, N), float("nan"), device=dev) for _ in range(nb)]
    wsb = L.gnn_gemm_p3_workspace_bytes(M, N, K, nb)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    arr = lambda ts: (ctypes.c_void_p * nb)(*[t.data_ptr() for t in ts])
    _lib.check(L.gnn_gemm_p3(M, N, K, nb, arr(pa), arr(pb), arr(C), N, ws.data_ptr(), wsb, st), "gnn_gemm_p3")
    torch.cuda.synchronize()
    for c, r in zip(C, ref):
        assert torch.equal(c, r)
    # a row-indexed m-major A (x[sampled]) packs to the same pieces as its gathered copy
    if not a_km:
        src = torch.randn(M + 50, As[0].shape[1], device=dev, generator=torch.Generator(device=dev).manual_seed(5))
        idx = torch.randperm(M + 50, device=dev)[:M]
        assert torch.equal(pack(src, False, M, idx), pack(src[idx].contiguous(), False, M))


def test_split3_tail_tiles(dev, monkeypatch):
    """Tail tiles (gemm.hip tail_plan) on the layer-1 forward shape: 544 tiles = 2 x 256 whole + 32
    tail tiles computed as 4 k pieces each and added in piece order. Against fp64 within the module
    tolerance; the whole tiles bit-identical to the unsplit launch (GNN_GEMM_TAIL=0), the tail tiles
    (batch 1, rows >= 7,680) within fp32 rounding of it; deterministic."""
    M, N, K = 8680, 512, 1024
    _check(False, False, M, N, K, 2, dev, algo="split3")
    g = torch.Generator().manual_seed(5)
    As = [_operand(False, M, K, K, g, dev) for _ in range(2)]
    Bs = [_operand(False, N, K, K, g, dev) for _ in range(2)]
    on = gemm(False, False, As, Bs, M, N, K, algo="split3")
    again = gemm(False, False, As, Bs, M, N, K, algo="split3")
    monkeypatch.setenv("GNN_GEMM_TAIL", "0")
    off = gemm(False, False, As, Bs, M, N, K, algo="split3")
    torch.cuda.synchronize()
    assert all(torch.equal(x, y) for x, y in zip(on, again))
    assert torch.equal(on[0], off[0]) and torch.equal(on[1][:7680], off[1][:7680])
    d = (on[1][7680:] - off[1][7680:]).abs().max().item()
    assert 0 < d <= 1e-4 * off[1][7680:].abs().max().item()


@pytest.mark.parametrize("a_km,b_km", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K,nb", [(300, 256, 77, 1), (130, 513, 602, 2), (257, 700, 1024, 1), (512, 602, 5000, 2),
                                      (1000, 512, 33, 2)])
def test_split3_wide_fp64_bound_and_whole_tiles_bit_identical(dev, monkeypatch, a_km, b_km, M, N, K, nb):
    """The wide split3 kernel (GNN_GEMM_WIDE=1: 128 x 256 tiles, a wave owns 64 x 128) within the fp64
    bound on every layout, edge tiles, split-k and batches; where it runs k unsplit (every shape
    here but the long-k one) each output sums the same pieces in the same order as split3, so it
    must be bit-identical to split3 with its tail tiles off."""
    monkeypatch.setenv("GNN_GEMM_WIDE", "1")
    _check(a_km, b_km, M, N, K, nb, dev, algo="split3")
    g = torch.Generator().manual_seed(5)
    As = [_operand(a_km, K if a_km else M, M if a_km else K, M if a_km else K, g, dev) for _ in range(nb)]
    Bs = [_operand(b_km, K if b_km else N, N if b_km else K, N if b_km else K, g, dev) for _ in range(nb)]
    wide = gemm(a_km, b_km, As, Bs, M, N, K, algo="split3")
    monkeypatch.setenv("GNN_GEMM_WIDE", "0")
    monkeypatch.setenv("GNN_GEMM_TAIL", "0")
    base = gemm(a_km, b_km, As, Bs, M, N, K, algo="split3")
    torch.cuda.synchronize()
    if K < 4000:  # neither kernel splits k here
        for x, y in zip(wide, base):
            assert torch.equal(x, y)


@pytest.mark.parametrize("case", ["a_fwd", "b_wgrad"])
def test_split3_wide_row_indexed_equals_gathered(dev, monkeypatch, case):
    """The wide kernel's indexed operands (x[sampled] read in place) equal the gathered operand bit for bit."""
    monkeypatch.setenv("GNN_GEMM_WIDE", "1")
    test_split3_row_indexed_equals_gathered(dev, case, 4100, 512, 602, 6000)
