"""CPU: the oracle is pinned against the reference's golden vectors before it is trusted."""
import numpy as np
import torch

import oracle as O
from oracle.fixtures import powerlaw_lens, random_csr


def _coo_to_csr(indices, values, shape):
    M = int(shape[0])
    rows, cols = indices
    rowptr = np.zeros(M + 1, np.int32)
    np.add.at(rowptr, rows + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), cols.astype(np.int32), values.astype(np.float32)


def test_operand_builder_matches_reference_adjs(golden):
    """oracle_build_operand on the inputs the reference passed to create_coo_tensor equals
    the coalesced COO the reference returned (formula of cuda_spmm.cu:800, double math)."""
    z = golden("ladies_tiny.npz")
    for c in range(4):
        for li in range(3):
            p = f"c{c}_call{li}_"
            col, val = O.build_operand(z[p + "fullrowptr"], z[p + "rowptr"], z[p + "colidx"].astype(np.int32),
                                       z[p + "normfact"])
            q = f"c{c}_adj{2 - li}_"
            assert np.array_equal(col, z[q + "indices"][1])
            assert np.array_equal(val, z[q + "values"])


def test_spmm_oracle_matches_torch_sparse_mm_golden(golden):
    z = golden("ladies_tiny.npz")
    s = golden("spmm_tiny.npz")
    for li in range(3):
        shape = z[f"c2_adj{li}_shape"]
        rowptr, col, val = _coo_to_csr(z[f"c2_adj{li}_indices"], z[f"c2_adj{li}_values"], shape)
        trp, trc, trv = O.csr_transpose(rowptr, col, val, int(shape[1]))
        for F in (1, 26, 64, 100, 602):
            g = torch.Generator().manual_seed(1000 * li + F)
            X = torch.randn(int(shape[1]), F, generator=g).numpy()
            G = torch.randn(int(shape[0]), F, generator=g).numpy()
            np.testing.assert_allclose(O.spmm_f32(rowptr, col, val, X), s[f"l{li}_F{F}_Y"], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(O.spmm_f64(rowptr, col, val, X), s[f"l{li}_F{F}_Y"], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(O.spmm_f32(trp, trc, trv, G), s[f"l{li}_F{F}_dX"], rtol=1e-5, atol=1e-5)


WIDE_CASES = (("c2", (0, 1, 2)), ("c0", (2,)))  # tests/golden/make_golden.py spmm_wide_goldens


def wide_inputs(z, case, li, F=1024):
    """X, G of one spmm_wide.npz entry, regenerated from the seed make_golden.py used."""
    shape = tuple(int(v) for v in z[f"{case}_adj{li}_shape"])
    g = torch.Generator().manual_seed(7000 + 100 * li + int(case[1:]))
    return shape, torch.randn(shape[1], F, generator=g), torch.randn(shape[0], F, generator=g)


def test_spmm_oracle_matches_wide_golden(golden):
    """F = 1024 (the hidden width of the layer-1/2 aggregations): the oracle's fp32 chain and
    its canonical transpose against the reference CPU path's outputs (spmm_wide.npz)."""
    z = golden("ladies_tiny.npz")
    s = golden("spmm_wide.npz")
    for case, layers in WIDE_CASES:
        for li in layers:
            shape, X, G = wide_inputs(z, case, li)
            rowptr, col, val = _coo_to_csr(z[f"{case}_adj{li}_indices"], z[f"{case}_adj{li}_values"], shape)
            trp, trc, trv = O.csr_transpose(rowptr, col, val, int(shape[1]))
            np.testing.assert_allclose(O.spmm_f32(rowptr, col, val, X.numpy()), s[f"{case}_l{li}_Y"],
                                       rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(O.spmm_f32(trp, trc, trv, G.numpy()), s[f"{case}_l{li}_dX"],
                                       rtol=1e-5, atol=1e-5)


def test_transpose_matches_torch_coalesce():
    rng = np.random.default_rng(0)
    M, K = 300, 200
    full, rowptr, col, nf = random_csr(M, K, powerlaw_lens(M, 20, 1.4, rng, K), rng)
    col, val = O.build_operand(full, rowptr, col, nf)
    rows = np.repeat(np.arange(M), np.diff(rowptr))
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, col])), torch.from_numpy(val), (M, K)).coalesce()
    At = A.t().coalesce()
    trp, trc, trv = O.csr_transpose(rowptr, col, val, K)
    trows = np.repeat(np.arange(K), np.diff(trp))
    assert np.array_equal(np.stack([trows, trc]), At.indices().numpy())
    assert np.array_equal(trv, At.values().numpy())


def test_f32_oracle_error_bound():
    """fp32 CSR-order sums stay within 1e-5 relative of fp64 w.r.t. sum |a||x|."""
    rng = np.random.default_rng(1)
    M, K, F = 200, 400, 64
    full, rowptr, col, nf = random_csr(M, K, powerlaw_lens(M, 150, 1.0, rng, K), rng)
    col, val = O.build_operand(full, rowptr, col, nf)
    X = rng.standard_normal((K, F)).astype(np.float32)
    y32 = O.spmm_f32(rowptr, col, val, X)
    y64 = O.spmm_f64(rowptr, col, val, X)
    scale = O.spmm_abs(rowptr, col, val, X)
    assert np.max(np.abs(y32 - y64) / np.maximum(scale, 1e-30)) < 1e-5


def test_gather_rows_oracle():
    rng = np.random.default_rng(2)
    src = rng.standard_normal((50, 7)).astype(np.float32)
    si = rng.integers(0, 50, 20)
    di = rng.permutation(30)[:20]
    dst = np.zeros((30, 7), np.float32)
    O.gather_rows(src, si, dst, di)
    ref = np.zeros_like(dst)
    ref[di] = src[si]
    assert np.array_equal(dst, ref)
