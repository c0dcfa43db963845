"""The PyTorch-ROCm extension (gnn_amd/csrc/spmm_ext.cpp): the reference's native module `spmm`
(spmm_cpp/spmm.cpp:52-56, loaded by custom_sparse_ops.py:8) and the registered operators
torch.ops.gnn.* (fake kernels + autograd from gnn_amd/torch_ops.py).

CPU: the module imports as `spmm` with the reference's three functions; the operators' schemas
and fake (shape) kernels; the reference's TORCH_CHECK messages (spmm.cpp:10-21).
GPU: `spmm.spmm_load_balance` / `spmm_naive` / `create_coo_tensor` against the C oracle (operand
values bit-exact; aggregation within the module tolerance), torch.ops.gnn.spmm forward + backward
against the oracle (backward = Aᵀ·G, custom_sparse_ops.py:33-37), and a function using the op
compiled with torch.compile(fullgraph=True) (dynamo + AOTAutograd trace the op through its fake
kernel and autograd formula) equal to eager, outputs and gradients.
"""
import numpy as np
import pytest
import torch

import oracle as O
from gnn_amd import torch_ops
from oracle.fixtures import random_csr

RTOL = ATOL = 1e-5  # the aggregation tolerance of every parity test


def test_module_and_ops_registered():
    mod = torch_ops.load()
    assert mod.__name__ == "spmm"
    for name in ("spmm_load_balance", "spmm_naive", "create_coo_tensor"):
        assert callable(getattr(mod, name))
    for op in ("spmm", "spmm_csr", "csr_transpose"):
        assert hasattr(torch.ops.gnn, op)
    s = str(torch.ops.gnn.spmm.default._schema)
    assert s.startswith("gnn::spmm(Tensor rowptr, Tensor col, Tensor val, Tensor t_rowptr")


def test_fake_kernels_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    torch_ops.load()
    with FakeTensorMode():
        rp = torch.empty(11, dtype=torch.int32, device="cuda")
        c = torch.empty(30, dtype=torch.int32, device="cuda")
        v = torch.empty(30, device="cuda")
        x = torch.empty(7, 5, device="cuda")
        y = torch.ops.gnn.spmm(rp, c, v, rp, c, v, 10, 7, x)
        assert tuple(y.shape) == (10, 5) and y.dtype == torch.float32
        t = torch.ops.gnn.csr_transpose(rp, c, v, 10, 7)
        assert [tuple(a.shape) for a in t] == [(8,), (30,), (30,)]


def test_reference_error_messages():
    mod = torch_ops.load()
    A = torch.eye(3).to_sparse()
    with pytest.raises(RuntimeError, match="sparseMat must be a CUDA tensor"):
        mod.spmm_load_balance(A, torch.zeros(3, 2))
    with pytest.raises(RuntimeError, match="must be CUDA tensors"):
        mod.create_coo_tensor(torch.zeros(4, dtype=torch.int32), torch.zeros(4, dtype=torch.int32),
                              torch.zeros(0, dtype=torch.int16), torch.zeros(3), 3, 3)


def _case(seed, M=300, K=500, F=602):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 120, M)
    lens[5] = 0
    lens[9] = K  # a dense row: cut across work units
    full, rowptr, col, normfact = random_csr(M, K, lens, rng)
    X = rng.standard_normal((K, F)).astype(np.float32)
    G = rng.standard_normal((M, F)).astype(np.float32)
    return full, rowptr, col, normfact, X, G


@pytest.mark.gpu
def test_module_functions_vs_oracle(dev):
    mod = torch_ops.load()
    full, rowptr, col, normfact, X, _ = _case(1)
    M, K = len(rowptr) - 1, X.shape[0]
    t = lambda a: torch.from_numpy(a).to(dev)
    A = mod.create_coo_tensor(t(full), t(rowptr), t(col.astype(np.int16)), t(normfact), M, K)
    assert A.is_sparse and A.is_coalesced() and tuple(A.shape) == (M, K)
    ocol, oval = O.build_operand(full, rowptr, col, normfact)
    idx = A._indices().cpu().numpy()
    assert np.array_equal(idx[1], ocol) and np.array_equal(np.diff(np.searchsorted(idx[0], np.arange(M + 1))),
                                                           np.diff(rowptr))
    assert np.array_equal(A._values().cpu().numpy().view(np.uint32), oval.view(np.uint32)), "values bit-exact"
    want = O.spmm_f32(rowptr, ocol, oval, X)
    for fn in (mod.spmm_load_balance, mod.spmm_naive):
        Y = fn(A, t(X))
        torch.cuda.synchronize()
        np.testing.assert_allclose(Y.cpu().numpy(), want, rtol=RTOL, atol=ATOL)
    with pytest.raises(RuntimeError, match="denseMat must be contiguous"):
        mod.spmm_load_balance(A, t(np.ascontiguousarray(X.T)).T)
    with pytest.raises(RuntimeError, match="sparseMat must be coalesced"):
        B = torch.sparse_coo_tensor(A._indices().flip(1), A._values().flip(0), A.shape)
        mod.spmm_load_balance(B, t(X))


def _csr_pieces(dev, seed):
    from gnn_amd import custom_sparse_ops as cso

    full, rowptr, col, normfact, X, G = _case(seed)
    M, K = len(rowptr) - 1, X.shape[0]
    t = lambda a: torch.from_numpy(a).to(dev)
    op, _ = cso.build_operand(t(full), t(rowptr), t(col), t(normfact), M, K, with_coo=False)
    return op, X, G, (rowptr, *O.build_operand(full, rowptr, col, normfact))


@pytest.mark.gpu
def test_registered_op_forward_backward_vs_oracle(dev):
    torch_ops.load()
    op, X, G, (rowptr, ocol, oval) = _csr_pieces(dev, 2)
    M, K = op.shape
    Xd = torch.from_numpy(X).to(dev).requires_grad_(True)
    Y = torch_ops.spmm(op, Xd)
    Y.backward(torch.from_numpy(G).to(dev))
    torch.cuda.synchronize()
    np.testing.assert_allclose(Y.detach().cpu().numpy(), O.spmm_f32(rowptr, ocol, oval, X), rtol=RTOL, atol=ATOL)
    trp, trc, trv = O.csr_transpose(rowptr, ocol, oval, K)
    np.testing.assert_allclose(Xd.grad.cpu().numpy(), O.spmm_f32(trp, trc, trv, G), rtol=RTOL, atol=ATOL)
    # the operator's own transpose is the canonical one, bit for bit
    r, c, v = torch.ops.gnn.csr_transpose(op.rowptr, op.col, op.val, M, K)
    assert np.array_equal(r.cpu().numpy(), trp) and np.array_equal(c.cpu().numpy(), trc)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), trv.view(np.uint32))


@pytest.mark.gpu
def test_torch_compile_traces_the_op(dev):
    torch_ops.load()
    op, X, G, _ = _csr_pieces(dev, 3)
    t = op.transpose()
    M, K = op.shape
    W = torch.randn(X.shape[1], 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0))

    def layer(x, w):  # GraphSAGE-like: aggregate, project, activate
        h = torch.ops.gnn.spmm(op.rowptr, op.col, op.val, t.rowptr, t.col, t.val, M, K, x)
        return torch.nn.functional.elu(h @ w)

    compiled = torch.compile(layer, backend="aot_eager", fullgraph=True)
    outs = []
    for fn in (layer, compiled):
        x = torch.from_numpy(X).to(dev).requires_grad_(True)
        w = W.clone().requires_grad_(True)
        y = fn(x, w)
        y.sum().backward()
        torch.cuda.synchronize()
        outs.append((y.detach(), x.grad, w.grad))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_module_in_the_reference_autograd_pattern(dev):
    """The reference's SparseDenseMM (custom_sparse_ops.py:16-37) unchanged but for the module
    object: forward spmm_load_balance(A, X), backward spmm_load_balance on A.transpose(0,1)
    .coalesce() — a foreign coalesced COO the module has never seen (no cached CSR)."""
    mod = torch_ops.load()

    class RefSparseDenseMM(torch.autograd.Function):
        @staticmethod
        def forward(ctx, mat1, mat2):
            ctx.save_for_backward(mat1)
            return mod.spmm_load_balance(mat1, mat2)

        @staticmethod
        def backward(ctx, grad_output):
            mat1, = ctx.saved_tensors
            return None, mod.spmm_load_balance(mat1.transpose(0, 1).coalesce(), grad_output.contiguous())

    full, rowptr, col, normfact, X, G = _case(4)
    M, K = len(rowptr) - 1, X.shape[0]
    t = lambda a: torch.from_numpy(a).to(dev)
    A = mod.create_coo_tensor(t(full), t(rowptr), t(col.astype(np.int16)), t(normfact), M, K)
    Xd = t(X).requires_grad_(True)
    Y = RefSparseDenseMM.apply(A, Xd)
    Y.backward(t(G))
    torch.cuda.synchronize()
    ocol, oval = O.build_operand(full, rowptr, col, normfact)
    np.testing.assert_allclose(Y.detach().cpu().numpy(), O.spmm_f32(rowptr, ocol, oval, X), rtol=RTOL, atol=ATOL)
    trp, trc, trv = O.csr_transpose(rowptr, ocol, oval, K)
    np.testing.assert_allclose(Xd.grad.cpu().numpy(), O.spmm_f32(trp, trc, trv, G), rtol=RTOL, atol=ATOL)


@pytest.mark.gpu
def test_module_create_coo_tensor_sums_duplicate_columns(dev):
    from oracle.fixtures import coalesced_reference, duplicate_columns_case

    mod = torch_ops.load()
    M, K, full, rowptr, col, nf = duplicate_columns_case()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    A = mod.create_coo_tensor(t(full), t(rowptr), t(col.astype(np.int32)), t(nf), M, K)
    ref = coalesced_reference(M, K, full, rowptr, col, nf)
    assert A.is_coalesced()
    X = torch.randn(K, 40, device=dev)
    Y = mod.spmm_load_balance(A, X)  # the first aggregation merges the flagged repeat in place
    assert A._nnz() == 10
    assert torch.equal(A._indices().cpu(), ref._indices())
    np.testing.assert_allclose(A._values().cpu().numpy(), ref._values().numpy(), rtol=1e-6)
    np.testing.assert_allclose(Y.cpu().numpy(), torch.sparse.mm(ref, X.cpu()).numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_module_create_coo_tensor_graph_capture(dev):
    """The module's create_coo_tensor reads nothing back (no duplicate check on the host): it
    captures into a HIP graph and the replay builds the reference's values bit for bit."""
    import oracle as O
    from oracle.fixtures import random_csr

    mod = torch_ops.load()
    rng = np.random.default_rng(12)
    M, K = 150, 260
    full, rowptr, col, nf = random_csr(M, K, rng.integers(0, 30, M), rng)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ins = (t(full), t(rowptr), t(col.astype(np.int16)), t(nf))
    mod.create_coo_tensor(*ins, M, K)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        A = mod.create_coo_tensor(*ins, M, K)
    g.replay()
    torch.cuda.synchronize()
    ocol, oval = O.build_operand(full, rowptr, col, nf)
    assert np.array_equal(A._indices()[1].cpu().numpy(), ocol)
    assert np.array_equal(A._values().cpu().numpy(), oval)


@pytest.mark.gpu
def test_module_uses_the_builders_csr(dev):
    """create_coo_tensor keeps the CSR its builder made on the tensor (no per-call
    COO->CSR in spmm_load_balance); the result equals the per-call COO->CSR path on a plain torch
    COO tensor with the same entries bit for bit, and a coalesce that merges duplicates drops it."""
    mod = torch_ops.load()
    full, rowptr, col, normfact, X, _ = _case(4)
    M, K = len(rowptr) - 1, X.shape[0]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    A = mod.create_coo_tensor(t(full), t(rowptr), t(col.astype(np.int32)), t(normfact), M, K)
    assert hasattr(A, "_gnn_ext_csr")
    plain = torch.sparse_coo_tensor(A._indices(), A._values(), A.shape, is_coalesced=True)
    Xd = t(X)
    assert torch.equal(mod.spmm_load_balance(A, Xd), mod.spmm_load_balance(plain, Xd))
    from oracle.fixtures import coalesced_reference, duplicate_columns_case

    M2, K2, full2, rowptr2, col2, nf2 = duplicate_columns_case()
    B = mod.create_coo_tensor(t(full2), t(rowptr2), t(col2.astype(np.int32)), t(nf2), M2, K2)
    X2 = torch.randn(K2, 16, device=dev)
    ref = coalesced_reference(M2, K2, full2, rowptr2, col2, nf2)
    np.testing.assert_allclose(mod.spmm_load_balance(B, X2).cpu().numpy(), torch.sparse.mm(ref, X2.cpu()).numpy(),
                               rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_module_reference_pattern_at_config2_size(dev):
    """The reference's SparseDenseMM pattern through `import spmm` at BASELINE config-2 sizes
    (bench.py's `dropin` shapes): forward spmm_load_balance(A, X) on the module's create_coo_tensor
    (15.8 k x 22.2 k, ~1.8 M nonzeros, contiguous F = 602) and backward
    spmm_load_balance(A.transpose(0, 1).coalesce(), G) (A 8.7 k x 15.8 k, ~0.86 M nonzeros,
    F = 1024) against the C oracle, rtol / atol 1e-5."""
    from tests.test_spmm_gpu import _config2_operand

    mod = torch_ops.load()
    rng = np.random.default_rng(77)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    M, K, F = 15809, 22176, 602
    full, rowptr, col, nf = _config2_operand(M, K, 1.81e6, rng)
    A = mod.create_coo_tensor(t(full), t(rowptr), t(col), t(nf), M, K)
    ocol, oval = O.build_operand(full, rowptr, col, nf)
    X = rng.standard_normal((K, F)).astype(np.float32)
    Y = mod.spmm_load_balance(A, t(X))
    np.testing.assert_allclose(Y.cpu().numpy(), O.spmm_f32(rowptr, ocol, oval, X), rtol=RTOL, atol=ATOL)
    M1, K1, F1 = 8689, 15809, 1024
    full, rowptr, col, nf = _config2_operand(M1, K1, 0.86e6, rng)
    A1 = mod.create_coo_tensor(t(full), t(rowptr), t(col), t(nf), M1, K1)
    ocol, oval = O.build_operand(full, rowptr, col, nf)
    G = rng.standard_normal((M1, F1)).astype(np.float32)
    dX = mod.spmm_load_balance(A1.transpose(0, 1).coalesce(), t(G))
    trp, trc, trv = O.csr_transpose(rowptr, ocol, oval, K1)
    # 16 M outputs summed in a different order from the oracle's: a cancelling row can leave 1e-5
    # absolute by plain fp32 rounding, so each output is held to rtol 1e-5 of its summation scale
    # |A|·|G| (the forward error bound of a sum) as well as to atol 1e-5 everywhere but such rows.
    got, want = dX.cpu().numpy(), O.spmm_f32(trp, trc, trv, G)
    scale = O.spmm_f32(trp, trc, np.abs(trv), np.abs(G))
    err = np.abs(got - want)
    assert bool((err <= RTOL * scale + ATOL).all())
    assert np.count_nonzero(err > RTOL * np.abs(want) + ATOL) <= 16
