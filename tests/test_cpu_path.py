"""CPU: BASELINE config 1 — the product's CPU device branch (custom_sparse_ops.py:25,36:
torch.sparse.mm forward, A.t().coalesce() backward; create_coo_tensor's formula in torch)
against the goldens the reference itself produced (tests/golden/make_golden.py). Nothing
here imports oracle/: the checks are against the committed reference outputs only.

Tolerances: operands (indices and values) bit-exact; aggregation outputs bit-exact (the
same torch.sparse.mm call the reference makes on the same inputs); the training step
rtol 1e-5 (the same CPU kernels, so in practice exact)."""
import numpy as np
import pytest
import torch

from gnn_amd import custom_sparse_ops as cso
from gnn_amd.models import build_model, loss


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


@pytest.mark.parametrize("case", [0, 1, 2, 3])
def test_create_coo_tensor_cpu_matches_reference(golden, case):
    """Every create_coo_tensor call the reference's ladies_sampler made (c0/c1: samp 512,
    batch 128 — config 1's geometry on the tiny graph) rebuilt by the CPU branch."""
    z = golden("ladies_tiny.npz")
    p = f"c{case}_"
    calls = sorted({k.split("_")[1] for k in z.files if k.startswith(p + "call")})
    assert len(calls) == 3
    for li, call in enumerate(calls):
        a = cso.create_coo_tensor(*(_t(z[f"{p}{call}_{k}"]) for k in ("fullrowptr", "rowptr", "colidx", "normfact")),
                                  *(int(v) for v in z[f"{p}{call}_shape"]))
        assert a.is_coalesced() and a.device.type == "cpu"
        bl = 2 - li  # calls are top-down, adjs bottom-up
        assert np.array_equal(a.indices().numpy(), z[f"{p}adj{bl}_indices"])
        assert np.array_equal(a.values().numpy(), z[f"{p}adj{bl}_values"])


def test_spmm_cpu_matches_reference_goldens(golden):
    z = golden("ladies_tiny.npz")
    sm = golden("spmm_tiny.npz")
    for li in range(3):
        a = torch.sparse_coo_tensor(_t(z[f"c2_adj{li}_indices"]), _t(z[f"c2_adj{li}_values"]),
                                    tuple(int(v) for v in z[f"c2_adj{li}_shape"])).coalesce()
        for F in (1, 26, 64, 100, 602):
            g = torch.Generator().manual_seed(1000 * li + F)
            X = torch.randn(a.shape[1], F, generator=g)
            G = torch.randn(a.shape[0], F, generator=g)
            Xr = X.clone().requires_grad_(True)
            Y = cso.spmm(a, Xr)
            Y.backward(G)
            assert np.array_equal(Y.detach().numpy(), sm[f"l{li}_F{F}_Y"])
            assert np.array_equal(Xr.grad.numpy(), sm[f"l{li}_F{F}_dX"])


def test_cpu_branch_does_not_swallow_device_errors():
    a = torch.sparse_coo_tensor(torch.tensor([[0, 1], [1, 0]]), torch.ones(2), (2, 2)).coalesce()
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        cso.spmm_load_balance(a, torch.ones(2, 3))  # the native entry point stays CUDA-only
    dense = torch.ones(2, 3)
    assert torch.equal(cso.spmm(a, dense), torch.sparse.mm(a, dense))


@pytest.mark.parametrize("name", ["graphsage", "gcn"])
def test_cpu_training_step_matches_reference(golden, name):
    """One GraphSAGE/GCN training step through the product's CPU branch (unfused modules,
    cso.spmm on CPU tensors) reproduces the reference's seeded step: logits, loss, gradients
    and the post-Adam weights."""
    st = golden("model_step_tiny.npz")
    z = golden("ladies_tiny.npz")
    adjs = [torch.sparse_coo_tensor(_t(z[f"c2_adj{li}_indices"]), _t(z[f"c2_adj{li}_values"]),
                                    tuple(int(v) for v in z[f"c2_adj{li}_shape"])).coalesce() for li in range(3)]
    sampled = [_t(z[f"c2_sampled{li}"]) for li in range(3)]
    g = torch.Generator().manual_seed(77)
    x0 = torch.randn(int(z["c2_nin"]), 602, generator=g)
    y = _t(z["c2_labels"])
    torch.manual_seed(0)
    net = build_model(name, 602, 32, [1, 1, 1], 41, dropout=0.1)
    net.eval()
    opt = torch.optim.Adam(net.parameters(), lr=0.01)
    out = net(x0, adjs, sampled)
    lo = loss(out, y, True, "cpu")
    lo.backward()
    np.testing.assert_allclose(out.detach().numpy(), st[f"{name}_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(lo), float(st[f"{name}_loss"]), rtol=1e-6)
    for pname, prm in net.named_parameters():
        np.testing.assert_allclose(prm.grad.numpy(), st[f"{name}_grad_{pname}"], rtol=1e-5, atol=1e-7, err_msg=pname)
    torch.nn.utils.clip_grad_norm_(net.parameters(), 5)
    opt.step()
    for pname, prm in net.named_parameters():
        np.testing.assert_allclose(prm.detach().numpy(), st[f"{name}_step_{pname}"], rtol=1e-5, atol=1e-6,
                                   err_msg=pname)
