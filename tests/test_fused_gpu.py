"""GPU: the fused layer epilogue (gnn_layers.h) against the reference's torch expression,
and whole GraphSAGE/GCN training steps on the GPU against the reference's golden step.

Floating-point tolerance: the epilogue reduces 512-2048 values per row (mean, variance)
and 15k rows per column (d(scale), d(offset)) in a different order than torch: compared
with rtol = 1e-4, atol = 1e-5 against an fp64 evaluation of the same expression, the
same bound torch's own fp32 kernels meet (checked alongside).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gnn_amd.fused import sage_norm
from gnn_amd.models import build_model, loss

pytestmark = pytest.mark.gpu


def _ref(hB, hW, scale, offset, bB=None, bW=None):
    if bW is not None:
        hW = hW + bW
    if hB is not None and bB is not None:
        hB = hB + bB
    h = hW if hB is None else torch.cat([hB, hW], 1)
    out = F.elu(h)
    mean = out.mean(dim=1).view(out.shape[0], 1)
    var = out.var(dim=1, unbiased=False).view(out.shape[0], 1) + 1e-9
    return (out - mean) * scale * torch.rsqrt(var) + offset


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("D1,D2,M", [(512, 512, 1000), (0, 512, 777), (512, 512, 1), (256, 256, 5), (0, 100, 33),
                                     (1024, 1024, 300)])
def test_sage_norm_matches_torch(dev, D1, D2, M, bias):
    g = torch.Generator().manual_seed(D1 + D2 + M)
    hB = torch.randn(M, D1, generator=g) * 2 if D1 else None
    hW = torch.randn(M, D2, generator=g) * 2
    scale = torch.rand(D1 + D2, generator=g) + 0.5
    offset = torch.randn(D1 + D2, generator=g)
    bB = torch.randn(D1, generator=g) if (bias and D1) else None
    bW = torch.randn(D2, generator=g) if bias else None
    gY = torch.randn(M, D1 + D2, generator=g)
    # fp64 reference on the CPU
    leaves64 = [t.double().requires_grad_(True) if t is not None else None for t in (hB, hW, scale, offset, bB, bW)]
    y64 = _ref(*leaves64)
    y64.backward(gY.double())
    # fused on the GPU
    leaves = [t.to(dev).requires_grad_(True) if t is not None else None for t in (hB, hW, scale, offset, bB, bW)]
    y = sage_norm(*leaves[:4], p=0.1, training=False, biasB=leaves[4], biasW=leaves[5])
    y.backward(gY.to(dev))
    np.testing.assert_allclose(y.detach().cpu().numpy(), y64.detach().numpy(), rtol=1e-4, atol=1e-5)
    for a, b in zip(leaves, leaves64):
        if a is None:
            continue
        np.testing.assert_allclose(a.grad.cpu().numpy(), b.grad.numpy(), rtol=1e-4, atol=1e-4)


def test_sage_norm_dropout_masks(dev):
    M, D1, D2, p = 2000, 512, 512, 0.1
    torch.manual_seed(3)
    hB = torch.randn(M, D1, device=dev, requires_grad=True)
    hW = torch.randn(M, D2, device=dev, requires_grad=True)
    scale = torch.ones(D1 + D2, device=dev, requires_grad=True)
    offset = torch.full((D1 + D2,), 0.25, device=dev, requires_grad=True)
    y = sage_norm(hB, hW, scale, offset, p=p, training=True)
    ref = _ref(hB.detach(), hW.detach(), scale.detach(), offset.detach())
    kept = y != 0
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.005
    torch.testing.assert_close(y[kept], (ref / (1 - p))[kept], rtol=1e-4, atol=1e-5)
    # backward regenerates the same mask: d(offset) only sees kept elements
    y.backward(torch.ones_like(y))
    torch.testing.assert_close(offset.grad, kept.float().sum(0) / (1 - p), rtol=1e-5, atol=1e-3)
    # same seed -> same mask; torch.manual_seed makes it reproducible
    torch.manual_seed(3)
    y2 = sage_norm(hB, hW, scale, offset, p=p, training=True)
    assert torch.equal(y.detach(), y2.detach())


def test_index_rows_matches_torch(dev):
    from gnn_amd.fused import index_rows

    g = torch.Generator().manual_seed(0)
    base = torch.randn(500, 608, generator=g).to(dev)
    x = base[:, :602].requires_grad_(False).clone().requires_grad_(True)
    xv = base[:, :602]  # strided view (the staging buffer's layout)
    idx = torch.randperm(500, generator=g)[:300].to(dev)
    assert torch.equal(index_rows(xv, idx), xv[idx])
    y = index_rows(x, idx)
    gy = torch.randn(300, 602, generator=g).to(dev)
    y.backward(gy)
    ref = torch.zeros(500, 602, device=dev)
    ref[idx] = gy
    assert torch.equal(x.grad, ref)


def _golden_inputs(golden, dev):
    z = golden("ladies_tiny.npz")
    adjs = [torch.sparse_coo_tensor(torch.from_numpy(z[f"c2_adj{li}_indices"]),
                                    torch.from_numpy(z[f"c2_adj{li}_values"]),
                                    tuple(int(v) for v in z[f"c2_adj{li}_shape"])).coalesce().to(dev)
            for li in range(3)]
    sampled = [torch.from_numpy(z[f"c2_sampled{li}"]).to(dev) for li in range(3)]
    g = torch.Generator().manual_seed(77)
    x0 = torch.randn(int(z["c2_nin"]), 602, generator=g).to(dev)
    y = torch.from_numpy(z["c2_labels"]).to(dev)
    return adjs, sampled, x0, y


@pytest.mark.parametrize("name", ["graphsage", "gcn"])
@pytest.mark.parametrize("fused", [False, True])
def test_gpu_model_step_matches_reference(dev, golden, name, fused):
    """One training step on the GPU (HIP aggregation fwd/bwd, optionally the fused
    epilogue) reproduces the reference's seeded CPU step (eval mode: dropout off)."""
    st = golden("model_step_tiny.npz")
    adjs, sampled, x0, y = _golden_inputs(golden, dev)
    torch.manual_seed(0)
    net = build_model(name, 602, 32, [1, 1, 1], 41, dropout=0.1, fused=fused).to(dev)
    net.eval()
    opt = torch.optim.Adam(net.parameters(), lr=0.01)
    opt.zero_grad()
    out = net(x0, adjs, sampled)
    lo = loss(out, y, True, dev)
    lo.backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), st[f"{name}_out"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(lo), float(st[f"{name}_loss"]), rtol=1e-5)
    for pname, prm in net.named_parameters():
        np.testing.assert_allclose(prm.grad.cpu().numpy(), st[f"{name}_grad_{pname}"], rtol=2e-3, atol=1e-5,
                                   err_msg=pname)
    torch.nn.utils.clip_grad_norm_(net.parameters(), 5)
    opt.step()
    # Adam's first step moves every weight by ~lr * sign(grad): compare where the golden
    # gradient is clearly non-zero (its sign is then the same on both sides).
    for pname, prm in net.named_parameters():
        g = st[f"{name}_grad_{pname}"]
        sure = np.abs(g) > 1e-5 * max(np.abs(g).max(), 1e-12)
        got = prm.detach().cpu().numpy()
        np.testing.assert_allclose(got[sure], st[f"{name}_step_{pname}"][sure], rtol=1e-4, atol=1e-5, err_msg=pname)
