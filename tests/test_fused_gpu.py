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


def _assert_rel_l2(got, ref, what, tol=1e-5):
    """Norm-wise gradient check beside the elementwise one (rtol 2e-3 elementwise is
    needed only for entries that cancel to near zero): ||got - ref|| <= tol * ||ref||."""
    g = got.detach().cpu().double().numpy()
    r = np.asarray(ref, dtype=np.float64)
    rel = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30))
    assert rel <= tol, f"{what}: relative L2 error {rel:.2e} > {tol:.0e}"


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
        _assert_rel_l2(prm.grad, st[f"{name}_grad_{pname}"], pname)
    torch.nn.utils.clip_grad_norm_(net.parameters(), 5)
    opt.step()
    # Adam's first step moves every weight by ~lr * sign(grad): compare where the golden
    # gradient is clearly non-zero (its sign is then the same on both sides).
    for pname, prm in net.named_parameters():
        g = st[f"{name}_grad_{pname}"]
        sure = np.abs(g) > 1e-5 * max(np.abs(g).max(), 1e-12)
        got = prm.detach().cpu().numpy()
        np.testing.assert_allclose(got[sure], st[f"{name}_step_{pname}"][sure], rtol=1e-4, atol=1e-5, err_msg=pname)


def _head_ref(x, W, b, y, mask=None, p=0.0):
    """GNN's tail (models.py:90-97) + utils.loss (utils.py:129-140) in torch; `mask` replaces
    the dropout draw (1 kept / 0 dropped)."""
    h = F.normalize(x, p=2, dim=1)
    if mask is not None:
        h = h * mask / (1 - p)
    z = F.linear(h, W, b)
    return loss(z, y, True, x.device), z


@pytest.mark.parametrize("M,D,C", [(512, 1024, 41), (37, 512, 41), (1, 64, 3), (100, 2048, 64), (5, 4, 1),
                                   (512, 1024, 172), (33, 2048, 256), (7, 512, 65)])
def test_head_bce_matches_torch(dev, M, D, C):
    """Fused head + BCE (gnn_head_bce_*), eval mode, against an fp64 torch evaluation:
    rtol 1e-4 / atol 1e-5 (row reductions of up to 2048 terms in another order)."""
    from gnn_amd.fused import head_bce_loss

    g = torch.Generator().manual_seed(M * 7 + D + C)
    x = torch.randn(M, D, generator=g)
    x[0] *= 1e-3
    if M > 3:
        x[3] = 0.0  # a zero row: the norm is clamped to 1e-12
    W = torch.randn(C, D, generator=g) * 0.1
    b = torch.randn(C, generator=g)
    y = (torch.rand(M, C, generator=g) < 0.3).float()
    leaves64 = [t.double().requires_grad_(True) for t in (x, W, b)]
    l64, z64 = _head_ref(*leaves64, y.double())
    l64.backward()
    leaves = [t.to(dev).requires_grad_(True) for t in (x, W, b)]
    lo, z = head_bce_loss(*leaves, y.to(dev), p=0.1, training=False)
    lo.backward()
    np.testing.assert_allclose(z.cpu().numpy(), z64.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(lo), float(l64), rtol=1e-5)
    for a, r in zip(leaves[1:], leaves64[1:]):
        np.testing.assert_allclose(a.grad.cpu().numpy(), r.grad.numpy(), rtol=1e-4, atol=1e-5)
    # d(x) = (d(xn) - xn (xn · d(xn))) / ||x||: the projection cancels, so the error scales
    # with the row's gradient magnitude — tolerance per row
    got, ref = leaves[0].grad.cpu().double().numpy(), leaves64[0].grad.numpy()
    rowmax = np.abs(ref).max(axis=1, keepdims=True)
    assert np.all(np.abs(got - ref) <= 1e-4 * np.abs(ref) + 1e-5 * np.maximum(rowmax, 1.0))


def test_head_bce_dropout(dev):
    """Training mode: the mask the forward drew (read back from the stored dropout output)
    reproduces the loss, and the backward regenerates the same mask."""
    from gnn_amd import _lib

    M, D, C, p = 512, 1024, 41, 0.1
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, D, generator=g).to(dev)
    W = (torch.randn(C, D, generator=g) * 0.1).to(dev)
    b = torch.randn(C, generator=g).to(dev)
    y = (torch.rand(M, C, generator=g) < 0.3).float().to(dev)
    xd = torch.empty(M, D, device=dev)
    z = torch.empty(M, C, device=dev)
    nrm = torch.empty(M, device=dev)
    rl = torch.empty(M, device=dev)
    lo = torch.empty((), device=dev)
    st = _lib.stream_of(dev)
    L = _lib.lib()
    _lib.check(L.gnn_head_bce_fwd_f32(x.data_ptr(), D, M, D, W.data_ptr(), b.data_ptr(), C, y.data_ptr(), C, p, 1234,
                                      1, xd.data_ptr(), z.data_ptr(), nrm.data_ptr(), rl.data_ptr(), lo.data_ptr(),
                                      st), "fwd")
    gl = torch.full((), 2.0, device=dev)
    dz = torch.empty(M, C, device=dev)
    dx = torch.empty(M, D, device=dev)
    _lib.check(L.gnn_head_bce_bwd_f32(x.data_ptr(), D, M, D, W.data_ptr(), C, y.data_ptr(), C, gl.data_ptr(), p, 1234,
                                      1, z.data_ptr(), nrm.data_ptr(), dz.data_ptr(), dx.data_ptr(), D, st), "bwd")
    torch.cuda.synchronize()
    mask = (xd != 0).float()
    assert abs(mask.mean().item() - (1 - p)) < 0.005
    xr = x.clone().requires_grad_(True)
    lr, zr = _head_ref(xr, W, b, y, mask, p)
    (2.0 * lr).backward()
    torch.testing.assert_close(xd, F.normalize(x, dim=1) * mask / (1 - p), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(z, zr, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(lo, lr.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dx, xr.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", ["graphsage", "gcn"])
def test_gpu_forward_loss_matches_reference(dev, golden, name):
    """GNN.forward_loss (fused encoder + fused head/BCE) reproduces the reference's seeded
    CPU step: loss, logits and every parameter gradient (eval mode)."""
    st = golden("model_step_tiny.npz")
    adjs, sampled, x0, y = _golden_inputs(golden, dev)
    torch.manual_seed(0)
    net = build_model(name, 602, 32, [1, 1, 1], 41, dropout=0.1, fused=True).to(dev)
    net.eval()
    lo, out = net.forward_loss(x0, adjs, sampled, y, True)
    lo.backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), st[f"{name}_out"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(lo), float(st[f"{name}_loss"]), rtol=1e-5)
    for pname, prm in net.named_parameters():
        np.testing.assert_allclose(prm.grad.cpu().numpy(), st[f"{name}_grad_{pname}"], rtol=2e-3, atol=1e-5,
                                   err_msg=pname)
        _assert_rel_l2(prm.grad, st[f"{name}_grad_{pname}"], pname)


def _keep_mask_ref(seed, e, p):
    """Per-element dropout keep mask of the layer tail, restated in numpy from its definition
    (sage.hip `drop4`): h = mix32(lo32(e) ^ mix32(hi32(e) ^ mix32(lo32(seed) ^ 0x9e3779b9) ^
    hi32(seed))), keep = float(h >> 8) * 2^-24 >= p."""
    def mix32(x):
        x = x.astype(np.uint64) & 0xFFFFFFFF
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        x ^= x >> 16
        return x

    e = np.asarray(e, dtype=np.uint64)
    s = mix32(np.uint64((seed & 0xFFFFFFFF) ^ 0x9E3779B9)) ^ np.uint64(seed >> 32)
    h = mix32((e & np.uint64(0xFFFFFFFF)) ^ mix32((e >> np.uint64(32)) ^ s))
    return (h >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0) >= np.float32(p)


def _tail_fwd_abi(hB, M, D, p, seed, offset_val=1.0):
    """gnn_sage_norm_fwd_f32 on hB (M x D, D2 = 0) with scale 1 and a constant offset, so every
    kept output is nonzero: returns Y."""
    from gnn_amd import _lib

    dev = hB.device
    scale = torch.ones(D, device=dev)
    offset = torch.full((D,), offset_val, device=dev)
    Y = torch.empty(M, D, device=dev)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    _lib.check(_lib.lib().gnn_sage_norm_fwd_f32(hB.data_ptr(), D, D, None, 0, 0, None, None, scale.data_ptr(),
                                                offset.data_ptr(), M, p, seed, 1, Y.data_ptr(), D,
                                                mean.data_ptr(), rstd.data_ptr(), _lib.stream_of(dev)),
               "gnn_sage_norm_fwd_f32")
    torch.cuda.synchronize()
    return Y


@pytest.mark.parametrize("p,seed", [(0.1, 0x123456789ABCDEF), (0.5, 7), (0.3, (1 << 63) + 12345)])
def test_dropout_mask_matches_hash_definition(dev, p, seed):
    M, D = 777, 1000
    hB = torch.randn(M, D, device=dev)
    Y = _tail_fwd_abi(hB, M, D, p, seed, offset_val=50.0)  # |normalised| << 50: kept => nonzero
    e = np.arange(M * D, dtype=np.uint64)
    ref = _keep_mask_ref(seed, e, p).reshape(M, D)
    assert np.array_equal((Y != 0).cpu().numpy(), ref)


def test_dropout_mask_past_2_32_elements(dev):
    """M * D >= 2^32 (the per-float4 hi32 path): the row holding element 2^32 straddles the
    boundary (D = 1000); its mask and its neighbours' match the definition."""
    D = 1000
    M = (1 << 32) // D + 3
    free, _ = torch.cuda.mem_get_info()
    if free < 2 * M * D * 4 + (4 << 30):
        pytest.skip("needs ~35 GB of free HBM")
    hB = torch.ones(M, D, device=dev)  # every row constant: y = offset exactly where kept
    Y = _tail_fwd_abi(hB, M, D, 0.25, 99, offset_val=1.0)
    del hB
    r0 = (1 << 32) // D - 1
    rows = Y[r0:r0 + 4].cpu().numpy()
    del Y
    e = (np.arange(r0 * D, (r0 + 4) * D, dtype=np.uint64))
    ref = _keep_mask_ref(99, e, 0.25).reshape(4, D)
    assert np.array_equal(rows != 0, ref)
    assert np.all(rows[ref] == np.float32(1.0) / np.float32(0.75))

