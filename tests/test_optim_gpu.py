"""GPU: gnn_amd.optim.ClipAdam (clip_grad_norm_ + Adam in two HIP launches) against
torch.nn.utils.clip_grad_norm_ + torch.optim.Adam, over several steps, with and without
clipping, and the N > 1 form (clip into the flat buffer, then plain Adam).
Tolerance: fp32 with a different norm summation order: rtol 2e-6 on the parameters."""
import pytest
import torch

from gnn_amd.optim import ClipAdam

pytestmark = pytest.mark.gpu


def _params(dev, seed, shapes):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(*s, generator=g).to(dev) for s in shapes]


SHAPES = [(512, 602), (512,), (1024,), (41, 1024), (41,), (3, 5, 7), (9000,)] + [(17,)] * 30  # > 32 tensors


@pytest.mark.parametrize("scale", [1.0, 50.0])  # grads below / above the clip norm
def test_clip_adam_matches_torch(dev, scale):
    ref = [p.clone().requires_grad_(True) for p in _params(dev, 1, SHAPES)]
    mine = [p.clone().requires_grad_(True) for p in _params(dev, 1, SHAPES)]
    opt_ref = torch.optim.Adam(ref, lr=0.01)
    opt = ClipAdam(mine, lr=0.01, max_norm=5.0)
    for step in range(4):
        grads = _params(dev, 100 + step, SHAPES)
        for p, q, g in zip(ref, mine, grads):
            p.grad = (g * scale / 40).clone()
            q.grad = (g * scale / 40).clone()
        torch.nn.utils.clip_grad_norm_(ref, 5.0)
        opt_ref.step()
        opt.step()
    torch.cuda.synchronize()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=2e-6, atol=2e-7)


def test_clip_to_flat_then_step(dev):
    ref = [p.clone().requires_grad_(True) for p in _params(dev, 2, SHAPES[:6])]
    mine = [p.clone().requires_grad_(True) for p in _params(dev, 2, SHAPES[:6])]
    opt_ref = torch.optim.Adam(ref, lr=0.003)
    opt = ClipAdam(mine, lr=0.003, max_norm=5.0)
    grads = _params(dev, 7, SHAPES[:6])
    for p, q, g in zip(ref, mine, grads):
        p.grad = g.clone()
        q.grad = g.clone()
    torch.nn.utils.clip_grad_norm_(ref, 5.0)
    opt_ref.step()
    flat = opt.clip_to_flat()
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, torch.cat([p.grad.reshape(-1) for p in ref]), rtol=2e-6, atol=1e-8)
    opt.step(clipped=True)
    torch.cuda.synchronize()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=2e-6, atol=2e-7)


def test_clip_adam_flat_views_unaligned(dev):
    """Parameters and gradients as views of one flat buffer (the executor's layout): tensors
    start at offsets that are not 16-byte aligned, so full chunks take the per-element path
    and aligned ones the float4 path; both match torch."""
    shapes = [(41,), (512, 602), (3,), (1024, 7), (9000,)]
    sizes = [int(torch.Size(s).numel()) for s in shapes]
    base = _params(dev, 5, [(sum(sizes),)])[0]
    gbase = _params(dev, 6, [(sum(sizes),)])[0] / 10

    def views(buf):
        out, off = [], 0
        for s, n in zip(shapes, sizes):
            out.append(buf[off:off + n].view(*s))
            off += n
        return out

    ref = [p.clone().requires_grad_(True) for p in views(base)]
    flat = base.clone()
    mine = [p.requires_grad_(True) for p in views(flat)]
    gflat = gbase.clone()
    for p, q, g in zip(ref, mine, views(gflat)):
        p.grad = g.clone()
        q.grad = g  # a view of gflat: unaligned where the offset is
    opt_ref = torch.optim.Adam(ref, lr=0.01)
    opt = ClipAdam(mine, lr=0.01, max_norm=5.0)
    for _ in range(3):
        torch.nn.utils.clip_grad_norm_(ref, 5.0)
        opt_ref.step()
        opt.step()
        for p, g in zip(ref, views(gbase / 10)):
            p.grad = g.clone()
        gflat.copy_(gbase / 10)
    torch.cuda.synchronize()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=2e-6, atol=2e-7)
