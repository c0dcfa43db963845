"""Fused layer epilogue of GraphSAGE / GCN (HIP, include/gnn_layers.h) as an autograd op.

``sage_norm(hB, hW, scale, offset, p, training, biasB, biasW)`` computes, per row,
    dropout_p( (elu(cat[hB + biasB, hW + biasW]) - mean) * scale * rsqrt(var + 1e-9) + offset )
which is GraphSageConvolution.forward's tail (models.py:18-25) plus the dropout that
GraphSage.forward applies to every layer output (models.py:43); with hB = None it is
GraphConvolution's (models.py:58-64, 82). One HIP pass forward, one (+ a column reduction)
backward. Dropout masks: a counter hash of (seed, element) with the seed drawn from torch's
CPU generator, so torch.manual_seed makes runs reproducible; the mask stream differs from
torch's Philox stream (same distribution).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _lib


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(dev) -> int:
    return _lib.stream_of(dev)


class SageNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hB, hW, scale, offset, biasB, biasW, p: float, training: bool, seed: int):
        for t in (hW, scale, offset) + tuple(t for t in (hB, biasB, biasW) if t is not None):
            if not t.is_cuda:
                raise RuntimeError("sage_norm: tensors must be CUDA tensors")
            if t.dtype != torch.float32:
                raise RuntimeError("sage_norm: tensors must be float32")
        hW = hW.contiguous()
        hB = hB.contiguous() if hB is not None else None
        if hB is None:
            biasB = None
        biasB = biasB.contiguous() if biasB is not None else None
        biasW = biasW.contiguous() if biasW is not None else None
        M, D2 = hW.shape
        D1 = 0 if hB is None else hB.shape[1]
        D = D1 + D2
        dev = hW.device
        scale = scale.contiguous()
        offset = offset.contiguous()
        Y = torch.empty((M, D), dtype=torch.float32, device=dev)
        mean = torch.empty(M, dtype=torch.float32, device=dev)
        rstd = torch.empty(M, dtype=torch.float32, device=dev)
        L = _lib.lib()
        _lib.check(L.gnn_sage_norm_fwd_f32(_ptr(hB), D1 or 4, D1, _ptr(hW), D2, D2, _ptr(biasB), _ptr(biasW),
                                           _ptr(scale), _ptr(offset), M, float(p), seed, int(training), _ptr(Y), D,
                                           _ptr(mean), _ptr(rstd), _stream(dev)), "gnn_sage_norm_fwd_f32")
        ctx.save_for_backward(hB, hW, scale, mean, rstd, biasB, biasW)
        ctx.cfg = (float(p), int(training), int(seed))
        return Y

    @staticmethod
    def backward(ctx, gY):
        hB, hW, scale, mean, rstd, biasB, biasW = ctx.saved_tensors
        p, training, seed = ctx.cfg
        gY = gY.contiguous()
        M, D2 = hW.shape
        D1 = 0 if hB is None else hB.shape[1]
        dev = hW.device
        dhB = torch.empty_like(hB) if hB is not None else None
        dhW = torch.empty_like(hW)
        dscale = torch.empty(D1 + D2, dtype=torch.float32, device=dev)
        doffset = torch.empty(D1 + D2, dtype=torch.float32, device=dev)
        dbB = torch.empty_like(biasB) if biasB is not None else None
        dbW = torch.empty_like(biasW) if biasW is not None else None
        L = _lib.lib()
        wsb = L.gnn_sage_norm_bwd_workspace_bytes(M, D1 + D2)
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
        _lib.check(L.gnn_sage_norm_bwd_f32(_ptr(gY), D1 + D2, _ptr(hB), D1 or 4, D1, _ptr(hW), D2, D2, _ptr(biasB),
                                           _ptr(biasW), _ptr(scale), _ptr(mean), _ptr(rstd), M, p, seed, training,
                                           _ptr(dhB), _ptr(dhW), _ptr(dscale), _ptr(doffset), _ptr(dbB), _ptr(dbW),
                                           _ptr(ws), wsb, _stream(dev)),
                   "gnn_sage_norm_bwd_f32")
        return dhB, dhW, dscale, doffset, dbB, dbW, None, None, None


class SageAggregateFn(torch.autograd.Function):
    """Both inputs of GraphSageConvolution (models.py:18-21): (A·x, x[sampled]).

    Forward: the HIP aggregation and the HIP row gather. Backward: ONE aggregation kernel
    d(x) = Aᵀ·d(A·x) + scatter(d(x[sampled])) — the scatter is fused into its row stores as a
    residual (gnn_spmm_csr_f32_ex with rmap[sampled[i]] = i), instead of zeros + scatter +
    an autograd add over the whole K x F gradient. ``sampled`` rows must be unique (they are
    positions of the previous layer's nodes, sampler.py:143)."""

    @staticmethod
    def forward(ctx, adj, x, sampled):
        from . import custom_sparse_ops as cso

        op = cso.csr_of(adj)
        feat = cso.spmm_csr(op, x, tag="fwd")
        # x[sampled] in the same row layout as A·x (padded rows for the 602-wide layer-0
        # input), so the pair of linear products runs as one batched GEMM
        F = x.shape[1]
        ld = feat.stride(0) if feat.dim() == 2 and feat.shape[0] > 1 else F
        xs = torch.empty((sampled.numel(), ld), dtype=x.dtype, device=x.device)[:, :F]
        cso.gather_rows(x, sampled, xs, None, n=sampled.numel())
        ctx.op = op
        ctx.rmap = getattr(sampled, "_gnn_rmap", None)  # precomputed by HostBatch.to_device
        ctx.save_for_backward(sampled)
        return feat, xs

    @staticmethod
    def backward(ctx, g_feat, g_xs):
        from . import custom_sparse_ops as cso

        if not ctx.needs_input_grad[1]:
            return None, None, None
        (sampled,) = ctx.saved_tensors
        op_t = ctx.op.transpose()
        K = op_t.shape[0]
        rmap = ctx.rmap
        if rmap is None or rmap.numel() != K:
            rmap = torch.full((K,), -1, dtype=torch.int32, device=sampled.device)
            rmap[sampled] = torch.arange(sampled.numel(), dtype=torch.int32, device=sampled.device)
        return None, cso.spmm_csr(op_t, g_feat.contiguous(), tag="bwd", residual=g_xs.contiguous(), rmap=rmap), None


def sage_aggregate(adj, x: torch.Tensor, sampled: torch.Tensor):
    """(A·x, x[sampled]) with the fused backward of SageAggregateFn."""
    if sampled.dtype != torch.int64 or not sampled.is_contiguous():
        sampled = sampled.long().contiguous()
    return SageAggregateFn.apply(adj, x, sampled)


def _gemm_ok(*ts) -> bool:
    """gnn_gemm_f32's operand contract: fp32 CUDA, unit column stride, even row stride,
    8-byte aligned."""
    for t in ts:
        if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1
                and (t.stride(0) % 2 == 0 or t.shape[0] <= 1) and t.data_ptr() % 8 == 0):
            return False
    return True


def _ld(t: torch.Tensor) -> int:
    return t.stride(0) if t.shape[0] > 1 else t.shape[1] + (t.shape[1] & 1)


GEMM_ALGOS = ("split3", "f32")


def gemm_algo() -> str:
    """The fp32 GEMM kernel (include/gnn_layers.h): "split3" (bf16 matrix cores on an exact
    three-way split of every operand, six products, fp32 accumulation) or "f32" (f32-input
    MFMA). GNN_GEMM_ALGO overrides the default."""
    a = os.environ.get("GNN_GEMM_ALGO", "split3")
    if a not in GEMM_ALGOS:
        raise RuntimeError(f"GNN_GEMM_ALGO must be one of {GEMM_ALGOS}, got {a!r}")
    return a


def gemm(a_kmajor: bool, b_kmajor: bool, As, Bs, M: int, N: int, K: int, algo: Optional[str] = None):
    """Batched fp32 GEMM on the matrix cores (gnn_gemm_f32 / gnn_gemm_f32_split3):
    C[b] = A[b]·B[b] with the layouts of include/gnn_layers.h; all problems share shapes and
    row strides. Returns new (M x N) tensors."""
    import ctypes

    algo = algo or gemm_algo()
    dev = As[0].device
    nb = len(As)
    Cs = [torch.empty((M, N), dtype=torch.float32, device=dev) for _ in range(nb)]
    L = _lib.lib()
    if algo == "split3":
        wsf, fn, name = L.gnn_gemm_f32_split3_workspace_bytes, L.gnn_gemm_f32_split3, "gnn_gemm_f32_split3"
    else:
        wsf, fn, name = L.gnn_gemm_f32_workspace_bytes, L.gnn_gemm_f32, "gnn_gemm_f32"
    wsb = wsf(M, N, K, nb)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev) if wsb else None
    arr = lambda ts: (ctypes.c_void_p * nb)(*[t.data_ptr() for t in ts])
    _lib.check(fn(int(a_kmajor), int(b_kmajor), M, N, K, nb, arr(As), _ld(As[0]), arr(Bs), _ld(Bs[0]),
                  arr(Cs), N, _ptr(ws), wsb, _stream(dev)), name)
    return Cs


_GEMM_SLOTS = 512  # workgroup slots of the MFMA kernel (2 per CU, 256 CUs): gemm.hip SLOTS


def _mfma_fills(M: int, N: int, nb: int) -> bool:
    """Whether our GEMM takes an unsplit (M x N) x nb product. split3 does when the tiles
    cover the CUs: it beats the vendor GEMM on every such layer shape (scripts/gemm_bench.py:
    116-150 µs per pair against 160-256). The f32-input kernel only when it fills its
    workgroup rounds (>= 90 %):
    measured, it beats the vendor GEMM when it does (15.8k x 602 -> 512 pair: 175 vs 189 µs)
    and loses when a last round runs half empty (8.7k x 1024 -> 512 pair: 202 vs 171 µs)."""
    tiles = -(-M // 128) * -(-N // 128) * nb
    if gemm_algo() == "split3":
        # at least one 128 x 128 tile per CU: the layer-2 products (512 rows: 32-64 tiles)
        # run 22-31 µs here against ~10 µs in the vendor's small-tile kernels
        return tiles >= 256
    rounds = -(-tiles // _GEMM_SLOTS)
    return tiles >= 0.9 * rounds * _GEMM_SLOTS


def _same_layout(ts) -> bool:
    return all(t.shape == ts[0].shape and t.stride() == ts[0].stride() for t in ts)


class LinearPairFn(torch.autograd.Function):
    """y_i = x_i·W_iᵀ for the (x, W) pairs of one layer (GraphSAGE: linearB(x[sampled]) and
    linearW(A·x); GCN: one pair), bias-free (the biases live in the fused epilogue). The
    products run as fp32 MFMA GEMMs (gemm.hip), the pairs batched into one launch: always
    the weight gradients G_iᵀ·x_i (split over the sampled rows), and the forward / input
    gradients when their tiles fill the chip (else rocBLAS through torch, which wins those
    shapes). Same math as F.linear; operands outside the kernel's contract run through torch."""

    @staticmethod
    def forward(ctx, n, *args):
        xs, Ws = list(args[:n]), list(args[n:])
        ctx.n = n
        ctx.save_for_backward(*xs, *Ws)
        M, K = xs[0].shape
        N = Ws[0].shape[0]
        if _gemm_ok(*xs, *Ws) and _same_layout(xs) and _same_layout(Ws) and _mfma_fills(M, N, n):
            return tuple(gemm(False, False, xs, Ws, M, N, K))
        return tuple(torch.mm(x, W.t()) for x, W in zip(xs, Ws))

    @staticmethod
    def backward(ctx, *gs):
        n = ctx.n
        saved = ctx.saved_tensors
        xs, Ws = list(saved[:n]), list(saved[n:])
        gs = [g.contiguous() for g in gs]
        M, K = xs[0].shape
        N = Ws[0].shape[0]
        ok = _gemm_ok(*xs, *Ws, *gs) and _same_layout(xs) and _same_layout(Ws)
        dxs = [None] * n
        if any(ctx.needs_input_grad[1:1 + n]):
            if ok and _mfma_fills(M, K, n):
                dxs = gemm(False, True, gs, Ws, M, K, N)
            else:
                dxs = [torch.mm(g, W) for g, W in zip(gs, Ws)]
        dWs = [None] * n
        if any(ctx.needs_input_grad[1 + n:]):
            # split over the sampled rows (gemm.hip pick_splits); split3 from 2048 rows (the
            # layer-2 weight gradient, 512 rows: 19 + 5 µs here vs ~7 µs in the vendor GEMM)
            if ok and ((gemm_algo() == "split3" and M >= 2048) or (gemm_algo() == "f32" and K % 128)):
                # Measured (scripts/gemm_sweep.py, in the step): for 602 features the vendor
                # kernels run at 66 TF/s (145 µs per product) against 95 µs here; for the
                # 1024-wide layers hipBLASLt's tiles fit exactly and it is faster (79 vs 93 µs).
                dWs = gemm(True, True, gs, xs, N, K, M)
            elif gemm_algo() == "split3":
                # small products on torch's default BLAS: switching the preferred library per
                # call cost ~0.5 ms of host time per step (host-issue bound steps, measured)
                dWs = [torch.mm(g.t(), x) for g, x in zip(gs, xs)]
            else:
                with _BlasLibrary("cublaslt"):
                    dWs = [torch.mm(g.t(), x) for g, x in zip(gs, xs)]
        return (None, *dxs, *dWs)


def linear_pair(xs, Ws):
    """(x_i·W_iᵀ for each pair) — see LinearPairFn."""
    if xs[0].is_cuda:
        return LinearPairFn.apply(len(xs), *xs, *Ws)
    return tuple(torch.nn.functional.linear(x, W) for x, W in zip(xs, Ws))


class _BlasLibrary:
    """Route the GEMMs issued inside the block to one BLAS backend ("cublas" = rocBLAS,
    "cublaslt" = hipBLASLt on ROCm builds of torch); restores the previous choice."""

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        self.prev = torch.backends.cuda.preferred_blas_library()
        torch.backends.cuda.preferred_blas_library(self.name)

    def __exit__(self, *exc):
        torch.backends.cuda.preferred_blas_library(self.prev)
        return False


class LinearNoBiasFn(torch.autograd.Function):
    """y = x·Wᵀ (the bias lives in the fused epilogue). Same math as F.linear; the backward
    picks the BLAS backend per GEMM from measurements on MI355X (scripts/gemm_layouts.py):
    the weight gradient Gᵀ·X (a long reduction over the sampled rows) runs 1.7-1.9x faster
    on hipBLASLt than on rocBLAS at these shapes, while rocBLAS wins the forward / input
    gradient."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return torch.mm(x, W.t())

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        dx = torch.mm(g, W) if ctx.needs_input_grad[0] else None
        dW = None
        if ctx.needs_input_grad[1]:
            with _BlasLibrary("cublaslt"):
                dW = torch.mm(g.t(), x)
        return dx, dW


def linear_nobias(x: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    if x.is_cuda:
        return LinearNoBiasFn.apply(x, W)
    return torch.nn.functional.linear(x, W)


class IndexRowsFn(torch.autograd.Function):
    """x[idx] for UNIQUE row indices (sampled_nodes: positions of the previous layer's nodes
    among the sampled ones, sampler.py:143). Forward: HIP row gather (reads strided rows in
    place). Backward: zeros + one HIP row scatter — no index sort, which torch's generic
    index backward needs because it must allow repeated indices."""

    @staticmethod
    def forward(ctx, x, idx):
        from . import custom_sparse_ops as cso

        out = torch.empty((idx.numel(), x.shape[1]), dtype=x.dtype, device=x.device)
        cso.gather_rows(x, idx, out, None, n=idx.numel())
        ctx.save_for_backward(idx)
        ctx.n = x.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        from . import custom_sparse_ops as cso

        (idx,) = ctx.saved_tensors
        gx = torch.zeros((ctx.n, g.shape[1]), dtype=g.dtype, device=g.device)
        cso.gather_rows(g.contiguous(), None, gx, idx, n=idx.numel())
        return gx, None


def index_rows(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    if idx.dtype != torch.int64 or not idx.is_contiguous():
        idx = idx.long().contiguous()
    return IndexRowsFn.apply(x, idx)


def sage_norm(hB: Optional[torch.Tensor], hW: torch.Tensor, scale: torch.Tensor, offset: torch.Tensor,
              p: float = 0.0, training: bool = False, biasB: Optional[torch.Tensor] = None,
              biasW: Optional[torch.Tensor] = None) -> torch.Tensor:
    """hB / hW are the bias-free linear outputs; the linear biases (optional) are added, and
    their gradients reduced, inside the fused kernels."""
    seed = int(torch.randint(0, 2**62, (1,)).item()) if (training and p > 0) else 0
    return SageNormFn.apply(hB, hW, scale, offset, biasB, biasW, float(p), bool(training and p > 0), seed)


class HeadBCEFn(torch.autograd.Function):
    """GNN's head and loss (models.py:90-97 + utils.py:129-140, sigmoid_loss):
    BCEWithLogits(linear(dropout(normalize(x))), labels, weight 1/M, "sum") in one HIP pass
    (gnn_head_bce_fwd_f32) + a fixed-order row sum; backward one HIP pass for dx and dz, then
    dW = dzᵀ·xd (C x D, a small GEMM) and db = Σ_rows dz. Returns (loss, logits)."""

    @staticmethod
    def forward(ctx, x, W, b, labels, p: float, training: bool, seed: int):
        M, D = x.shape
        C = W.shape[0]
        dev = x.device
        W = W.contiguous()
        b = b.contiguous() if b is not None else None
        labels = labels if (labels.dim() == 2 and labels.stride(1) == 1) else labels.contiguous()
        if labels.dtype != torch.float32:
            labels = labels.float()
        xd = torch.empty((M, D), dtype=torch.float32, device=dev)
        z = torch.empty((M, C), dtype=torch.float32, device=dev)
        nrm = torch.empty(M, dtype=torch.float32, device=dev)
        rowloss = torch.empty(max(M, 1), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().gnn_head_bce_fwd_f32(x.data_ptr(), x.stride(0), M, D, W.data_ptr(), _ptr(b), C,
                                                   labels.data_ptr(), labels.stride(0), float(p), seed,
                                                   int(training), xd.data_ptr(), z.data_ptr(), nrm.data_ptr(),
                                                   rowloss.data_ptr(), loss.data_ptr(), _stream(dev)),
                   "gnn_head_bce_fwd_f32")
        ctx.save_for_backward(x, W, labels, xd, z, nrm)
        ctx.cfg = (float(p), int(training), int(seed), b is not None)
        ctx.mark_non_differentiable(z)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the logits output
        return loss, z

    @staticmethod
    def backward(ctx, gloss, _gz):
        x, W, labels, xd, z, nrm = ctx.saved_tensors
        p, training, seed, has_bias = ctx.cfg
        M, D = x.shape
        C = W.shape[0]
        dev = x.device
        gloss = gloss.contiguous()
        dz = torch.empty((M, C), dtype=torch.float32, device=dev)
        dx = torch.empty((M, D), dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().gnn_head_bce_bwd_f32(x.data_ptr(), x.stride(0), M, D, W.data_ptr(), C,
                                                   labels.data_ptr(), labels.stride(0), gloss.data_ptr(), p, seed,
                                                   training, z.data_ptr(), nrm.data_ptr(), dz.data_ptr(),
                                                   dx.data_ptr(), D, _stream(dev)),
                   "gnn_head_bce_bwd_f32")
        dW = torch.mm(dz.t(), xd) if ctx.needs_input_grad[1] else None
        db = dz.sum(0) if (has_bias and ctx.needs_input_grad[2]) else None
        return dx, dW, db, None, None, None, None


def head_supported(x: torch.Tensor, W: torch.Tensor, labels: torch.Tensor) -> bool:
    M, D = x.shape
    return (x.is_cuda and x.dtype == torch.float32 and W.dtype == torch.float32 and x.stride(1) == 1
            and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0 and D % 4 == 0 and D <= 2048
            and W.shape[0] <= 256 and labels.shape == (M, W.shape[0]))


def head_bce_loss(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor], labels: torch.Tensor,
                  p: float = 0.0, training: bool = False):
    """(loss, logits) of GNN's head with the sigmoid loss — see HeadBCEFn. Raises when the
    operands are outside the kernel's contract (callers check head_supported first)."""
    if not head_supported(x, W, labels):
        raise RuntimeError("head_bce_loss: fp32 CUDA x (M x D, D % 4 == 0, D <= 2048, 16-byte rows), "
                           "at most 64 classes, labels M x C")
    tr = bool(training and p > 0)
    seed = int(torch.randint(0, 2**62, (1,)).item()) if tr else 0
    return HeadBCEFn.apply(x, W, b, labels, float(p), tr, seed)
