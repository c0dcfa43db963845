"""Gradient clipping + Adam on the GPU in two launches (include/gnn_optim.h).

Semantics of the reference step (main.py:146-170): clip_grad_norm_(params, 5) on each
rank's own gradients, the SUM of the clipped gradients across ranks (no averaging), then
torch.optim.Adam (betas (0.9, 0.999), eps 1e-8, no weight decay). At N = 1 the clip factor
is applied inside the Adam kernel; at N > 1 the clipped gradients are written straight into
the flat all-reduce buffer (one kernel instead of a cat), summed over RCCL, and Adam reads
them from there.
"""
from __future__ import annotations

import ctypes
from typing import List

import torch

from . import _lib

_MAXT = 32  # GNN_OPTIM_MAX_TENSORS


def _arr(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


class ClipAdam:
    def __init__(self, params, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, max_norm: float = 5.0):
        self.params: List[torch.Tensor] = [p for p in params]
        for p in self.params:
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                raise RuntimeError("ClipAdam: parameters must be contiguous float32 CUDA tensors")
        self.lr, self.betas, self.eps, self.max_norm = float(lr), betas, float(eps), float(max_norm)
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.step_count = 0
        self.groups = [list(range(i, min(i + _MAXT, len(self.params)))) for i in range(0, len(self.params), _MAXT)]
        L = _lib.lib()
        self._n = [(ctypes.c_int64 * len(g))(*[self.params[i].numel() for i in g]) for g in self.groups]
        self._chunks = [int(L.gnn_optim_chunks(len(g), n)) for g, n in zip(self.groups, self._n)]
        self.nchunks = sum(self._chunks)
        dev = self.params[0].device
        self.partial = torch.empty(max(self.nchunks, 1), dtype=torch.float32, device=dev)
        self.scale = torch.ones(1, dtype=torch.float32, device=dev)  # the clip factor (device)
        self._p = [_arr([self.params[i].data_ptr() for i in g]) for g in self.groups]
        self._m = [_arr([self.m[i].data_ptr() for i in g]) for g in self.groups]
        self._v = [_arr([self.v[i].data_ptr() for i in g]) for g in self.groups]
        self.numel = sum(p.numel() for p in self.params)

    def _grads(self):
        gs = []
        for p in self.params:
            g = p.grad
            if g is None:
                g = torch.zeros_like(p)
                p.grad = g
            elif not g.is_contiguous():
                g = g.contiguous()
                p.grad = g
            gs.append(g)
        return gs

    def _clip_scale(self, gs, st):
        """Partial sums of squares per chunk, then the clip factor into self.scale."""
        L = _lib.lib()
        off = 0
        for g, n, c in zip(self.groups, self._n, self._chunks):
            _lib.check(L.gnn_grad_sqnorm_f32(len(g), _arr([gs[i].data_ptr() for i in g]), n,
                                             self.partial.data_ptr() + 4 * off, st), "gnn_grad_sqnorm_f32")
            off += c
        _lib.check(L.gnn_clip_scale_f32(self.partial.data_ptr(), self.nchunks, self.max_norm, self.scale.data_ptr(),
                                        st), "gnn_clip_scale_f32")

    def clip_to_flat(self) -> torch.Tensor:
        """Per-rank clip, written into a new flat buffer (the all-reduce input); the
        parameters' .grad become views of it."""
        gs = self._grads()
        dev = self.params[0].device
        st = _lib.stream_of(dev)
        scale = None
        if self.max_norm > 0:
            self._clip_scale(gs, st)
            scale = self.scale.data_ptr()
        flat = torch.empty(self.numel, dtype=torch.float32, device=dev)
        L = _lib.lib()
        base = 0
        for g, n in zip(self.groups, self._n):
            _lib.check(L.gnn_scale_into_f32(len(g), _arr([gs[i].data_ptr() for i in g]), n, scale,
                                            flat.data_ptr() + 4 * base, st), "gnn_scale_into_f32")
            base += sum(self.params[i].numel() for i in g)
        off = 0
        for p in self.params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return flat

    def step(self, clipped: bool = False):
        """Adam step. clipped=False: clip (from this rank's gradients) inside the update;
        clipped=True: the gradients were already clipped (and summed) — plain Adam."""
        gs = self._grads()
        dev = self.params[0].device
        st = _lib.stream_of(dev)
        L = _lib.lib()
        scale = None
        if not clipped and self.max_norm > 0:
            self._clip_scale(gs, st)
            scale = self.scale.data_ptr()
        self.step_count += 1
        b1, b2 = self.betas
        for g, n, pp, mm, vv in zip(self.groups, self._n, self._p, self._m, self._v):
            _lib.check(L.gnn_adam_f32(len(g), pp, _arr([gs[i].data_ptr() for i in g]), mm, vv, n, scale, self.lr, b1,
                                      b2, self.eps, self.step_count, st), "gnn_adam_f32")
