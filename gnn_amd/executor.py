"""Native training-step executor (include/gnn_step.h): the fused GraphSAGE / GCN model's
forward + backward as ONE C call per step.

Reference: main.py:122-146 (model forward, utils.loss, loss.backward()). The Python fused path
(gnn_amd.models with fused=True) runs the same HIP kernels through ~45 autograd Functions and
ctypes calls per step — 1.2-1.5 ms of host time against a 1.8 ms GPU step; here the host fills
one int64 descriptor and makes one call. Same kernels, same GEMM routing, same dropout seeds
(drawn from torch's CPU generator in the same order as the Python path), so the two paths agree
to the last bit except the few small products on the vendor GEMM (tests/test_executor_gpu.py).
Gradients land in one persistent flat buffer; the parameters' ``.grad`` are views of it, so
gnn_amd.optim.ClipAdam (clip, all-reduce, Adam) runs unchanged after the call.
"""
from __future__ import annotations

import os
import struct
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from . import custom_sparse_ops as cso

VERSION, MAX_LAYERS, HEADER, LAYER_SLOTS, SAGE, GCN = 1, 4, 24, 32, 0, 1
(H_VERSION, H_LAYERS, H_KIND, H_X0, H_LDX0, H_F0, H_HEAD_W, H_HEAD_B, H_HEAD_GW, H_HEAD_GB, H_CLASSES, H_LABELS,
 H_LDL, H_HEAD_SEED, H_PDROP_BITS, H_TRAINING, H_LOSS, H_NHID, H_TIMING, H_GRAD_EVENTS, H_STAGE_EVENT,
 H_STAGE_LAYER, H_PHASE) = range(23)
TIMING_SLOTS = 16
(L_ROWPTR, L_COL, L_VAL, L_M, L_K, L_NNZ, L_TROWPTR, L_TCOL, L_TVAL, L_SAMPLED, L_NSAMPLED, L_RMAP, L_WW, L_BW,
 L_WB, L_BB, L_SCALE, L_OFFSET, L_GWW, L_GBW, L_GWB, L_GBB, L_GSCALE, L_GOFFSET, L_SEED) = range(25)


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def enabled() -> bool:
    """GNN_NATIVE_STEP=0 keeps the Python autograd path (A/B measurements)."""
    return os.environ.get("GNN_NATIVE_STEP", "1") != "0"


class NativeStep:
    """Binds a fused ``models.GNN`` (GraphSage or GCN encoder, every layer of order 1) to
    gnn_train_step_f32. ``step(x0, adjs, sampled_nodes, labels)`` runs forward + backward and
    returns the loss (a device scalar); the gradients are in the parameters' ``.grad``."""

    def __init__(self, model):
        from . import models

        enc = model.encoder
        if not getattr(enc, "fused", False):
            raise ValueError("NativeStep needs the fused model (build_model(..., fused=True))")
        if isinstance(enc, models.GraphSage):
            self.kind = SAGE
        elif isinstance(enc, models.GCN):
            self.kind = GCN
        else:
            raise ValueError(f"NativeStep: unsupported encoder {type(enc).__name__}")
        if any(g.order != 1 for g in enc.gcs) or not 1 <= len(enc.gcs) <= MAX_LAYERS:
            raise ValueError("NativeStep: every layer must have order 1 (1-4 layers)")
        self.model = model
        self.enc = enc
        self.params: List[torch.nn.Parameter] = [p for p in model.parameters()]
        dev = self.params[0].device
        self.device = dev
        n = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grads, off = [], 0
        for p in self.params:
            self.grads.append(self.flat_grad[off:off + p.numel()].view_as(p))
            off += p.numel()
        g = {id(p): gr for p, gr in zip(self.params, self.grads)}
        d = np.zeros(HEADER + LAYER_SLOTS * len(enc.gcs), dtype=np.int64)
        d[H_VERSION] = VERSION
        d[H_LAYERS] = len(enc.gcs)
        d[H_KIND] = self.kind
        head = model.linear
        d[H_HEAD_W], d[H_HEAD_B] = _p(head.weight), _p(head.bias)
        d[H_HEAD_GW], d[H_HEAD_GB] = _p(g[id(head.weight)]), _p(g.get(id(head.bias)) if head.bias is not None else None)
        d[H_CLASSES] = head.weight.shape[0]
        d[H_NHID] = enc.gcs[0].n_out
        self.p_enc = float(enc.dropout.p)
        self.p_head = float(model.dropout.p)
        if self.p_enc != self.p_head:
            raise ValueError("NativeStep: the encoder and head dropout rates must match")
        d[H_PDROP_BITS] = struct.unpack("<i", struct.pack("<f", self.p_enc))[0]
        for li, gc in enumerate(enc.gcs):
            b = HEADER + li * LAYER_SLOTS
            if self.kind == SAGE:
                W, B = gc.linearW, gc.linearB
                d[b + L_WB], d[b + L_BB] = _p(B.weight), _p(B.bias)
                d[b + L_GWB], d[b + L_GBB] = _p(g[id(B.weight)]), _p(g[id(B.bias)])
            else:
                W = gc.linear
            d[b + L_WW], d[b + L_BW] = _p(W.weight), _p(W.bias)
            d[b + L_GWW], d[b + L_GBW] = _p(g[id(W.weight)]), _p(g[id(W.bias)])
            d[b + L_SCALE], d[b + L_OFFSET] = _p(gc.scale), _p(gc.offset)
            d[b + L_GSCALE], d[b + L_GOFFSET] = _p(g[id(gc.scale)]), _p(g[id(gc.offset)])
        for p in self.params:
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                raise ValueError("NativeStep: parameters must be contiguous float32 CUDA tensors")
        self.template = d

    def supports(self, x0, adjs, sampled_nodes, labels) -> bool:
        """Whether this batch fits the executor (CSR operands with their transposes, row maps)."""
        from .custom_sparse_ops import CsrOperand

        if not (x0.is_cuda and x0.dtype == torch.float32 and x0.stride(1) == 1 and labels.dtype == torch.float32
                and labels.dim() == 2 and labels.stride(1) == 1):
            return False
        C, D = self.model.linear.weight.shape
        if C > 256 or D % 4 or D > 2048 or labels.shape[1] != C:  # the fused head's contract (fused.head_supported)
            return False
        for li, op in enumerate(adjs):
            if not isinstance(op, CsrOperand):
                return False
            if li >= 1 and op._t is None:
                return False
            if self.kind == SAGE:
                s = sampled_nodes[li]
                if s.dtype != torch.int64 or not s.is_contiguous() or s.numel() != op.shape[0]:
                    return False
                if li >= 1 and getattr(s, "_gnn_rmap", None) is None:
                    return False
        return True

    def grad_stages(self):
        """Parameter indices (into self.params / the flat gradient) per backward stage, in the
        order the step finalises them: [head, layer L-1, ..., layer 0]."""
        head = {id(p) for p in self.model.linear.parameters()}
        stages = [[i for i, p in enumerate(self.params) if id(p) in head]]
        for gc in reversed(self.enc.gcs):
            mine = {id(p) for p in gc.parameters()}
            stages.append([i for i, p in enumerate(self.params) if id(p) in mine])
        return stages

    @staticmethod
    def _batch_key(x0, adjs, labels):
        return (x0.data_ptr(), tuple(x0.shape), x0.stride(0), labels.data_ptr(), tuple(id(op) for op in adjs))

    def prefetch(self, x0, adjs, sampled_nodes, labels, stage_gate=None) -> None:
        """Issue ONLY this batch's layer-0 forward aggregation A_0·x0 (GNN_SH_PHASE 1) into a
        workspace kept for its step, on the current stream; the next ``step`` on the same batch
        (same x0, operands and labels) runs without issuing it again (phase 2). It reads only the
        batch, never a parameter, so a data-parallel trainer issues it between the gradient
        all-reduce's launch and the optimizer step: it runs while the all-reduce does (reference:
        main.py:122-168, where the next batch's forward starts after the exchange and the step).
        No dropout seed is drawn here: the step draws them, in the same order as without it."""
        d = self._desc(x0, adjs, sampled_nodes, labels, seeds=False)
        if stage_gate is not None and int(stage_gate[1]) == 0:
            self._set_gate(d, stage_gate)
        d[H_PHASE] = 1
        ws, wsb = self._workspace(d, x0.device)
        L = _lib.lib()
        with _lib.on_device(x0.device):
            _lib.check(L.gnn_train_step_f32(d.ctypes.data, ws.data_ptr(), wsb, _lib.stream_of(x0.device)),
                       "gnn_train_step_f32 (phase 1)")
        # the batch's tensors and operands are held with the key, so no other batch can take
        # their addresses or ids while the prefetched aggregation waits for its step
        self._pre = (self._batch_key(x0, adjs, labels), ws, wsb, (x0, tuple(adjs), labels))

    def drop_prefetch(self) -> None:
        self._pre = None

    @staticmethod
    def _set_gate(d, stage_gate):
        ev, layer = stage_gate
        if not getattr(ev, "_gnn_created", False):
            ev.record()  # creates the underlying hipEvent once; the step re-records it
            ev._gnn_created = True
        d[H_STAGE_EVENT], d[H_STAGE_LAYER] = ev.cuda_event, int(layer)

    @staticmethod
    def _workspace(d, device):
        wsb = _lib.lib().gnn_train_step_workspace_bytes(d.ctypes.data)
        if wsb == 0:
            raise RuntimeError("gnn_train_step_workspace_bytes: " + _lib.lib().gnn_last_error().decode(errors="replace"))
        return torch.empty(wsb, dtype=torch.uint8, device=device), wsb

    def step(self, x0, adjs, sampled_nodes, labels, grad_events=None, stage_gate=None) -> torch.Tensor:
        """grad_events: optional [head event, layer 0 event, layer 1 event, ...] (torch.cuda.Event)
        recorded on the step's stream once those gradients are final (GNN_SH_GRAD_EVENTS).
        stage_gate: optional (torch.cuda.Event, layer): the event is recorded right after that
        layer's forward aggregation (GNN_SH_STAGE_EVENT; staging.Stager waits on it).
        A ``prefetch`` of this same batch (the last one issued) supplies the layer-0 aggregation."""
        d = self._desc(x0, adjs, sampled_nodes, labels, seeds=True)
        pre, self._pre = getattr(self, "_pre", None), None
        if pre is not None and pre[0] == self._batch_key(x0, adjs, labels):
            d[H_PHASE] = 2
            ws, wsb = pre[1], pre[2]
            if stage_gate is not None and int(stage_gate[1]) == 0:
                stage_gate = None  # recorded by the prefetch, after the layer-0 aggregation
        else:
            ws, wsb = None, 0
        loss = torch.empty((), dtype=torch.float32, device=x0.device)
        d[H_LOSS] = loss.data_ptr()
        timing = self._arm_timing(d, len(adjs)) if cso.timing_enabled() else None
        E = None
        if grad_events is not None:
            E = np.zeros(1 + len(grad_events), dtype=np.int64)
            E[0] = len(E)
            for i, ev in enumerate(grad_events):
                if ev is not None:
                    ev.record()  # creates the underlying hipEvent; the step re-records it
                    E[1 + i] = ev.cuda_event
            d[H_GRAD_EVENTS] = E.ctypes.data
        if stage_gate is not None:
            self._set_gate(d, stage_gate)
        L = _lib.lib()
        dp = d.ctypes.data
        if ws is None:
            ws, wsb = self._workspace(d, x0.device)
        with _lib.on_device(x0.device):
            _lib.check(L.gnn_train_step_f32(dp, ws.data_ptr(), wsb, _lib.stream_of(x0.device)), "gnn_train_step_f32")
        if timing is not None:
            self._collect_timing(*timing)
        for p, gr in zip(self.params, self.grads):
            p.grad = gr
        return loss

    def _desc(self, x0, adjs, sampled_nodes, labels, seeds: bool):
        model = self.model
        training = model.training
        tr = bool(training and self.p_enc > 0)
        d = self.template.copy()
        d[H_X0], d[H_LDX0], d[H_F0] = x0.data_ptr(), x0.stride(0) if x0.shape[0] > 1 else x0.shape[1], x0.shape[1]
        d[H_LABELS], d[H_LDL] = labels.data_ptr(), labels.stride(0) if labels.shape[0] > 1 else labels.shape[1]
        d[H_TRAINING] = int(tr)
        # the Python path draws one seed per layer tail, then one for the head (fused.py): one
        # randint call for all of them gives the same values from the CPU generator (one call
        # instead of nl + 1: ~15 us less host issue per step)
        sv = torch.randint(0, 2**62, (len(adjs) + 1,)).tolist() if (tr and seeds) else None
        for li, op in enumerate(adjs):
            b = HEADER + li * LAYER_SLOTS
            d[b + L_ROWPTR], d[b + L_COL], d[b + L_VAL] = op.rowptr.data_ptr(), op.col.data_ptr(), op.val.data_ptr()
            d[b + L_M], d[b + L_K], d[b + L_NNZ] = op.shape[0], op.shape[1], op.nnz
            if li >= 1:
                t = op._t
                d[b + L_TROWPTR], d[b + L_TCOL], d[b + L_TVAL] = t.rowptr.data_ptr(), t.col.data_ptr(), t.val.data_ptr()
            if self.kind == SAGE:
                s = sampled_nodes[li]
                d[b + L_SAMPLED], d[b + L_NSAMPLED] = s.data_ptr(), s.numel()
                r = getattr(s, "_gnn_rmap", None)
                d[b + L_RMAP] = _p(r) if li >= 1 else 0
            d[b + L_SEED] = sv[li] if sv is not None else 0
        d[H_HEAD_SEED] = sv[len(adjs)] if sv is not None else 0
        return d

    @staticmethod
    def _arm_timing(d, nl):
        """custom_sparse_ops timing is on (bench roofline): one event pair per aggregation launch
        (nl forwards + nl - 1 backwards), armed by the executor around its SpMM kernels."""
        n = 2 * nl - 1
        T = np.zeros(1 + TIMING_SLOTS * n, dtype=np.int64)
        T[0] = n
        evs = []
        for i in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()  # creates the underlying hipEvent; the library re-records it
            e1.record()
            T[1 + TIMING_SLOTS * i], T[2 + TIMING_SLOTS * i] = e0.cuda_event, e1.cuda_event
            evs.append((e0, e1))
        d[H_TIMING] = T.ctypes.data
        return T, evs

    @staticmethod
    def _collect_timing(T, evs):
        for i, (e0, e1) in enumerate(evs):
            r = T[1 + TIMING_SLOTS * i: 1 + TIMING_SLOTS * (i + 1)]
            if r[14] != 1:
                continue
            kind, l, M, K, nnz, F, Fk, ldx, ldy, xp, yp, res = (int(v) for v in r[2:14])
            cso.record_timing(("fwd" if kind == 0 else "bwd") + f"_L{l}", e0, e1, M, K, nnz, F, Fk, ldx, ldy, xp, yp,
                              0, res, kind == 1 and res > 0)
