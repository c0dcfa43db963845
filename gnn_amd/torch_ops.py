"""The aggregation as registered PyTorch operators (torch.ops.gnn.*) and the reference's native
module `spmm`, from the PyTorch-ROCm extension gnn_amd/csrc/spmm_ext.cpp.

Reference: custom_sparse_ops.py:8 JIT-builds a pybind module named ``spmm`` (spmm_cpp/spmm.cpp:
52-56: ``spmm_load_balance``, ``spmm_naive``, ``create_coo_tensor``) and wraps it in an
``autograd.Function`` (custom_sparse_ops.py:16-37). Here the module of the same name is the
in-tree extension (``import spmm`` from the repository root — what the reference's ``load()``
returns), and the aggregation is also a dispatcher operator with a fake (shape) kernel and an
autograd formula, so ``torch.compile`` traces it as one op:

  torch.ops.gnn.spmm(rowptr, col, val, t_rowptr, t_col, t_val, M, K, X) -> Y = A·X
      backward: dX = Aᵀ·dY on the given transpose (the reference's backward,
      custom_sparse_ops.py:33-37), no gradient to the sparse values.
  torch.ops.gnn.spmm_csr(rowptr, col, val, M, K, X) -> A·X      (no autograd)
  torch.ops.gnn.csr_transpose(rowptr, col, val, M, K) -> canonical Aᵀ (A.t().coalesce())

The operator bodies are C++ calling libgnn_spmm.so's C ABI on torch's current HIP stream; a
missing extension raises (no fallback).
"""
from __future__ import annotations

import importlib
import os
import sys

import torch

_loaded = False


def load():
    """Import the extension module `spmm` (registers torch.ops.gnn.*) and the Python-side fake
    kernels and autograd formula; returns the module. Raises if the extension is not built."""
    global _loaded
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    try:
        mod = importlib.import_module("spmm")
    except ImportError as e:
        raise RuntimeError("the PyTorch extension `spmm` is not built (gnn_amd.build.build_torch_ext): "
                           f"{e}") from e
    if not _loaded:
        _register()
        _loaded = True
    return mod


def _register():
    @torch.library.register_fake("gnn::spmm_csr")
    def _spmm_csr_fake(rowptr, col, val, M, K, dense):
        return dense.new_empty((M, dense.shape[1]))

    @torch.library.register_fake("gnn::spmm")
    def _spmm_fake(rowptr, col, val, t_rowptr, t_col, t_val, M, K, dense):
        return dense.new_empty((M, dense.shape[1]))

    @torch.library.register_fake("gnn::csr_transpose")
    def _csr_transpose_fake(rowptr, col, val, M, K):
        nnz = col.shape[0]
        return rowptr.new_empty((K + 1,)), col.new_empty((nnz,)), val.new_empty((nnz,))

    def _setup(ctx, inputs, output):
        _, _, _, t_rowptr, t_col, t_val, M, K, _ = inputs
        ctx.save_for_backward(t_rowptr, t_col, t_val)
        ctx.MK = (M, K)

    def _backward(ctx, grad):
        t_rowptr, t_col, t_val = ctx.saved_tensors
        M, K = ctx.MK
        gx = None
        if ctx.needs_input_grad[8]:
            gx = torch.ops.gnn.spmm_csr(t_rowptr, t_col, t_val, K, M, grad.contiguous())
        return None, None, None, None, None, None, None, None, gx

    torch.library.register_autograd("gnn::spmm", _backward, setup_context=_setup)


def spmm(adj, x: torch.Tensor) -> torch.Tensor:
    """custom_sparse_ops.spmm as the registered operator: ``adj`` a CsrOperand (its cached
    transpose is passed along for the backward) or a coalesced CUDA COO tensor."""
    from .custom_sparse_ops import csr_of

    load()
    op = csr_of(adj)
    t = op.transpose()
    M, K = op.shape
    return torch.ops.gnn.spmm(op.rowptr, op.col, op.val, t.rowptr, t.col, t.val, M, K, x)
