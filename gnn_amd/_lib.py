"""ctypes binding of libgnn_spmm.so (the C ABI declared in include/gnn_spmm.h).

The shared library is built in-tree by ``gnn_amd.build.build_library()`` (hipcc,
--offload-arch=gfx950) and travels with the repository snapshot. There is deliberately no
fallback: if the library is missing or fails to load, every operator raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GNN_SPMM_LIBRARY") or os.path.join(_HERE, "libgnn_spmm.so")  # override: experiments

_lock = threading.Lock()
_lib = None

c_i32p = ctypes.c_void_p  # all device pointers travel as void*
_VP = ctypes.c_void_p
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t
_INT = ctypes.c_int

# name -> (restype, argtypes)
_SIGNATURES = {
    "gnn_last_error": (ctypes.c_char_p, []),
    "gnn_version": (ctypes.c_char_p, []),
    "gnn_spmm_default_unit_nnz": (_I64, [_I64, _I64, _I64]),
    "gnn_spmm_workspace_bytes": (_SZ, [_I64, _I64, _I64, _I64]),
    "gnn_spmm_csr_f32": (_INT, [_VP, _VP, _VP, _I64, _I64, _I64, _VP, _I64, _VP, _I64, _I64, _VP, _SZ, _I64, _VP]),
    "gnn_spmm_csr_f32_ex": (_INT, [_VP, _VP, _VP, _I64, _I64, _I64, _VP, _I64, _VP, _I64, _I64, _VP, _I64, _VP,
                                   _VP, _SZ, _I64, _VP]),
    "gnn_spmm_kernel_name": (_INT, [_I64, _I64, _I64, _I64, _I64, _I64, _VP, _VP, _I64, _INT, ctypes.c_char_p, _SZ]),
    "gnn_spmm_config":(_INT, [_I64, _I64, _I64, _I64, _I64, _I64, _VP, _VP, _I64, ctypes.POINTER(ctypes.c_int32)]),
    "gnn_spmm_set_timing_events": (None, [_VP, _VP]),
    "gnn_segsort_workspace_bytes": (_SZ, [_I64]),
    "gnn_build_operand_workspace_bytes": (_SZ, []),
    "gnn_build_operand_f32": (_INT, [_VP, _VP, _VP, _INT, _VP, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _SZ, _VP]),
    "gnn_build_operand_t_f32": (_INT, [_VP, _VP, _VP, _VP, _I64, _I64, _I64, _VP, _VP]),
    "gnn_build_operand_sorted_f32": (_INT, [_VP, _VP, _VP, _INT, _VP, _I64, _I64, _I64, _VP, _VP, _VP, _VP]),
    "gnn_coo_to_csr": (_INT, [_VP, _VP, _I64, _I64, _VP, _VP, _VP]),
    "gnn_csr_transpose_workspace_bytes": (_SZ, [_I64, _I64, _I64]),
    "gnn_csr_transpose": (_INT, [_VP, _VP, _VP, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _SZ, _VP]),
    "gnn_gather_rows_f32": (_INT, [_VP, _I64, _VP, _VP, _I64, _VP, _I64, _I64, _VP]),
    "gnn_gather_rows2_f32": (_INT, [_VP, _I64, _VP, _VP, _I64, _VP, _I64, _VP, _VP, _I64, _VP, _I64, _I64, _VP]),
    "gnn_gather_rows_host_f32": (_INT, [_VP, _I64, _VP, _VP, _I64, _VP, _I64, _I64, _VP]),
    "gnn_host_register": (_INT, [_VP, _SZ]),
    "gnn_host_unregister": (_INT, [_VP]),
    "gnn_memcpy_h2d_async": (_INT, [_VP, _VP, _SZ, _VP]),
    # include/gnn_stage.h
    "gnn_stage_plan": (_SZ, [_VP, _VP]),
    "gnn_stage_batch_f32": (_INT, [_VP, _VP]),
    "gnn_stream_create_cu_masked": (_INT, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(_VP)]),
    "gnn_stream_destroy": (_INT, [_VP]),
    "gnn_ipc_export": (_INT, [_VP, _VP, ctypes.POINTER(_I64)]),
    "gnn_ipc_open": (_INT, [_VP, _I64, _INT, ctypes.POINTER(_VP)]),
    "gnn_ipc_close": (_INT, [_VP, _I64]),
    # include/gnn_layers.h
    "gnn_sage_norm_fwd_f32": (_INT, [_VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP, _VP, _VP, _I64, ctypes.c_float,
                                     ctypes.c_uint64, _INT, _VP, _I64, _VP, _VP, _VP]),
    "gnn_sage_norm_bwd_workspace_bytes": (_SZ, [_I64, _I64]),
    "gnn_sage_norm_bwd_f32": (_INT, [_VP, _I64, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP, _VP, _VP, _VP, _I64,
                                     ctypes.c_float, ctypes.c_uint64, _INT, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _SZ,
                                     _VP]),
    "gnn_sage_norm_bwd_agg_f32": (_INT, [_VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP, _I64, _I64, _VP, _I64, _I64,
                                         _VP, _VP, _VP, _VP, _VP, _I64, ctypes.c_float, ctypes.c_uint64, _INT, _VP,
                                         _VP, _VP, _VP, _VP, _VP, _VP, _SZ, _VP]),
    "gnn_gemm_p3_packed_bytes": (_SZ, [_I64, _I64]),
    "gnn_gemm_p3_pack_f32": (_INT, [_VP, _I64, _INT, _VP, _I64, _I64, _VP, _SZ, _VP]),
    "gnn_gemm_p3_workspace_bytes": (_SZ, [_I64, _I64, _I64, _INT]),
    "gnn_gemm_p3": (_INT, [_I64, _I64, _I64, _INT, _VP, _VP, _VP, _I64, _VP, _SZ, _VP]),
    # include/gnn_optim.h
    "gnn_optim_chunks": (_I64, [_INT, _VP]),
    "gnn_grad_sqnorm_f32": (_INT, [_INT, _VP, _VP, _VP, _VP]),
    "gnn_clip_scale_f32": (_INT, [_VP, _I64, ctypes.c_float, _VP, _VP]),
    "gnn_scale_into_f32": (_INT, [_INT, _VP, _VP, _VP, _VP, _VP]),
    "gnn_adam_f32": (_INT, [_INT, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                            ctypes.c_float, _I64, _VP]),
    "gnn_head_bce_fwd_f32": (_INT, [_VP, _I64, _I64, _I64, _VP, _VP, _I64, _VP, _I64, ctypes.c_float,
                                    ctypes.c_uint64, _INT, _VP, _VP, _VP, _VP, _VP, _VP]),
    "gnn_head_bce_bwd_f32": (_INT, [_VP, _I64, _I64, _I64, _VP, _I64, _VP, _I64, _VP, ctypes.c_float,
                                    ctypes.c_uint64, _INT, _VP, _VP, _VP, _VP, _I64, _VP]),
    # include/gnn_extract.h
    "gnn_ladies_extract_workspace_bytes": (_SZ, [_I64, _I64, _I64, ctypes.c_int32, _I64, _I64]),
    "gnn_colcount_create": (_INT, [ctypes.c_int32, _I64, _VP, _VP, ctypes.POINTER(_VP)]),
    "gnn_colcount_add": (_INT, [_VP, _VP, _I64, ctypes.POINTER(_I64), ctypes.POINTER(_VP), ctypes.POINTER(_VP)]),
    "gnn_colcount_reset": (_INT, [_VP]),
    "gnn_colcount_destroy": (None, [_VP]),
    "gnn_colcount_set_cus": (_INT, [ctypes.c_int32]),
    "gnn_ladies_extract_f32": (_INT, [_VP, _VP, _VP, _I64, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _I64,
                                      _I64, _VP, _VP, _VP, _VP, _VP, _VP, _SZ, _VP, _VP]),
    # include/gnn_step.h
    "gnn_train_step_workspace_bytes": (_SZ, [_VP]),
    "gnn_train_step_f32": (_INT, [_VP, _VP, _SZ, _VP]),
    "gnn_gemm_f32_workspace_bytes": (_SZ, [_I64, _I64, _I64, _INT]),
    "gnn_gemm_f32": (_INT, [_INT, _INT, _I64, _I64, _I64, _INT, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _SZ, _VP]),
    "gnn_gemm_f32_split3_workspace_bytes": (_SZ, [_I64, _I64, _I64, _INT]),
    "gnn_gemm_f32_split3_indexed": (_INT, [_INT, _INT, _I64, _I64, _I64, _INT, _VP, _I64, _VP, _I64, _VP, _I64, _VP,
                                           _I64, _VP, _I64, _VP, _SZ, _VP]),
    "gnn_gemm_f32_split3": (_INT, [_INT, _INT, _I64, _I64, _I64, _INT, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _SZ,
                                   _VP]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

# libgnn_sampler.so (include/gnn_sampler.h): host-only, g++
SAMPLER_PATH = os.path.join(_HERE, "libgnn_sampler.so")
_SAMPLER_SIGNATURES = {
    "gnn_sampler_last_error": (ctypes.c_char_p, []),
    "gnn_ladies_sample": (_INT, [_VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_uint32,
                                 ctypes.POINTER(_VP)]),
    "gnn_ladies_sample_dev": (_INT, [_VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_uint32,
                                     ctypes.c_int32, ctypes.POINTER(_VP)]),
    "gnn_ladies_layer_device": (_INT, [_VP, ctypes.c_int32, _VP, _VP, _VP, _VP, _VP]),
    "gnn_subgraph_sample": (_INT, [_VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_uint32,
                                   ctypes.POINTER(_VP)]),
    "gnn_fastgcn_sample": (_INT, [_VP, _VP, _VP, _I64, _VP, _VP, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_uint32,
                                  ctypes.POINTER(_VP)]),
    "gnn_fastgcn_p_changed": (None, []),
    "gnn_ladies_layer_dims": (_INT, [_VP, ctypes.c_int32, ctypes.POINTER(_I64)]),
    "gnn_ladies_layer_copy": (_INT, [_VP, ctypes.c_int32, _VP, _VP, _VP, _VP, _VP]),
    "gnn_ladies_layer_csc": (_INT, [_VP, ctypes.c_int32, _VP, _VP]),
    "gnn_ladies_num_input_nodes": (_I64, [_VP]),
    "gnn_ladies_input_nodes": (_INT, [_VP, _VP]),
    "gnn_ladies_free": (None, [_VP]),
    "gnn_mt19937_random_sample": (_INT, [ctypes.c_uint32, _I64, _VP]),
    "gnn_sampler_profile": (_INT, [_VP, ctypes.c_int32, ctypes.c_int32]),
    "gnn_host_gather_rows_f32": (_INT, [_VP, _I64, _I64, _VP, _I64, _I64, _VP, _I64]),
    "gnn_loader_create": (_VP, [_VP, _VP, _VP, _VP, _I64, _VP, _VP, _VP, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_int32,
                                _VP, _VP, _I64, _I64, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_int32, _VP,
                                ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "gnn_loader_submit": (_INT, [_VP, ctypes.c_uint32, _VP, _I64]),
    "gnn_loader_set_colcount": (_INT, [_VP, _VP]),
    "gnn_loader_set_colcount_workers": (_INT, [_VP, ctypes.c_int32]),
    "gnn_ladies_sample_cc": (_INT, [_VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP, ctypes.c_int32, ctypes.c_uint32,
                                    ctypes.c_int32, _VP, _VP, ctypes.POINTER(_VP)]),
    "gnn_loader_next": (_INT, [_VP, ctypes.POINTER(_VP)]),
    "gnn_batch_desc": (ctypes.POINTER(_I64), [_VP, ctypes.POINTER(_I64)]),
    "gnn_batch_blob": (_VP, [_VP]),
    "gnn_batch_release": (None, [_VP]),
    "gnn_loader_destroy": (None, [_VP]),
}
SAMPLER_EXPORTED_SYMBOLS = tuple(_SAMPLER_SIGNATURES)
_sampler = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library. Raises if it is missing: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"gnn_amd: native library {LIB_PATH} is missing; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def sampler_lib() -> ctypes.CDLL:
    """Load (once) the host sampler library. Raises if it is missing."""
    global _sampler
    if _sampler is not None:
        return _sampler
    with _lock:
        if _sampler is None:
            if not os.path.exists(SAMPLER_PATH):
                raise RuntimeError(f"gnn_amd: native sampler {SAMPLER_PATH} is missing; build it with "
                                   "`python -c 'import __graft_entry__ as g; g.build()'`")
            handle = ctypes.CDLL(SAMPLER_PATH)
            for name, (res, args) in _SAMPLER_SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _sampler = handle
    return _sampler


def check_sampler(rc: int, what: str) -> None:
    if rc != 0:
        msg = sampler_lib().gnn_sampler_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


_NULLCTX = contextlib.nullcontext()


def stream_of(dev) -> int:
    """Raw hipStream_t of torch's current stream on `dev` (no Python Stream object)."""
    return torch._C._cuda_getCurrentRawStream(dev.index if dev.index is not None else torch.cuda.current_device())


def on_device(dev):
    """torch.cuda.device(dev) only when dev is not already current (the context manager
    costs ~10 µs a call on the host; one process per GPU keeps its device current)."""
    if dev.index is None or dev.index == torch._C._cuda_getDevice():
        return _NULLCTX
    return torch.cuda.device(dev)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().gnn_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")
