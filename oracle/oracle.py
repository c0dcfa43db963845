"""TEST INFRASTRUCTURE: numpy front end of liboracle.so (see oracle/__init__.py)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None

__all__ = ["build_oracle", "build_operand", "spmm_f32", "spmm_f64", "spmm_abs", "csr_transpose", "gather_rows",
           "load"]


def build_oracle(force: bool = False) -> str:
    src = os.path.join(_HERE, "oracle_spmm.c")
    if force or not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return _SO


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build_oracle()
        L = ctypes.CDLL(_SO)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.oracle_build_operand.argtypes = [vp, vp, vp, vp, i64, vp, vp]
        for name in ("oracle_spmm_csr_f32", "oracle_spmm_csr_f64", "oracle_spmm_abs_f64"):
            getattr(L, name).argtypes = [vp, vp, vp, i64, vp, i64, i64, vp, i64]
        L.oracle_csr_transpose.argtypes = [vp, vp, vp, i64, i64, vp, vp, vp]
        L.oracle_gather_rows.argtypes = [vp, i64, vp, vp, i64, vp, i64, i64]
        for name in ("oracle_build_operand", "oracle_spmm_csr_f32", "oracle_spmm_csr_f64", "oracle_spmm_abs_f64",
                     "oracle_csr_transpose", "oracle_gather_rows"):
            getattr(L, name).restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def build_operand(fullrowptr, rowptr, colidx, normfact):
    """-> (col int32, val float32), rows sorted by column (coalesced order)."""
    fullrowptr, rowptr = _c(fullrowptr, np.int32), _c(rowptr, np.int32)
    colidx, normfact = _c(colidx, np.int32), _c(normfact, np.float32)
    nnz = int(rowptr[-1])
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, np.float32)
    load().oracle_build_operand(_p(fullrowptr), _p(rowptr), _p(colidx), _p(normfact), len(rowptr) - 1, _p(col), _p(val))
    return col, val


def _spmm(fn, out_dt, rowptr, col, val, X):
    rowptr, col, val = _c(rowptr, np.int32), _c(col, np.int32), _c(val, np.float32)
    X = _c(X, np.float32)
    M = len(rowptr) - 1
    F = X.shape[1]
    Y = np.empty((M, F), out_dt)
    getattr(load(), fn)(_p(rowptr), _p(col), _p(val), M, _p(X), F, F, _p(Y), F)
    return Y


def spmm_f32(rowptr, col, val, X):
    return _spmm("oracle_spmm_csr_f32", np.float32, rowptr, col, val, X)


def spmm_f64(rowptr, col, val, X):
    return _spmm("oracle_spmm_csr_f64", np.float64, rowptr, col, val, X)


def spmm_abs(rowptr, col, val, X):
    return _spmm("oracle_spmm_abs_f64", np.float64, rowptr, col, val, X)


def csr_transpose(rowptr, col, val, K):
    rowptr, col, val = _c(rowptr, np.int32), _c(col, np.int32), _c(val, np.float32)
    M = len(rowptr) - 1
    nnz = int(rowptr[-1])
    tr_rowptr = np.empty(K + 1, np.int32)
    tr_col = np.empty(nnz, np.int32)
    tr_val = np.empty(nnz, np.float32)
    load().oracle_csr_transpose(_p(rowptr), _p(col), _p(val), M, K, _p(tr_rowptr), _p(tr_col), _p(tr_val))
    return tr_rowptr, tr_col, tr_val


def gather_rows(src, src_idx, dst, dst_idx):
    src = _c(src, np.float32)
    assert dst.flags.c_contiguous and dst.dtype == np.float32
    si = None if src_idx is None else _c(src_idx, np.int64)
    di = None if dst_idx is None else _c(dst_idx, np.int64)
    n = len(si) if si is not None else (len(di) if di is not None else src.shape[0])
    F = dst.shape[1]
    load().oracle_gather_rows(_p(src), src.shape[1], _p(si), _p(dst), dst.shape[1], _p(di), n, F)
    return dst
