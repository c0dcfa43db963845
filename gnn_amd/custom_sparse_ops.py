"""Sparse x dense aggregation operator — drop-in for the reference's ``custom_sparse_ops``.

Reference interface (custom_sparse_ops.py:1-43, spmm_cpp/spmm.cpp:1-56):
  * ``spmm = SparseDenseMM.apply`` — Y = A·X for a coalesced sparse COO ``A`` (M x K) on
    the GPU and a dense fp32 ``X`` (K x F); backward returns ``(None, Aᵀ·G)``
    (custom_sparse_ops.py:16-37). No gradient flows to the sparse values.
  * ``create_coo_tensor(fullrowptr, rowptr, colidx, normfact, nrows, ncols)`` — the
    sampled-adjacency builder (spmm.cpp:44-50, cuda_spmm.cu:787-827).
  * module floats ``spmm_forward_time`` / ``spmm_backward_time`` read by main.py:196.
  * native entry points ``spmm_load_balance`` / ``spmm_naive`` (spmm.cpp:23-42).

Here every call lands in libgnn_spmm.so (HIP, gfx950) through its C ABI, stream-ordered on
torch's current stream with no host synchronisation. The CSR image of an operand is built
once (by ``create_coo_tensor`` or on first use of a foreign COO tensor) and cached on the
tensor; the transpose needed by backward is built on the GPU once and cached too, instead
of the reference's per-backward ``A.transpose(0,1).coalesce()`` sort.

Error behaviour mirrors the reference's TORCH_CHECKs (spmm.cpp:10-21): RuntimeError
"<arg> must be a CUDA tensor" / "must be coalesced" / "must be contiguous".

Device dispatch (BASELINE config 1, "single process on CPU via torch.sparse.mm"): when BOTH
operands of ``spmm`` live on the CPU it runs the reference's own CPU expression
(custom_sparse_ops.py:25,36: ``mat1.mm(mat2)`` forward, ``mat1.t().mm(grad)`` backward), and
``create_coo_tensor`` with CPU inputs builds the COO with the same double-precision formula
in torch. This is a device branch, not a fallback: a CUDA operand never leaves the HIP path
(a missing libgnn_spmm.so raises), mixed devices raise, and the native entry points
``spmm_load_balance`` / ``spmm_naive`` stay CUDA-only like spmm.cpp:10-21.
"""
from __future__ import annotations

import ctypes
import weakref
from typing import List, Optional, Tuple

import torch

from . import _lib

# Reference module-level timers (custom_sparse_ops.py:11-12). Accumulated in seconds from the
# aggregation kernels' own dispatch timestamps when timing is enabled (enable_timing(True)); 0.0
# otherwise, as upstream. A backward aggregation the native step executor folds into the layer
# tail below it (gnn_sage_norm_bwd_agg_f32: the top layer's, when its rows are short) has no
# launch of its own and is not in spmm_backward_time.
spmm_forward_time = 0.0
spmm_backward_time = 0.0

_timing_enabled = False
_timing_records: List[Tuple[str, "torch.cuda.Event", "torch.cuda.Event", int]] = []


def enable_timing(flag: bool = True) -> None:
    """Time every aggregation kernel (main kernel only) by its dispatch's start / end timestamps."""
    global _timing_enabled
    _timing_enabled = bool(flag)


def take_timing_records(sync: bool = True):
    """Return [(tag, ms, algorithmic_bytes, kernel_name, dims)] for recorded calls and clear
    the list (kernel_name as rocprofv3 lists the main kernel: spmm_unit_kernel<VW, G, NJ, U, RES> or,
    small operands, spmm_row_kernel<VW, NJ, U, WPR, RES>;
    dims = {M, K, nnz, F, res_rows}: the call's shape, residual rows read if any).

    Also folds the times into spmm_forward_time / spmm_backward_time (seconds)."""
    global spmm_forward_time, spmm_backward_time
    if sync and _timing_records:
        _timing_records[-1][2].synchronize()
    out = []
    for tag, e0, e1, nbytes, kname, dims in _timing_records:
        ms = e0.elapsed_time(e1)
        out.append((tag, ms, nbytes, kname, dims))
        if tag.startswith("fwd"):
            spmm_forward_time += ms * 1e-3
        else:
            spmm_backward_time += ms * 1e-3
    _timing_records.clear()
    return out


def timing_enabled() -> bool:
    return _timing_enabled


def record_timing(tag, e0, e1, M, K, nnz, F, Fk, ldx, ldy, xptr, yptr, unit_nnz, res_rows, residual) -> None:
    """Append one timed aggregation launch (events e0 / e1 armed around its main kernel) — also
    used by the native step executor, whose launches are armed from C (gnn_amd.executor)."""
    L = _lib.lib()
    name = ctypes.create_string_buffer(128)
    _lib.check(L.gnn_spmm_kernel_name(M, K, nnz, Fk, ldx, ldy, xptr, yptr, unit_nnz, int(bool(residual)), name, 128),
               "gnn_spmm_kernel_name")
    nbytes = algorithmic_bytes(M, nnz, F)
    if residual:  # residual rows read + the row map
        nbytes += res_rows * F * 4 + M * 4
    _timing_records.append((tag, e0, e1, nbytes, name.value.decode(),
                            dict(M=M, K=K, nnz=nnz, F=F, res_rows=res_rows if residual else 0)))


def algorithmic_bytes(M: int, nnz: int, F: int) -> int:
    """gathered X rows + (col, val) + rowptr + Y write."""
    return nnz * F * 4 + nnz * 8 + (M + 1) * 4 + M * F * 4


def _stream(device: torch.device) -> int:
    return _lib.stream_of(device)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError(msg)


class CsrOperand:
    """Device CSR image of a sampled adjacency A (M x K).

    rowptr int32[M+1], col int32[nnz], val fp32[nnz], columns ascending inside each row.
    ``transpose()`` returns (and caches) the canonical CSR of Aᵀ (K x M)."""

    __slots__ = ("rowptr", "col", "val", "shape", "nnz", "_t", "_tw", "_dup_word", "__weakref__")

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, shape: Tuple[int, int]):
        self.rowptr = rowptr
        self.col = col
        self.val = val
        self.shape = (int(shape[0]), int(shape[1]))
        self.nnz = int(col.numel())
        self._t: Optional["CsrOperand"] = None  # the cached transpose (strong)
        self._tw = None  # on a transpose: weakref back to the operand it was made from (no cycle,
        # so refcounting frees an operand pair as soon as the staged batch drops it)
        self._dup_word = None  # create_coo_tensor: the builder's repeated-column word (device int64)

    @property
    def device(self) -> torch.device:
        return self.val.device

    def tensors(self) -> tuple:
        """The device tensors of the operand and of its cached transpose (for record_stream
        when the operand is built on another stream than the one that reads it)."""
        ts = (self.rowptr, self.col, self.val)
        if self._t is not None:
            ts += (self._t.rowptr, self._t.col, self._t.val)
        return ts

    def _link(self, t: "CsrOperand") -> None:
        self._t = t
        t._tw = weakref.ref(self)

    def transpose(self) -> "CsrOperand":
        if self._t is None and self._tw is not None:
            back = self._tw()
            if back is not None:
                return back
        if self._t is None:
            M, K = self.shape
            dev = self.device
            with _lib.on_device(dev):
                L = _lib.lib()
                tr_rowptr = torch.empty(K + 1, dtype=torch.int32, device=dev)
                tr_col = torch.empty(self.nnz, dtype=torch.int32, device=dev)
                tr_val = torch.empty(self.nnz, dtype=torch.float32, device=dev)
                wsb = L.gnn_csr_transpose_workspace_bytes(M, K, self.nnz)
                ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
                _lib.check(L.gnn_csr_transpose(_ptr(self.rowptr), _ptr(self.col), _ptr(self.val), M, K, self.nnz,
                                               _ptr(tr_rowptr), _ptr(tr_col), _ptr(tr_val), _ptr(ws), wsb,
                                               _stream(dev)), "gnn_csr_transpose")
            self._link(CsrOperand(tr_rowptr, tr_col, tr_val, (K, M)))
        return self._t

    def to_torch_coo(self) -> torch.Tensor:
        """Coalesced torch COO view of the operand (int64 indices, shared values)."""
        M, _ = self.shape
        rows = torch.repeat_interleave(torch.arange(M, device=self.device),
                                       (self.rowptr[1:] - self.rowptr[:-1]).long())
        idx = torch.stack([rows, self.col.long()])
        return torch.sparse_coo_tensor(idx, self.val, self.shape, is_coalesced=True)


def _resolve_duplicates(mat: torch.Tensor) -> None:
    """create_coo_tensor's deferred half of the reference's .coalesce() (cuda_spmm.cu:825): the
    builder flags a repeated (row, col) pair on the GPU (the second word of its workspace) and
    the returned tensor is marked coalesced without a host read; the first aggregation on the
    tensor reads that word (one synchronisation, like the reference's coalesce) and, if it is
    set, coalesces the tensor in place (the duplicates summed, nnz shrinks) and drops the CSR
    image built from the uncoalesced entries."""
    word = mat._gnn_dup
    mat._gnn_dup = None
    if int(word.item()) == 0:
        return
    coal = torch.sparse_coo_tensor(mat._indices(), mat._values(), mat.shape).coalesce()
    mat.copy_(coal)
    mat._gnn_csr = None


def finalize_coalesce(mat: torch.Tensor) -> torch.Tensor:
    """Complete create_coo_tensor's deferred coalesce now (one synchronisation) and return the
    tensor: afterwards its indices hold no repeated (row, col) pair, so any torch operator may
    consume it. The aggregation entry points (spmm, spmm_load_balance, csr_of) call this
    themselves; other consumers of a create_coo_tensor result whose inputs may repeat a column
    within a row call it first. A no-op for every other tensor."""
    if getattr(mat, "_gnn_dup", None) is not None:
        _resolve_duplicates(mat)
    return mat


def csr_of(mat: "torch.Tensor | CsrOperand") -> CsrOperand:
    """CSR image of a sampled operand: cached one, or built on the GPU from a coalesced COO."""
    if isinstance(mat, CsrOperand):
        return mat
    if getattr(mat, "_gnn_dup", None) is not None:
        _resolve_duplicates(mat)
    plan = getattr(mat, "_gnn_csr", None)
    if plan is not None:
        return plan
    _require(isinstance(mat, torch.Tensor) and mat.is_sparse, "sparseMat must be a sparse COO tensor")
    _require(mat.is_cuda, "sparseMat must be a CUDA tensor")
    _require(mat.is_coalesced(), "sparseMat must be coalesced")
    _require(mat.dtype == torch.float32, "sparseMat must be float32")
    M, K = mat.shape
    nnz = mat._nnz()
    _require(M < 2**31 and K < 2**31 and nnz < 2**31, "sparseMat dims and nnz must be < 2^31")
    dev = mat.device
    idx = mat._indices()
    with _lib.on_device(dev):
        rowptr = torch.empty(M + 1, dtype=torch.int32, device=dev)
        col = torch.empty(nnz, dtype=torch.int32, device=dev)
        L = _lib.lib()
        row_ptr = idx[0].data_ptr() if nnz else None
        col_ptr = idx[1].data_ptr() if nnz else None
        if nnz and not idx.is_contiguous():
            idx = idx.contiguous()
            row_ptr, col_ptr = idx[0].data_ptr(), idx[1].data_ptr()
        _lib.check(L.gnn_coo_to_csr(row_ptr, col_ptr, nnz, M, _ptr(rowptr), _ptr(col) if nnz else None,
                                    _stream(dev)), "gnn_coo_to_csr")
    plan = CsrOperand(rowptr, col, mat._values().contiguous(), (M, K))
    try:
        mat._gnn_csr = plan
    except AttributeError:  # pragma: no cover - tensors normally accept attributes
        pass
    return plan


def spmm_csr(op: CsrOperand, dense: torch.Tensor, tag: str = "fwd", unit_nnz: int = 0,
             residual: Optional[torch.Tensor] = None, rmap: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Y = A·X on the GPU. ``dense`` must be fp32, row-major rows (stride(1) == 1); a padded
    row stride (stride(0) > F) is accepted and read in place.

    With ``rmap`` (int32[M], -1 = none) the rows ``residual[rmap[r]]`` are added to the
    output rows in the same kernel (gnn_spmm_csr_f32_ex)."""
    _require(dense.is_cuda, "denseMat must be a CUDA tensor")
    _require(dense.dim() == 2, "denseMat must be 2-D")
    _require(dense.dtype == torch.float32, "denseMat must be float32")
    _require(dense.stride(1) == 1 or dense.shape[1] <= 1, "denseMat must be contiguous")
    M, K = op.shape
    _require(dense.shape[0] == K, f"size mismatch: sparse {tuple(op.shape)} @ dense {tuple(dense.shape)}")
    _require(dense.device == op.device, "sparseMat and denseMat must be on the same device")
    F = dense.shape[1]
    ldx = dense.stride(0) if dense.shape[0] > 1 else max(F, 1)
    dev = dense.device
    # Padded rows (the layer-0 staging buffer: 602 floats in 608-float rows): let the
    # kernel run over the padded width Fk = round_up(F, 4) so it can use 16-byte loads, into
    # an output with the same padded stride; the caller gets the (M x F) view.
    if rmap is not None:
        _require(residual is not None and residual.is_cuda and residual.dtype == torch.float32,
                 "residual must be a float32 CUDA tensor")
        _require(rmap.is_cuda and rmap.dtype == torch.int32 and rmap.is_contiguous() and rmap.numel() == M,
                 "rmap must be a contiguous int32 CUDA tensor of M entries")
        _require(residual.dim() == 2 and residual.shape[1] == F and residual.stride(1) == 1,
                 "residual rows must be contiguous with F columns")
    Fk = F
    if F % 4 and ldx % 4 == 0 and dense.data_ptr() % 16 == 0 and rmap is None:
        F4 = F + (4 - F % 4)
        avail = dense.untyped_storage().nbytes() // 4 - dense.storage_offset()
        if ldx >= F4 and (K - 1) * ldx + F4 <= avail:
            Fk = F4
    # A padded input gets an output with the same row stride (line-aligned rows for the
    # consumer GEMM and whole-line row stores).
    ldo = ldx if (Fk != F and ldx <= 2 * Fk) else Fk
    with _lib.on_device(dev):
        out = torch.empty((M, ldo), dtype=torch.float32, device=dev)
        if M == 0 or F == 0:
            return out[:, :F]
        L = _lib.lib()
        wsb = L.gnn_spmm_workspace_bytes(M, op.nnz, Fk, unit_nnz)
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
        st = _stream(dev)
        if _timing_enabled:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()  # creates the underlying hipEvent; the library re-records it
            e1.record()
            L.gnn_spmm_set_timing_events(e0.cuda_event, e1.cuda_event)
            record_timing(tag, e0, e1, M, K, op.nnz, F, Fk, ldx, ldo, dense.data_ptr(), out.data_ptr(), unit_nnz,
                          residual.shape[0] if rmap is not None else 0, rmap is not None)
        if rmap is None:
            _lib.check(L.gnn_spmm_csr_f32(_ptr(op.rowptr), _ptr(op.col), _ptr(op.val), M, K, op.nnz,
                                          dense.data_ptr(), ldx, out.data_ptr(), ldo, Fk,
                                          ws.data_ptr(), wsb, unit_nnz, st), "gnn_spmm_csr_f32")
        else:
            ldr = residual.stride(0) if residual.shape[0] > 1 else max(F, 1)
            _lib.check(L.gnn_spmm_csr_f32_ex(_ptr(op.rowptr), _ptr(op.col), _ptr(op.val), M, K, op.nnz,
                                             dense.data_ptr(), ldx, out.data_ptr(), ldo, Fk,
                                             residual.data_ptr(), ldr, rmap.data_ptr(),
                                             ws.data_ptr(), wsb, unit_nnz, st), "gnn_spmm_csr_f32_ex")
    return out if Fk == F else out[:, :F]


def _on_cpu(mat1, mat2) -> bool:
    """Both operands on the CPU: the config-1 torch.sparse.mm branch."""
    return (isinstance(mat1, torch.Tensor) and isinstance(mat2, torch.Tensor) and mat1.device.type == "cpu"
            and mat2.device.type == "cpu")


class SparseDenseMM(torch.autograd.Function):
    """custom_sparse_ops.py:16-37: forward A·X, backward (None, Aᵀ·G)."""

    @staticmethod
    def forward(ctx, mat1, mat2):
        if _on_cpu(mat1, mat2):
            # custom_sparse_ops.py:25 (the reference's CPU expression)
            _require(mat1.is_sparse, "sparseMat must be a sparse COO tensor")
            ctx.cpu_mat1 = mat1
            return torch.sparse.mm(mat1, mat2)
        op = csr_of(mat1)
        _require(mat2.is_cuda, "denseMat must be a CUDA tensor")
        ctx.op = op
        return spmm_csr(op, mat2, tag="fwd")

    @staticmethod
    def backward(ctx, grad_output):
        if not ctx.needs_input_grad[1]:
            return None, None
        if getattr(ctx, "cpu_mat1", None) is not None:
            # custom_sparse_ops.py:36, with the coalesce() torch needs for a transposed COO
            return None, torch.sparse.mm(ctx.cpu_mat1.t().coalesce(), grad_output.contiguous())
        op_t = ctx.op.transpose()
        return None, spmm_csr(op_t, grad_output.contiguous(), tag="bwd")


spmm = SparseDenseMM.apply


def spmm_load_balance(sparseMat, denseMat) -> torch.Tensor:
    """Native entry point of spmm.cpp:23-27 (no autograd)."""
    _require(isinstance(sparseMat, CsrOperand) or sparseMat.is_cuda, "sparseMat must be a CUDA tensor")
    if isinstance(sparseMat, torch.Tensor):
        _require(sparseMat.is_coalesced(), "sparseMat must be coalesced")
    _require(denseMat.is_cuda, "denseMat must be a CUDA tensor")
    _require(denseMat.is_contiguous(), "denseMat must be contiguous")
    return spmm_csr(csr_of(sparseMat), denseMat)


# spmm.cpp:38-42 binds a second kernel with the same math; one kernel serves both here.
spmm_naive = spmm_load_balance



def build_operand(fullrowptr: torch.Tensor, rowptr: torch.Tensor, colidx: torch.Tensor, normfact: torch.Tensor,
                  nrows: int, ncols: int, with_coo: bool = True, sorted_rows: bool = False):
    """Device operand from the sampler's CSR pieces. Returns (CsrOperand, coo_indices|None).
    sorted_rows=True: the caller guarantees column-ascending rows (the native samplers' output)
    and the unsorted-row pass is not launched."""
    for name, t in (("fullrowptr", fullrowptr), ("rowptr", rowptr), ("normfact", normfact)):
        _require(t.is_cuda, f"{name} must be a CUDA tensor")
        _require(t.is_contiguous(), f"{name} must be contiguous")
    _require(colidx.is_cuda, "colidx must be a CUDA tensor")
    _require(fullrowptr.dtype == torch.int32 and rowptr.dtype == torch.int32, "row pointers must be int32")
    _require(normfact.dtype == torch.float32, "normfact must be float32")
    _require(colidx.dtype in (torch.int16, torch.int32, torch.int64), "colidx must be int16/int32/int64")
    _require(rowptr.numel() == nrows + 1 and fullrowptr.numel() == nrows + 1, "row pointer length != nrows + 1")
    colidx = colidx.contiguous()
    nnz = colidx.numel()
    dev = colidx.device
    with _lib.on_device(dev):
        col32 = torch.empty(nnz, dtype=torch.int32, device=dev)
        val = torch.empty(nnz, dtype=torch.float32, device=dev)
        coo = torch.empty((2, nnz), dtype=torch.int64, device=dev) if with_coo else None
        if sorted_rows:
            _lib.check(_lib.lib().gnn_build_operand_sorted_f32(
                _ptr(fullrowptr), _ptr(rowptr), _ptr(colidx), colidx.element_size(), _ptr(normfact),
                nrows, ncols, nnz, _ptr(col32), _ptr(val), _ptr(coo), _stream(dev)), "gnn_build_operand_sorted_f32")
        else:
            wsb = _lib.lib().gnn_build_operand_workspace_bytes()
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)  # the unsorted-row and repeated-column words
            _lib.check(_lib.lib().gnn_build_operand_f32(
                _ptr(fullrowptr), _ptr(rowptr), _ptr(colidx), colidx.element_size(), _ptr(normfact),
                nrows, ncols, nnz, _ptr(col32), _ptr(val), _ptr(coo), _ptr(ws), wsb, _stream(dev)),
                "gnn_build_operand_f32")
    op = CsrOperand(rowptr, col32, val, (nrows, ncols))
    if not sorted_rows and nrows > 0 and nnz > 1:
        op._dup_word = ws.view(torch.int64)[1:2]  # set on the GPU iff a row repeats a column
    return op, coo


def extract_operand(graph, rows: torch.Tensor, cols: torch.Tensor, normfact: torch.Tensor, nnz: int,
                    rowseg: torch.Tensor, colseg: Optional[torch.Tensor] = None,
                    colptr: Optional[torch.Tensor] = None, rowseg_total: Optional[int] = None,
                    colseg_total: Optional[int] = None) -> CsrOperand:
    """adj = lap[rows, :][:, cols] with create_coo_tensor's values, built on the GPU from the
    graph resident there (gnn_ladies_extract_f32; ``graph`` a sampler.DeviceGraph): the
    operand of a LADIES layer whose draw ran on the host (sampler.py:114-139). ``nnz`` is the
    host-known entry count (the column counts of U over cols); ``rowseg`` U's row pointer (M+1).
    With ``colseg`` (offsets of lapᵀ's rows of cols, K+1) and ``colptr`` (the CSC column
    pointer, K+1; rows must be unique and ascending) the transpose is built too and cached on
    the operand — the canonical Aᵀ (A.t().coalesce()). ``rowseg_total`` / ``colseg_total`` =
    rowseg[M] / colseg[K] (the graph entries scanned per direction; they size the launch): pass
    the host's values — if omitted they are read back from the device (a synchronisation)."""
    for name, t in (("rows", rows), ("cols", cols), ("rowseg", rowseg)):
        _require(t.is_cuda and t.dtype == torch.int32 and t.is_contiguous(), f"{name} must be contiguous int32 CUDA")
    _require(normfact.is_cuda and normfact.dtype == torch.float32 and normfact.numel() == cols.numel(),
             "normfact must be float32 CUDA with one entry per column")
    M, K, nnz = rows.numel(), cols.numel(), int(nnz)
    dev = rows.device
    with _lib.on_device(dev):
        rowptr = torch.empty(M + 1, dtype=torch.int32, device=dev)
        col = torch.empty(nnz, dtype=torch.int32, device=dev)
        val = torch.empty(nnz, dtype=torch.float32, device=dev)
        rows_t = val_t = None
        _require(rowseg.numel() == M + 1, "rowseg must have M + 1 entries")
        _require((colptr is None) == (colseg is None), "colptr and colseg come together")
        if colptr is not None:
            for name, t in (("colptr", colptr), ("colseg", colseg)):
                _require(t.is_cuda and t.dtype == torch.int32 and t.numel() == K + 1,
                         f"{name} must be int32 CUDA with K + 1 entries")
            rows_t = torch.empty(nnz, dtype=torch.int32, device=dev)
            val_t = torch.empty(nnz, dtype=torch.float32, device=dev)
        if rowseg_total is None:
            rowseg_total = int(rowseg[M].item())
        if colptr is not None and colseg_total is None:
            colseg_total = int(colseg[K].item())
        L = _lib.lib()
        wsb = L.gnn_ladies_extract_workspace_bytes(graph.num_nodes, M, K, int(colptr is not None),
                                                   int(rowseg_total), int(colseg_total or 0))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        st = _stream(dev)
        _lib.check(L.gnn_ladies_extract_f32(
            _ptr(graph.indptr), _ptr(graph.indices), _ptr(graph.degree), graph.num_nodes, _ptr(graph.indptr_t),
            _ptr(graph.indices_t),
            _ptr(rows), M, _ptr(cols), K, _ptr(normfact), nnz, _ptr(rowseg), _ptr(colseg), _ptr(colptr),
            int(rowseg_total), int(colseg_total or 0), _ptr(rowptr), _ptr(col), _ptr(val), _ptr(rows_t), _ptr(val_t), ws.data_ptr(), wsb, _ptr(graph.err), st),
            "gnn_ladies_extract_f32")
    op = CsrOperand(rowptr, col, val, (M, K))
    if colptr is not None:
        op._link(CsrOperand(colptr, rows_t, val_t, (K, M)))
    return op


def attach_transpose(op: CsrOperand, fullrowptr: torch.Tensor, colptr: torch.Tensor, rows: torch.Tensor,
                     normfact: torch.Tensor) -> CsrOperand:
    """Cache on ``op`` its transpose built from a caller-provided CSC structure (colptr,
    rows: rows ascending per column, e.g. from the native sampler) — only the values are
    computed on the GPU (gnn_build_operand_t_f32); the result equals op.transpose()."""
    M, K = op.shape
    _require(colptr.numel() == K + 1 and rows.numel() == op.nnz, "CSC structure does not match the operand")
    for name, t in (("colptr", colptr), ("rows", rows)):
        _require(t.is_cuda and t.dtype == torch.int32 and t.is_contiguous(), f"{name} must be contiguous int32 CUDA")
    dev = op.device
    with _lib.on_device(dev):
        val = torch.empty(op.nnz, dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().gnn_build_operand_t_f32(_ptr(fullrowptr), _ptr(colptr), _ptr(rows), _ptr(normfact),
                                                      M, K, op.nnz, _ptr(val), _stream(dev)),
                   "gnn_build_operand_t_f32")
    t = CsrOperand(colptr, rows, val, (K, M))
    op._link(t)
    return t


def _create_coo_tensor_cpu(fullrowptr, rowptr, colidx, normfact, nrows: int, ncols: int) -> torch.Tensor:
    """The config-1 CPU branch of create_coo_tensor: cuda_spmm.cu:795-802's formula in torch,
    value = (float)((1.0 / full_degree(row)) * (double)normfact[col]) (two double roundings
    then one to fp32, the same operations as the HIP builder), then .coalesce()
    (cuda_spmm.cu:825)."""
    rp = rowptr.to(torch.int64)
    rows = torch.repeat_interleave(torch.arange(nrows, dtype=torch.int64), rp[1:] - rp[:-1])
    col = colidx.to(torch.int64)  # int16 sign-extends like the reference's accessor
    deg = (fullrowptr[1:] - fullrowptr[:-1]).to(torch.float64)
    val = ((1.0 / deg)[rows] * normfact.to(torch.float64)[col]).to(torch.float32)
    return torch.sparse_coo_tensor(torch.stack([rows, col]), val, (nrows, ncols)).coalesce()


def create_coo_tensor(fullrowptr, rowptr, colidx, normfact, nrows, ncols) -> torch.Tensor:
    """spmm.cpp:44-50 / cuda_spmm.cu:806-827: coalesced sparse COO of the sampled layer with
    value = (1/full_degree(row)) * normfact[col] (double math, fp32 store). The CSR image
    is cached on the returned tensor for the aggregation kernels. CPU inputs (all four)
    take the config-1 CPU branch.

    Coalescing contract (GPU inputs): the call reads nothing back to the host, so it stays
    stream-ordered and graph-capturable. Columns come out ascending per row and the tensor is
    marked coalesced. If the inputs repeat a column within a row (the reference's samplers never
    do: LADIES' after nodes are unique, sampler.py:135-139), the repeats are summed, as the
    reference's .coalesce() does (cuda_spmm.cu:825), by the first aggregation on the tensor or by
    ``finalize_coalesce(t)``. Until then ``_nnz()`` / ``_indices()`` / ``_values()`` show the
    unmerged entries: a caller that hands such a tensor to another torch operator calls
    ``finalize_coalesce`` first."""
    ins = (fullrowptr, rowptr, colidx, normfact)
    if all(isinstance(t, torch.Tensor) and t.device.type == "cpu" for t in ins):
        return _create_coo_tensor_cpu(*ins, int(nrows), int(ncols))
    op, coo = build_operand(fullrowptr, rowptr, colidx, normfact, int(nrows), int(ncols), with_coo=True)
    t = torch.sparse_coo_tensor(coo, op.val, (int(nrows), int(ncols)), is_coalesced=True)
    t._gnn_csr = op
    # A repeated column within a row (the reference's samplers never make one: LADIES' after nodes
    # are unique, sampler.py:135-139) is flagged by the builder on the GPU; no host read here (the
    # call stays stream-ordered and graph-capturable): the first aggregation on the tensor reads
    # the flag and, if set, sums the duplicates in place as the reference's .coalesce() does
    # (cuda_spmm.cu:825; _resolve_duplicates).
    t._gnn_dup = getattr(op, "_dup_word", None)
    return t


def _padded_width(src: torch.Tensor, dst: torch.Tensor, F: int) -> int:
    """Rows of a 602-wide layer live in 608-float (whole 128-byte line) rows: when both row
    strides are multiples of 4 and every row's storage holds the padded width, copy F rounded
    up to 4 floats so the kernel moves 16-byte vectors (the padding columns are don't-care:
    no consumer reads them). Layer-0 x[sampled]: 19 -> ~12 µs."""
    F4 = (F + 3) & ~3
    if F4 == F:
        return F
    for t in (src, dst):
        r = t.shape[0]
        if (t.stride(0) % 4 or t.stride(0) < F4 or t.data_ptr() % 16
                or (r > 0 and (t.storage_offset() + (r - 1) * t.stride(0) + F4) * 4 > t.untyped_storage().nbytes())):
            return F
    return F4


def gather_rows(src: torch.Tensor, src_idx: Optional[torch.Tensor], dst: torch.Tensor,
                dst_idx: Optional[torch.Tensor], n: Optional[int] = None) -> None:
    """dst[dst_idx] = src[src_idx] row copy on the GPU (int64 indices, fp32 rows)."""
    _require(src.is_cuda and dst.is_cuda, "gather_rows tensors must be CUDA tensors")
    _require(src.dtype == torch.float32 and dst.dtype == torch.float32, "gather_rows tensors must be float32")
    _require(src.stride(1) == 1 and dst.stride(1) == 1, "gather_rows rows must be contiguous")
    F = dst.shape[1]
    _require(src.shape[1] >= F, "gather_rows: source rows narrower than destination")
    F = _padded_width(src, dst, F)
    if n is None:
        n = int((src_idx if src_idx is not None else dst_idx).numel()) if (src_idx is not None or dst_idx is not None) \
            else int(src.shape[0])
    for t in (src_idx, dst_idx):
        if t is not None:
            _require(t.is_cuda and t.dtype == torch.int64 and t.is_contiguous(), "gather_rows indices must be int64 CUDA")
    dev = dst.device
    with _lib.on_device(dev):
        _lib.check(_lib.lib().gnn_gather_rows_f32(src.data_ptr(), src.stride(0), _ptr(src_idx), dst.data_ptr(),
                                                  dst.stride(0), _ptr(dst_idx), n, F, _stream(dev)),
                   "gnn_gather_rows_f32")


def gather_rows2(src0: torch.Tensor, idx0: Optional[torch.Tensor], pos0: Optional[torch.Tensor], n0: int,
                 src1: torch.Tensor, idx1: Optional[torch.Tensor], pos1: Optional[torch.Tensor], n1: int,
                 dst: torch.Tensor) -> None:
    """dst[pos0] = src0[idx0] (n0 rows) and dst[pos1] = src1[idx1] (n1 rows) in one launch
    (gnn_gather_rows2_f32): X0's own-buffer and host rows."""
    for t in (src0, src1, dst):
        _require(t.is_cuda and t.dtype == torch.float32 and t.stride(1) == 1,
                 "gather_rows2 tensors must be float32 CUDA tensors with contiguous rows")
    for t in (idx0, pos0, idx1, pos1):
        if t is not None:
            _require(t.is_cuda and t.dtype == torch.int64 and t.is_contiguous(), "gather_rows2 indices must be int64 CUDA")
    F = dst.shape[1]
    _require(src0.shape[1] >= F and src1.shape[1] >= F, "gather_rows2: source rows narrower than destination")
    F = min(_padded_width(src0, dst, F), _padded_width(src1, dst, F))
    dev = dst.device
    with _lib.on_device(dev):
        _lib.check(_lib.lib().gnn_gather_rows2_f32(src0.data_ptr(), src0.stride(0), _ptr(idx0), _ptr(pos0), int(n0),
                                                   src1.data_ptr(), src1.stride(0), _ptr(idx1), _ptr(pos1), int(n1),
                                                   dst.data_ptr(), dst.stride(0), F, _stream(dev)),
                   "gnn_gather_rows2_f32")


def gather_rows_host(host: torch.Tensor, src_idx: torch.Tensor, dst: torch.Tensor,
                     dst_idx: Optional[torch.Tensor], n: Optional[int] = None) -> None:
    """dst[dst_idx] = host[src_idx], read by the GPU over PCIe from a host table registered
    with gnn_host_register (FeatureStore(zero_copy=True)); int64 device indices."""
    _require(not host.is_cuda and host.dtype == torch.float32 and host.stride(1) == 1,
             "gather_rows_host: host must be a registered fp32 CPU table with contiguous rows")
    _require(dst.is_cuda and dst.dtype == torch.float32 and dst.stride(1) == 1,
             "gather_rows_host: dst must be a float32 CUDA tensor with contiguous rows")
    _require(src_idx.is_cuda and src_idx.dtype == torch.int64 and src_idx.is_contiguous(),
             "gather_rows_host: src_idx must be int64 CUDA")
    if dst_idx is not None:
        _require(dst_idx.is_cuda and dst_idx.dtype == torch.int64 and dst_idx.is_contiguous(),
                 "gather_rows_host: dst_idx must be int64 CUDA")
    F = dst.shape[1]
    _require(host.shape[1] >= F, "gather_rows_host: source rows narrower than destination")
    n = int(src_idx.numel()) if n is None else n
    dev = dst.device
    with _lib.on_device(dev):
        _lib.check(_lib.lib().gnn_gather_rows_host_f32(host.data_ptr(), host.stride(0), src_idx.data_ptr(),
                                                       dst.data_ptr(), dst.stride(0), _ptr(dst_idx), n, F,
                                                       _stream(dev)),
                   "gnn_gather_rows_host_f32")


def spmm_config(M: int, nnz: int, F: int, ldx: Optional[int] = None, ldy: Optional[int] = None,
                unit_nnz: int = 0, K: int = 0) -> dict:
    """Kernel configuration the library picks for a call shape (16-byte aligned buffers)."""
    out = (ctypes.c_int32 * 6)()
    _lib.check(_lib.lib().gnn_spmm_config(M, K, nnz, F, ldx or F, ldy or F, 256, 256, unit_nnz, out),
               "gnn_spmm_config")
    name = ctypes.create_string_buffer(128)
    _lib.check(_lib.lib().gnn_spmm_kernel_name(M, K, nnz, F, ldx or F, ldy or F, 256, 256, unit_nnz, 0, name, 128),
               "gnn_spmm_kernel_name")
    return dict(vw=out[0], g=out[1], nj=out[2], tiles=out[3], unit_nnz=out[4], units=out[5],
                kernel=name.value.decode())
