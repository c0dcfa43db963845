"""LADIES layer-wise importance sampler and the batch scheduler (host side).

Restates sampler.py:90-160 (``ladies_sampler``) and sampler.py:164-193 (``prepare_data``)
of the reference with the same numpy call sequence, so a given seed yields the same
sampled nodes, sub-graph CSR and masks (pinned by tests/golden). The split is:

  * ``ladies_sample_host`` — pure numpy/scipy; returns a ``HostBatch`` (CSR pieces per
    layer, feature-placement indices, labels). Runs in sampler worker processes: no GPU.
  * ``HostBatch.to_device`` — H2D of the index arrays and the GPU operand build
    (``custom_sparse_ops.build_operand``, the create_coo_tensor kernel).
  * ``ladies_sampler`` — the reference's signature and return tuple, both steps in one.

Deviation (documented, values unchanged): column ids travel as int32 instead of int16
(sampler.py:136), lifting the 32,767-column cap; the values are identical whenever the
reference's int16 would not have overflowed.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import scipy.sparse as sp
import torch


@dataclass
class HostLayer:
    fullrowptr: Optional[np.ndarray]  # int32 [M+1]: indptr of U = lap[previous, :]
    rowptr: Optional[np.ndarray]      # int32 [M+1]: indptr of U[:, after]
    colidx: Optional[np.ndarray]      # int32 [nnz]
    normfact: np.ndarray    # float32 [K]: 1 / float32(clip(s_num * p[after], 1e-10, 1))
    shape: tuple            # (M, K)
    csc_colptr: Optional[np.ndarray] = None  # int32 [K+1]: CSC of the sub-graph (= CSR of its
    csc_rows: Optional[np.ndarray] = None    # transpose, rows ascending per column), if made
    # A layer left to the GPU extraction (gnn_ladies_extract_f32): rowptr / colidx are None;
    # rows = U's rows (node ids, ascending), cols = after_nodes, csc_colptr from the column
    # counts, fullrowptr = U's row pointer (the forward segments), colseg = the offsets of lapᵀ's
    # rows of cols (the transposed segments), dev_nnz = its exact nnz.
    rows: Optional[np.ndarray] = None
    cols: Optional[np.ndarray] = None
    dev_nnz: int = -1
    colseg: Optional[np.ndarray] = None

    @property
    def on_device(self) -> bool:
        return self.colidx is None and self.rows is not None

    @property
    def nnz(self) -> int:
        return int(self.dev_nnz) if self.on_device else int(self.colidx.size)


@dataclass
class HostBatch:
    layers: List[Optional[HostLayer]]          # bottom-up (layer 0 first), as adjs
    sampled_nodes: List[np.ndarray]            # bottom-up
    input_nodes: np.ndarray                    # ids of the layer-0 input rows (sorted)
    input_nodes_mask_on_devices: List[np.ndarray]
    input_nodes_mask_on_cpu: np.ndarray
    nodes_idx_on_devices: List[np.ndarray]
    nodes_idx_on_cpu: np.ndarray
    batch_nodes: np.ndarray
    labels: np.ndarray                         # dense float32 [batch, classes]
    seed: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def num_input_nodes(self) -> int:
        return int(len(self.input_nodes))

    def nnz(self) -> int:
        return int(sum(l.nnz for l in self.layers if l is not None))

    def pin(self) -> "HostBatch":
        """Copy the arrays the GPU needs into pinned host tensors (done by the batch producer
        thread, so the training thread only issues asynchronous copies)."""
        if "pinned" not in self.extra:
            pin = torch.cuda.is_available()
            t = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a, dtype=dt))
            p = lambda x: None if x is None else (t(x).pin_memory() if pin else t(x))
            layers = [None if L is None else
                      (p(L.fullrowptr), p(L.rowptr), p(L.colidx), p(L.normfact), p(L.csc_colptr), p(L.csc_rows),
                       p(L.rows), p(L.cols), p(L.colseg))
                      for L in self.layers]
            sampled = [p(t(s, np.int64)) for s in self.sampled_nodes]
            self.extra["pinned"] = (layers, sampled, p(t(self.labels)))
        if "rmaps" not in self.extra:
            # inverse of sampled_nodes over the layer's input rows (rmap[sampled[i]] = i, -1 else):
            # the row map of the fused backward residual (gnn_spmm_csr_f32_ex), made here so the
            # training step launches no fill/arange/index_put for it
            pin = torch.cuda.is_available()
            rm = []
            for li, (L, sn) in enumerate(zip(self.layers, self.sampled_nodes)):
                if L is None or li == 0 or len(sn) == 0:
                    rm.append(None)
                    continue
                r = np.full(L.shape[1], -1, dtype=np.int32)
                r[np.asarray(sn, dtype=np.int64)] = np.arange(len(sn), dtype=np.int32)
                x = torch.from_numpy(r)
                rm.append(x.pin_memory() if pin else x)
            self.extra["rmaps"] = rm
        return self

    def cpu_inputs(self, feat_data: torch.Tensor):
        """BASELINE config 1 (single process on the CPU): (adjs, x0, sampled_nodes, labels)
        with the operands built by create_coo_tensor's CPU branch and X0 = the layer-0 input
        rows of the host feature table (main.py:129-134 with every row on the host)."""
        from . import custom_sparse_ops as cso

        adjs = []
        for L in self.layers:
            if L is None:
                adjs.append(None)
                continue
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
            adjs.append(cso.create_coo_tensor(t(L.fullrowptr), t(L.rowptr), t(L.colidx), t(L.normfact), *L.shape))
        x0 = feat_data[torch.from_numpy(np.asarray(self.input_nodes, dtype=np.int64))]
        sampled = [torch.from_numpy(np.asarray(s, dtype=np.int64)) for s in self.sampled_nodes]
        return adjs, x0, sampled, torch.from_numpy(self.labels)

    def to_device(self, device, with_coo: bool = True, build: bool = True, graph: "Optional[DeviceGraph]" = None):
        """Materialise on the GPU (H2D of the CSR pieces — or, for layers left to the GPU
        extraction, of their rows / columns / CSC column pointer — labels, sampled_nodes) and,
        unless build=False, run the operand builder / extraction. Returns a DeviceBatch.
        ``graph``: the graph resident on the device (default: device_graph() of the batch's
        sampler graph), needed only by GPU-extracted layers."""
        dev = torch.device(device)
        layers, sampled, labels = self.pin().extra["pinned"]
        d = lambda x: None if x is None else x.to(dev, non_blocking=True)
        raw = [None if P is None else (d(P[0]), d(P[1]), d(P[2]), d(P[3]), L.shape, d(P[4]), d(P[5]), d(P[6]),
                                       d(P[7]), L.nnz, d(P[8]))
               for P, L in zip(layers, self.layers)]
        sn = [d(s) for s in sampled]
        for x, r in zip(sn, self.extra["rmaps"]):
            if r is not None:
                x._gnn_rmap = d(r)  # read by fused.SageAggregateFn's backward
        if graph is None and any(L is not None and L.on_device for L in self.layers):
            graph = device_graph(self.extra["graph"], dev)
        db = DeviceBatch(self, raw, None, sn, d(labels), graph)
        if build:
            db.build_operands(with_coo=with_coo)
        return db


@dataclass
class DeviceBatch:
    host: HostBatch
    raw: list            # per layer: device (fullrowptr, rowptr, colidx, normfact, shape, csc_colptr|None,
                         # csc_rows|None, rows|None, cols|None, nnz, colseg|None) or None
    adjs: Optional[list]
    sampled_nodes: list
    labels: torch.Tensor
    graph: Optional["DeviceGraph"] = None
    # pinned host copy of the graph's extraction error flag, taken on the build stream right after
    # this batch's GPU extractions (None when no layer was extracted on the GPU)
    err_host: Optional[torch.Tensor] = None
    # a natively staged batch (loader.NativeBatch.stage): raw is None, the operands are views of
    # these allocations (the device blob and the staging arena)
    keep: Optional[list] = None

    def check_extraction(self, err_host: Optional[torch.Tensor] = None) -> None:
        """Raise if a GPU extraction up to and including this batch's saw a device count that
        disagrees with the host's (``err_host``: the flag of a given build; default the latest).
        The caller makes sure the build stream has passed the flag's copy (StagedX0.wait
        synchronises on the staging event first)."""
        flag = self.err_host if err_host is None else err_host
        if flag is not None and int(flag[0]):
            raise RuntimeError(f"gnn_ladies_extract_f32: device counts disagree with the host's "
                               f"(flag {int(flag[0])}); the batch's operand is not used")

    def tensors(self) -> list:
        """Every device tensor the step reads: CSR pieces, sampled_nodes (+ residual row
        maps), labels and the built operands (record_stream across streams)."""
        ts = [t for r in (self.raw or []) if r is not None
              for t in (r[0], r[1], r[2], r[3], r[5], r[6], r[7], r[8], r[10]) if t is not None]
        ts.extend(self.keep or [])
        for x in self.sampled_nodes:
            ts.append(x)
            if getattr(x, "_gnn_rmap", None) is not None:
                ts.append(x._gnn_rmap)
        ts.append(self.labels)
        for a in self.adjs or []:
            if a is not None:
                ts.extend(a.tensors() if hasattr(a, "tensors") else a._gnn_csr.tensors())
        return ts

    def build_operands(self, with_coo: bool = False) -> list:
        """create_coo_tensor for every layer (stream-ordered on the current stream)."""
        from . import custom_sparse_ops as cso

        if self.raw is None:
            raise RuntimeError("DeviceBatch: staged natively (gnn_stage_batch_f32); its operands are built")
        adjs = []
        csc_from = int(self.host.extra.get("csc_from", 1))
        for li, r in enumerate(self.raw):
            if r is None:
                adjs.append(None)
                continue
            fr, rp, ci, nf, shape, cp, cr, rows, cols, nnz, cs = r
            if ci is None:  # left to the GPU extraction (rows / cols / column counts from the draw)
                _require_graph(self.graph)
                tr = li >= csc_from
                hl = self.host.layers[li]  # host views of the same offsets: their totals size the launch
                op = cso.extract_operand(self.graph, rows, cols, nf, nnz, fr, cs if tr else None, cp if tr else None,
                                         rowseg_total=int(hl.fullrowptr[-1]),
                                         colseg_total=int(hl.colseg[-1]) if tr else None)
                coo = op.to_torch_coo()._indices() if with_coo else None
            else:
                op, coo = cso.build_operand(fr, rp, ci, nf, shape[0], shape[1], with_coo=with_coo,
                                            sorted_rows=bool(self.host.extra.get("sorted_rows", False)))
                if cp is not None:  # host-made CSC: the backward's operand without a GPU transpose
                    cso.attach_transpose(op, fr, cp, cr, nf)
            if with_coo:
                a = torch.sparse_coo_tensor(coo, op.val, shape, is_coalesced=True)
                a._gnn_csr = op
                adjs.append(a)
            else:
                adjs.append(op)
        self.adjs = adjs
        if self.graph is not None and any(r is not None and r[2] is None for r in self.raw):
            # the error flag as it stands after this batch's extractions, into pinned host memory on
            # the same stream: read once the staging event has completed, before the step that
            # consumes the operands is issued (StagedX0.wait)
            # a flag of its own per build: a rebuilt batch must not overwrite the flag a
            # staged copy of its previous build is about to read
            self.err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self.err_host.copy_(self.graph.err, non_blocking=True)
        return adjs


def _require_graph(graph) -> None:
    if graph is None:
        raise RuntimeError("a GPU-extracted layer needs the graph on the device (DeviceGraph)")


class DeviceGraph:
    """A NativeGraph's structure resident in device memory for gnn_ladies_extract_f32: canonical
    CSR of lap (int64 indptr, int32 indices, int32 row degrees) and of lapᵀ (the same arrays when
    the structure is symmetric), and an error flag the extraction raises if a device count disagrees with the host's."""

    def __init__(self, graph: "NativeGraph", device):
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())  # where a bare 'cuda' allocates
        self.device = dev
        self.num_nodes = graph.num_nodes
        self.indptr = torch.from_numpy(graph.indptr).to(dev)
        self.indices = torch.from_numpy(graph.indices).to(dev)
        # row degrees as int32 (one 4-byte load per kept entry for the transposed values)
        self.degree = torch.from_numpy(np.diff(graph.indptr).astype(np.int32)).to(dev)
        self.symmetric, ipt, ixt = graph.transpose_structure
        if self.symmetric:
            self.indptr_t, self.indices_t = self.indptr, self.indices
        else:
            self.indptr_t = torch.from_numpy(ipt).to(dev)
            self.indices_t = torch.from_numpy(ixt).to(dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)

    def check(self) -> None:
        """Raise if any extraction so far saw a count that disagrees with the host's (syncs)."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f"gnn_ladies_extract_f32: device counts disagree with the host's (flag {e})")


def device_graph(graph, device) -> DeviceGraph:
    """The DeviceGraph of a NativeGraph (or lap matrix) on `device`, made once and cached."""
    g = native_graph(graph)
    dev = torch.device(device)
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    dg = g._device_graphs.get(key)
    if dg is None:
        dg = DeviceGraph(g, dev)
        g._device_graphs[key] = dg
    return dg


def column_nnz_counts(U: sp.csr_matrix, num_nodes: int) -> np.ndarray:
    """sp.linalg.norm(U, ord=0, axis=0) (sampler.py:117): nonzeros per column, int64."""
    idx = U.indices if U.data.size == 0 or np.all(U.data != 0) else U.indices[U.data != 0]
    return np.bincount(idx, minlength=num_nodes).astype(np.int64)


class NativeGraph:
    """The lap matrix as the native sampler reads it: canonical CSR (sorted, duplicate-free
    rows — what sp.linalg.norm makes of U in place, sampler.py:117), int64 indptr, int32
    indices, float32 data. Built once per graph; shared read-only by sampler threads."""

    def __init__(self, lap: sp.csr_matrix):
        self.src = lap  # the caller's matrix (cache key; kept alive so its id stays unique)
        if not sp.isspmatrix_csr(lap):
            lap = sp.csr_matrix(lap)
        if not lap.has_canonical_format:
            lap = lap.copy()
            lap.sum_duplicates()
        self.num_nodes = int(lap.shape[0])
        if lap.shape[1] != lap.shape[0]:
            raise ValueError("lap_matrix must be square")
        self.indptr = np.ascontiguousarray(lap.indptr, dtype=np.int64)
        self.indices = np.ascontiguousarray(lap.indices, dtype=np.int32)
        data = np.asarray(lap.data)
        # data == 0 entries are structure but not counted (ord-0 norm); skip the array if none
        self.data = None if np.all(data != 0) else np.ascontiguousarray(data, dtype=np.float32)
        self.lap = lap
        self._fastgcn_p = None
        self._device_graphs = {}
        self._tstruct = None

    @property
    def transpose_structure(self):
        """(symmetric, indptr_t, indices_t): lapᵀ's canonical structure, computed once; the two
        arrays are None when it equals lap's (then lap's serve for both)."""
        if self._tstruct is None:
            lt = self.lap.T.tocsr()
            lt.sum_duplicates()
            lt.sort_indices()
            sym = bool(np.array_equal(lt.indptr, self.indptr) and np.array_equal(lt.indices, self.indices))
            self._tstruct = (sym, None if sym else np.ascontiguousarray(lt.indptr, dtype=np.int64),
                             None if sym else np.ascontiguousarray(lt.indices, dtype=np.int32))
        return self._tstruct

    @property
    def fastgcn_p(self) -> np.ndarray:
        if self._fastgcn_p is None:
            from . import _lib

            p = fastgcn_probability(self.lap)
            p.flags.writeable = False  # the native draw caches per-p state: no in-place edits
            # a fresh array may reuse a freed one's address: drop every thread's cached candidates
            _lib.sampler_lib().gnn_fastgcn_p_changed()
            self._fastgcn_p = p
        return self._fastgcn_p


_native_graphs: "dict[int, NativeGraph]" = {}


def native_graph(lap) -> NativeGraph:
    if isinstance(lap, NativeGraph):
        return lap
    g = _native_graphs.get(id(lap))
    if g is None or g.src is not lap:
        g = NativeGraph(lap)
        _native_graphs.clear()  # one graph per process in practice; do not pin old ones
        _native_graphs[id(lap)] = g
    return g


class _ColCountApi(ctypes.Structure):
    """gnn_colcount_api (include/gnn_sampler.h): libgnn_spmm.so's gnn_colcount_* by address."""
    _fields_ = [("create", ctypes.c_void_p), ("add", ctypes.c_void_p), ("reset", ctypes.c_void_p),
                ("destroy", ctypes.c_void_p), ("device", ctypes.c_int32), ("indptr", ctypes.c_void_p),
                ("indices", ctypes.c_void_p)]


def colcount_api(graph, device) -> "_ColCountApi":
    """The device column-count API over the graph's DeviceGraph on `device` (made if needed)."""
    from . import _lib

    dg = device_graph(graph, device)
    L = _lib.lib()
    fp = lambda f: ctypes.cast(f, ctypes.c_void_p).value
    # the device that holds the graph's arrays (device_graph resolves a bare 'cuda' the same way)
    index = dg.device.index if dg.device.index is not None else torch.cuda.current_device()
    api = _ColCountApi(fp(L.gnn_colcount_create), fp(L.gnn_colcount_add), fp(L.gnn_colcount_reset),
                       fp(L.gnn_colcount_destroy), index, dg.indptr.data_ptr(), dg.indices.data_ptr())
    api._dg = dg  # the device arrays stay alive with the struct
    return api


class ColumnCounter:
    """A device column-count context for calls from THIS thread (gnn_ladies_sample_cc): U's column
    counts of the LADIES draw summed on the GPU; the draw and its outputs are unchanged."""

    def __init__(self, graph, device):
        from . import _lib

        self.api = colcount_api(graph, device)
        ctx = ctypes.c_void_p()
        _lib.check(_lib.lib().gnn_colcount_create(self.api.device, native_graph(graph).num_nodes, self.api.indptr,
                                                  self.api.indices, ctypes.byref(ctx)), "gnn_colcount_create")
        self.ctx = ctx

    def close(self) -> None:
        from . import _lib

        if self.ctx:
            _lib.lib().gnn_colcount_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def extract_mask(device_extract) -> int:
    """device_extract (True = every layer below the top one, False / None = none, or an iterable
    of bottom-up layer indices) as the native samplers' layer mask (-1 = all)."""
    if device_extract is True:
        return -1
    if not device_extract:
        return 0
    m = 0
    for li in device_extract:
        m |= 1 << int(li)
    return m


def _native_layers(seed, batch_nodes, samp_num_list, graph: NativeGraph, orders, kind: str = "ladies",
                   csc_from: int = 1, device_extract=False, colcount: "Optional[ColumnCounter]" = None):
    """Run gnn_ladies_sample / gnn_subgraph_sample / gnn_fastgcn_sample and copy the result
    out: (layers, sampled_nodes, input_nodes, pinned tensors). Layers >= csc_from (those
    whose input needs a gradient; layer 0's input is the features) also get their CSC.
    device_extract (LADIES; see extract_mask): those layers below the top one are left to the GPU
    extraction — only their rows, columns, segment offsets, CSC column pointer and nnz come back."""
    from . import _lib

    L = _lib.sampler_lib()
    bn = np.ascontiguousarray(batch_nodes, dtype=np.int64)
    nl = len(orders)
    sn = np.ascontiguousarray([int(samp_num_list[d]) for d in range(nl)], dtype=np.int64)
    od = np.ascontiguousarray(orders, dtype=np.int32)
    ptr = lambda a: None if a is None else a.ctypes.data
    h = ctypes.c_void_p()
    g3 = (ptr(graph.indptr), ptr(graph.indices), ptr(graph.data), graph.num_nodes)
    rest = (ptr(bn), bn.size, ptr(sn), ptr(od), nl, int(seed) & 0xFFFFFFFF, ctypes.byref(h))
    if kind == "fastgcn":
        rc = L.gnn_fastgcn_sample(*g3, ptr(graph.fastgcn_p), *rest)
    elif kind == "ladies" and colcount is not None:
        ipt = graph.transpose_structure[1] if device_extract else None
        rc = L.gnn_ladies_sample_cc(ptr(graph.indptr), ptr(graph.indices), ptr(graph.data), ptr(ipt), graph.num_nodes,
                                    *rest[:-1], extract_mask(device_extract), ctypes.byref(colcount.api), colcount.ctx,
                                    rest[-1])
    elif kind == "ladies" and device_extract:
        ipt = graph.transpose_structure[1]
        rc = L.gnn_ladies_sample_dev(ptr(graph.indptr), ptr(graph.indices), ptr(graph.data), ptr(ipt), graph.num_nodes,
                                     *rest[:-1], extract_mask(device_extract), rest[-1])
    else:
        rc = (L.gnn_ladies_sample if kind == "ladies" else L.gnn_subgraph_sample)(*g3, *rest)
    _lib.check_sampler(rc, f"gnn_{kind}_sample")
    # Outputs land straight in pinned host tensors (when a GPU is present): HostBatch.pin()
    # then has nothing left to copy and the H2D copies can be asynchronous.
    pin = torch.cuda.is_available()
    pinned_layers, pinned_sampled = [], []

    def buf(n, dt):
        t = torch.empty(int(n), dtype=dt, pin_memory=pin)
        return t, t.numpy()

    try:
        layers: List[Optional[HostLayer]] = []
        sampled: List[np.ndarray] = []
        dims = (ctypes.c_int64 * 5)()
        for li in range(nl):
            absent = L.gnn_ladies_layer_dims(h, li, dims)
            if absent:
                layers.append(None)
                sampled.append(np.zeros(0, dtype=np.int64))
                pinned_layers.append(None)
                pinned_sampled.append(buf(0, torch.int64)[0])
                continue
            M, K, nnz, ns = dims[0], dims[1], dims[2], dims[3]
            (tnf, nf), (tsa, sa) = buf(K, torch.float32), buf(ns, torch.int64)
            if device_extract and L.gnn_ladies_layer_device(h, li, None, None, None, None, None) == 0:
                (trw, rw), (tcl, cl), (tcp, cp) = buf(M, torch.int32), buf(K, torch.int32), buf(K + 1, torch.int32)
                (tfr, fr), (tcs, cs) = buf(M + 1, torch.int32), buf(K + 1, torch.int32)
                _lib.check_sampler(L.gnn_ladies_layer_device(h, li, ptr(rw), ptr(cl), ptr(cp), ptr(fr), ptr(cs)) & ~1,
                                   "gnn_ladies_layer_device")
                _lib.check_sampler(L.gnn_ladies_layer_copy(h, li, None, None, None, ptr(nf), ptr(sa)),
                                   "gnn_ladies_layer_copy")
                pinned_layers.append((tfr, None, None, tnf, tcp, None, trw, tcl, tcs))
                pinned_sampled.append(tsa)
                layers.append(HostLayer(fullrowptr=fr, rowptr=None, colidx=None, normfact=nf, shape=(int(M), int(K)),
                                        csc_colptr=cp, rows=rw, cols=cl, dev_nnz=int(nnz), colseg=cs))
                sampled.append(sa)
                continue
            (tfr, fr), (trp, rp), (tci, ci) = buf(M + 1, torch.int32), buf(M + 1, torch.int32), buf(nnz, torch.int32)
            tcp = tcr = cp = cr = None
            if li >= csc_from:  # layers whose input needs a gradient: the backward's operand
                (tcp, cp), (tcr, cr) = buf(K + 1, torch.int32), buf(nnz, torch.int32)
            pinned_layers.append((tfr, trp, tci, tnf, tcp, tcr, None, None, None))
            pinned_sampled.append(tsa)
            _lib.check_sampler(L.gnn_ladies_layer_copy(h, li, ptr(fr), ptr(rp), ptr(ci), ptr(nf), ptr(sa)),
                               "gnn_ladies_layer_copy")
            if cp is not None:
                _lib.check_sampler(L.gnn_ladies_layer_csc(h, li, ptr(cp), ptr(cr)), "gnn_ladies_layer_csc")
            layers.append(HostLayer(fullrowptr=fr, rowptr=rp, colidx=ci, normfact=nf, shape=(int(M), int(K)),
                                    csc_colptr=cp, csc_rows=cr))
            sampled.append(sa)
        inp = np.empty(L.gnn_ladies_num_input_nodes(h), np.int64)
        _lib.check_sampler(L.gnn_ladies_input_nodes(h, ptr(inp)), "gnn_ladies_input_nodes")
    finally:
        L.gnn_ladies_free(h)
    return layers, sampled, inp, (pinned_layers, pinned_sampled)


def ladies_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full,
                       orders: Sequence[int], device_id_of_nodes, idx_of_nodes_on_device,
                       skewed_sampling_nodes=None, scale_factor: float = 1.0, devices=(0,),
                       native: bool = True, device_extract=False,
                       colcount: "Optional[ColumnCounter]" = None) -> HostBatch:
    """sampler.py:90-160 without the device work.

    native=True runs the C++ sampler (libgnn_sampler.so, bit-identical; releases the GIL, so
    batches sample concurrently on threads); native=False (and scale_factor > 1, a branch the
    reference never reaches) runs the numpy restatement below. device_extract (native, a graph
    without stored zeros; True = every layer below the top one, or bottom-up layer indices):
    those layers are extracted on the GPU by ``to_device`` (gnn_ladies_extract_f32) instead of on
    the host — same operands. colcount (native): a ColumnCounter made on this thread — U's column
    counts summed on the GPU, same batch."""
    batch_nodes = np.asarray(batch_nodes)
    if native and not scale_factor > 1:
        g = native_graph(lap_matrix)
        if g.num_nodes != num_nodes:
            raise ValueError("num_nodes does not match lap_matrix")
        dx = device_extract if (extract_mask(device_extract) and g.data is None) else False
        layers, sampled_nodes, previous_nodes, pinned = _native_layers(seed, batch_nodes, samp_num_list, g,
                                                                       list(orders), device_extract=dx,
                                                                       colcount=colcount)
        hb = _finish_batch(layers, sampled_nodes, previous_nodes, batch_nodes, labels_full, device_id_of_nodes,
                           idx_of_nodes_on_device, devices, seed)
        lab = torch.from_numpy(hb.labels)
        hb.extra["pinned"] = (pinned[0], pinned[1], lab.pin_memory() if torch.cuda.is_available() else lab)
        hb.extra["sorted_rows"] = True  # native samplers emit column-ascending rows by construction
        hb.extra["graph"] = g
        return hb
    if isinstance(lap_matrix, NativeGraph):
        lap_matrix = lap_matrix.lap
    np.random.seed(seed)
    batch_nodes = np.asarray(batch_nodes)
    previous_nodes = batch_nodes
    layers: List[Optional[HostLayer]] = []
    sampled_nodes: List[np.ndarray] = []
    orders1 = list(orders)[::-1]
    for d in range(len(orders1)):
        if orders1[d] == 0:
            layers.append(None)
            sampled_nodes.append(np.zeros(0, dtype=np.int64))
            continue
        U = lap_matrix[previous_nodes, :]
        # The reference's sp.linalg.norm(U, ord=0) canonicalises U in place (sorted,
        # duplicate-free indices) before U[:, after] is taken, so its sub-graph columns
        # come out ascending even when lap_matrix is unsorted (row_normalize's product).
        U.sum_duplicates()
        pi = column_nnz_counts(U, num_nodes)
        if scale_factor > 1:
            # int64 counts scaled in place: the product is truncated on assignment, as in
            # the reference (sampler.py:119-121; never reached there since scale_factor=1).
            nodes_on_this_gpu = skewed_sampling_nodes[len(orders1) - d - 1]
            pi[nodes_on_this_gpu] = pi[nodes_on_this_gpu] * scale_factor
        p = pi / np.sum(pi)
        samp_num_d = samp_num_list[d]
        s_num = np.min([np.sum(p > 0), samp_num_d])
        after_nodes = np.random.choice(num_nodes, s_num, p=p, replace=False)
        after_nodes = np.unique(np.concatenate((after_nodes, previous_nodes)))
        adj = U[:, after_nodes]
        layers.append(HostLayer(
            fullrowptr=U.indptr.astype(np.int32),
            rowptr=adj.indptr.astype(np.int32),
            colidx=adj.indices.astype(np.int32),
            # sampler.py:137 casts the clipped value to float32 BEFORE the reciprocal, so the
            # division is a float32 one: keep that precedence.
            normfact=1 / np.clip(s_num * p[after_nodes], 1e-10, 1).astype(np.float32),
            shape=(int(adj.shape[0]), int(adj.shape[1])),
        ))
        sampled_nodes.append(np.where(np.isin(after_nodes, previous_nodes))[0])
        previous_nodes = after_nodes
    layers.reverse()
    sampled_nodes.reverse()
    return _finish_batch(layers, sampled_nodes, previous_nodes, batch_nodes, labels_full, device_id_of_nodes,
                         idx_of_nodes_on_device, devices, seed)


def _finish_batch(layers, sampled_nodes, previous_nodes, batch_nodes, labels_full, device_id_of_nodes,
                  idx_of_nodes_on_device, devices, seed) -> HostBatch:
    """Feature-placement masks and labels of a sampled batch (sampler.py:150-160)."""
    input_nodes_devices = device_id_of_nodes[previous_nodes]
    input_nodes_mask_on_cpu = input_nodes_devices == -1
    nodes_idx_on_cpu = previous_nodes[input_nodes_mask_on_cpu]
    masks, idxs = [], []
    for dv in devices:
        m = input_nodes_devices == dv
        masks.append(m)
        idxs.append(idx_of_nodes_on_device[previous_nodes[m]].copy())
    labels = np.asarray(labels_full[batch_nodes].todense(), dtype=np.float32)
    return HostBatch(layers=layers, sampled_nodes=sampled_nodes, input_nodes=previous_nodes,
                     input_nodes_mask_on_devices=masks, input_nodes_mask_on_cpu=input_nodes_mask_on_cpu,
                     nodes_idx_on_devices=idxs, nodes_idx_on_cpu=nodes_idx_on_cpu, batch_nodes=batch_nodes,
                     labels=labels, seed=int(seed))


def subgraph_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full,
                         orders: Sequence[int], device_id_of_nodes, idx_of_nodes_on_device,
                         skewed_sampling_nodes=None, scale_factor: float = 1.0, devices=(0,),
                         native: bool = True, device=None) -> HostBatch:
    """subgraph_sampler (sampler.py:7-88) without the device work: one importance draw, then
    the top-most non-zero-order layer takes lap[batch, :][:, after] and every layer below it
    the square lap[after, :][:, after] (whatever its order, as the reference does), all with
    the same normfact. native=False (and scale_factor > 1, where the reference scales the
    counts of the columns placed on ``device``) runs the numpy restatement."""
    batch_nodes = np.asarray(batch_nodes)
    if native and not scale_factor > 1:
        g = native_graph(lap_matrix)
        if g.num_nodes != num_nodes:
            raise ValueError("num_nodes does not match lap_matrix")
        layers, sampled_nodes, after, pinned = _native_layers(seed, batch_nodes, samp_num_list, g, list(orders),
                                                              kind="subgraph")
        hb = _finish_batch(layers, sampled_nodes, after, batch_nodes, labels_full, device_id_of_nodes,
                           idx_of_nodes_on_device, devices, seed)
        lab = torch.from_numpy(hb.labels)
        hb.extra["pinned"] = (pinned[0], pinned[1], lab.pin_memory() if torch.cuda.is_available() else lab)
        hb.extra["sorted_rows"] = True  # native samplers emit column-ascending rows by construction
        return hb
    if isinstance(lap_matrix, NativeGraph):
        lap_matrix = lap_matrix.lap
    np.random.seed(seed)
    orders1 = list(orders)[::-1]
    U = lap_matrix[batch_nodes, :]
    U.sum_duplicates()
    pi = column_nnz_counts(U, num_nodes)
    if scale_factor > 1:
        on_gpu = device_id_of_nodes == device
        pi[on_gpu] = pi[on_gpu] * scale_factor
    p = pi / np.sum(pi)
    s_num = np.min([np.sum(p > 0), samp_num_list[0]])
    after = np.random.choice(num_nodes, s_num, p=p, replace=False)
    after = np.unique(np.concatenate((after, batch_nodes)))
    normfact = 1 / np.clip(s_num * p[after], 1e-10, 1).astype(np.float32)

    def layer(Ur):
        adj = Ur[:, after]
        return HostLayer(fullrowptr=Ur.indptr.astype(np.int32), rowptr=adj.indptr.astype(np.int32),
                         colidx=adj.indices.astype(np.int32), normfact=normfact.copy(),
                         shape=(int(adj.shape[0]), int(adj.shape[1])))

    layers: List[Optional[HostLayer]] = []
    sampled_nodes: List[np.ndarray] = []
    layer_idx = 0
    for d in range(len(orders1)):
        layer_idx += 1
        if orders1[d] == 0:
            layers.append(None)
            sampled_nodes.append(np.zeros(0, dtype=np.int64))
        else:
            layers.append(layer(U))
            sampled_nodes.append(np.where(np.isin(after, batch_nodes))[0])
            break
    for d in range(layer_idx, len(orders1)):
        Ua = lap_matrix[after, :]
        Ua.sum_duplicates()
        layers.append(layer(Ua))
        sampled_nodes.append(np.arange(len(after)))
    layers.reverse()
    sampled_nodes.reverse()
    return _finish_batch(layers, sampled_nodes, after, batch_nodes, labels_full, device_id_of_nodes,
                         idx_of_nodes_on_device, devices, seed)


def fastgcn_probability(lap) -> np.ndarray:
    """FastGCN's layer-independent importance q(u) ∝ ||lap[:, u]||² (Chen et al. 2018; the
    form LADIES' reference code uses: column sums of lap∘lap), float64, normalised."""
    lap = sp.csr_matrix(lap)
    d = np.asarray(lap.data, dtype=np.float64)
    pi = np.bincount(lap.indices, weights=d * d, minlength=lap.shape[1])
    return pi / np.sum(pi)


def fastgcn_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full,
                        orders: Sequence[int], device_id_of_nodes, idx_of_nodes_on_device,
                        skewed_sampling_nodes=None, scale_factor: float = 1.0, devices=(0,),
                        native: bool = True) -> HostBatch:
    """FastGCN sampler (BASELINE config 5; NOT in the reference, so parity is unpinned — the
    native and numpy versions below are checked against each other and for their sampling
    law). Per layer, top-down: s_num = min(#(p > 0), samp_num[d]) nodes drawn with the global
    importance p (np.random.choice without replacement, same RNG stream as LADIES), the
    sub-graph U[:, after] with the reference operator's normfact convention. Layers are
    independent (no union with the previous nodes), so it suits GCN, not GraphSAGE's
    x[sampled_nodes] self features."""
    batch_nodes = np.asarray(batch_nodes)
    g = native_graph(lap_matrix)
    if native:
        layers, sampled_nodes, inp, pinned = _native_layers(seed, batch_nodes, samp_num_list, g, list(orders),
                                                            kind="fastgcn")
        hb = _finish_batch(layers, sampled_nodes, inp, batch_nodes, labels_full, device_id_of_nodes,
                           idx_of_nodes_on_device, devices, seed)
        lab = torch.from_numpy(hb.labels)
        hb.extra["pinned"] = (pinned[0], pinned[1], lab.pin_memory() if torch.cuda.is_available() else lab)
        hb.extra["sorted_rows"] = True  # native samplers emit column-ascending rows by construction
        return hb
    lap = g.lap
    p = g.fastgcn_p
    np.random.seed(seed)
    previous = batch_nodes
    layers: List[Optional[HostLayer]] = []
    sampled_nodes: List[np.ndarray] = []
    orders1 = list(orders)[::-1]
    for d in range(len(orders1)):
        if orders1[d] == 0:
            layers.append(None)
            sampled_nodes.append(np.zeros(0, dtype=np.int64))
            continue
        U = lap[previous, :]
        s_num = np.min([np.sum(p > 0), samp_num_list[d]])
        after = np.unique(np.random.choice(num_nodes, s_num, p=p, replace=False))
        adj = U[:, after]
        layers.append(HostLayer(fullrowptr=U.indptr.astype(np.int32), rowptr=adj.indptr.astype(np.int32),
                                colidx=adj.indices.astype(np.int32),
                                normfact=1 / np.clip(s_num * p[after], 1e-10, 1).astype(np.float32),
                                shape=(int(adj.shape[0]), int(adj.shape[1]))))
        sampled_nodes.append(np.where(np.isin(after, previous))[0])
        previous = after
    layers.reverse()
    sampled_nodes.reverse()
    return _finish_batch(layers, sampled_nodes, previous, batch_nodes, labels_full, device_id_of_nodes,
                         idx_of_nodes_on_device, devices, seed)


def fastgcn_sampler(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                    device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, rank, devices):
    """Same signature and return tuple as the reference's samplers (sampler.py:7, :90)."""
    dev = devices[rank]
    hb = fastgcn_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                             device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, devices)
    db = hb.to_device(torch.device("cuda", dev) if isinstance(dev, int) else dev)
    return (db.adjs, hb.input_nodes_mask_on_devices, hb.input_nodes_mask_on_cpu, hb.nodes_idx_on_devices,
            hb.nodes_idx_on_cpu, hb.num_input_nodes, db.labels, hb.sampled_nodes)


def subgraph_sampler(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                     device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, rank, devices):
    """Reference signature and return tuple (sampler.py:7, :88)."""
    dev = devices[rank]
    hb = subgraph_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                              device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor,
                              devices, device=dev)
    db = hb.to_device(torch.device("cuda", dev) if isinstance(dev, int) else dev)
    return (db.adjs, hb.input_nodes_mask_on_devices, hb.input_nodes_mask_on_cpu, hb.nodes_idx_on_devices,
            hb.nodes_idx_on_cpu, hb.num_input_nodes, db.labels, hb.sampled_nodes)


def ladies_sampler(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                   device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, rank, devices):
    """Reference signature and return tuple (sampler.py:90, :160)."""
    hb = ladies_sample_host(seed, batch_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                            device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes, scale_factor, devices)
    dev = devices[rank]
    db = hb.to_device(torch.device("cuda", dev) if isinstance(dev, int) else dev)
    return (db.adjs, hb.input_nodes_mask_on_devices, hb.input_nodes_mask_on_cpu, hb.nodes_idx_on_devices,
            hb.nodes_idx_on_cpu, hb.num_input_nodes, db.labels, hb.sampled_nodes)


def rank_batches(target_nodes, batch_size: int, rank: int, world_size: int, iter_num: int,
                 local_shuffle: bool = False):
    """Batch node lists of one epoch for one rank (sampler.py:168-189): a torch.manual_seed
    permutation, a contiguous per-rank chunk of ceil(n/world) positions, batch_size slices."""
    n = len(target_nodes)
    chunk_size = n // world_size + (1 if n % world_size else 0)
    chunk_start = rank * chunk_size
    chunk_end = min((rank + 1) * chunk_size, n)
    num_batches = (chunk_end - chunk_start) // batch_size
    if (chunk_end - chunk_start) % batch_size:
        num_batches += 1
    if not local_shuffle:
        g = torch.Generator().manual_seed(iter_num)
        idxs = torch.randperm(n, generator=g).numpy()
    else:
        g = torch.Generator().manual_seed(iter_num)
        idxs = np.empty(n, dtype=np.int64)
        idxs[chunk_start:chunk_end] = torch.randperm(chunk_end - chunk_start, generator=g).numpy() + chunk_start
    out = []
    for j in range(num_batches):
        sl = idxs[chunk_start + j * batch_size: min(chunk_start + (j + 1) * batch_size, chunk_end)]
        out.append(np.asarray(target_nodes)[sl])
    return out
