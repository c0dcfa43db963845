"""Mini-batch producer: LADIES sampling + host-side feature staging in worker threads.

Reference: ``prepare_data`` (sampler.py:163-210) submits ``ladies_sampler`` calls to a
ThreadPoolExecutor (main.py:77, ``--pool_num`` 4) in groups of 32 and yields the futures;
each call re-seeds numpy's GLOBAL RNG (sampler.py:96) while the driver draws the next seeds
from that same global RNG, so concurrent threads race on it.

Here the worker threads run the native sampler (libgnn_sampler.so: bit-identical to the
numpy path, its own MT19937 per call, GIL released) and the host half of the X0 staging
(native row gather into a pinned buffer), so sampling scales with threads and the training
thread only issues asynchronous copies. Seeds come from the loader's own RandomState, so a
run is reproducible whatever the thread timing.
"""
from __future__ import annotations

import collections
import ctypes
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, Optional, Sequence

import numpy as np
import torch

from . import sampler as smp
from . import staging


def prepare_data(pool, sampler_fn, target_nodes, samp_num_list, num_nodes, lap_matrix, labels_full, orders,
                 batch_size, rank, world_size, device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes,
                 device, devices, scale_factor=1.0, local_shuffle=False, mode="train", iter_num=1, rng=None):
    """Reference signature (sampler.py:163): yields futures of ``sampler_fn`` calls.

    ``iter_num`` replaces the reference's module-global epoch counter (torch.manual_seed of
    the train permutation); ``rng`` (default: numpy's global RNG, as the reference) supplies
    the per-batch seeds."""
    rng = np.random if rng is None else rng
    target_nodes = np.asarray(target_nodes)

    def submit(nodes):
        return pool.submit(sampler_fn, int(rng.randint(2**32 - 1)), nodes, samp_num_list, num_nodes, lap_matrix,
                           labels_full, orders, device_id_of_nodes, idx_of_nodes_on_device, skewed_sampling_nodes,
                           scale_factor, rank, devices)

    if mode == "train":
        for chunk in smp.rank_batches(target_nodes, batch_size, rank, world_size, iter_num, local_shuffle):
            yield submit(chunk)
    elif mode == "val":
        import torch

        idx = torch.randperm(len(target_nodes))[:batch_size].numpy()
        yield submit(target_nodes[idx])
    elif mode == "test":
        # sampler.py:199-201: num_batches = len // bs, +1 when (num_batches % bs) != 0 (sic)
        num_batches = len(target_nodes) // batch_size
        if num_batches % batch_size:
            num_batches += 1
        for j in range(num_batches):
            chunk = target_nodes[batch_size * j: min((j + 1) * batch_size, len(target_nodes))]
            if len(chunk):
                yield submit(chunk)
    else:
        raise ValueError(f"unknown mode {mode!r}")


@dataclass
class LoadedBatch:
    host: smp.HostBatch
    plan: Optional[staging.StagePlan]


class BatchLoader:
    """Ordered, bounded-prefetch stream of sampled + host-staged training batches of one rank.

    ``workers`` threads each run: native LADIES sampling -> pinned copies of the batch's
    index arrays -> (with a FeatureStore) the pinned host-row gather of its X0 plan. The
    iterator hands batches out in submission order, keeping ``prefetch`` in flight."""

    def __init__(self, lap, labels_full, train_nodes, samp_num: int, batch_size: int, orders: Sequence[int],
                 device_id_of_nodes, idx_of_nodes_on_device, rank: int = 0, world_size: int = 1,
                 store: Optional[staging.FeatureStore] = None, workers: int = 8, prefetch: int = 0,
                 seed: int = 0, devices=None, kind: str = "ladies", device_extract=False,
                 skewed_sampling_nodes=None, scale_factor: float = 1.0):
        """skewed_sampling_nodes / scale_factor: --locality_sampling (main.py:284-287,
        preprocess.py:414-423), passed to every sampler call as the reference's prepare_data does
        (sampler.py:163-193); they change the LADIES draw only when scale_factor > 1
        (sampler.py:119-121; the reference fixes scale_factor = 1.0, main.py:256), which takes
        the numpy restatement."""
        fns = {"ladies": smp.ladies_sample_host, "subgraph": smp.subgraph_sample_host,
               "fastgcn": smp.fastgcn_sample_host}
        if kind not in fns:
            raise ValueError("sampler configuration is wrong")  # main.py:88
        self.sample_fn = fns[kind]
        # LADIES: leave the layers below the top one to the GPU extraction (to_device), so the
        # worker threads only draw (sampler.ladies_sample_host(device_extract=True))
        self.kw = {"device_extract": device_extract} if device_extract and kind == "ladies" else {}
        self.graph = smp.native_graph(lap)
        self.labels = labels_full
        self.train = np.asarray(train_nodes)
        self.samp = np.array([samp_num] * 5)
        self.batch_size = batch_size
        self.orders = list(orders)
        self.dev_of = device_id_of_nodes
        self.idx_on = idx_of_nodes_on_device
        self.rank = rank
        self.world = world_size
        self.devices = list(range(world_size)) if devices is None else list(devices)
        self.store = store
        self.workers = max(1, int(workers))
        self.prefetch = prefetch if prefetch > 0 else 2 * self.workers
        self.rng = np.random.RandomState(seed + 7919 * rank)
        self.skewed = skewed_sampling_nodes
        self.scale_factor = float(scale_factor)
        self.pool = ThreadPoolExecutor(max_workers=self.workers, thread_name_prefix="gnn-sampler")

    def _produce(self, seed: int, nodes: np.ndarray) -> LoadedBatch:
        hb = self.sample_fn(seed, nodes, self.samp, self.graph.num_nodes, self.graph, self.labels, self.orders,
                            self.dev_of, self.idx_on, self.skewed, self.scale_factor, self.devices, **self.kw)
        hb.pin()
        plan = staging.make_plan(hb, self.store, self.rank, self.world, self.devices) if self.store else None
        return LoadedBatch(hb, plan)

    def epoch(self, iter_num: int) -> Iterator[LoadedBatch]:
        chunks = smp.rank_batches(self.train, self.batch_size, self.rank, self.world, iter_num)
        return self._stream(chunks)

    def forever(self, first_epoch: int = 1) -> Iterator[LoadedBatch]:
        def chunks():
            e = first_epoch
            while True:
                yield from smp.rank_batches(self.train, self.batch_size, self.rank, self.world, e)
                e += 1
        return self._stream(chunks())

    def _stream(self, chunks) -> Iterator[LoadedBatch]:
        q = collections.deque()
        it = iter(chunks)
        done = False
        while True:
            while not done and len(q) < self.prefetch:
                try:
                    nodes = next(it)
                except StopIteration:
                    done = True
                    break
                q.append(self.pool.submit(self._produce, int(self.rng.randint(2**32 - 1)), nodes))
            if not q:
                return
            yield q.popleft().result()

    def close(self):
        self.pool.shutdown(wait=True, cancel_futures=True)


# ----------------------------------------------------------------------------------------
# Native batch producer (libgnn_sampler.so gnn_loader_*, include/gnn_sampler.h): the worker
# threads are C++ and never take the GIL, so the training thread keeps the interpreter to itself;
# each batch is ONE blob uploaded with ONE host-to-device copy.
# ----------------------------------------------------------------------------------------
# descriptor layout (mirrors GNN_BLOB_* / GNN_H_* / GNN_L_* / GNN_B_* of gnn_sampler.h)
BLOB_VERSION, BLOB_HEADER, BLOB_LAYER_SLOTS, BLOB_BATCH_SLOTS = 1, 16, 32, 16
H_VERSION, H_LAYERS, H_BYTES, H_BATCH, H_CLASSES, H_INPUTS, H_WORLD, H_LD_X0, H_SEED, H_PINNED = range(10)
(L_PRESENT, L_ON_DEVICE, L_M, L_K, L_NNZ, L_SNUM, L_NSAMPLED, L_HAS_RMAP) = range(8)
L_FULLROWPTR, L_ROWPTR, L_COLIDX, L_NORMFACT, L_CSC_COLPTR, L_CSC_ROWS, L_ROWS, L_COLS, L_SAMPLED, L_RMAP, \
    L_COLSEG = range(8, 30, 2)
B_LABELS, B_HOST_ROWS, B_OWN_POS, B_OWN_SRC, B_HOST_POS, B_HOST_SRC, B_INPUT_NODES = range(0, 14, 2)
KINDS = {"ladies": 0, "subgraph": 1, "fastgcn": 2}
# include/gnn_stage.h (gnn_stage_batch_f32's argument slots and per-layer arena offsets)
STAGE_SLOTS, STAGE_OUT_SLOTS, BLOB_MAX_LAYERS = 24, 6, 16
(ST_DESC, ST_HOST_BLOB, ST_DEV_BLOB, ST_UPLOAD, ST_BUFFER, ST_LD_BUFFER, ST_X0, ST_LD_X0, ST_F, ST_INDPTR, ST_INDICES,
 ST_DEGREE, ST_NUM_NODES, ST_INDPTR_T, ST_INDICES_T, ST_ERR, ST_ERR_HOST, ST_GATE, ST_CSC_FROM, ST_ARENA,
 ST_ARENA_BYTES) = range(21)
SO_ROWPTR, SO_COL, SO_VAL, SO_ROWS_T, SO_VAL_T = range(5)
_I32, _I64, _F32 = np.dtype(np.int32), np.dtype(np.int64), np.dtype(np.float32)
_TDT = {_I32: torch.int32, _I64: torch.int64, _F32: torch.float32}


def _release_blob(release, handle, uploads) -> None:
    """weakref.finalize of a NativeBatch: wait for the blob's uploads, then return it to the pool."""
    for ev in uploads:
        ev.synchronize()
    uploads.clear()
    release(handle)


class NativeBatch:
    """One batch of the native loader: the host blob, its descriptor and views of its sections.

    Duck-types the parts of ``sampler.HostBatch`` the training pipeline and the benchmark read
    (``layers``, ``sampled_nodes``, ``input_nodes``, ``labels``, ``nnz()``, ``to_device``) and
    carries the X0 staging plan (``plan``). The blob goes back to the loader's pool when this
    object dies, and not before its uploads (``device_blob``) have completed: the device side
    only reads the uploaded copy, so dropping the host batch early is safe."""

    def __init__(self, handle: int, store: Optional[staging.FeatureStore]):
        import weakref

        from . import _lib

        L = _lib.sampler_lib()
        n = ctypes.c_int64()
        dp = L.gnn_batch_desc(handle, ctypes.byref(n))
        self.desc = np.ctypeslib.as_array(dp, shape=(n.value,)).copy()
        self.nbytes = int(self.desc[H_BYTES])
        self.ptr = int(L.gnn_batch_blob(handle))
        # the pinned blob goes back to the loader's pool (where a worker may refill it at once)
        # only after every upload that read it has completed: device_blob() records an event
        # after its H2D into this holder, and the release waits for it
        self._uploads = []
        self._release = weakref.finalize(self, _release_blob, L.gnn_batch_release, handle, self._uploads)
        self.blob = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))
        self.num_layers = int(self.desc[H_LAYERS])
        self.world = int(self.desc[H_WORLD])
        self.seed = int(self.desc[H_SEED])
        self.pinned = bool(self.desc[H_PINNED])
        self.extra = {"sorted_rows": True, "csc_from": 1}
        self.store = store
        self._dev = None  # (device, device blob) once uploaded
        self._layers = None
        bb = BLOB_HEADER + self.num_layers * BLOB_LAYER_SLOTS
        self._bb = bb
        self.input_nodes = self._h(bb + B_INPUT_NODES, _I64)
        self.num_input_nodes = int(self.desc[H_INPUTS])
        C = int(self.desc[H_CLASSES])
        self.labels = self._h(bb + B_LABELS, _F32).reshape(-1, C) if C else np.zeros((0, 0), np.float32)
        self.sampled_nodes = [self._h(self._lb(li) + L_SAMPLED, _I64) for li in range(self.num_layers)]
        self.nodes_idx_on_cpu = self._h(bb + B_HOST_SRC, _I64)

    # -- host views ------------------------------------------------------------------------
    def _lb(self, li: int) -> int:
        return BLOB_HEADER + li * BLOB_LAYER_SLOTS

    def _count(self, slot: int) -> int:
        return int(self.desc[slot + 1])

    def _h(self, slot: int, dt: np.dtype) -> np.ndarray:
        off, cnt = int(self.desc[slot]), int(self.desc[slot + 1])
        return self.blob[off:off + cnt * dt.itemsize].view(dt)

    @property
    def layers(self) -> list:
        if self._layers is None:
            from .sampler import HostLayer

            out = []
            for li in range(self.num_layers):
                b = self._lb(li)
                if not self.desc[b + L_PRESENT]:
                    out.append(None)
                    continue
                shape = (int(self.desc[b + L_M]), int(self.desc[b + L_K]))
                if self.desc[b + L_ON_DEVICE]:
                    out.append(HostLayer(fullrowptr=self._h(b + L_FULLROWPTR, _I32), rowptr=None, colidx=None,
                                         normfact=self._h(b + L_NORMFACT, _F32), shape=shape,
                                         csc_colptr=self._h(b + L_CSC_COLPTR, _I32),
                                         rows=self._h(b + L_ROWS, _I32), cols=self._h(b + L_COLS, _I32),
                                         dev_nnz=int(self.desc[b + L_NNZ]), colseg=self._h(b + L_COLSEG, _I32)))
                else:
                    has_t = self._count(b + L_CSC_COLPTR) > 0
                    out.append(HostLayer(fullrowptr=self._h(b + L_FULLROWPTR, _I32), rowptr=self._h(b + L_ROWPTR, _I32),
                                         colidx=self._h(b + L_COLIDX, _I32), normfact=self._h(b + L_NORMFACT, _F32),
                                         shape=shape, csc_colptr=self._h(b + L_CSC_COLPTR, _I32) if has_t else None,
                                         csc_rows=self._h(b + L_CSC_ROWS, _I32) if has_t else None))
            self._layers = out
        return self._layers

    def nnz(self) -> int:
        return int(sum(self.desc[self._lb(li) + L_NNZ] for li in range(self.num_layers)
                       if self.desc[self._lb(li) + L_PRESENT]))

    @property
    def plan(self) -> staging.StagePlan:
        """The X0 staging plan (views of the blob). Made per access and not kept here: the plan
        references this batch, and a cycle would hold the blob until the cyclic GC runs."""
        bb = self._bb
        W = self.world
        peer_pos = [self._h(bb + BLOB_BATCH_SLOTS + 4 * j, _I64) for j in range(W)]
        peer_src = [self._h(bb + BLOB_BATCH_SLOTS + 4 * j + 2, _I64) for j in range(W)]
        return staging.StagePlan(self.num_input_nodes, self._h(bb + B_OWN_POS, _I64), self._h(bb + B_OWN_SRC, _I64),
                                 self._h(bb + B_HOST_POS, _I64), None, peer_pos, peer_src, (), blob=self)

    # -- device side -----------------------------------------------------------------------
    def device_blob(self, dev) -> torch.Tensor:
        """The blob on `dev`: one allocation + ONE host-to-device copy on the current stream
        (made once; later calls return the same tensor)."""
        from . import _lib

        dev = torch.device(dev)
        if self._dev is None or self._dev[0] != dev:
            with _lib.on_device(dev):
                d = torch.empty(self.nbytes, dtype=torch.uint8, device=dev)
                _lib.check(_lib.lib().gnn_memcpy_h2d_async(d.data_ptr(), self.ptr, self.nbytes, _lib.stream_of(dev)),
                           "gnn_memcpy_h2d_async")
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
            # completed uploads need no wait at release time: keep the list short
            self._uploads[:] = [e for e in self._uploads if not e.query()] + [ev]
            self._dev = (dev, d)
        return self._dev[1]

    def drop_device(self) -> None:
        """Forget the uploaded copy: the next device_blob() uploads the blob again (the
        benchmark's second pass over pre-sampled batches times a real H2D per batch)."""
        self._dev = None

    def _d(self, slot: int, dt: np.dtype) -> torch.Tensor:
        off, cnt = int(self.desc[slot]), int(self.desc[slot + 1])
        return self._dev[1][off:off + cnt * dt.itemsize].view(_TDT[dt])

    def stage_views(self, dev):
        """(own_pos, own_src, host_pos, host rows | host_src) on the device for Stager.issue."""
        self.device_blob(dev)
        bb = self._bb
        ld = int(self.desc[H_LD_X0])
        rows = self._d(bb + B_HOST_ROWS, _F32)
        host = rows.view(-1, ld) if self._count(bb + B_HOST_ROWS) else self._d(bb + B_HOST_SRC, _I64)
        return (self._d(bb + B_OWN_POS, _I64), self._d(bb + B_OWN_SRC, _I64), self._d(bb + B_HOST_POS, _I64), host)

    def peer_views(self, dev, j: int):
        """(X0 positions, slots in rank j's buffer) of the rows rank j supplies, on the device
        (views of the uploaded blob) — for staging.PeerDirect."""
        self.device_blob(dev)
        b = self._bb + BLOB_BATCH_SLOTS + 4 * j
        return self._d(b, _I64), self._d(b + 2, _I64)

    def stage(self, device, x0: torch.Tensor, store: "staging.FeatureStore", gate=None):
        """The DeviceBatch of this batch, with X0's own-buffer and host rows gathered into ``x0``,
        by ONE native call on the current stream (gnn_stage_batch_f32, include/gnn_stage.h): the
        blob's upload (unless already on the device), [a wait for ``gate``, a torch.cuda.Event],
        the X0 gather and every layer's operand — the library calls Stager.issue + to_device
        make, with the same arguments (bit-identical results). Copy-mode stores only."""
        from . import _lib
        from .custom_sparse_ops import CsrOperand
        from .sampler import DeviceBatch, device_graph

        dev = torch.device(device)
        desc, nl = self.desc, self.num_layers
        lbs = [self._lb(li) for li in range(nl)]
        on_dev = any(desc[b + L_PRESENT] and desc[b + L_ON_DEVICE] for b in lbs)
        graph = device_graph(self.graph, dev) if on_dev else None
        upload = self._dev is None or self._dev[0] != dev
        blob = torch.empty(self.nbytes, dtype=torch.uint8, device=dev) if upload else self._dev[1]
        a = np.zeros(STAGE_SLOTS, np.int64)
        a[ST_DESC], a[ST_HOST_BLOB], a[ST_DEV_BLOB], a[ST_UPLOAD] = desc.ctypes.data, self.ptr, blob.data_ptr(), upload
        buf = store.gpu_buffer
        a[ST_BUFFER], a[ST_LD_BUFFER] = buf.data_ptr(), buf.stride(0)
        a[ST_X0], a[ST_LD_X0], a[ST_F] = x0.data_ptr(), x0.stride(0), x0.shape[1]
        err_host = None
        if graph is not None:
            a[ST_INDPTR], a[ST_INDICES], a[ST_DEGREE] = (graph.indptr.data_ptr(), graph.indices.data_ptr(),
                                                         graph.degree.data_ptr())
            a[ST_NUM_NODES], a[ST_INDPTR_T], a[ST_INDICES_T] = (graph.num_nodes, graph.indptr_t.data_ptr(),
                                                                graph.indices_t.data_ptr())
            a[ST_ERR] = graph.err.data_ptr()
            # a flag of its own per build (as DeviceBatch.build_operands: ADVICE r4)
            err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            a[ST_ERR_HOST] = err_host.data_ptr()
        a[ST_GATE] = gate.cuda_event if gate is not None else 0  # 0 until first recorded: no wait
        a[ST_CSC_FROM] = int(self.extra.get("csc_from", 1))
        L = _lib.lib()
        out = np.empty(BLOB_MAX_LAYERS * STAGE_OUT_SLOTS, np.int64)
        nbytes = L.gnn_stage_plan(a.ctypes.data, out.ctypes.data)
        if nbytes == 0:
            raise RuntimeError("gnn_stage_plan: " + L.gnn_last_error().decode(errors="replace"))
        arena = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        a[ST_ARENA], a[ST_ARENA_BYTES] = arena.data_ptr(), nbytes
        with _lib.on_device(dev):
            st = _lib.stream_of(dev)
            _lib.check(L.gnn_stage_batch_f32(a.ctypes.data, st), "gnn_stage_batch_f32")
            if upload:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
                self._uploads[:] = [e for e in self._uploads if not e.query()] + [ev]
                self._dev = (dev, blob)

        def av(off, n, tdt):
            return arena[off:off + n * 4].view(tdt)

        adjs, sn = [], []
        for li, b in enumerate(lbs):
            x = self._d(b + L_SAMPLED, _I64)
            if not desc[b + L_PRESENT]:
                adjs.append(None)
                sn.append(x)
                continue
            if desc[b + L_HAS_RMAP]:
                x._gnn_rmap = self._d(b + L_RMAP, _I32)  # read by fused.SageAggregateFn's backward
            sn.append(x)
            M, K, nnz = int(desc[b + L_M]), int(desc[b + L_K]), int(desc[b + L_NNZ])
            o = out[li * STAGE_OUT_SLOTS:(li + 1) * STAGE_OUT_SLOTS]
            rowptr = av(int(o[SO_ROWPTR]), M + 1, torch.int32) if o[SO_ROWPTR] >= 0 else self._d(b + L_ROWPTR, _I32)
            op = CsrOperand(rowptr, av(int(o[SO_COL]), nnz, torch.int32), av(int(o[SO_VAL]), nnz, torch.float32), (M, K))
            if o[SO_VAL_T] >= 0:
                rows_t = av(int(o[SO_ROWS_T]), nnz, torch.int32) if o[SO_ROWS_T] >= 0 else self._d(b + L_CSC_ROWS, _I32)
                op._link(CsrOperand(self._d(b + L_CSC_COLPTR, _I32), rows_t, av(int(o[SO_VAL_T]), nnz, torch.float32),
                                    (K, M)))
            adjs.append(op)
        C = int(desc[H_CLASSES])
        labels = self._d(self._bb + B_LABELS, _F32).view(-1, C)
        return DeviceBatch(self, None, adjs, sn, labels, graph, err_host=err_host, keep=[blob, arena])

    def to_device(self, device, with_coo: bool = True, build: bool = True, graph=None):
        """The DeviceBatch of this batch: views of the uploaded blob (no further copies), then
        (build=True) the operand builds / GPU extractions on the current stream."""
        from .sampler import DeviceBatch, device_graph

        dev = torch.device(device)
        self.device_blob(dev)
        raw = []
        for li in range(self.num_layers):
            b = self._lb(li)
            if not self.desc[b + L_PRESENT]:
                raw.append(None)
                continue
            shape = (int(self.desc[b + L_M]), int(self.desc[b + L_K]))
            if self.desc[b + L_ON_DEVICE]:
                raw.append((self._d(b + L_FULLROWPTR, _I32), None, None, self._d(b + L_NORMFACT, _F32), shape,
                            self._d(b + L_CSC_COLPTR, _I32), None, self._d(b + L_ROWS, _I32),
                            self._d(b + L_COLS, _I32), int(self.desc[b + L_NNZ]), self._d(b + L_COLSEG, _I32)))
            else:
                has_t = self._count(b + L_CSC_COLPTR) > 0
                raw.append((self._d(b + L_FULLROWPTR, _I32), self._d(b + L_ROWPTR, _I32), self._d(b + L_COLIDX, _I32),
                            self._d(b + L_NORMFACT, _F32), shape, self._d(b + L_CSC_COLPTR, _I32) if has_t else None,
                            self._d(b + L_CSC_ROWS, _I32) if has_t else None, None, None, int(self.desc[b + L_NNZ]),
                            None))
        sn = []
        for li in range(self.num_layers):
            b = self._lb(li)
            x = self._d(b + L_SAMPLED, _I64)
            if self.desc[b + L_PRESENT] and self.desc[b + L_HAS_RMAP]:
                x._gnn_rmap = self._d(b + L_RMAP, _I32)  # read by fused.SageAggregateFn's backward
            sn.append(x)
        C = int(self.desc[H_CLASSES])
        labels = self._d(self._bb + B_LABELS, _F32).view(-1, C)
        if graph is None and any(self.desc[self._lb(li) + L_PRESENT] and self.desc[self._lb(li) + L_ON_DEVICE]
                                 for li in range(self.num_layers)):
            graph = device_graph(self.graph, dev)
        db = DeviceBatch(self, raw, None, sn, labels, graph)
        if build:
            db.build_operands(with_coo=with_coo)
        return db


class ToDevice:
    """batch_fn of staging.Stager.issue for a native-loader batch: ``host.to_device(dev,
    with_coo=False)``. Stager.issue recognises it and, when it can (copy-mode store, no copy
    timing), stages the batch through one native call instead (NativeBatch.stage); either way
    ``on_built`` (optional) receives the DeviceBatch."""

    __slots__ = ("host", "dev", "on_built")

    def __init__(self, host, dev, on_built=None):
        self.host, self.dev, self.on_built = host, dev, on_built

    def __call__(self):
        db = self.host.to_device(self.dev, with_coo=False)
        if self.on_built is not None:
            self.on_built(db)
        return db


class NativeLoader:
    """BatchLoader with C++ workers (gnn_loader_*): same batches (same seeds, same chunks,
    same sampler calls), same ``epoch`` / ``forever`` interface, yielding LoadedBatch(host=
    NativeBatch, plan=its StagePlan). ``store`` (copy mode) supplies the host feature table the
    workers gather the non-buffered rows from; zero-copy stores leave the rows to the GPU."""

    def __init__(self, lap, labels_full, train_nodes, samp_num: int, batch_size: int, orders: Sequence[int],
                 device_id_of_nodes, idx_of_nodes_on_device, rank: int = 0, world_size: int = 1,
                 store: Optional[staging.FeatureStore] = None, workers: int = 8, prefetch: int = 0,
                 seed: int = 0, devices=None, kind: str = "ladies", device_extract=False,
                 pinned: Optional[bool] = None, device_count=None, skewed_sampling_nodes=None,
                 scale_factor: float = 1.0, device_count_workers: Optional[int] = None):
        """device_count (LADIES, a graph without stored zeros): a torch device — the workers sum
        U's column counts on it (gnn_colcount_*, the graph resident there) instead of on the host.
        device_count_workers = k (0 < k < workers): only k of the workers count on the device, the
        others on the host, and the device contexts get hardware queues of their own on 64 CUs
        (gnn_loader_set_colcount_workers, gnn_colcount_set_cus); the batches are the same.
        skewed_sampling_nodes (--locality_sampling, preprocess.py:414-423) are accepted at the
        reference's scale_factor 1.0 (main.py:256), where they leave the draw unchanged
        (sampler.py:119-121); scale_factor > 1 is the numpy branch (BatchLoader)."""
        if float(scale_factor) > 1:
            raise ValueError("NativeLoader draws at the reference's scale_factor 1.0 (main.py:256); "
                             "scale_factor > 1 runs the numpy restatement: use BatchLoader")
        self.skewed = skewed_sampling_nodes
        import scipy.sparse as sp

        from . import _lib

        if kind not in KINDS:
            raise ValueError("sampler configuration is wrong")  # main.py:88
        self.graph = smp.native_graph(lap)
        g = self.graph
        self.train = np.asarray(train_nodes)
        self.batch_size = batch_size
        self.rank, self.world = rank, world_size
        self.store = store
        self.workers = max(1, int(workers))
        self.prefetch = prefetch if prefetch > 0 else 2 * self.workers
        self.rng = np.random.RandomState(seed + 7919 * rank)
        lab = sp.csr_matrix(labels_full)
        nl = len(orders)
        # borrowed by the C++ loader: kept alive here
        self._keep = dict(
            lab_ptr=np.ascontiguousarray(lab.indptr, dtype=np.int64),
            lab_idx=np.ascontiguousarray(lab.indices, dtype=np.int32),
            lab_val=np.ascontiguousarray(lab.data, dtype=np.float32),
            dev_of=np.ascontiguousarray(device_id_of_nodes, dtype=np.int64),
            idx_on=np.ascontiguousarray(idx_of_nodes_on_device, dtype=np.int64),
            devices=np.ascontiguousarray(list(range(world_size)) if devices is None else list(devices), dtype=np.int64),
            samp=np.ascontiguousarray([int(samp_num)] * nl, dtype=np.int64),
            orders=np.ascontiguousarray(orders, dtype=np.int32),
            p=g.fastgcn_p if kind == "fastgcn" else None)
        feat, ld_feat, F, ld_x0 = None, 0, 0, 0
        if store is not None:
            F, ld_x0 = store.F, store.ld
            if not store.zero_copy:
                host = store.host
                assert host.dtype == torch.float32 and host.stride(1) == 1
                feat, ld_feat = host.data_ptr(), host.stride(0)
                self._keep["feat"] = host
        k = self._keep
        ptr = lambda a: None if a is None else a.ctypes.data
        if pinned is None:
            pinned = torch.cuda.is_available()
        L = _lib.sampler_lib()
        dx = smp.extract_mask(device_extract) if (kind == "ladies" and g.data is None) else 0
        ipt = g.transpose_structure[1] if dx else None
        self.handle = L.gnn_loader_create(
            ptr(g.indptr), ptr(g.indices), ptr(g.data), ptr(ipt), g.num_nodes, ptr(k["lab_ptr"]), ptr(k["lab_idx"]),
            ptr(k["lab_val"]), int(lab.shape[1]), ptr(k["dev_of"]), ptr(k["idx_on"]), rank, world_size,
            ptr(k["devices"]), feat, ld_feat, F, ld_x0, ptr(k["samp"]), ptr(k["orders"]), nl, KINDS[kind],
            ptr(k["p"]), dx, 1, self.workers, int(bool(pinned)))
        if not self.handle:
            raise RuntimeError("gnn_loader_create failed: " + L.gnn_sampler_last_error().decode(errors="replace"))
        self.device_count = device_count is not None and kind == "ladies" and g.data is None
        self.device_count_workers = 0
        if self.device_count:
            self._keep["cc"] = smp.colcount_api(g, device_count)
            _lib.check_sampler(L.gnn_loader_set_colcount(self.handle, ctypes.byref(self._keep["cc"])),
                               "gnn_loader_set_colcount")
            k = int(device_count_workers or 0)
            if 0 < k < self.workers:
                _lib.check_sampler(L.gnn_loader_set_colcount_workers(self.handle, k), "gnn_loader_set_colcount_workers")
                # the counting streams off the step's hardware queues, on 64 of the CUs (contexts are
                # made on first use). Products, interleaved: 64 CUs 631 / 631 / 640 / 574 and 521 /
                # 596 / 583 / 642 / 640 end to end, 32 CUs 636 / 637 / 500 / 461, 128 CUs 636 / 641 /
                # 597 / 538, all CUs 483 / 636 / 483 / 567 / 627 (profiles/round6/mixed_counts/)
                _lib.check(_lib.lib().gnn_colcount_set_cus(64), "gnn_colcount_set_cus")
                self.device_count_workers = k
        self._pending = 0

    def _submit(self, nodes) -> None:
        from . import _lib

        nodes = np.ascontiguousarray(nodes, dtype=np.int64)
        seed = int(self.rng.randint(2**32 - 1))
        _lib.check_sampler(_lib.sampler_lib().gnn_loader_submit(self.handle, seed, nodes.ctypes.data, nodes.size),
                           "gnn_loader_submit")
        self._pending += 1

    def _next(self) -> LoadedBatch:
        from . import _lib

        h = ctypes.c_void_p()
        self._pending -= 1
        _lib.check_sampler(_lib.sampler_lib().gnn_loader_next(self.handle, ctypes.byref(h)), "gnn_loader_next")
        nb = NativeBatch(h.value, self.store)
        nb.graph = self.graph
        return LoadedBatch(nb, nb.plan)

    def epoch(self, iter_num: int) -> Iterator[LoadedBatch]:
        return self._stream(smp.rank_batches(self.train, self.batch_size, self.rank, self.world, iter_num))

    def forever(self, first_epoch: int = 1) -> Iterator[LoadedBatch]:
        def chunks():
            e = first_epoch
            while True:
                yield from smp.rank_batches(self.train, self.batch_size, self.rank, self.world, e)
                e += 1
        return self._stream(chunks())

    def _stream(self, chunks) -> Iterator[LoadedBatch]:
        it = iter(chunks)
        done = False
        while True:
            while not done and self._pending < self.prefetch:
                try:
                    self._submit(next(it))
                except StopIteration:
                    done = True
            if self._pending == 0:
                return
            yield self._next()

    def close(self):
        from . import _lib

        if self.handle:
            _lib.sampler_lib().gnn_loader_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
