"""Layer-0 feature staging: assemble X0 for a batch from the placement's three sources.

Reference (main.py:129-134): an uninitialised (n_input x F) tensor filled by masked scatters —
per source GPU i, ``gpu_buffers[i][idx].to(device)`` (gather on GPU i + P2P copy), then the
non-buffered rows ``feat_data[idx_cpu].to(device, non_blocking=True)`` from PAGEABLE host
memory, bracketed by device-wide synchronisations.

Here (DESIGN.md §Feature staging):
  * X0 is allocated with a padded row stride ``ld`` (602 -> 608 floats: every row starts on a
    128-byte cache line, so a 64-column tile of a row is 2 lines, not 3 — the layer-0
    aggregation went 386 -> 284 us on MI355X; the model sees the (n_input x F) view.
  * Own-buffer rows: one gather kernel (gnn_gather_rows_f32) from this GPU's buffer straight
    into their X0 positions.
  * Host rows, zero-copy (an option; measured slower on MI355X — the PCIe reads slow the
    concurrent compute kernels, GPU step 2.18 -> 2.5 ms): the host table lives in pinned, device-mapped
    memory and one gather kernel on the side stream reads the batch's rows over PCIe straight
    into their X0 positions (gnn_gather_rows_host_f32) — no host thread touches the rows.
    Copy mode: gathered on the host into a PINNED staging tensor (by the batch producer, off
    the critical path), then one contiguous hipMemcpyAsync on the side stream, then a scatter
    kernel into X0. Either way the side stream runs ahead, overlapping the previous batch's
    aggregation kernels; the compute stream waits on an event only when it needs X0.
  * Peer rows (world_size > 1), two forms:
    - ``PeerDirect`` (``--peer-rows direct``, the N > 1 default of bench.py; provisional until a
      multi-GPU record's ``peer_rows_ab`` confirms it): every peer's buffer is mapped
      once (IPC) and the staging stream's gather kernels read the batch's peer rows straight from
      the peers' HBM over xGMI — no negotiation and no per-batch collective;
    - ``PeerExchange`` (``--peer-rows alltoall``, and the fallback when any rank cannot map a
      peer): RCCL all-to-all — the request sizes and slot ids are negotiated on the host over a
      gloo group (no GPU sync), each rank gathers the rows its peers asked for from its own
      buffer, one all_to_all_single moves them over xGMI, and a scatter kernel places them.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys
import weakref
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import custom_sparse_ops as cso


# The training thread's host waits on GPU events: HIP's event wait spins, also for events made
# with hipEventBlockingSync (profiles/round6/blocking_wait/), so the thread burned a whole CPU of
# the cgroup's quota that the batch producers share. The wait polls the event and sleeps
# GNN_WAIT_SLEEP_US (default 20) between polls instead, with the thread's timer slack lowered to
# 1 µs so a sleep is not rounded up to the default 50 µs; 0 restores HIP's spinning wait.
# Measured (profiles/round6/sleep_wait/): the training thread's CPU 1.63 -> 0.70-0.90 ms per step,
# the same rates.
_WAIT_SLEEP_S = max(0.0, float(os.environ.get("GNN_WAIT_SLEEP_US", "20")) * 1e-6)
_slack_set = set()


def wait_event(ev) -> None:
    """Block the host until `ev` (a torch.cuda.Event) has completed: spin in HIP's wait, or with
    GNN_WAIT_SLEEP_US poll-and-sleep (see above)."""
    if _WAIT_SLEEP_S <= 0.0:
        ev.synchronize()
        return
    if ev.query():
        return
    import threading
    import time

    tid = threading.get_ident()
    if tid not in _slack_set:
        _slack_set.add(tid)
        try:
            ctypes.CDLL(None).prctl(29, ctypes.c_ulong(1000), 0, 0, 0)  # PR_SET_TIMERSLACK, 1 µs
        except (OSError, AttributeError):
            pass
    while not ev.query():
        time.sleep(_WAIT_SLEEP_S)


def _host_unregister(ptr: int, device) -> None:
    from . import _lib

    with _lib.on_device(device):
        _lib.lib().gnn_host_unregister(ptr)


def padded_ld(F: int, align: Optional[int] = None) -> int:
    """Row stride (floats) of X0, the feature buffer and the pinned host rows: F rounded up to
    whole 128-byte lines (32 floats; GNN_X0_ALIGN overrides it for measurements)."""
    if align is None:
        align = int(os.environ.get("GNN_X0_ALIGN", "32"))
    return (F + align - 1) // align * align


class FeatureStore:
    """Placement-resident features of one rank: its GPU buffer + the host table.

    ``zero_copy``: the host table is kept in ld-wide rows, pinned and mapped for the device
    (gnn_host_register); the GPU then reads a batch's non-buffered rows straight from it over
    PCIe (gnn_gather_rows_host_f32 on the staging stream) and no host thread copies rows.
    Otherwise the batch producer gathers them into a pinned buffer for one hipMemcpyAsync."""

    def __init__(self, feat_data: torch.Tensor, buffer_nodes: np.ndarray, device, rank: int = 0,
                 pin_host: bool = False, zero_copy: bool = False):
        assert feat_data.dtype == torch.float32 and feat_data.dim() == 2
        self.device = torch.device(device)
        self.rank = rank
        self.F = int(feat_data.shape[1])
        self.ld = padded_ld(self.F)
        self.zero_copy = bool(zero_copy)
        if self.zero_copy:
            from . import _lib

            if self.device.type != "cuda":
                raise RuntimeError("FeatureStore(zero_copy=True) needs a CUDA device")
            tab = torch.zeros((feat_data.shape[0], self.ld), dtype=torch.float32)
            tab[:, : self.F] = feat_data
            with _lib.on_device(self.device):
                _lib.check(_lib.lib().gnn_host_register(tab.data_ptr(), tab.numel() * 4), "gnn_host_register")
            self._unregister = weakref.finalize(self, _host_unregister, tab.data_ptr(), self.device)
            self.host = tab
        else:
            self.host = feat_data.pin_memory() if pin_host else feat_data.contiguous()
        idx = torch.from_numpy(np.asarray(buffer_nodes, dtype=np.int64))
        buf = torch.zeros((len(idx), self.ld), dtype=torch.float32)
        buf[:, : self.F] = feat_data[idx]
        self.gpu_buffer = buf.to(self.device)  # (k x ld), row i = node buffer_nodes[i]

    def host_rows_pinned(self, node_ids: np.ndarray) -> torch.Tensor:
        """Host gather of non-buffered rows into a pinned (n x ld) tensor (zero padding):
        one native row-copy loop (gnn_host_gather_rows_f32, GIL released) straight into
        the pinned buffer, so sampler worker threads stage concurrently."""
        from . import _lib

        idx = np.ascontiguousarray(node_ids, dtype=np.int64)
        n = len(idx)
        out = torch.empty((n, self.ld), dtype=torch.float32, pin_memory=torch.cuda.is_available())
        if n:
            host = self.host
            _lib.check_sampler(_lib.sampler_lib().gnn_host_gather_rows_f32(
                host.data_ptr(), host.stride(0), host.shape[0], idx.ctypes.data, n, self.F, out.data_ptr(), self.ld),
                "gnn_host_gather_rows_f32")
        return out


@dataclass
class StagePlan:
    """Host-side description of one batch's X0 assembly (all int64 index arrays)."""
    n_input: int
    own_pos: np.ndarray      # X0 rows filled from this rank's buffer
    own_src: np.ndarray      # their slots in the buffer
    host_pos: np.ndarray     # X0 rows filled from host memory
    host_rows: Optional[torch.Tensor]  # pinned (n_host x ld) rows gathered on the host (None: zero-copy)
    peer_pos: List[np.ndarray]   # per peer rank: X0 rows it supplies
    peer_src: List[np.ndarray]   # per peer rank: slots in that peer's buffer
    pinned: tuple = ()           # pinned host copies of (own_pos, own_src, host_pos[, host_src])
    blob: object = None          # a loader.NativeBatch: every array above lives in its blob, uploaded once
    peer_meta: object = None     # a Future of PeerExchange.prepare(plan), negotiated ahead (NegotiatedStream)


def make_plan(host_batch, store: FeatureStore, rank: int, world_size: int, devices=None) -> StagePlan:
    devices = list(range(world_size)) if devices is None else list(devices)
    masks = host_batch.input_nodes_mask_on_devices
    idxs = host_batch.nodes_idx_on_devices
    own_pos = np.flatnonzero(masks[rank]).astype(np.int64)
    own_src = np.asarray(idxs[rank], dtype=np.int64)
    host_pos = np.flatnonzero(host_batch.input_nodes_mask_on_cpu).astype(np.int64)
    # zero-copy stores: the GPU reads the rows itself (Stager.issue); else gather them here
    host_src = np.ascontiguousarray(host_batch.nodes_idx_on_cpu, dtype=np.int64)
    host_rows = None if store.zero_copy else store.host_rows_pinned(host_src)
    peer_pos, peer_src = [], []
    for j in range(world_size):
        if j == rank:
            peer_pos.append(np.zeros(0, np.int64))
            peer_src.append(np.zeros(0, np.int64))
        else:
            peer_pos.append(np.flatnonzero(masks[j]).astype(np.int64))
            peer_src.append(np.asarray(idxs[j], dtype=np.int64))
    cuda = torch.cuda.is_available()
    arrs = (own_pos, own_src, host_pos) + ((host_src,) if store.zero_copy else ())
    pin = tuple(torch.from_numpy(a).pin_memory() if cuda else torch.from_numpy(a) for a in arrs)
    return StagePlan(host_batch.num_input_nodes, own_pos, own_src, host_pos, host_rows, peer_pos, peer_src, pin)


def _staging_stream(device):
    """The staging stream: a plain torch stream, or with GNN_STAGE_CUS = n a stream whose kernels
    run on n of the device's CUs only (gnn_stream_create_cu_masked; experiments: the X0 gathers and
    layer extractions then never hold LDS / wave slots on the other CUs that the step's GEMMs and
    aggregations fill)."""
    cus = int(os.environ.get("GNN_STAGE_CUS", "0"))
    if cus <= 0:
        return torch.cuda.Stream(device=device)
    import ctypes

    from . import _lib

    ptr = ctypes.c_void_p()
    idx = torch.device(device).index or 0
    _lib.check(_lib.lib().gnn_stream_create_cu_masked(idx, cus, 0, ctypes.byref(ptr)), "gnn_stream_create_cu_masked")
    return torch.cuda.ExternalStream(ptr.value, device=device)


class Stager:
    """Issues X0 assembly on a side stream; ``wait`` hands X0 to the compute stream."""

    def __init__(self, store: FeatureStore, exchange: Optional["PeerExchange"] = None):
        self.store = store
        self.device = store.device
        self.stream = _staging_stream(self.device)
        self.exchange = exchange
        self.timing: Optional[list] = None  # set to [] to record (event, event, bytes) per host copy
        # optional torch.cuda.Event the staging kernels wait for (Trainer.stage_gate's event): the
        # step re-records it after the gating layer's forward aggregation
        self.gate: Optional[torch.cuda.Event] = None

    def take_timing(self):
        """(host bytes, seconds) summed over the recorded host-row copies; clears the record."""
        recs, self.timing = self.timing or [], None
        if not recs:
            return 0, 0.0
        recs[-1][1].synchronize()
        return sum(b for _, _, b in recs), sum(a.elapsed_time(b) for a, b, _ in recs) * 1e-3

    def issue(self, plan: StagePlan, batch_fn=None):
        """Issue X0's assembly (and, with ``batch_fn``, the batch's device side: batch_fn() runs
        on the staging stream and returns the DeviceBatch — its H2D copies and operand
        builds then overlap the previous step too). ``wait()`` on the result orders the
        compute stream after all of it."""
        dev = self.device
        st = self.stream
        meta = None
        if self.exchange is not None:
            # host-side metadata all-to-all (gloo), in batch order, paid for every issue: the
            # negotiation is part of each step (never cached on a plan that is issued again) —
            # made ahead on the NegotiatedStream's thread when the batch came through one
            fut = plan.peer_meta
            if fut is not None:
                plan.peer_meta = None
                meta = fut.result()
            else:
                meta = self.exchange.prepare(plan)
        # No wait on the compute stream: staging only reads static buffers and its own
        # uploads, so batch i+1's X0 assembles while batch i computes.
        with torch.cuda.stream(st):
            x0 = torch.empty((plan.n_input, self.store.ld), dtype=torch.float32, device=dev)
            if _NATIVE_STAGE and plan.blob is not None and self.timing is None and not self.store.zero_copy:
                from .loader import ToDevice

                if isinstance(batch_fn, ToDevice) and batch_fn.host is plan.blob:
                    # the native loader's batch: blob upload, X0 gather and operands in ONE call
                    batch = plan.blob.stage(dev, x0, self.store, self.gate)
                    if batch_fn.on_built is not None:
                        batch_fn.on_built(batch)
                    extra = self.exchange.exchange(plan, x0, self.store, meta) if self.exchange is not None else ()
                    ev = torch.cuda.Event()
                    ev.record(st)
                    return StagedX0(x0, ev, tuple(extra) + tuple(batch.tensors()), self.store.F, batch)
            nh = len(plan.host_pos)
            if self.timing is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
            if plan.blob is not None:  # native loader: ONE H2D of the whole batch blob, views of it
                own_pos, own_src, host_pos, host_dev = plan.blob.stage_views(dev)
                if self.store.zero_copy:  # host_dev = the host rows' node ids
                    cso.gather_rows_host(self.store.host, host_dev, x0, host_pos, n=nh)
            else:
                idx = [t.to(dev, non_blocking=True) for t in plan.pinned]
                own_pos, own_src, host_pos = idx[:3]
                if plan.host_rows is None:  # zero-copy: the GPU reads the rows from the mapped table
                    host_dev = idx[3]
                    cso.gather_rows_host(self.store.host, host_dev, x0, host_pos, n=nh)
                else:
                    host_dev = plan.host_rows.to(dev, non_blocking=True)  # one contiguous H2D
            if self.timing is not None:
                e1.record(st)
                self.timing.append((e0, e1, plan.blob.nbytes if plan.blob is not None else nh * self.store.ld * 4))
            if self.gate is not None:
                # the uploads above go ahead at once (copy engine); the gathers and layer extractions
                # below wait for the gate the step records after its layer-0 aggregation, so they run
                # beside the MFMA-bound GEMMs and tails instead of competing for L2 with the gather
                st.wait_event(self.gate)
            host_rows_here = nh and (plan.host_rows is not None or (plan.blob is not None and not self.store.zero_copy))
            if host_rows_here and _GATHER2:
                # the own-buffer rows and the host rows in one launch (gnn_gather_rows2_f32)
                cso.gather_rows2(self.store.gpu_buffer, own_src, own_pos, len(plan.own_pos), host_dev, None, host_pos,
                                 nh, x0)
            else:
                cso.gather_rows(self.store.gpu_buffer, own_src, x0, own_pos, n=len(plan.own_pos))
                if host_rows_here:
                    cso.gather_rows(host_dev, None, x0, host_pos, n=nh)
            extra = ()
            if self.exchange is not None:
                extra = self.exchange.exchange(plan, x0, self.store, meta)
            batch = batch_fn() if batch_fn is not None else None
            ev = torch.cuda.Event()
            ev.record(st)
        keep = (own_pos, own_src, host_pos, host_dev) + tuple(extra)
        if batch is not None:
            keep += tuple(batch.tensors())
        return StagedX0(x0, ev, keep, self.store.F, batch)


_EXTRACT_CHECK = os.environ.get("GNN_EXTRACT_CHECK", "step")
# X0's own-buffer and host rows in one gather launch (GNN_GATHER2=0: two launches, the round-5 form)
_GATHER2 = os.environ.get("GNN_GATHER2", "1") != "0"
# a native-loader batch staged by one native call (gnn_stage_batch_f32; GNN_NATIVE_STAGE=0: the
# Python sequence of calls, the round-5 form); it gathers X0 in one launch, so GNN_GATHER2=0 also
# selects the Python sequence
_NATIVE_STAGE = os.environ.get("GNN_NATIVE_STAGE", "1") != "0" and _GATHER2


class StagedX0:
    def __init__(self, x0, event, keep, F, batch=None):
        self._x0 = x0
        self.event = event
        self._keep = keep
        self.F = F
        self.batch = batch  # the DeviceBatch built on the staging stream, if any
        # its operands as built by this issue (a later issue may rebuild the same batch), and the
        # pinned copy of the extraction error flag taken by this build
        self.adjs = list(batch.adjs) if batch is not None and batch.adjs is not None else None
        self.err_host = getattr(batch, "err_host", None) if batch is not None else None

    def wait(self, retire: Optional["Retirement"] = None) -> torch.Tensor:
        """Make the current stream wait for the staging and return the (n x F) view. The
        staged buffers were allocated on the staging stream and are read on this one: either
        each is marked with record_stream (default), or ``retire`` keeps them alive until the
        consuming step has run on the GPU (one event instead of ~40 record_stream calls)."""
        b = self.batch
        if b is not None and self.err_host is not None and _EXTRACT_CHECK == "step":
            # GPU-extracted layers: their error flag is read before this step is issued, so a
            # device count that disagrees with the host's raises before any kernel consumes the
            # operand (a host wait on the staging event, which the staged work was issued a step
            # ahead of; GNN_EXTRACT_CHECK=end defers the check to DeviceGraph.check at the end)
            wait_event(self.event)
            b.check_extraction(self.err_host)
        cur = torch.cuda.current_stream(self._x0.device)
        cur.wait_event(self.event)
        if retire is None:
            self._x0.record_stream(cur)
            for t in self._keep:
                t.record_stream(cur)
        return self._x0[:, : self.F]


class Retirement:
    """Keeps staged batches alive until the GPU has finished the step that read them: after
    the step is issued, ``retire(staged)`` records an event on the current stream and holds
    the batch; held batches are released once their event has completed, and the host waits
    for the oldest when more than ``depth`` are held (so it never runs further ahead)."""

    def __init__(self, depth: int = 3):
        import collections

        self.depth = depth
        self.q = collections.deque()
        self.wait_s = 0.0  # host time spent waiting for the GPU (so callers can report issue cost)

    def retire(self, staged) -> None:
        ev = torch.cuda.Event()
        ev.record()
        self.q.append((ev, staged))
        while self.q and self.q[0][0].query():
            self.q.popleft()
        if len(self.q) > self.depth:
            import time

            t0 = time.perf_counter()
            while len(self.q) > self.depth:
                ev0, _ = self.q.popleft()
                wait_event(ev0)
            self.wait_s += time.perf_counter() - t0

    def drain(self) -> None:
        while self.q:
            ev0, _ = self.q.popleft()
            ev0.synchronize()


class NegotiatedStream:
    """Wraps a stream of loader batches (LoadedBatch) and runs each batch's peer negotiation
    (PeerExchange.prepare: two gloo all-to-alls of request sizes and slot ids) on ONE background
    thread, ``depth`` batches ahead of the consumer, so the training thread never blocks on the
    other ranks' hosts inside a step. Every rank pulls the same number of batches (consumed +
    depth), so the collectives pair up in batch order across ranks; only this thread uses the
    metadata group."""

    def __init__(self, it, exchange: "PeerExchange", depth: int = 4):
        import collections
        from concurrent.futures import ThreadPoolExecutor

        self.it = iter(it)
        self.exchange = exchange
        self.depth = max(0, int(depth))
        self.q = collections.deque()
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="gnn-peer-meta")

    def __iter__(self):
        return self

    def __next__(self):
        while self.it is not None and len(self.q) <= self.depth:
            try:
                lb = next(self.it)
            except StopIteration:
                self.it = None
                break
            lb.plan.peer_meta = self.pool.submit(self.exchange.prepare, lb.plan)
            self.q.append(lb)
        if not self.q:
            raise StopIteration
        return self.q.popleft()

    def close(self):
        self.pool.shutdown(wait=True)


@contextlib.contextmanager
def stdout_to_stderr():
    """Send file descriptor 1 to stderr for the duration (native libraries' prints included)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class PeerExchange:
    """All-to-all exchange of buffered rows held by peer GPUs (RCCL over xGMI).

    Rank r needs, from each peer j, the rows at slots ``plan.peer_src[j]`` of j's buffer.
    ``prepare`` (host, in batch order on every rank): the per-peer request counts and the
    requested slot ids move by two all-to-alls on a CPU (gloo) group — metadata only, so the
    host never waits on the GPU queue. ``exchange`` (device, on the staging stream): each rank
    gathers the rows its peers asked for from its own buffer (HIP gather), ONE RCCL
    all_to_all_single with the sizes ``prepare`` learnt moves them over xGMI, and a scatter
    kernel drops them at their X0 positions. Replaces the reference's per-peer P2P
    ``gpu_buffers[i][idx].to(device)`` copies (main.py:129-133)."""

    needs_negotiation = True

    def __init__(self, group=None, meta_group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if meta_group is None:
            # always a group of its own: the negotiation may run on another thread
            # (NegotiatedStream) while this thread's row all-to-all / gradient all-reduce use
            # `group` — two threads on one communicator would interleave their collectives
            from .train import new_gloo_group

            meta_group = new_gloo_group()  # with the package's collective timeout
        self.meta_group = meta_group

    def prepare(self, plan: StagePlan) -> tuple:
        """Host-side negotiation for one batch: (send counts, recv counts, wanted slots, X0
        positions). Collective: call on every rank, for the same batch sequence, once per
        exchange (the result is not cached: every step pays its own negotiation)."""
        dist, W = self.dist, self.world
        sc = [len(plan.peer_src[j]) for j in range(W)]
        rc_t = torch.empty(W, dtype=torch.int64)
        dist.all_to_all_single(rc_t, torch.tensor(sc, dtype=torch.int64), group=self.meta_group)
        rc = rc_t.tolist()
        req = torch.from_numpy(np.concatenate(plan.peer_src).astype(np.int64) if W else np.zeros(0, np.int64))
        want = torch.empty(sum(rc), dtype=torch.int64)
        dist.all_to_all_single(want, req, output_split_sizes=rc, input_split_sizes=sc, group=self.meta_group)
        pos = torch.from_numpy(np.concatenate(plan.peer_pos).astype(np.int64) if W else np.zeros(0, np.int64))
        pin = torch.cuda.is_available()
        return (sc, rc, want.pin_memory() if pin else want, pos.pin_memory() if pin else pos)

    def exchange(self, plan: StagePlan, x0: torch.Tensor, store: FeatureStore, meta: Optional[tuple] = None):
        sc, rc, want_h, pos_h = self.prepare(plan) if meta is None else meta
        dev = x0.device
        want = want_h.to(dev, non_blocking=True)
        pos = pos_h.to(dev, non_blocking=True)
        ld = store.ld
        send_rows = torch.empty((sum(rc), ld), dtype=torch.float32, device=dev)
        if sum(rc):
            cso.gather_rows(store.gpu_buffer, want, send_rows, None, n=sum(rc))
        recv_rows = torch.empty((sum(sc), ld), dtype=torch.float32, device=dev)
        self.dist.all_to_all_single(recv_rows, send_rows, output_split_sizes=sc, input_split_sizes=rc,
                                    group=self.group)
        if sum(sc):
            cso.gather_rows(recv_rows, None, x0, pos, n=sum(sc))
        return (want, pos, send_rows, recv_rows)


def _ipc_close_all(mapped, device) -> None:
    """Unmap the peers' buffers. The device is synchronised first, so no gather kernel still in
    flight on any stream reads a mapping being closed (also when this runs as the finalizer of a
    PeerDirect dropped without close())."""
    from . import _lib

    if not mapped:
        return
    try:
        torch.cuda.synchronize(device)
    except RuntimeError:  # interpreter shutdown / a device already in error: unmap anyway
        pass
    with _lib.on_device(device):
        for ptr, off in mapped:
            _lib.lib().gnn_ipc_close(ptr, off)
    mapped.clear()


class PeerDirect:
    """Peer rows read directly from the peers' feature buffers over xGMI.

    Reference: main.py:129-133 copies ``gpu_buffers[i][idx]`` from every peer GPU by a P2P
    ``.to(device)`` per batch. Here each rank maps every peer's buffer ONCE at start-up (an IPC
    handle + offset per rank, exchanged by one all_gather_object on a gloo group,
    ``gnn_ipc_export`` / ``gnn_ipc_open``) and a batch's peer rows are then gathered by HIP
    kernels that read the peers' HBM straight into their X0 positions (one gnn_gather_rows_f32
    per peer, on the staging stream). The slots come from the placement every rank computes
    identically (``plan.peer_src``), so there is no per-batch negotiation and no collective:
    ranks never wait for each other while staging. The buffers never change after start-up,
    so no per-batch synchronisation with the peers is needed either. Same X0 as PeerExchange,
    bit for bit (tests/test_dist_gpu.py).

    Callers must call the collective ``close()`` when staging is done (bench.py does so in a
    ``finally``): it unmaps after a device sync and a barrier, so no rank frees its exported buffer
    while a peer still reads it. The finalizer of an object dropped without close() only unmaps
    this rank's mappings (after a device sync); it cannot wait for the peers."""

    needs_negotiation = False

    def __init__(self, store: FeatureStore, group=None, feats: Optional[torch.Tensor] = None,
                 buffer_nodes: Optional[list] = None):
        """Collective (every rank of `group`). Raises on every rank if any rank could not map a
        peer's buffer — all ranks agree before anyone raises, so none is left waiting. With
        `feats` (the full feature table) and `buffer_nodes` (every rank's buffered node ids,
        the placement's gpu_buffer_group), a few rows of every peer are read through the new
        mapping and checked bit for bit before the first batch."""
        import torch.distributed as dist
        from . import _lib

        self.dist = dist
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = dev = store.device
        buf = store.gpu_buffer
        self.ld = int(buf.stride(0))
        self.peers = [None] * self.world  # (mapped pointer, rows, ld) per peer rank
        self.verified_rows = 0  # rows read through the mappings and checked against the feature table
        mapped = []
        self._closer = weakref.finalize(self, _ipc_close_all, mapped, dev)
        from .train import new_gloo_group

        self.group = new_gloo_group()
        err, info = "", None
        try:
            if buf.shape[0]:
                h = (ctypes.c_char * 64)()
                off = ctypes.c_int64()
                with _lib.on_device(dev):
                    _lib.check(_lib.lib().gnn_ipc_export(buf.data_ptr(), h, ctypes.byref(off)), "gnn_ipc_export")
                info = (bytes(h), int(off.value), dev.index, int(buf.shape[0]), self.ld)
            torch.cuda.synchronize(dev)  # the buffer is final before any peer reads it
        except Exception as e:  # noqa: BLE001 — reported to every rank below
            err = f"rank {self.rank}: {e}"
        infos = [None] * self.world
        dist.all_gather_object(infos, (err, info), group=self.group)
        err = "; ".join(e for e, _ in infos if e)
        if not err:
            try:
                for j, (_, inf) in enumerate(infos):
                    if j == self.rank or inf is None:
                        continue
                    handle, off, pdev, rows, ld = inf
                    if ld != self.ld:
                        raise RuntimeError(f"rank {j}'s buffer rows are {ld} floats, this rank's {self.ld}")
                    ptr = ctypes.c_void_p()
                    with _lib.on_device(dev):
                        _lib.check(_lib.lib().gnn_ipc_open(handle, off, pdev if pdev != dev.index else -1,
                                                           ctypes.byref(ptr)), "gnn_ipc_open")
                    mapped.append((ptr.value, off))
                    self.peers[j] = (ptr.value, rows, ld)
                if feats is not None and buffer_nodes is not None:
                    self._verify(feats, buffer_nodes)
            except Exception as e:  # noqa: BLE001
                err = f"rank {self.rank}: {e}"
            errs = [None] * self.world
            dist.all_gather_object(errs, err, group=self.group)
            err = "; ".join(e for e in errs if e)
        if err:
            self._closer()
            raise RuntimeError(f"PeerDirect unavailable: {err}")

    def _verify(self, feats: torch.Tensor, buffer_nodes) -> None:
        """Read the first, middle and last slot of every peer's buffer through the mapping and
        compare with the feature table (catches a wrong offset or a mapping of the wrong GPU)."""
        from . import _lib

        dev, F = self.device, int(feats.shape[1])
        for j, peer in enumerate(self.peers):
            if peer is None:
                continue
            ptr, rows, ld = peer
            slots = np.unique(np.array([0, rows // 2, rows - 1], np.int64))
            src = torch.from_numpy(slots).to(dev)
            out = torch.full((len(slots), ld), float("nan"), device=dev)
            with _lib.on_device(dev):
                _lib.check(_lib.lib().gnn_gather_rows_f32(ptr, ld, src.data_ptr(), out.data_ptr(), ld, None,
                                                          len(slots), ld, _lib.stream_of(dev)), "gnn_gather_rows_f32")
            got = out.cpu()
            nodes = torch.from_numpy(np.asarray(buffer_nodes[j], np.int64)[slots])
            if not torch.equal(got[:, :F], feats[nodes]):
                raise RuntimeError(f"rows read from rank {j}'s mapped buffer differ from the feature table")
            self.verified_rows += len(slots)

    def prepare(self, plan: StagePlan):
        return None

    def close(self) -> None:
        """Unmap the peers' buffers (after the last batch was staged; collective, so no rank
        frees its buffer while a peer still has it mapped)."""
        torch.cuda.synchronize(self.device)
        self._closer()
        self.dist.barrier(group=self.group)

    def close_local(self) -> None:
        """Unmap this rank's mappings after a device sync, without waiting for the peers (the
        error path: a peer may never reach close()'s barrier)."""
        self._closer()

    def exchange(self, plan: StagePlan, x0: torch.Tensor, store: FeatureStore, meta=None):
        from . import _lib

        dev = x0.device
        keep = []
        for j in range(self.world):
            n = len(plan.peer_src[j])
            if j == self.rank or n == 0:
                continue
            peer = self.peers[j]
            if peer is None:
                raise RuntimeError(f"PeerDirect: the plan wants {n} rows from rank {j}, which buffers none")
            ptr, rows, ld = peer
            hi = int(np.max(plan.peer_src[j]))
            if hi >= rows or int(np.min(plan.peer_src[j])) < 0:  # never read outside a peer's buffer
                raise RuntimeError(f"PeerDirect: slot {hi} outside rank {j}'s buffer of {rows} rows")
            if plan.blob is not None:
                pos, src = plan.blob.peer_views(dev, j)
            else:
                pos = torch.from_numpy(np.ascontiguousarray(plan.peer_pos[j], np.int64)).to(dev, non_blocking=True)
                src = torch.from_numpy(np.ascontiguousarray(plan.peer_src[j], np.int64)).to(dev, non_blocking=True)
            keep += [pos, src]
            with _lib.on_device(dev):
                _lib.check(_lib.lib().gnn_gather_rows_f32(ptr, ld, src.data_ptr(), x0.data_ptr(), x0.stride(0),
                                                          pos.data_ptr(), n, min(ld, x0.shape[1]),
                                                          _lib.stream_of(dev)), "gnn_gather_rows_f32 (peer)")
        return tuple(keep)
