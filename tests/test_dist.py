"""CPU, world_size 2 (gloo): the data-parallel pieces of the path.

* Trainer: per-rank clip then all-reduce(SUM) of the flat gradient equals the reference's
  thread-sum semantics (main.py:146-168): grad = Σ_r clip_r(grad_r), no averaging; initial
  weights are broadcast from rank 0.
* PeerExchange: every rank receives exactly the rows it requested from each peer's buffer
  (host-side negotiation of sizes and slot ids, then the row all-to-all).
The HIP row gather is replaced by a torch index copy here (no GPU on this host).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _trainer_worker(rank, world, port, q):
    _init(rank, world, port)
    from gnn_amd.train import Trainer

    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    tr = Trainer(model, lr=0.01, device="cpu")
    # reference semantics on the same data, computed independently on every rank
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(4, 6, generator=g) for _ in range(world)]
    ys = [torch.rand(4, 3, generator=g).round() for _ in range(world)]
    init = [p.detach().clone() for p in model.parameters()]
    ref_grads = []
    for r in range(world):
        m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
        with torch.no_grad():
            for p, p0 in zip(m.parameters(), init):
                p.copy_(p0)
        out = m(xs[r])
        loss = torch.nn.BCEWithLogitsLoss(weight=torch.full((4, 1), 0.25), reduction="sum")(out, ys[r])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 5)
        ref_grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
    ref = sum(ref_grads)
    # the same through the Trainer (model forward signature differs: call pieces directly)
    out = model(xs[rank])
    loss = torch.nn.BCEWithLogitsLoss(weight=torch.full((4, 1), 0.25), reduction="sum")(out, ys[rank])
    loss.backward()
    torch.nn.utils.clip_grad_norm_(tr.params, 5)
    flat = tr.allreduce_grads()
    got = torch.cat([p.grad.reshape(-1) for p in tr.params])
    q.put((rank, torch.allclose(flat, ref, rtol=1e-6, atol=1e-7) and torch.allclose(got, ref, rtol=1e-6, atol=1e-7),
           [p.detach().numpy().copy() for p in model.parameters()]))
    dist.destroy_process_group()


def _exchange_worker(rank, world, port, q):
    _init(rank, world, port)
    from gnn_amd import custom_sparse_ops as cso
    from gnn_amd import staging

    def cpu_gather(src, src_idx, dst, dst_idx, n=None):  # test stand-in for the HIP kernel
        s = src if src_idx is None else src[src_idx]
        if dst_idx is None:
            dst[: s.shape[0], : dst.shape[1]] = s[:, : dst.shape[1]]
        else:
            dst[dst_idx] = s[:, : dst.shape[1]]

    cso.gather_rows = cpu_gather
    staging.cso.gather_rows = cpu_gather
    F, k = 5, 10
    store = staging.FeatureStore.__new__(staging.FeatureStore)
    store.F, store.ld, store.rank, store.device = F, 8, rank, torch.device("cpu")
    buf = torch.zeros(k, 8)
    buf[:, :F] = torch.arange(k * F, dtype=torch.float32).view(k, F) + 1000 * rank
    store.gpu_buffer = buf
    rng = np.random.default_rng(rank)
    n_in = 12
    peer = 1 - rank
    pos = np.sort(rng.choice(n_in, 5, replace=False)).astype(np.int64)
    src = rng.integers(0, k, 5).astype(np.int64)
    peer_pos = [np.zeros(0, np.int64)] * world
    peer_src = [np.zeros(0, np.int64)] * world
    peer_pos[peer], peer_src[peer] = pos, src
    plan = staging.StagePlan(n_in, np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64),
                             torch.zeros(0, F), peer_pos, peer_src)
    x0 = torch.full((n_in, 8), -1.0)
    ex = staging.PeerExchange()
    meta = ex.prepare(plan)
    assert ex.prepare(plan)[:2] == meta[:2]  # same negotiation when repeated
    ex.exchange(plan, x0, store, meta)
    expect = torch.arange(k * F, dtype=torch.float32).view(k, F)[torch.from_numpy(src)] + 1000 * peer
    ok = torch.equal(x0[torch.from_numpy(pos), :F], expect)
    q.put((rank, ok))
    dist.destroy_process_group()


def _negotiated_worker(rank, world, port, q):
    """NegotiatedStream: the metadata negotiated ahead on its thread equals the synchronous
    PeerExchange.prepare of the same batches, in order."""
    _init(rank, world, port)
    from gnn_amd import loader, staging

    rng = np.random.default_rng(10 + rank)
    plans = []
    for b in range(7):
        peer_pos = [np.zeros(0, np.int64)] * world
        peer_src = [np.zeros(0, np.int64)] * world
        n = int(rng.integers(0, 6))
        peer_pos[1 - rank] = np.sort(rng.choice(20, n, replace=False)).astype(np.int64)
        peer_src[1 - rank] = rng.integers(0, 50, n).astype(np.int64)
        plans.append(staging.StagePlan(20, np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64),
                                       None, peer_pos, peer_src))
    ex = staging.PeerExchange()
    ref = [ex.prepare(p) for p in plans]
    stream = staging.NegotiatedStream((loader.LoadedBatch(None, p) for p in plans), ex, depth=3)
    ok = True
    n = 0
    for i, lb in enumerate(stream):
        n += 1
        got = lb.plan.peer_meta.result()
        ok &= got[0] == ref[i][0] and got[1] == ref[i][1]
        ok &= torch.equal(got[2], ref[i][2]) and torch.equal(got[3], ref[i][3])
    stream.close()
    q.put((rank, bool(ok) and n == len(plans)))
    dist.destroy_process_group()


def _spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


def test_trainer_allreduce_matches_thread_sum():
    out = _spawn(_trainer_worker)
    assert all(ok for _, ok, _ in out)
    for a, b in zip(out[0][2], out[1][2]):
        assert np.array_equal(a, b)  # broadcast made the ranks weights identical


def test_peer_exchange_rows():
    out = _spawn(_exchange_worker)
    assert all(ok for _, ok in out)


def test_negotiated_stream_matches_prepare():
    out = _spawn(_negotiated_worker)
    assert all(ok for _, ok in out)
