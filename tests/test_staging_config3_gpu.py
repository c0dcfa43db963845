"""GPU, world_size 4 on the one GPU (gloo): BASELINE config 3's feature placement and X0 staging
at its own geometry.

Config 3 is ogbn-products GraphSAGE / LADIES with buffer_size = 0.1 over 4 GPUs
(preprocess.py:343-386: every rank caches 10 % of the nodes, chosen by the placement every rank
computes identically) and X0 assembled per batch from three sources (main.py:129-134): this
rank's buffer, the peers' buffers (P2P in the reference; here IPC-mapped direct reads —
staging.PeerDirect, the N > 1 default — and the RCCL all-to-all — staging.PeerExchange, the
fallback) and the host table for the rest. Here each of 4 ranks (all on cuda:0, gloo for the
collectives) builds the products-shaped test graph (500 k nodes, F = 100), the placement over 4
ranks, draws a samp 8192 / batch 512 LADIES batch through the native producer (the bench's path:
one blob per batch, the placement split made by the C++ workers) and stages X0 with each peer-row
form. X0 must equal oracle.gather_rows of the host feature table at the batch's input nodes, bit
for bit, and each source must really be used (rows from this rank's buffer, from every peer, and
from the host).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
WORLD = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GNN_DIST_BACKEND="gloo")
    import torch.distributed as dist

    try:
        import oracle as O
        from gnn_amd import graphs, loader, placement, staging
        from gnn_amd.train import init_distributed

        init_distributed()
        dev = torch.device("cuda", 0)
        A, labels, feats, ncls, train, *_ = graphs.make_dataset(graphs.PRODUCTS_TEST, seed=0)
        lap = graphs.lap_matrix(A, "graphsage")
        N = A.shape[0]
        pl = placement.create_buffer(lap, train, int(0.1 * N), list(range(world)), 3, alpha=0)
        store = staging.FeatureStore(feats, pl.gpu_buffer_group[rank], dev, rank)
        direct = staging.PeerDirect(store, feats=feats, buffer_nodes=pl.gpu_buffer_group)
        alltoall = staging.PeerExchange()
        ld = loader.NativeLoader(lap, labels, train, 8192, 512, [1, 1, 1], pl.device_id_of_nodes_group[rank],
                                 pl.idx_of_nodes_on_device_group[rank], rank=rank, world_size=world, store=store,
                                 workers=2, seed=4242, device_extract=True)
        counts, ok = [], True
        try:
            it = ld.epoch(1)
            for _ in range(2):
                lb = next(it)
                plan = lb.plan
                inp = np.asarray(lb.host.input_nodes, np.int64)
                want = np.zeros((inp.size, store.F), np.float32)
                O.gather_rows(feats.numpy(), inp, want, None)  # the host table at the input nodes
                got = {}
                for name, ex in (("direct", direct), ("alltoall", alltoall)):
                    stager = staging.Stager(store, ex)
                    staged = stager.issue(plan, None)  # collective for the all-to-all (same order on every rank)
                    x0 = staged.wait()
                    torch.cuda.synchronize()
                    got[name] = x0.cpu().numpy()
                    ok = ok and np.array_equal(got[name], want)
                ok = ok and np.array_equal(got["direct"], got["alltoall"])
                counts.append((len(plan.own_pos), len(plan.host_pos),
                               [len(plan.peer_pos[j]) for j in range(world) if j != rank]))
        finally:
            ld.close()
            direct.close()
        q.put((rank, "ok" if ok else "X0 differs from the host table", counts))
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, f"error: {e!r}", None))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_config3_placement_and_staging_world4():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=280) for _ in range(WORLD)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, status, counts in out:
        assert status == "ok", (rank, status)
        for own, host, peers in counts:
            # every source is used: own buffer, the host table, and each of the 3 peers
            assert own > 0 and host > 0 and len(peers) == WORLD - 1 and all(n > 0 for n in peers), (rank, counts)
