"""GPU: the N > 1 collectives through a real RCCL ("nccl") process group, on the one GPU.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so every multi-rank GPU test
(tests/test_dist_gpu.py) runs over gloo, and the driver's multi-GPU run would be the first time
RCCL itself executes (the reference's exchange is main.py:149-168, started from one command at
main.py:289-297). Here a 1-rank RCCL group on cuda:0 runs every collective call the N > 1 path
makes, with the package's collective timeout (gnn_amd.train.init_group):

* Trainer.broadcast_parameters (initial weights from rank 0);
* the flat exchange: ClipAdam.clip_to_flat -> all_reduce(SUM) -> Adam on the views (Trainer.step's
  data-parallel branch, forced on at world 1), through the native step executor;
* the bucketed exchange (gnn_amd.dp.BucketedExchange: all-to-alls on a side stream as the
  executor's gradient-ready events fire, all_gather_into_tensor of the clip factors, gather);
* PeerExchange: the host negotiation on its gloo side group + RCCL all_to_all_single of rows;
* Trainer.check_ranks_agree (all_gather_object).

The same script runs once more over gloo; the two runs must agree bit for bit (losses,
parameters, exchanged rows), and the exchanged rows must equal the buffer rows they came from.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
LR = 0.01
NSPEC = dict(name="rccl-native", num_nodes=6000, num_edge_samples=40_000, num_feats=100, num_classes=41,
             train_frac=0.5, valid_frac=0.1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(backend, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      GNN_DIST_TIMEOUT_S="120")
    import torch.distributed as dist

    try:
        from gnn_amd import graphs, sampler, staging
        from gnn_amd.dp import BucketedExchange
        from gnn_amd.models import build_model
        from gnn_amd.train import Trainer, init_group

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        init_group(backend, rank=0, world=1, local=0)
        assert dist.get_backend() == backend
        out = {"backend": dist.get_backend()}

        spec = graphs.GraphSpec(*NSPEC.values())
        A, labels, feats, ncls, train, *_ = graphs.make_dataset(spec, seed=3)
        lap = graphs.lap_matrix(A, "graphsage")
        N = A.shape[0]
        chunk = sampler.rank_batches(train, 64, 0, 1, 1)[0]
        hb = sampler.ladies_sample_host(50, chunk, np.array([700] * 5), N, lap, labels, [1, 1, 1],
                                        np.full(N, -1, np.int64), np.zeros(N, np.int64), None, 1.0, [0],
                                        device_extract=True)
        F = feats.shape[1]
        torch.manual_seed(200)
        net = build_model("graphsage", F, 32, [1, 1, 1], ncls, dropout=0.0, fused=True).to(dev)
        tr = Trainer(net, LR, dev)
        before = tr.param_digest()
        tr.broadcast_parameters()
        torch.cuda.synchronize()
        out["broadcast_kept_params"] = tr.param_digest() == before

        db = hb.to_device(dev, with_coo=False)
        x = torch.zeros((hb.num_input_nodes, staging.padded_ld(F)), dtype=torch.float32)
        x[:, :F] = feats[torch.from_numpy(np.asarray(hb.input_nodes, np.int64))]
        x0 = x.to(dev)[:, :F]
        assert tr.executor is not None and tr.executor.supports(x0, db.adjs, db.sampled_nodes, db.labels)
        tr.dp = True  # the N > 1 branch: clip_to_flat -> all_reduce(SUM) -> Adam(clipped)
        losses = [float(tr.step(x0, db.adjs, db.sampled_nodes, db.labels)) for _ in range(2)]
        tr.bucketed = tr.exchange = BucketedExchange(tr.executor, tr.optimizer)
        losses += [float(tr.step(x0, db.adjs, db.sampled_nodes, db.labels)) for _ in range(2)]
        torch.cuda.synchronize()
        out["losses"] = losses
        out["params"] = [p.detach().cpu().numpy().copy() for p in net.parameters()]
        agree = tr.check_ranks_agree()
        out["agree"] = agree["identical"] and len(agree["digests"]) == 1

        # PeerExchange: this rank asks itself for rows (the only peer of a 1-rank group)
        k, n_in, Fp = 300, 500, 602
        table = torch.arange(k * Fp, dtype=torch.float32).view(k, Fp) * 1e-3
        store = staging.FeatureStore(table, np.arange(k), dev, 0)
        rng = np.random.default_rng(5)
        pos = np.sort(rng.choice(n_in, 200, replace=False)).astype(np.int64)
        src = rng.integers(0, k, 200).astype(np.int64)
        empty = np.zeros(0, np.int64)
        plan = staging.StagePlan(n_in, empty, empty, empty, None, [pos], [src])
        x0b = torch.full((n_in, store.ld), -1.0, device=dev)
        ex = staging.PeerExchange()
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            for _ in range(2):
                keep = ex.exchange(plan, x0b, store)
        torch.cuda.synchronize()
        del keep
        got = x0b.cpu()
        rows_ok = torch.equal(got[torch.from_numpy(pos), :Fp], table[torch.from_numpy(src)])
        untouched = np.setdiff1d(np.arange(n_in), pos)
        out["rows_ok"] = rows_ok and bool((got[torch.from_numpy(untouched)] == -1.0).all())
        out["rows"] = got.numpy()
        q.put(("ok", out))
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((f"error: {e!r}", None))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(backend):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(backend, _free_port(), q))
    p.start()
    try:
        status, out = q.get(timeout=150)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert status == "ok", f"{backend}: {status}"
    assert p.exitcode == 0, f"{backend}: exit code {p.exitcode}"
    return out


def test_rccl_group_runs_every_dp_collective_like_gloo():
    rccl = _run("nccl")
    assert rccl["backend"] == "nccl"
    for key in ("broadcast_kept_params", "agree", "rows_ok"):
        assert rccl[key], key
    assert all(np.isfinite(rccl["losses"]))
    gloo = _run("gloo")
    assert gloo["rows_ok"] and gloo["agree"]
    assert rccl["losses"] == gloo["losses"], (rccl["losses"], gloo["losses"])
    for i, (a, b) in enumerate(zip(rccl["params"], gloo["params"])):
        assert np.array_equal(a, b), f"param {i} differs between RCCL and gloo"
    assert np.array_equal(rccl["rows"], gloo["rows"])
