"""GPU, world_size 2 (and 4): the data-parallel step the benchmark runs at N > 1, on the one GPU.

All ranks run on cuda:0 with GNN_DIST_BACKEND=gloo (RCCL refuses two ranks on one GPU;
gloo moves the same CUDA tensors through the host), spawned as fresh processes.

* Trainer on CUDA: the native branch — ClipAdam.clip_to_flat (this rank's clip_grad_norm_(5)
  written into the flat all-reduce buffer), all_reduce(SUM), ClipAdam.step(clipped=True) —
  for 2 steps on rank-specific batches (the reference's LADIES goldens c2 / c3) must equal the
  reference's semantics computed independently in this process on the CPU (main.py:146-170:
  per-rank clip, SUM over ranks, no averaging, then Adam; initial weights broadcast from rank 0),
  through the product's CPU branch (torch.sparse.mm) and torch.optim.Adam.
  Tolerance: parameters within rtol 1e-4 / atol 1e-6 where the summed gradient is clearly
  non-zero (Adam's first steps move a weight by ~lr·sign(g), so weights whose gradient sits at
  the fp32 noise level are excluded, as in tests/test_fused_gpu.py).
* PeerExchange with the HIP gathers: every rank receives exactly the rows it requested from
  the peer's GPU buffer (bit-exact), through the per-step host negotiation + all_to_all.
* The benchmark's own N > 1 branch (native step executor on GPU-extracted CsrOperands) with the
  flat all-reduce and with the bucketed exchange (gnn_amd/dp.py) against the same semantics;
  bucketed ≡ flat bit for bit at world 2; the bucketed exchange at world 4 (uneven shards).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = (2, 3)  # ladies_tiny cases per rank
LR = 0.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(rank, device):
    z = np.load(os.path.join(GOLDEN, "ladies_tiny.npz"))
    c = CASES[rank]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    adjs = [torch.sparse_coo_tensor(t(z[f"c{c}_adj{li}_indices"]), t(z[f"c{c}_adj{li}_values"]),
                                    tuple(int(v) for v in z[f"c{c}_adj{li}_shape"])).coalesce() for li in range(3)]
    sampled = [t(z[f"c{c}_sampled{li}"]) for li in range(3)]
    g = torch.Generator().manual_seed(77 + rank)
    x0 = torch.randn(int(z[f"c{c}_nin"]), 602, generator=g)
    y = t(z[f"c{c}_labels"])
    if device != "cpu":
        adjs = [a.to(device) for a in adjs]
        sampled = [s.to(device) for s in sampled]
        x0, y = x0.to(device), y.to(device)
    return adjs, x0, sampled, y


def _model(seed):
    from gnn_amd.models import build_model

    torch.manual_seed(seed)
    # dropout 0: the CPU reference and the GPU run draw no masks (their RNGs differ)
    return build_model("graphsage", 602, 32, [1, 1, 1], 41, dropout=0.0)


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GNN_DIST_BACKEND="gloo")


def _trainer_worker(rank, world, port, q):
    _env(rank, world, port)
    import torch.distributed as dist

    try:
        from gnn_amd.models import build_model
        from gnn_amd.train import Trainer, init_distributed

        init_distributed()
        dev = torch.device("cuda", 0)
        torch.manual_seed(100 + rank)  # a different init per rank: the broadcast must fix it
        net = build_model("graphsage", 602, 32, [1, 1, 1], 41, dropout=0.0, fused=True).to(dev)
        tr = Trainer(net, LR, dev)
        assert tr.native and tr.world == world
        adjs, x0, sampled, y = _inputs(rank, dev)
        losses = [float(tr.step(x0, adjs, sampled, y)) for _ in range(2)]
        torch.cuda.synchronize()
        q.put((rank, "ok", losses, [p.detach().cpu().numpy().copy() for p in net.parameters()]))
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, f"error: {e!r}", None, None))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


NSPEC = dict(name="dist-native", num_nodes=6000, num_edge_samples=40_000, num_feats=100, num_classes=41,
             train_frac=0.5, valid_frac=0.1)
NSAMP, NBS = 700, 64


def _native_batch(rank, device_extract, world=2):
    """Rank `rank`'s batch of the native-executor case: LADIES with the lower layers extracted on
    the GPU (device_extract=True: CsrOperands + transposes + row maps, what the bench feeds the
    executor) or on the host (the CPU reference's operands; the draw is identical)."""
    from gnn_amd import graphs, sampler

    spec = graphs.GraphSpec(*NSPEC.values())
    A, labels, feats, ncls, train, *_ = graphs.make_dataset(spec, seed=3)
    lap = graphs.lap_matrix(A, "graphsage")
    N = A.shape[0]
    chunk = sampler.rank_batches(train, NBS, rank, world, 1)[0]
    hb = sampler.ladies_sample_host(50 + rank, chunk, np.array([NSAMP] * 5), N, lap, labels, [1, 1, 1],
                                    np.full(N, -1, np.int64), np.zeros(N, np.int64), None, 1.0, [0],
                                    device_extract=device_extract)
    return hb, feats, ncls


def _native_model(seed, F, ncls, fused):
    from gnn_amd.models import build_model

    torch.manual_seed(seed)
    return build_model("graphsage", F, 32, [1, 1, 1], ncls, dropout=0.0, fused=fused)


def _native_trainer_worker(rank, world, port, q, buckets=True, prefetch=False):
    """The benchmark's N > 1 branch: the executor step, then (buckets=True, GNN_DP_BUCKETS=1) the
    bucketed exchange overlapped with the backward (gnn_amd.dp) or (buckets=False, the default)
    ClipAdam.clip_to_flat -> all_reduce(SUM); then Adam (train.py, Trainer.step)."""
    _env(rank, world, port)
    os.environ["GNN_DP_BUCKETS"] = "1" if buckets else "0"
    import torch.distributed as dist

    try:
        from gnn_amd import staging
        from gnn_amd.train import Trainer, init_distributed

        init_distributed()
        dev = torch.device("cuda", 0)
        hb, feats, ncls = _native_batch(rank, True, world)
        F = feats.shape[1]
        net = _native_model(200 + rank, F, ncls, True).to(dev)  # rank-specific init: the broadcast fixes it
        tr = Trainer(net, LR, dev)
        db = hb.to_device(dev, with_coo=False)
        x = torch.zeros((hb.num_input_nodes, staging.padded_ld(F)), dtype=torch.float32)
        x[:, :F] = feats[torch.from_numpy(np.asarray(hb.input_nodes, np.int64))]
        x0 = x.to(dev)[:, :F]
        assert tr.executor is not None and tr.executor.supports(x0, db.adjs, db.sampled_nodes, db.labels), \
            "the executor branch must be the one exercised"
        assert (tr.exchange is not None) == buckets, "the exchange variant under test must be the one in use"
        losses, taken = [], []
        for s in range(2):
            # prefetch: the batch of the next step (the same one here) — its layer-0 aggregation
            # issued while this step's all-reduce runs, then not issued again by the next step
            nxt = (x0, db.adjs, db.sampled_nodes, db.labels) if prefetch and s == 0 else None
            losses.append(float(tr.step(x0, db.adjs, db.sampled_nodes, db.labels, prefetch=nxt)))
            taken.append(getattr(tr.executor, "_pre", None) is not None)
        torch.cuda.synchronize()
        if taken != [prefetch, False]:
            raise AssertionError(f"prefetch taken {taken}")
        q.put((rank, "ok", losses, [p.detach().cpu().numpy().copy() for p in net.parameters()]))
    except Exception as e:
        q.put((rank, f"error: {e!r}", None, None))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _native_reference_two_steps(world=2):
    """main.py:146-170 on the CPU for the native case: per-rank grads of the host-extracted
    batches through the CPU branch (torch.sparse.mm), per-rank clip_grad_norm_(5), SUM, Adam."""
    from gnn_amd.models import loss as loss_fn

    batches = [_native_batch(r, False, world) for r in range(world)]
    F, ncls = batches[0][1].shape[1], batches[0][2]
    nets = [_native_model(200, F, ncls, False) for _ in range(world)]  # rank 0's init on all
    params = list(nets[0].parameters())
    opt = torch.optim.Adam(params, lr=LR)
    inputs = [hb.cpu_inputs(feats) for hb, feats, _ in batches]
    sums, losses = [], []
    for _ in range(2):
        with torch.no_grad():
            for net in nets[1:]:
                for p0, p1 in zip(nets[0].parameters(), net.parameters()):
                    p1.copy_(p0)
        grads = []
        for r in range(world):
            net = nets[r]
            net.zero_grad()
            adjs, x0, sampled, y = inputs[r]
            lo = loss_fn(net(x0, adjs, sampled), y, True, "cpu")
            lo.backward()
            losses.append(float(lo.detach()))
            torch.nn.utils.clip_grad_norm_(net.parameters(), 5)
            grads.append([p.grad.detach().clone() for p in net.parameters()])
        total = [sum(gs[1:], gs[0]) for gs in zip(*grads)]
        for p, g in zip(params, total):
            p.grad = g
        sums.append(total)
        opt.step()
    return [p.detach().numpy() for p in params], sums, losses


_native_out = {}


@pytest.mark.parametrize("buckets", [True, False], ids=["bucketed", "flat"])
def test_trainer_executor_dp_step_matches_reference(buckets):
    """The branch bench.py runs at N > 1 (executor + the gradient exchange + Adam on views), with
    GPU-extracted CsrOperands as the bench feeds them, against main.py:146-170 semantics — for the
    bucketed exchange overlapped with the backward and the flat all-reduce (the default)."""
    out = _spawn(_native_trainer_worker, extra=(buckets,))
    for rank, status, _, _ in out:
        assert status == "ok", f"rank {rank}: {status}"
    _native_out[buckets] = out
    ref, sums, ref_losses = _native_reference_two_steps()
    for rank in range(2):
        for s in range(2):
            got, want = out[rank][2][s], ref_losses[2 * s + rank]
            assert abs(got - want) <= 1e-4 * abs(want) + 1e-6, (rank, s, got, want)
    p0, p1 = out[0][3], out[1][3]
    for a, b in zip(p0, p1):
        assert np.array_equal(a, b), "ranks disagree after the summed update"
    for i, (got, want) in enumerate(zip(p0, ref)):
        sure = np.ones(got.shape, bool)
        for s in sums:
            gg = s[i].numpy()
            sure &= np.abs(gg) > 1e-4 * max(np.abs(gg).max(), 1e-12)
        assert sure.mean() > 0.5
        np.testing.assert_allclose(got[sure], want[sure], rtol=1e-4, atol=1e-6, err_msg=f"param {i}")


def test_dp_layer0_prefetch_is_bit_identical():
    """The flat data-parallel step with the next batch's layer-0 aggregation issued while the
    all-reduce runs (Trainer.step(prefetch=...), the bench's N > 1 default) against the same two
    steps without it: losses and parameters bit for bit on both ranks."""
    outs = {}
    for pf in (False, True):
        out = _spawn(_native_trainer_worker, extra=(False, pf))
        for rank, status, _, _ in out:
            assert status == "ok", f"prefetch={pf} rank {rank}: {status}"
        outs[pf] = out
    for rank in range(2):
        assert outs[True][rank][2] == outs[False][rank][2], rank
        for a, b in zip(outs[True][rank][3], outs[False][rank][3]):
            assert np.array_equal(a, b), rank


def _exchange_worker(rank, world, port, q):
    _env(rank, world, port)
    import torch.distributed as dist

    try:
        from gnn_amd import staging
        from gnn_amd.train import init_distributed

        init_distributed()
        dev = torch.device("cuda", 0)
        F, k, n_in = 602, 300, 500
        feats = torch.arange(2 * k * F, dtype=torch.float32).view(2 * k, F) * 1e-3
        # rank r buffers nodes [r*k, (r+1)*k) of the feature table, slot i = node r*k + i
        store = staging.FeatureStore(feats, np.arange(rank * k, (rank + 1) * k), dev, rank)
        rng = np.random.default_rng(rank)
        peer = 1 - rank
        pos = np.sort(rng.choice(n_in, 200, replace=False)).astype(np.int64)
        src = rng.integers(0, k, 200).astype(np.int64)
        empty = np.zeros(0, np.int64)
        peer_pos, peer_src = [empty, empty], [empty, empty]
        peer_pos[peer], peer_src[peer] = pos, src
        plan = staging.StagePlan(n_in, empty, empty, empty, None, peer_pos, peer_src)
        x0 = torch.full((n_in, store.ld), -1.0, device=dev)
        ex = staging.PeerExchange()
        for _ in range(2):  # negotiated afresh each time
            ex.exchange(plan, x0, store)
        torch.cuda.synchronize()
        expect = feats[torch.from_numpy(peer * k + src)]
        ok = torch.equal(x0[torch.from_numpy(pos).to(dev), :F].cpu(), expect)
        untouched = np.setdiff1d(np.arange(n_in), pos)
        ok = ok and bool((x0[torch.from_numpy(untouched).to(dev)] == -1.0).all())
        q.put((rank, "ok" if ok else "rows differ", None, None))
    except Exception as e:
        q.put((rank, f"error: {e!r}", None, None))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _direct_worker(rank, world, port, q):
    """staging.PeerDirect: each rank maps the other's buffer once (IPC) and gathers the rows it
    needs straight from it into X0 — same rows as the all-to-all exchange, bit for bit, and
    nothing else in X0 touched."""
    _env(rank, world, port)
    import torch.distributed as dist

    try:
        from gnn_amd import staging
        from gnn_amd.train import init_distributed

        init_distributed()
        dev = torch.device("cuda", 0)
        F, k, n_in = 602, 300, 500
        feats = torch.arange(world * k * F, dtype=torch.float32).view(world * k, F) * 1e-3
        store = staging.FeatureStore(feats, np.arange(rank * k, (rank + 1) * k), dev, rank)
        ex = staging.PeerDirect(store)
        rng = np.random.default_rng(10 + rank)
        empty = np.zeros(0, np.int64)
        peer_pos, peer_src = [empty] * world, [empty] * world
        perm = rng.permutation(n_in)
        expect_rows, cut = [], 0
        for j in range(world):
            if j == rank:
                continue
            m = 120
            peer_pos[j] = np.sort(perm[cut:cut + m]).astype(np.int64)
            peer_src[j] = rng.integers(0, k, m).astype(np.int64)
            peer_src[j][0] = k - 1  # the last slot of the peer's buffer
            cut += m
        plan = staging.StagePlan(n_in, empty, empty, empty, None, peer_pos, peer_src)
        x0 = torch.full((n_in, store.ld), -1.0, device=dev)
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            for _ in range(2):
                ex.exchange(plan, x0, store)
        torch.cuda.synchronize()
        ok = True
        got = x0.cpu()
        for j in range(world):
            if j == rank:
                continue
            want = torch.zeros((len(peer_src[j]), store.ld))
            want[:, :F] = feats[torch.from_numpy(j * k + peer_src[j])]
            ok = ok and torch.equal(got[torch.from_numpy(peer_pos[j])], want)
        touched = np.concatenate([p for p in peer_pos if len(p)])
        untouched = np.setdiff1d(np.arange(n_in), touched)
        ok = ok and bool((got[torch.from_numpy(untouched)] == -1.0).all())
        bad = False
        try:  # a slot outside the peer's buffer is refused on the host, before any kernel
            peer_src2 = list(peer_src)
            peer_src2[1 - rank if world == 2 else (rank + 1) % world] = np.array([k], np.int64)
            peer_pos2 = list(peer_pos)
            peer_pos2[1 - rank if world == 2 else (rank + 1) % world] = np.array([0], np.int64)
            ex.exchange(staging.StagePlan(n_in, empty, empty, empty, None, peer_pos2, peer_src2), x0, store)
        except RuntimeError as e:
            bad = "outside" in str(e)
        ex.close()
        q.put((rank, "ok" if ok and bad else f"rows differ or bound unchecked (rows ok {ok}, bound {bad})",
               None, None))
    except Exception as e:
        q.put((rank, f"error: {e!r}", None, None))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(fn, world=2, extra=()):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = [q.get(timeout=100) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return sorted(out, key=lambda t: t[0])


def _reference_two_steps():
    """main.py:146-170 on the CPU: per-rank grads, per-rank clip_grad_norm_(5), SUM, Adam."""
    from gnn_amd.models import loss as loss_fn

    nets = [_model(100) for _ in range(2)]  # rank 0's init on both (the broadcast)
    params = list(nets[0].parameters())
    opt = torch.optim.Adam(params, lr=LR)
    inputs = [_inputs(r, "cpu") for r in range(2)]
    sums = []
    for _ in range(2):
        with torch.no_grad():
            for p0, p1 in zip(nets[0].parameters(), nets[1].parameters()):
                p1.copy_(p0)
        grads = []
        for r in range(2):
            net = nets[r]
            net.zero_grad()
            adjs, x0, sampled, y = inputs[r]
            lo = loss_fn(net(x0, adjs, sampled), y, True, "cpu")
            lo.backward()
            torch.nn.utils.clip_grad_norm_(net.parameters(), 5)
            grads.append([p.grad.detach().clone() for p in net.parameters()])
        total = [a + b for a, b in zip(*grads)]
        for p, g in zip(params, total):
            p.grad = g
        sums.append(total)
        opt.step()
    return [p.detach().numpy() for p in params], sums


def test_trainer_native_dp_step_matches_reference():
    out = _spawn(_trainer_worker)
    for rank, status, _, _ in out:
        assert status == "ok", f"rank {rank}: {status}"
    ref, sums = _reference_two_steps()
    p0, p1 = out[0][3], out[1][3]
    for a, b in zip(p0, p1):
        assert np.array_equal(a, b), "ranks disagree after the summed update"
    for i, (got, want) in enumerate(zip(p0, ref)):
        sure = np.ones(got.shape, bool)
        for s in sums:
            gg = s[i].numpy()
            sure &= np.abs(gg) > 1e-4 * max(np.abs(gg).max(), 1e-12)
        assert sure.mean() > 0.5
        np.testing.assert_allclose(got[sure], want[sure], rtol=1e-4, atol=1e-6, err_msg=f"param {i}")


def test_peer_exchange_hip_gathers_bit_exact():
    out = _spawn(_exchange_worker)
    for rank, status, _, _ in out:
        assert status == "ok", f"rank {rank}: {status}"


def test_bucketed_exchange_equals_flat():
    """At world size 2 the bucketed exchange's sum (c_0 g_0 + c_1 g_1 per element, each product
    rounded once) is the flat all-reduce's, bit for bit."""
    for b in (True, False):
        if b not in _native_out:
            out = _spawn(_native_trainer_worker, extra=(b,))
            assert all(st == "ok" for _, st, _, _ in out), out
            _native_out[b] = out
    for rank in range(2):
        for a, c in zip(_native_out[True][rank][3], _native_out[False][rank][3]):
            assert np.array_equal(a, c), "bucketed and flat exchanges disagree"


def _check_against_reference(out, world):
    ref, sums, ref_losses = _native_reference_two_steps(world)
    for rank in range(world):
        for s in range(2):
            got, want = out[rank][2][s], ref_losses[world * s + rank]
            assert abs(got - want) <= 1e-4 * abs(want) + 1e-6, (rank, s, got, want)
    for r in range(1, world):
        for a, b in zip(out[0][3], out[r][3]):
            assert np.array_equal(a, b), f"rank {r} disagrees with rank 0 after the summed update"
    for i, (got, want) in enumerate(zip(out[0][3], ref)):
        sure = np.ones(got.shape, bool)
        for s in sums:
            gg = s[i].numpy()
            sure &= np.abs(gg) > 1e-4 * max(np.abs(gg).max(), 1e-12)
        assert sure.mean() > 0.5
        np.testing.assert_allclose(got[sure], want[sure], rtol=1e-4, atol=1e-6, err_msg=f"param {i}")


def test_bucketed_exchange_world4():
    """Four ranks on the one GPU (gloo): uneven shards of every bucket (the bucket sizes are not
    multiples of 4), four clip factors riding with the last bucket, the gather of four ranks'
    shards — every rank ends with the same parameters, main.py:146-170 semantics."""
    out = _spawn(_native_trainer_worker, world=4, extra=(True,))
    for rank, status, _, _ in out:
        assert status == "ok", f"rank {rank}: {status}"
    _check_against_reference(out, 4)


@pytest.mark.parametrize("world", [2, 3])
def test_peer_direct_rows_bit_exact(world):
    out = _spawn(_direct_worker, world=world)
    for rank, status, _, _ in out:
        assert status == "ok", f"rank {rank}: {status}"
