"""Benchmark: Reddit GraphSAGE / LADIES mini-batch training on MI355X (BASELINE.json config 2).

One step = one data-parallel mini-batch training iteration of the reference's hot path
(main.py:122-170) on a pre-sampled LADIES batch whose operands and index arrays are resident
in HBM: X0 staging (own-GPU buffer gather + pinned-host rows H2D on a side stream, peer rows
by RCCL all-to-all when N > 1), 3 HIP aggregation forwards + 2 backwards inside GraphSAGE
(samp_num 8192, batch 512, nhid 512, orders 1,1,1, F = 602, 41 classes), loss, backward,
clip_grad_norm_(5), RCCL all-reduce(SUM) of the flat gradient, Adam.
Synthetic Reddit-shaped graph: Chung-Lu lognormal sigma 1.3, N = 232,965,
~23.1 M nnz, N(0,1) fp32 features (StandardScaler'd analogue), buffer_size = 0.1.

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under torch.distributed.run.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from gnn_amd import custom_sparse_ops as cso  # noqa: E402
from gnn_amd import graphs, placement, sampler, staging  # noqa: E402
from gnn_amd.models import build_model  # noqa: E402
from gnn_amd.train import Trainer, init_distributed  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


GRAPH_NAMES = {"reddit": "Reddit", "products": "ogbn-products", "papers": "ogbn-papers100M-scaled", "tiny": "tiny"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batches", type=int, default=4, help="distinct pre-sampled batches per rank (cycled)")
    ap.add_argument("--model", default="graphsage", choices=["graphsage", "gcn"])
    ap.add_argument("--sampler", default="ladies", choices=["ladies", "subgraph", "fastgcn"])
    ap.add_argument("--samp-num", type=int, default=8192)
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--nhid", type=int, default=512)
    ap.add_argument("--buffer-size", type=float, default=0.1)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--graph", default="reddit", choices=["reddit", "products", "papers", "tiny"],
                    help="synthetic graph shape: reddit (configs 1-2), products (configs 3, 5), papers "
                         "(config 4's per-batch geometry on a graph scaled to the box), tiny (smoke)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic child run")
    ap.add_argument("--unfused", action="store_true", help="torch elementwise layer tail instead of the HIP one")
    ap.add_argument("--e2e-steps", type=int, default=60, help="steps of the live-sampling end-to-end run")
    ap.add_argument("--no-e2e", action="store_true", help="skip the live-sampling end-to-end run")
    ap.add_argument("--workers", type=int, default=0, help="sampler threads per rank (0: auto)")
    ap.add_argument("--compute-priority", default="high", choices=["high", "normal"],
                    help="priority of the stream the training step runs on (the staging stream stays normal)")
    ap.add_argument("--staging", default="copy", choices=["copy", "zerocopy"],
                    help="non-buffered feature rows: host gather into pinned memory + one hipMemcpyAsync "
                         "(copy), or the GPU reads the mapped host table over PCIe (zerocopy: measured "
                         "slower, it slows the concurrent compute kernels)")
    ap.add_argument("--cprofile", default="", help="after the timed run, cProfile 20 steps into this text file")
    ap.add_argument("--torch-profile", default="", help="after the timed run, write a torch.profiler op table here")
    ap.add_argument("--dump-batch", default="", help="save rank-0 batch 0 operands (.npz) for kernel profiling")
    return ap.parse_args()


def sample_batches(args, lap, labels, train, pl, rank, world):
    batches = sampler.rank_batches(train, args.batch_size, rank, world, iter_num=1)[: args.batches]
    rs = np.random.RandomState(1234 + rank)
    seeds = rs.randint(2**31 - 1, size=len(batches))
    out = []
    fn = {"ladies": sampler.ladies_sample_host, "subgraph": sampler.subgraph_sample_host,
          "fastgcn": sampler.fastgcn_sample_host}[args.sampler]
    for s, b in zip(seeds, batches):
        out.append(fn(int(s), b, np.array([args.samp_num] * 5), lap.shape[0], lap, labels,
                                              [1, 1, 1], pl.device_id_of_nodes_group[rank],
                                              pl.idx_of_nodes_on_device_group[rank], None, 1.0, list(range(world))))
    return out


def _counter_rows(d):
    import csv
    import glob

    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def _kernel_symbol(name: str) -> str:
    """'void (anonymous namespace)::spmm_unit_kernel<4, 16, 1, 4, false>(int const*, ...)' ->
    'spmm_unit_kernel<4, 16, 1, 4, false>' (the form the bench's timing records use)."""
    name = name.split("(anonymous namespace)::")[-1]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i].strip()
    return name.strip()


def pmc_traffic(hb, F, hidden, workdir="/tmp/gnn_bench_pmc"):
    """Bytes per launch leaving L2 (toward the Infinity Cache / HBM) for each aggregation
    kernel instantiation, from rocprofv3 PMC counters (FETCH_SIZE and WRITE_SIZE in separate
    passes) over the forward calls of batch 0 laid out as the benchmark runs them, each
    counter corrected by a calibration gather of known bytes with the same 16-byte row
    vectors (MI355X_MICROARCH.md §HBM). Runs the probe as a CHILD process before this process
    has touched the GPU. Returns {"by_kernel": {symbol: {...}}, corrections}, or None."""
    import shutil
    import subprocess

    if shutil.which("rocprofv3") is None:
        return None
    os.makedirs(workdir, exist_ok=True)
    npz = os.path.join(workdir, "batch0.npz")
    L0 = hb.layers
    np.savez(npz, **{f"l{i}_{k}": getattr(L, k) for i, L in enumerate(L0)
                     for k in ("fullrowptr", "rowptr", "colidx", "normfact")},
             **{f"l{i}_shape": np.array(L.shape) for i, L in enumerate(L0)})
    probe = os.path.join(REPO, "scripts", "pmc_probe.py")
    calib, kern = {}, {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(workdir, counter)
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "p", "--",
               sys.executable, probe, npz, "--feat", str(F), "--hidden", str(hidden)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            log(f"pmc pass {counter} failed rc={r.returncode}: {r.stderr[-500:]}")
            return None
        cal = []
        for row in _counter_rows(d):
            if row.get("Counter_Name") != counter:
                continue
            name, v = row.get("Kernel_Name", ""), float(row.get("Counter_Value", "nan"))
            if "gather_rows_kernel" in name:
                cal.append(v)
            elif "spmm_unit_kernel" in name:
                kern.setdefault(_kernel_symbol(name), {}).setdefault(counter, []).append(v)
        if not cal:
            return None
        calib[counter] = float(np.median(cal))
    ld = (F + 3) // 4 * 4
    n = int(1.2e9 // (ld * 4))
    known = n * ld * 4  # bytes read (and written) by one calibration gather
    read_corr = known / (calib["FETCH_SIZE"] * 1024.0)
    write_corr = known / (calib["WRITE_SIZE"] * 1024.0)
    by = {}
    for sym, c in kern.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        rd = float(np.mean(c["FETCH_SIZE"])) * 1024.0 * read_corr
        wr = float(np.mean(c["WRITE_SIZE"])) * 1024.0 * write_corr
        by[sym] = {"bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
                   "launches": len(c["FETCH_SIZE"])}
    return {"by_kernel": by, "read_correction": round(read_corr, 4), "write_correction": round(write_corr, 4)}


def cpu_baseline(args, hb, feats, num_classes):
    """Reference CPU path (torch.sparse.mm) full training step on the same batch, rank 0 / N=1."""
    from oracle.cpu_reference import cpu_inputs, cpu_train_step, torch_spmm

    torch.manual_seed(0)
    model = build_model(args.model, feats.shape[1], args.nhid, [1, 1, 1], num_classes, 0.1, spmm_fn=torch_spmm)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    adjs, x0, sampled, labels = cpu_inputs(hb, feats)
    cpu_train_step(model, opt, adjs, x0, sampled, labels)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        cpu_train_step(model, opt, adjs, x0, sampled, labels)
        n += 1
        if time.perf_counter() - t0 >= args.cpu_baseline_seconds or n >= 50:
            break
    dt = time.perf_counter() - t0
    # the aggregation calls alone: torch.sparse.mm forward, and backward
    # including the reference's A.transpose(0,1).coalesce()
    calls = {}
    g = torch.Generator().manual_seed(0)
    for li in (0, 1):
        a = adjs[li]
        X = x0 if li == 0 else torch.randn(a.shape[1], 2 * args.nhid, generator=g)
        reps, t = 0, time.perf_counter()
        while reps < 3 or (time.perf_counter() - t < 1.0 and reps < 20):
            torch.sparse.mm(a, X)
            reps += 1
        calls[f"fwd{li}"] = round(1e3 * (time.perf_counter() - t) / reps, 2)
        if li == 1:
            G = torch.randn(a.shape[0], 2 * args.nhid, generator=g)
            reps, t = 0, time.perf_counter()
            while reps < 3 or (time.perf_counter() - t < 1.0 and reps < 20):
                torch.sparse.mm(a.t().coalesce(), G)
                reps += 1
            calls["bwd1_incl_transpose"] = round(1e3 * (time.perf_counter() - t) / reps, 2)
    return {"value": n / dt, "unit": "mini-batches/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} full GraphSAGE training steps (torch.sparse.mm fwd/bwd, dense layers, Adam) on "
                      f"pre-sampled batch 0 (samp {args.samp_num}, bs {args.batch_size}), {dt:.1f} s",
            "spmm_call_ms": calls}


def cpu_budget() -> int:
    """Host CPUs this process may use: the affinity set, capped by a cgroup-v2 CPU quota
    (the GPU box grants 16 CPUs per GPU by quota while os.cpu_count() shows the machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 8)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def default_workers(world: int) -> int:
    # sampler threads per rank: the rank's CPU share minus the training thread and one spare
    # (measured on the 16-CPU box: 14 threads 288 mini-batches/s end to end, 10 threads 227)
    return max(2, min(14, cpu_budget() // max(world, 1) - 2))


def end_to_end(args, pipeline, lap, labels, train, pl, store, rank, world, dev):
    """Mini-batches/s with sampling in the loop: the native LADIES sampler + host-row staging
    in worker threads (gnn_amd.loader.BatchLoader) feeding the same training step. Also the
    single-thread sampler cost per batch, native and numpy (rank 0)."""
    from gnn_amd.loader import BatchLoader

    workers = args.workers or default_workers(world)
    ld = BatchLoader(lap, labels, train, args.samp_num, args.batch_size, [1, 1, 1], pl.device_id_of_nodes_group[rank],
                     pl.idx_of_nodes_on_device_group[rank], rank=rank, world_size=world, store=store,
                     workers=workers, seed=4242, kind=args.sampler)
    it = ld.forever()

    def nxt():
        lb = next(it)
        return lb.plan, lambda: lb.host.to_device(dev, with_coo=False)

    warm = max(2 * workers, 10)
    pipeline(nxt, warm)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipeline(nxt, args.e2e_steps)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    ld.close()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    out = {"value": round(world * args.e2e_steps / el, 3), "unit": "mini-batches/s", "steps": args.e2e_steps,
           "sampler_workers_per_rank": workers,
           "what": f"live {args.sampler} sampling (native, worker threads) + pinned host staging + H2D + the same step"}
    if rank == 0:
        chunks = sampler.rank_batches(train, args.batch_size, 0, 1, 99)[:4]
        fn = {"ladies": sampler.ladies_sample_host, "subgraph": sampler.subgraph_sample_host,
              "fastgcn": sampler.fastgcn_sample_host}[args.sampler]
        sm = np.array([args.samp_num] * 5)
        pdev, pidx = pl.device_id_of_nodes_group[rank], pl.idx_of_nodes_on_device_group[rank]
        t = time.perf_counter()
        for i, c in enumerate(chunks[:3]):
            fn(i, c, sm, lap.shape[0], lap, labels, [1, 1, 1], pdev, pidx, None, 1.0, list(range(world)))
        nat = (time.perf_counter() - t) / 3
        t = time.perf_counter()
        fn(3, chunks[3], sm, lap.shape[0], lap, labels, [1, 1, 1], pdev, pidx, None, 1.0, list(range(world)),
           native=False)
        npy = time.perf_counter() - t
        out["sampler_ms_per_batch_1thread"] = {"native": round(nat * 1e3, 1), "numpy": round(npy * 1e3, 1)}
    return out


def main():
    args = parse()
    rank, world, local = init_distributed()
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    dev = torch.device("cuda", local)

    t0 = time.time()
    spec = {"reddit": graphs.REDDIT, "products": graphs.PRODUCTS, "papers": graphs.PAPERS_SCALED,
            "tiny": graphs.TINY}[args.graph]
    A, labels, feats, num_classes, train, valid, test = graphs.make_dataset(spec, seed=0)
    lap = graphs.row_normalize(A)
    lap.sum_duplicates()
    N = A.shape[0]
    log(f"graph {spec.name}: N={N} nnz={A.nnz} ({time.time() - t0:.1f}s)")
    k = int(args.buffer_size * N)
    pl = placement.create_buffer(lap, train, k, list(range(world)), 3, alpha=0)
    log(f"placement k={k} per GPU ({time.time() - t0:.1f}s)")
    host_batches = sample_batches(args, lap, labels, train, pl, rank, world)
    log(f"sampled {len(host_batches)} batches ({time.time() - t0:.1f}s); nnz/batch={host_batches[0].nnz()}")
    traffic = None
    if rank == 0 and world == 1 and not args.no_traffic:
        # before this process initialises the GPU: the probe is a child process
        try:
            traffic = pmc_traffic(host_batches[0], feats.shape[1], 2 * args.nhid)
        except Exception as e:  # profiler trouble must not sink the benchmark
            log(f"pmc traffic measurement skipped: {e!r}")
        log(f"pmc traffic done ({time.time() - t0:.1f}s): {traffic}")
    torch.cuda.set_device(dev)

    store = staging.FeatureStore(feats, pl.gpu_buffer_group[rank], dev, rank, zero_copy=args.staging == "zerocopy")
    exchange = staging.PeerExchange() if world > 1 else None
    stager = staging.Stager(store, exchange)
    plans = [staging.make_plan(hb, store, rank, world) for hb in host_batches]
    # CSR pieces, labels and sampled_nodes resident in HBM; the operand builder (the
    # create_coo_tensor kernel) runs for every step, on the staging stream ahead of it.
    dbatches = [hb.to_device(dev, build=False) for hb in host_batches]
    if args.dump_batch and rank == 0:
        L0 = host_batches[0].layers
        np.savez(args.dump_batch, **{f"l{i}_{k}": getattr(L, k) for i, L in enumerate(L0)
                                     for k in ("fullrowptr", "rowptr", "colidx", "normfact")},
                 **{f"l{i}_shape": np.array(L.shape) for i, L in enumerate(L0)})

    torch.manual_seed(0)
    model = build_model(args.model, store.F, args.nhid, [1, 1, 1], num_classes, 0.1, fused=not args.unfused).to(dev)
    trainer = Trainer(model, args.lr, dev)
    torch.cuda.synchronize()
    log(f"setup done ({time.time() - t0:.1f}s); params={trainer.num_params}")

    nb = len(dbatches)
    retire = staging.Retirement()

    # The step runs on a high-priority stream: the staging stream's gathers and operand builds
    # for the next batch (default priority) then fill the compute stream's gaps instead of
    # taking CU slots from the layer-0 aggregation they overlap (--compute-priority normal: off).
    lo_pri, hi_pri = torch.cuda.Stream.priority_range()
    compute_stream = torch.cuda.Stream(device=dev, priority=hi_pri) if args.compute_priority == "high" else None

    def pipeline(next_item, steps):
        if compute_stream is None:
            return _pipeline(next_item, steps)
        compute_stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(compute_stream):
            loss = _pipeline(next_item, steps)
        torch.cuda.current_stream(dev).wait_stream(compute_stream)
        return loss

    def _pipeline(next_item, steps):
        """next_item() -> (StagePlan, batch_fn); batch_fn() makes the DeviceBatch (H2D when
        needed + the operand builds). Batch i+1's X0 staging and batch_fn run on the side
        stream, issued before batch i's step, so they overlap that step's kernels."""
        loss = None
        staged = stager.issue(*next_item())
        for i in range(steps):
            staged_next = stager.issue(*next_item()) if i + 1 < steps else None
            x0 = staged.wait(retire)
            db = staged.batch
            loss = trainer.step(x0, staged.adjs, db.sampled_nodes, db.labels)
            retire.retire(staged)  # held until the step has run (no per-tensor record_stream)
            staged = staged_next
        return loss

    def run(steps, start):
        """Pre-sampled batches, operands resident in HBM, cycled (the headline step)."""
        k = [start]

        def nxt():
            j = k[0] % nb
            k[0] += 1
            db = dbatches[j]
            return plans[j], lambda: (db.build_operands(), db)[1]
        return pipeline(nxt, steps)

    run(args.warmup, 0)
    cso.enable_timing(not args.no_roofline)
    stager.timing = []
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    retire.wait_s = 0.0
    t_start = time.perf_counter()
    loss = run(args.steps, args.warmup)
    # host time to issue the steps, without the waits that keep it <= 3 steps ahead of the GPU
    t_issued = time.perf_counter() - retire.wait_s
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    cso.enable_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    recs = cso.take_timing_records()
    h_bytes, h_sec = stager.take_timing()
    staging_info = {"mode": args.staging, "host_rows_MB_per_batch": round(h_bytes / args.steps / 1e6, 2),
                    "h2d_GBps": round(h_bytes / h_sec / 1e9, 1) if h_sec > 0 else None,
                    "h2d_ms_per_batch": round(1e3 * h_sec / args.steps, 3),
                    "note": ("GPU gather of the host rows from the pinned, device-mapped feature table over PCIe"
                             if args.staging == "zerocopy" else
                             "host rows gathered into pinned memory by the producer, one hipMemcpyAsync")
                            + " on the staging stream, overlapped with the previous step"}

    # ------------------------------------------------- end to end, live sampling
    e2e = None
    if not args.no_e2e and args.e2e_steps > 0:
        e2e = end_to_end(args, pipeline, lap, labels, train, pl, store, rank, world, dev)
    if args.cprofile and rank == 0:
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        run(20, 0)
        torch.cuda.synchronize()
        pr.disable()
        with open(args.cprofile, "w") as fh:
            st = pstats.Stats(pr, stream=fh)
            st.sort_stats("tottime").print_stats(45)
            st.sort_stats("cumulative").print_stats(45)
    if args.torch_profile and rank == 0:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            run(3, 0)
            torch.cuda.synchronize()
        with open(args.torch_profile, "w") as fh:
            fh.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=60,
                                                                        max_name_column_width=60,
                                                                        max_shapes_column_width=90))
            fh.write("\n\n")
            fh.write(prof.key_averages().table(sort_by="count", row_limit=80, max_name_column_width=60))
            fh.write("\n\n")
            fh.write(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=50, max_name_column_width=60))
            fh.write("\n\n")
            for ev in prof.events():
                if ev.device_type.name == "CUDA":
                    continue
                if ev.name in ("aten::mm", "aten::addmm", "aten::linear", "aten::matmul"):
                    kern = [(k.name[:70], round(float(getattr(k, "duration", 0)), 1)) for k in ev.kernels]
                    fh.write(f"{ev.name} {ev.input_shapes} {kern}\n")
    final_loss = float(loss.item()) if loss is not None else float("nan")

    # ---------------------------------------------------------------- roofline
    roof = None
    spmm_detail = {}
    if recs:
        # per call site, in call order within a step: 3 forwards, then the backwards of
        # layers 2 and 1 (layer 0's input needs no gradient)
        names = ["fwd_L0", "fwd_L1", "fwd_L2", "bwd_L2", "bwd_L1"]
        site, kname = {}, {}
        for i, (tag, ms, nbytes, kn) in enumerate(recs):
            key = names[i % len(names)]
            assert key.startswith(tag), (key, tag)
            e = site.setdefault(key, [0.0, 0, 0])
            e[0] += ms
            e[1] += nbytes
            e[2] += 1
            kname[key] = kn
        for key, (ms, nbytes, n) in site.items():
            spmm_detail[key] = {"avg_us": 1e3 * ms / n, "GB_per_launch": nbytes / n / 1e9,
                                "GBps": nbytes / (ms * 1e-3) / 1e9, "kernel": kname[key]}
        # the dominant kernel = the aggregation instantiation (as rocprofv3 names it) with the
        # most time per step; several call sites may share it (rocprof averages over them too)
        byk = {}
        for key, (ms_, nb_, n_) in site.items():
            e = byk.setdefault(kname[key], [0.0, 0, 0, []])
            e[0] += ms_
            e[1] += nb_
            e[2] += n_
            e[3].append(key)
        dom = max(byk, key=lambda k_: byk[k_][0])
        ms, nbytes, n, sites = byk[dom]
        achieved = nbytes / (ms * 1e-3) / 1e9
        tr = (traffic or {}).get("by_kernel", {}).get(dom)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # GB per launch leaving L2 for the Infinity Cache / HBM (PMC, calibrated)
                "traffic": round(tr["bytes_per_launch"] / 1e9, 4) if tr else None,
                "kernel": f"{dom} (call sites {' + '.join(sorted(sites))}), avg {1e3 * ms / n:.1f} us/launch over "
                          f"{n} launches, {nbytes / n / 1e9:.3f} GB algorithmic per launch"}
        if tr:
            roof["traffic_detail"] = dict(tr, read_correction=traffic["read_correction"],
                                          write_correction=traffic["write_correction"],
                                          all_kernels={k: round(v["bytes_per_launch"] / 1e9, 4)
                                                       for k, v in traffic["by_kernel"].items()})
        tot_ms = sum(v[0] for v in site.values())
        tot_b = sum(v[1] for v in site.values())
        roof["all_spmm_GBps"] = round(tot_b / (tot_ms * 1e-3) / 1e9, 1)
        roof["spmm_ms_per_step"] = round(tot_ms / args.steps, 3)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, host_batches[0], feats, num_classes)

    if rank == 0:
        value = world * args.steps / elapsed
        line = {
            "metric": "mini-batches/sec + SpMM HBM GB/s, Reddit GraphSAGE/LADIES at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "mini-batches/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "host_issue_ms_per_step": round(1e3 * (t_issued - t_start) / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (Chung-Lu {spec.name}-shaped graph, N(0,1) features, random-init "
                    f"{'GraphSAGE' if args.model == 'graphsage' else 'GCN'}); "
                    f"{nb} pre-sampled {args.sampler} batches per rank cycled, operands resident in HBM",
            "config": {"workload": (f"{GRAPH_NAMES[args.graph]} {'GraphSAGE' if args.model == 'graphsage' else 'GCN'} "
                                    f"{args.sampler.upper() if args.sampler != 'fastgcn' else 'FastGCN'} "
                                    f"samp_num={args.samp_num} batch_size={args.batch_size}"
                                    + (" (BASELINE config 2)" if (args.model, args.sampler, args.samp_num,
                                                                  args.batch_size) == ("graphsage", "ladies", 8192, 512)
                                       and args.graph == "reddit" else "")),
                       "sampler": args.sampler,
                       "model": args.model, "global_batch": args.batch_size * world, "samp_num": args.samp_num,
                       "nhid": args.nhid, "feat_dim": int(store.F), "num_nodes": int(N), "graph_nnz": int(A.nnz),
                       "buffer_size": args.buffer_size, "parallelism": f"dp{world}",
                       "nnz_per_batch": int(host_batches[0].nnz()),
                       "fused_epilogue": not args.unfused},
            "roofline": roof,
            "cpu_baseline": cpu,
            "spmm_per_callsite": spmm_detail,
            "end_to_end": e2e,
            "feature_staging": staging_info,
            "final_loss": round(final_loss, 5),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
