"""Benchmark: Reddit GraphSAGE / LADIES mini-batch training on MI355X (BASELINE.json config 2).

Headline `value` = END-TO-END mini-batches/s, as the reference's training loop runs
(main.py:115-170): every timed step takes a batch LIVE from the sampler pool (the native
LADIES sampler + the host gather of the non-buffered feature rows, in C++ worker threads; the
reference's prepare_data thread pool, sampler.py:163-193), stages it (one native call: the
batch blob's H2D on a side stream, X0 from the own-GPU buffer and the host rows, the lower
layers extracted on the GPU, the operands; peer rows read from the peers' mapped buffers when
N > 1), and runs 3 HIP aggregation forwards + 2 backwards inside GraphSAGE (samp_num 8192,
batch 512, nhid 512, orders 1,1,1, F = 602, 41 classes), loss, backward, clip_grad_norm_(5),
RCCL all-reduce(SUM) of the flat gradient, Adam. The warm-up drains the sampler's prefetch
queue first, so the timed steps run in steady state (nothing pre-sampled is consumed inside
the timed region).

Second figure `gpu_step`: the same step over DISTINCT pre-sampled batches (one per timed
step, none cycled), each blob uploaded afresh inside the timed region — the GPU side without
the producers. The SpMM roofline comes from that batch set (HIP events on the launch stream
around every aggregation, PMC counters in child processes). The line also carries where the
host's time went (`host_cpu_e2e`, `host_phases_ms_per_step_e2e`), the drop-in boundary per call
(`dropin`) and the split3-vs-exact-f32 GEMM A/B (`gemm_ab`); DESIGN.md §5.

Synthetic Reddit-shaped graph: Chung-Lu lognormal sigma 1.3, N = 232,965,
~23.1 M nnz, N(0,1) fp32 features (StandardScaler'd analogue), buffer_size = 0.1.
`--cpu`: BASELINE config 1 (samp 512, batch 128, one process on the CPU through the product's
torch.sparse.mm device branch).

Run: python bench.py [--gpus N --steps K --warmup W]. For N > 1 the command starts its own N rank
processes (gnn_amd.launch, before any GPU call; as the reference's one `python main.py` starts a
trainer per device, main.py:289-297) unless a launcher (torch.distributed.run) already set
WORLD_SIZE. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from gnn_amd import custom_sparse_ops as cso  # noqa: E402
from gnn_amd import graphs, launch, placement, sampler, staging  # noqa: E402
from gnn_amd.models import build_model  # noqa: E402
from gnn_amd.train import Trainer, init_distributed  # noqa: E402

METRIC = "mini-batches/sec + SpMM HBM GB/s, Reddit GraphSAGE/LADIES at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
# Row gathers served by an XCD's L2 (MI355X_MICROARCH.md §Indexed rows: 66-73 GB/s per CU,
# 16.8-18.8 TB/s chip-wide): the ceiling of a gather whose table is re-read from cache.
L2_GATHER_PEAK_GBS = 18800.0


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


GRAPH_NAMES = {"reddit": "Reddit", "products": "ogbn-products", "papers": "ogbn-papers100M-scaled", "tiny": "tiny"}
SAMPLERS = {"ladies": sampler.ladies_sample_host, "subgraph": sampler.subgraph_sample_host,
            "fastgcn": sampler.fastgcn_sample_host}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--gpu-step-batches", type=int, default=60,
                    help="distinct pre-sampled batches timed for the gpu_step field (at most --steps)")
    ap.add_argument("--model", default="graphsage", choices=["graphsage", "gcn"])
    ap.add_argument("--sampler", default="ladies", choices=["ladies", "subgraph", "fastgcn"])
    ap.add_argument("--samp-num", type=int, default=None, help="default 8192 (512 with --cpu)")
    ap.add_argument("--batch-size", type=int, default=None, help="default 512 (128 with --cpu)")
    ap.add_argument("--nhid", type=int, default=512)
    ap.add_argument("--buffer-size", type=float, default=0.1)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--graph", default="reddit", choices=["reddit", "products", "papers", "tiny"],
                    help="synthetic graph shape: reddit (configs 1-2), products (configs 3, 5), papers "
                         "(config 4's per-batch geometry on a graph scaled to the box), tiny (smoke)")
    ap.add_argument("--cpu", action="store_true", help="BASELINE config 1: one process on the CPU (no GPU)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic child runs")
    ap.add_argument("--no-site-trace", action="store_true",
                    help="skip the rocprofv3 kernel-trace child run that times the small aggregation call sites")
    ap.add_argument("--no-gpu-step", action="store_true", help="skip the distinct-batch GPU-step run")
    ap.add_argument("--unfused", action="store_true", help="torch elementwise layer tail instead of the HIP one")
    ap.add_argument("--workers", type=int, default=0, help="sampler threads per rank (0: auto)")
    ap.add_argument("--compute-priority", default="high", choices=["high", "normal"],
                    help="priority of the stream the training step runs on (the staging stream stays normal)")
    ap.add_argument("--staging", default="copy", choices=["copy", "zerocopy"],
                    help="non-buffered feature rows: host gather into pinned memory + one hipMemcpyAsync "
                         "(copy), or the GPU reads the mapped host table over PCIe (zerocopy: measured "
                         "slower, it slows the concurrent compute kernels)")
    ap.add_argument("--extract-layers", default="all",
                    help="LADIES: bottom-up layers (below the top one) whose sub-graph the GPU extracts "
                         "(gnn_ladies_extract_f32) instead of the sampler threads: comma list, 'all' or 'none'")
    ap.add_argument("--host-extract", action="store_true", help="= --extract-layers none")
    ap.add_argument("--column-counts", default="auto", choices=["auto", "host", "gpu", "mixed"],
                    help="LADIES draw: U's column counts summed by the sampler threads (host), on the GPU "
                         "(gnn_colcount_*, the graph resident in HBM), or mixed (half the sampler threads on "
                         "the GPU, on hardware queues of their own, the rest on the host); the draw itself "
                         "stays on the host. auto: mixed from 1 M nodes, host below (profiles/round6/"
                         "mixed_counts/; Reddit-shaped: the host draw is not the bound)")
    ap.add_argument("--peer-rows", default=os.environ.get("GNN_PEER_ROWS", "direct"), choices=["alltoall", "direct"],
                    help="N > 1: peer feature rows read directly from the peers' buffers over xGMI (IPC-mapped "
                         "once; default, falls back to alltoall if any rank cannot map) or by an RCCL all-to-all "
                         "per batch after a host negotiation; every N > 1 run also times the other form")
    ap.add_argument("--stage-ahead", type=int, default=int(os.environ.get("GNN_STAGE_AHEAD", "1")),
                    help="batches whose X0 staging / device side are issued ahead of the current step")
    ap.add_argument("--stage-gate", type=int,
                    default=int(os.environ["GNN_STAGE_GATE"]) if "GNN_STAGE_GATE" in os.environ else None,
                    help="the next batches' X0 gathers and layer extractions wait for this layer's forward "
                         "aggregation of the current step (an event the executor records; -1: no gate). "
                         "Default: 1 for graphs under 1 M nodes (Reddit: +2.4 %% end to end), none above "
                         "(the products-shaped staging needs the whole step: 475.5 vs 441.1 without / with, "
                         "profiles/round5/configs/)")
    ap.add_argument("--numa", default="off", choices=["gpu", "off"],
                    help="confine the process (training + producer threads) to the CPUs of the GPU's NUMA node "
                         "(A/B on one box, 3 runs each: 572 vs 584 mini-batches/s unpinned, so off by default)")
    ap.add_argument("--python-loader", action="store_true",
                    help="batch producer: Python worker threads calling the native sampler (BatchLoader) instead of "
                         "the C++ producer (NativeLoader: GIL-free workers, one blob and one H2D per batch)")
    ap.add_argument("--locality-sampling", action="store_true",
                    help="the reference's --locality_sampling (main.py:284-287): per-layer skewed node sets from the "
                         "placement (preprocess.py:414-423) handed to the sampler; at the reference's scale_factor "
                         "1.0 (main.py:256) they leave the draw unchanged (sampler.py:119-121)")
    ap.add_argument("--scale-factor", type=float, default=1.0,
                    help="sampler.py:119-121's boost of the skewed nodes' probability (the reference fixes 1.0); "
                         "> 1 takes the numpy restatement in Python producer threads")
    ap.add_argument("--cprofile", default="", help="after the timed runs, cProfile 20 GPU steps into this file")
    ap.add_argument("--dump-batch", default="", help="save rank-0 batch 0 operands (.npz) for kernel profiling")
    a = ap.parse_args()
    if a.samp_num is None:
        a.samp_num = 512 if a.cpu else 8192
    if a.batch_size is None:
        a.batch_size = 128 if a.cpu else 512
    return a


# ----------------------------------------------------------------------------- PMC traffic
def _counter_rows(d):
    import csv
    import glob

    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def _kernel_symbol(name: str) -> str:
    """'void (anonymous namespace)::spmm_unit_kernel<4, 16, 1, 4, false>(int const*, ...)' ->
    'spmm_unit_kernel<4, 16, 1, 4, false>' (the form the bench's timing records use)."""
    if name.startswith("void "):
        name = name[5:]
    if name.startswith("(anonymous namespace)::"):
        name = name[len("(anonymous namespace)::"):]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i].strip()
    return name.strip()


def _dump_batch(hb, path):
    np.savez(path, **{f"l{i}_{k}": getattr(L, k) for i, L in enumerate(hb.layers)
                      for k in ("fullrowptr", "rowptr", "colidx", "normfact")},
             **{f"l{i}_shape": np.array(L.shape) for i, L in enumerate(hb.layers)})


def pmc_traffic(hb, F, hidden, workdir="/tmp/gnn_bench_pmc"):
    """Per-launch bytes leaving L2 (toward the Infinity Cache / HBM) and the L2 hit rate of
    each aggregation kernel instantiation, from rocprofv3 PMC counters in three passes
    (FETCH_SIZE; WRITE_SIZE; TCC_HIT_sum + TCC_MISS_sum) over scripts/pmc_probe.py: batch 0's
    forward calls laid out as the benchmark runs them. FETCH_SIZE / WRITE_SIZE are corrected
    by a calibration launch of the SAME kernel instantiation (4 rows x 256 B per wave
    instruction) over an operand whose every X row is gathered once from a 2.4 GB table, so
    its bytes are known (MI355X_MICROARCH.md §HBM: calibrate in your own access pattern).
    Runs the probe as CHILD processes before this process has touched the GPU."""
    import shutil
    import subprocess

    if shutil.which("rocprofv3") is None:
        return None
    os.makedirs(workdir, exist_ok=True)
    npz = os.path.join(workdir, "batch0.npz")
    _dump_batch(hb, npz)
    probe = os.path.join(REPO, "scripts", "pmc_probe.py")
    calib, kern, info, dur = {}, {}, None, {}
    for counters in (["FETCH_SIZE"], ["WRITE_SIZE"], ["TCC_HIT_sum", "TCC_MISS_sum"]):
        d = os.path.join(workdir, counters[0])
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "p", "--",
               sys.executable, probe, npz, "--feat", str(F), "--hidden", str(hidden)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            log(f"pmc pass {counters} failed rc={r.returncode}: {r.stderr[-500:]}")
            return None
        for line in r.stdout.splitlines():
            if line.startswith("PMCPROBE "):
                info = json.loads(line[len("PMCPROBE "):])
        rows = sorted(_counter_rows(d), key=lambda row: int(row.get("Dispatch_Id", 0)))
        first_build = min((int(row["Dispatch_Id"]) for row in rows if "build_operand" in row.get("Kernel_Name", "")),
                          default=None)
        for row in rows:
            name, cn = row.get("Kernel_Name", ""), row.get("Counter_Name")
            if "spmm_unit_kernel" not in name or cn not in counters:
                continue
            v = float(row.get("Counter_Value", "nan"))
            if first_build is not None and int(row["Dispatch_Id"]) < first_build:
                calib.setdefault(cn, []).append(v)  # the calibration launches come first
            else:
                kern.setdefault(_kernel_symbol(name), {}).setdefault(cn, []).append(v)
                if counters[0] == "FETCH_SIZE" and row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    # the same dispatches' durations in this isolated run (ns)
                    dur.setdefault(_kernel_symbol(name), {})[row["Dispatch_Id"]] = (
                        int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    if info is None or "FETCH_SIZE" not in calib or "WRITE_SIZE" not in calib:
        return None
    read_corr = info["calib_known_read_bytes"] / (float(np.median(calib["FETCH_SIZE"])) * 1024.0)
    write_corr = info["calib_known_write_bytes"] / (float(np.median(calib["WRITE_SIZE"])) * 1024.0)
    by = {}
    for sym, c in kern.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        rd = float(np.mean(c["FETCH_SIZE"])) * 1024.0 * read_corr
        wr = float(np.mean(c["WRITE_SIZE"])) * 1024.0 * write_corr
        e = {"bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr, "launches": len(c["FETCH_SIZE"])}
        if dur.get(sym):
            e["probe_avg_us"] = float(np.mean(list(dur[sym].values()))) / 1e3
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = float(np.sum(c["TCC_HIT_sum"])), float(np.sum(c["TCC_MISS_sum"]))
            e["l2_hit_rate"] = round(h / (h + m), 4) if h + m > 0 else None
        by[sym] = e
    out = {"by_kernel": by, "read_correction": round(read_corr, 4), "write_correction": round(write_corr, 4),
           "calibration": {k: info[k] for k in ("calib_known_read_bytes", "calib_known_write_bytes", "calib_tiles")}}
    if "TCC_HIT_sum" in calib and "TCC_MISS_sum" in calib:
        h, m = float(np.sum(calib["TCC_HIT_sum"])), float(np.sum(calib["TCC_MISS_sum"]))
        out["calibration"]["l2_hit_rate"] = round(h / (h + m), 4) if h + m > 0 else None
    return out


def site_trace(workdir="/tmp/gnn_bench_sites", steps=30):
    """Per call site, the aggregation kernels' durations as rocprofv3 --kernel-trace times them in
    the step: a CHILD run of this benchmark (same workload flags, the end-to-end pass only, `steps`
    timed steps) under the tracer, its dispatches cut into steps at adam_kernel and the aggregation
    main kernels of each step named in call order (fwd_L0, fwd_L1, fwd_L2[, bwd_L2], bwd_L1). The
    in-process timings of small sites read high (fwd_L2 30.7 us by event pair vs 16.7
    by rocprofv3), so sites under 50 us report this figure. Runs before this process touches the GPU."""
    import csv
    import glob
    import shutil
    import subprocess

    if shutil.which("rocprofv3") is None:
        return None
    shutil.rmtree(workdir, ignore_errors=True)
    cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", workdir, "-o", "t", "--",
           sys.executable, os.path.abspath(__file__), *sys.argv[1:], "--steps", str(steps), "--warmup", "3",
           "--no-cpu-baseline", "--no-traffic", "--no-gpu-step", "--no-site-trace"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
    if r.returncode != 0:
        log(f"site trace failed rc={r.returncode}: {r.stderr[-500:]}")
        return None
    rows = []
    for f in glob.glob(os.path.join(workdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return sites_from_trace(rows, steps)


def sites_from_trace(rows, steps):
    """rocprofv3 kernel-trace rows -> {call site: rocprof_avg_us, launches, kernel} over the last
    `steps` steps (site_trace)."""
    rows = sorted(rows, key=lambda row: int(row["Start_Timestamp"]))
    per_step, cur = [], []
    for row in rows:
        name = row["Kernel_Name"]
        if "spmm_unit_kernel" in name or "spmm_row_kernel" in name:
            cur.append((_kernel_symbol(name), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3))
        elif "adam_kernel" in name:
            per_step.append(cur)
            cur = []
    per_step = per_step[-steps:]
    names = {4: ["fwd_L0", "fwd_L1", "fwd_L2", "bwd_L1"], 5: ["fwd_L0", "fwd_L1", "fwd_L2", "bwd_L2", "bwd_L1"]}
    out = {}
    for st in per_step:
        for site, (kn, us) in zip(names.get(len(st), []), st):
            e = out.setdefault(site, {"kernel": kn, "us": []})
            e["us"].append(us)
    return {k: {"rocprof_avg_us": round(float(np.mean(v["us"])), 2), "launches": len(v["us"]), "kernel": v["kernel"]}
            for k, v in out.items()}


# ----------------------------------------------------------------------------- CPU legs
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


def dropin_timing(hb, feats, dev, H, reps=20):
    """The drop-in boundary timed per call: the reference's own SparseDenseMM
    pattern (custom_sparse_ops.py:16-37) through the `spmm` extension module — forward
    spmm_load_balance(A, X) on a create_coo_tensor operand (spmm.cpp:23-27, 44-50), backward
    spmm_load_balance(A.transpose(0,1).coalesce(), G) with ATen's transpose + coalesce — beside the
    native call on the same operands (gnn_amd.custom_sparse_ops.spmm_csr on the CSR the builder
    made, and on its GPU-built canonical transpose). Config-2 layer-0 forward and layer-1 backward
    shapes; dense operands contiguous as the reference requires. Wall time per call over `reps`
    calls ended by one synchronize (the drop-in backward's coalesce synchronises by itself: ATen
    needs the unique count on the host), after one untimed call."""
    from gnn_amd import custom_sparse_ops as cso
    from gnn_amd import torch_ops

    ext = torch_ops.load()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    def per_call(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return round(1e6 * (time.perf_counter() - t0) / reps, 1)

    out = {}
    for li, site in ((0, "fwd_L0"), (1, "bwd_L1")):
        L = hb.layers[li]
        M, K = L.shape
        ins = (t(L.fullrowptr), t(L.rowptr), t(L.colidx), t(L.normfact))
        A = ext.create_coo_tensor(*ins, M, K)
        op, _ = cso.build_operand(*ins, M, K, with_coo=False)
        if li == 0:
            X = feats[torch.from_numpy(np.asarray(hb.input_nodes, np.int64))].contiguous().to(dev)
            d_us = per_call(lambda: ext.spmm_load_balance(A, X))
            n_us = per_call(lambda: cso.spmm_csr(op, X))
            foreign = torch.sparse_coo_tensor(A._indices(), A._values(), A.shape, is_coalesced=True)
            extra = {"dropin_foreign_coo_us": per_call(lambda: ext.spmm_load_balance(foreign, X)),
                     "what": "spmm_load_balance(A, X) with A from spmm.create_coo_tensor (the CSR the builder made "
                             "is kept on the tensor: no COO->CSR in the call); dropin_foreign_coo_us: the same "
                             "operand as a plain torch COO tensor, converted COO->CSR on the GPU every call"}
        else:
            G = torch.randn(M, H, device=dev)
            opt = op.transpose()  # built on the GPU once, kept on the operand
            d_us = per_call(lambda: ext.spmm_load_balance(A.transpose(0, 1).coalesce(), G))
            n_us = per_call(lambda: cso.spmm_csr(opt, G))
            c_us = per_call(lambda: A.transpose(0, 1).coalesce())
            extra = {"aten_transpose_coalesce_us": c_us,
                     "what": "spmm_load_balance(A.transpose(0,1).coalesce(), G): ATen's transpose + coalesce "
                             "(a sort, and a host sync for its unique count) every call, COO->CSR of the new "
                             "tensor, the aggregation; native: the canonical transpose built once on the GPU"}
        out[site] = {"dropin_us": d_us, "native_us": n_us, "overhead": round(d_us / n_us - 1.0, 4) if n_us else None,
                     "M": int(M), "K": int(K), "nnz": int(L.colidx.size), "F": int(X.shape[1] if li == 0 else H),
                     **extra}
    return out


def gpu_numa_cpus(dev) -> list:
    """The host CPUs of the GPU's NUMA node (sysfs; [] if unknown): the producer threads' blobs
    and the training thread's launches then stay on the socket the GPU hangs off."""
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
        if node < 0:
            return []
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
        cpus = []
        for part in spec.split(","):
            a, _, b = part.partition("-")
            cpus.extend(range(int(a), int(b or a) + 1))
        allowed = os.sched_getaffinity(0)
        return [c for c in cpus if c in allowed]
    except (OSError, ValueError, AttributeError):
        return []


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


def host_counters() -> dict:
    """CPU-time counters of this process and of its cgroup (cgroup v2 cpu.stat: usage and the
    CFS quota's throttling), read around a timed window."""
    c = {"wall": time.perf_counter(), "proc_cpu": time.process_time(), "thread_cpu": time.thread_time()}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    c["cg_" + k] = int(v)
    except (OSError, ValueError):
        pass
    return c


def host_delta(a: dict, b: dict) -> dict:
    return {k: b[k] - a[k] for k in a if k in b}


def host_report(d: dict, steps: int, workers: int) -> dict:
    """Where the host's CPU went over a timed window, per step: the training thread, the rest of
    the process (sampler / producer threads, HIP runtime threads), the whole cgroup, and whether the
    cgroup's CPU quota throttled it (nr_throttled > 0: every thread stalled for the rest of a period)."""
    if not d:
        return None
    ms = lambda s: round(1e3 * s / max(steps, 1), 3)
    out = {"trainer_thread_cpu_ms_per_step": ms(d["thread_cpu"]),
           "other_threads_cpu_ms_per_step": ms(d["proc_cpu"] - d["thread_cpu"]),
           "process_cpus_busy": round((d["proc_cpu"]) / d["wall"], 2) if d["wall"] > 0 else None,
           "cpu_budget": cpu_budget(), "sampler_workers": workers}
    if "cg_usage_usec" in d:
        out["cgroup"] = {"cpus_busy": round(d["cg_usage_usec"] * 1e-6 / d["wall"], 2) if d["wall"] > 0 else None,
                         "periods": d.get("cg_nr_periods"), "throttled_periods": d.get("cg_nr_throttled"),
                         "throttled_ms": round(d.get("cg_throttled_usec", 0) * 1e-3, 3)}
    out["what"] = ("CPU time over the timed window: the training thread (its waits for the GPU poll and "
                   "sleep: staging.wait_event), the process's other threads (the sampler producers and HIP's own "
                   "threads), and the cgroup's usage and CFS-quota throttling (cpu.stat)")
    return out


def default_workers(world: int) -> int:
    # sampler threads per rank: the rank's CPU share minus the training thread and one spare
    # (measured on the 16-CPU box: 14 threads 288 mini-batches/s end to end, 10 threads 227)
    return max(2, min(14, cpu_budget() // max(world, 1) - 2))


def workload_name(args, spec) -> str:
    model = "GraphSAGE" if args.model == "graphsage" else "GCN"
    smp = args.sampler.upper() if args.sampler != "fastgcn" else "FastGCN"
    w = f"{GRAPH_NAMES[args.graph]} {model} {smp} samp_num={args.samp_num} batch_size={args.batch_size}"
    if getattr(args, "locality_sampling", False):
        w += f" + locality_sampling (scale_factor {args.scale_factor:g})"
    if args.graph == "reddit" and (args.model, args.sampler) == ("graphsage", "ladies"):
        if (args.samp_num, args.batch_size) == (8192, 512) and not args.cpu:
            w += " (BASELINE config 2)"
        if (args.samp_num, args.batch_size) == (512, 128) and args.cpu:
            w += " (BASELINE config 1, CPU)"
    return w


def run_cpu(args, spec, A, lap, labels, feats, num_classes, train):
    """BASELINE config 1: one process on the CPU, the product's torch.sparse.mm device branch
    (gnn_amd.custom_sparse_ops), native LADIES sampling in the loader's worker threads."""
    from gnn_amd.loader import BatchLoader

    N = A.shape[0]
    pl = placement.create_buffer(lap, train, int(args.buffer_size * N), [0], 3, alpha=0)
    torch.manual_seed(0)
    model = build_model(args.model, feats.shape[1], args.nhid, [1, 1, 1], num_classes, 0.1)
    trainer = Trainer(model, args.lr, "cpu")
    workers = args.workers or max(1, min(4, cpu_budget() // 4))
    ld = BatchLoader(lap, labels, train, args.samp_num, args.batch_size, [1, 1, 1], pl.device_id_of_nodes_group[0],
                     pl.idx_of_nodes_on_device_group[0], workers=workers, seed=4242, kind=args.sampler)
    it = ld.forever()

    def step():
        adjs, x0, sampled, y = next(it).host.cpu_inputs(feats)
        return trainer.step(x0, adjs, sampled, y)

    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    el = time.perf_counter() - t0
    ld.close()
    line = {"metric": METRIC, "value": round(args.steps / el, 3), "unit": "mini-batches/s", "n_gpus": 0,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic (Chung-Lu {spec.name}-shaped graph, N(0,1) features, random-init model); live "
                    f"{args.sampler} sampling in {workers} worker threads",
            "config": {"workload": workload_name(args, spec), "device": "cpu", "torch_threads": torch.get_num_threads(),
                       "cpu_budget": cpu_budget(), "model": args.model, "global_batch": args.batch_size,
                       "samp_num": args.samp_num, "nhid": args.nhid, "feat_dim": int(feats.shape[1]),
                       "num_nodes": int(N), "parallelism": "none (one process)"},
            "roofline": None, "cpu_baseline": None, "final_loss": round(float(loss), 5)}
    print(json.dumps(line), flush=True)


# ----------------------------------------------------------------------------- roofline
def roofline_from(recs, step_batches, args, traffic, steps, sites=None):
    """Per call site and for the dominant aggregation kernel: algorithmic, compulsory and
    (PMC) L2-egress byte rates over the HIP-event launch durations of the distinct-batch run.
    Call sites per step, in call order: 3 forwards, then the backwards of layers 2 and 1 (the
    executor folds the layer-2 backward into the layer-1 tail when its rows are short: no record)."""
    names = ["fwd_L0", "fwd_L1", "fwd_L2", "bwd_L2", "bwd_L1"]
    site, kname = {}, {}
    uniq_cache = {}
    step_i, prev = 0, None
    for i, (tag, ms, nbytes, kn, dims) in enumerate(recs):
        if "_L" in tag:  # the executor names its call sites (a folded call site has no record)
            key = tag
            if prev is not None and names.index(key) <= names.index(prev):
                step_i += 1
            prev = key
        else:  # the autograd path: 5 calls per step in call order
            key = names[i % len(names)]
            assert key.startswith(tag), (key, tag)
            step_i = i // len(names)
        hb, db = step_batches[step_i % len(step_batches)]
        li = int(key[-1])
        L = hb.layers[li]
        ck = (id(hb), key)
        if ck not in uniq_cache:  # distinct X rows the call gathers (cols of A, or non-empty rows for Aᵀ)
            if L.on_device:  # GPU-extracted: the column counts (host) / the device row pointer
                uniq_cache[ck] = (int(np.count_nonzero(np.diff(L.csc_colptr))) if key.startswith("fwd")
                                  else int(torch.count_nonzero(torch.diff(db.adjs[li].rowptr)).item()))
            else:
                uniq_cache[ck] = (np.unique(L.colidx).size if key.startswith("fwd")
                                  else int(np.count_nonzero(np.diff(L.rowptr))))
        F, M, nnz = dims["F"], dims["M"], dims["nnz"]
        comp = uniq_cache[ck] * F * 4 + nnz * 8 + (M + 1) * 4 + M * F * 4 + dims["res_rows"] * F * 4
        if dims["res_rows"]:
            comp += M * 4
        e = site.setdefault(key, [0.0, 0, 0, 0])
        e[0] += ms
        e[1] += nbytes
        e[2] += 1
        e[3] += comp
        kname[key] = kn
    detail = {k: {"avg_us": round(1e3 * ms / n, 2), "GB_per_launch": round(nb / n / 1e9, 4),
                  "alg_GBps": round(nb / (ms * 1e-3) / 1e9, 1),
                  "compulsory_GB_per_launch": round(cb / n / 1e9, 4),
                  "compulsory_GBps": round(cb / (ms * 1e-3) / 1e9, 1), "kernel": kname[k]}
              for k, (ms, nb, n, cb) in site.items()}
    if "bwd_L2" not in detail and "bwd_L1" in detail:
        detail["bwd_L2"] = {"folded": "computed inside the layer-1 tail backward (gnn_sage_norm_bwd_agg_f32: each dY "
                                      "row as the tail reads it) - no launch of its own, so no time here and none in "
                                      "custom_sparse_ops.spmm_backward_time (the reference's main.py:196 figure)"}
    for k, v in detail.items():
        if "avg_us" not in v:
            continue
        v["timing"] = "the dispatch's own start/end timestamps (hipExtLaunchKernel events) in the timed pass"
        tr = (sites or {}).get(k)
        if tr and tr["kernel"] == v["kernel"]:
            v["rocprof_avg_us"] = tr["rocprof_avg_us"]
            if tr["rocprof_avg_us"] < 50.0:
                # small sites: the event figure reads high; report the traced kernel duration
                v["event_avg_us"] = v["avg_us"]
                v["avg_us"] = tr["rocprof_avg_us"]
                v["alg_GBps"] = round(v["GB_per_launch"] / (v["avg_us"] * 1e-6), 1)
                v["compulsory_GBps"] = round(v["compulsory_GB_per_launch"] / (v["avg_us"] * 1e-6), 1)
                v["timing"] = ("rocprofv3 --kernel-trace of a traced child run of this benchmark (sites under 50 us); "
                               "event_avg_us: the in-process dispatch timestamps")
    byk = {}
    for key, (ms_, nb_, n_, cb_) in site.items():
        e = byk.setdefault(kname[key], [0.0, 0, 0, 0, []])
        e[0] += ms_
        e[1] += nb_
        e[2] += n_
        e[3] += cb_
        e[4].append(key)
    dom = max(byk, key=lambda k_: byk[k_][0])
    ms, nbytes, n, cbytes, sites = byk[dom]
    t = ms * 1e-3 / n  # average launch duration, s
    alg = nbytes / n
    comp = cbytes / n
    tr = (traffic or {}).get("by_kernel", {}).get(dom)
    roof = {"bound": "hbm"}
    if tr:
        # the bytes that left L2 for the Infinity Cache / HBM (calibrated PMC), per launch, over the
        # duration of the SAME dispatches in the same isolated probe run (bytes and time measured
        # under one condition); the live in-step duration is avg_us below
        egress = tr["bytes_per_launch"]
        tp = tr.get("probe_avg_us", 1e6 * t) * 1e-6
        roof.update({"achieved": round(egress / tp / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(egress / tp / 1e9 / HBM_PEAK_GBS, 4), "traffic": round(egress / 1e9, 4),
                     "probe_avg_us": round(1e6 * tp, 2),
                     "basis": "PMC L2-egress bytes per launch (FETCH_SIZE + WRITE_SIZE, calibrated) / the duration "
                              "of the same dispatches in the isolated PMC probe run"})
    else:
        roof.update({"achieved": round(comp / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(comp / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                     "basis": "compulsory bytes per launch / HIP-event launch duration (no PMC pass in this run)"})
    roof.update({
        "kernel": f"{dom} (call sites {' + '.join(sorted(sites))}), avg {1e6 * t:.1f} us/launch over {n} launches",
        "avg_us": round(1e6 * t, 2),
        "compulsory": {"GB_per_launch": round(comp / 1e9, 4), "GBps": round(comp / t / 1e9, 1),
                       "frac_of_hbm_peak": round(comp / t / 1e9 / HBM_PEAK_GBS, 4),
                       "what": "distinct X rows gathered x F x 4 + (col, val) + rowptr + Y (+ residual rows)"},
        "algorithmic": {"GB_per_launch": round(alg / 1e9, 4), "GBps": round(alg / t / 1e9, 1),
                        "what": "SURVEY.md §8(d): every gathered X row counted (re-reads served by L2 / Infinity "
                                "Cache), no fraction: it is not an HBM quantity"},
        # the same launches against the three bases side by side (frac above: PMC L2-egress / HBM peak)
        "frac_alg_8d": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
        "frac_alg_8d_what": "SURVEY.md §8(d) algorithmic bytes (every gathered X row, L2 hits included) / "
                            "launch duration / 8 TB/s HBM peak: above 1 because re-reads are served by L2",
        "l2_gather": {"ceiling_GBps": L2_GATHER_PEAK_GBS, "frac": round(alg / t / 1e9 / L2_GATHER_PEAK_GBS, 4),
                      "what": "algorithmic gather rate / the L2-served row-gather rate of MI355X_MICROARCH.md "
                              "§Indexed rows (18.8 TB/s chip-wide)"},
    })
    if tr:
        roof["l2_hit_rate"] = tr.get("l2_hit_rate")
        roof["egress_over_compulsory"] = round(tr["bytes_per_launch"] / comp, 2)
        roof["pmc"] = {"read_correction": traffic["read_correction"], "write_correction": traffic["write_correction"],
                       "calibration": traffic["calibration"],
                       "all_kernels_GB_per_launch": {k: round(v["bytes_per_launch"] / 1e9, 4)
                                                     for k, v in traffic["by_kernel"].items()},
                       "all_kernels_l2_hit_rate": {k: v.get("l2_hit_rate") for k, v in traffic["by_kernel"].items()}}
    tot_ms = sum(v[0] for v in site.values())
    tot_b = sum(v[1] for v in site.values())
    roof["all_spmm_alg_GBps"] = round(tot_b / (tot_ms * 1e-3) / 1e9, 1)
    roof["spmm_ms_per_step"] = round(tot_ms / steps, 3)
    return roof, detail


def gather_ceiling(op, kernel_name, dev, reps=20, K=4096):
    """The dominant aggregation kernel's own access shape over a CACHE-RESIDENT table: the same
    instantiation (VW, G, NJ forced), the same row lengths (the operand's rowptr), F = 602 in
    608-float rows, columns uniform over K = 4096 rows (a 1 MB slice per XCD: every gather an
    L2 / L1 hit). Its algorithmic rate is the ceiling of the access pattern itself — 4 rows x
    256 B per wave instruction — on this chip, measured live (HIP events, median of reps)."""
    import re

    m = re.match(r"spmm_unit_kernel<(\d+), (\d+), (\d+)", kernel_name)
    if m is None:
        return None
    g, nj = int(m.group(2)), int(m.group(3))
    M, nnz = op.shape[0], op.nnz
    gen = torch.Generator(device=dev).manual_seed(1)
    rows = torch.repeat_interleave(torch.arange(M, device=dev), torch.diff(op.rowptr))
    col = torch.randint(0, K, (nnz,), device=dev, generator=gen, dtype=torch.int64)
    col = (torch.sort(rows * K + col).values - rows * K).to(torch.int32)  # ascending per row
    syn = cso.CsrOperand(op.rowptr, col, torch.rand(nnz, device=dev, generator=gen), (M, K))
    X = torch.randn(K, 608, device=dev, generator=gen)[:, :602]
    saved = {k: os.environ.get(k) for k in ("GNN_SPMM_G", "GNN_SPMM_NJ")}
    os.environ["GNN_SPMM_G"], os.environ["GNN_SPMM_NJ"] = str(g), str(nj)
    try:
        cso.spmm_csr(syn, X)
        cso.take_timing_records()
        cso.enable_timing(True)
        for _ in range(reps):
            cso.spmm_csr(syn, X)
        recs = cso.take_timing_records()
    finally:
        cso.enable_timing(False)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ms = float(np.median([r[1] for r in recs]))
    return {"GBps": round(recs[0][2] / (ms * 1e-3) / 1e9, 1), "us": round(ms * 1e3, 1), "kernel": recs[0][3],
            "what": f"same kernel instantiation and row lengths as the layer-0 operand, columns uniform over "
                    f"K = {K} rows (slice {K * 256 / 1e6:.1f} MB per XCD: cache-resident), median of {reps}"}


def access_shape_ceiling(K, kernel_name):
    """The aggregation's load stream with nothing else in it (scripts/gather_shape.hip, built by
    build()): 64/G row pieces of G x 16 B per wave instruction, 4 in flight per lane group, 32
    waves per CU, random rows of a K-row table with 608-float rows — at the dominant operand's
    own K (the same slice per XCD) and cache-resident (K = 4096). A child process, run after the
    timed passes; None if the probe is not built."""
    import re
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scripts", "bin", "gather_shape")
    m = re.match(r"spmm_unit_kernel<(\d+), (\d+), (\d+), (\d+)", kernel_name)
    if m is None or not os.path.exists(exe):
        return None
    g, u = m.group(2), m.group(4)
    out = {}
    for tag, k in (("at_operand_K", int(K)), ("cache_resident", 4096)):
        # long launches (1,024 row pieces per wave): the short default under-reads by the launch overhead
        r = subprocess.run([exe, str(k), g, u], capture_output=True, text=True, timeout=120, check=True,
                           env=dict(os.environ, PER_WAVE="1024"))
        out[tag] = json.loads(r.stdout.strip().splitlines()[-1])
    out["what"] = ("scripts/gather_shape.hip: the dominant kernel's load stream alone (row pieces of G x 16 B, "
                   "U in flight per lane group, 32 waves per CU, random rows, 1,024 pieces per wave), median of "
                   "20 launches")
    return out


# ----------------------------------------------------------------------------- main
def main():
    args = parse()
    if not args.cpu and launch.needs_launch(args.gpus):
        # one command starts every rank (no external torchrun needed); nothing above touched the GPU
        sys.exit(launch.relaunch_self(args.gpus))
    held = {}
    try:
        _main(args, held)
    except BaseException:
        # a failing rank unmaps its peers' buffers (after a device sync) without the collective
        # close(): the peers may never reach its barrier (the launcher stops them instead)
        if held.get("direct") is not None:
            held["direct"].close_local()
        raise


def _main(args, held):
    spec = {"reddit": graphs.REDDIT, "products": graphs.PRODUCTS, "papers": graphs.PAPERS_SCALED,
            "tiny": graphs.TINY}[args.graph]
    t0 = time.time()
    A, labels, feats, num_classes, train, valid, test = graphs.make_dataset(spec, seed=0)
    lap = graphs.lap_matrix(A, args.model)
    N = A.shape[0]
    log(f"graph {spec.name}: N={N} nnz={A.nnz} ({time.time() - t0:.1f}s)")
    if args.cpu:
        return run_cpu(args, spec, A, lap, labels, feats, num_classes, train)

    rank, world, local = init_distributed()
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    dev = torch.device("cuda", local)
    numa_cpus = gpu_numa_cpus(dev) if args.numa == "gpu" else []
    if len(numa_cpus) >= 4:
        os.sched_setaffinity(0, numa_cpus)  # before any worker thread exists: they inherit it
        log(f"pinned to the GPU's NUMA node: {len(numa_cpus)} CPUs")
    k = int(args.buffer_size * N)
    pl = placement.create_buffer(lap, train, k, list(range(world)), 3, alpha=0)
    pdev, pidx = pl.device_id_of_nodes_group[rank], pl.idx_of_nodes_on_device_group[rank]
    log(f"placement k={k} per GPU ({time.time() - t0:.1f}s)")
    samp = np.array([args.samp_num] * 5)
    fn = SAMPLERS[args.sampler]
    skewed = None
    if args.locality_sampling:  # main.py:284-287: on graph_data[0] + I, every rank's buffer
        import scipy.sparse as sp

        skewed = placement.get_skewed_sampled_nodes(A + sp.eye(N, dtype=A.dtype, format="csr"), pl.gpu_buffer_group,
                                                    [1, 1, 1])
        log(f"locality sampling: skewed node sets {[len(s) for s in skewed]} ({time.time() - t0:.1f}s)")
    if args.scale_factor > 1 and not args.python_loader:
        log("scale_factor > 1: the numpy restatement in Python producer threads (--python-loader)")
        args.python_loader = True
    probe_batch = fn(99, sampler.rank_batches(train, args.batch_size, rank, world, 0)[0], samp, N, lap, labels,
                     [1, 1, 1], pdev, pidx, skewed, args.scale_factor, list(range(world)))
    traffic = None
    if rank == 0 and world == 1 and not args.no_traffic and not args.no_roofline:
        # before this process initialises the GPU: the probes are child processes
        try:
            traffic = pmc_traffic(probe_batch, feats.shape[1], 2 * args.nhid if args.model == "graphsage" else args.nhid)
        except Exception as e:  # profiler trouble must not sink the benchmark
            log(f"pmc traffic measurement skipped: {e!r}")
        log(f"pmc traffic done ({time.time() - t0:.1f}s): {traffic}")
    sites = None
    if rank == 0 and world == 1 and not args.no_site_trace and not args.no_roofline and not args.no_gpu_step:
        try:
            sites = site_trace()
        except Exception as e:  # profiler trouble must not sink the benchmark
            log(f"site trace skipped: {e!r}")
        log(f"site trace done ({time.time() - t0:.1f}s): {sites}")
    if args.dump_batch and rank == 0:
        _dump_batch(probe_batch, args.dump_batch)
    torch.cuda.set_device(dev)

    store = staging.FeatureStore(feats, pl.gpu_buffer_group[rank], dev, rank, zero_copy=args.staging == "zerocopy")
    exchange = direct = alltoall = None
    peer_info = None
    if world > 1:
        alltoall = staging.PeerExchange()
        requested, direct_err = args.peer_rows, None
        if args.peer_rows == "direct" or os.environ.get("GNN_BENCH_PEER_AB", "1") == "1":
            try:  # collective; every rank gets the same outcome
                direct = staging.PeerDirect(store, feats=feats, buffer_nodes=pl.gpu_buffer_group)
            except RuntimeError as e:
                direct_err = str(e)
                log(f"{e} -> peer rows by all-to-all")
        held["direct"] = direct
        if args.peer_rows == "direct" and direct is None:
            args.peer_rows = "alltoall"
        exchange = direct if args.peer_rows == "direct" else alltoall
        peer_info = {"requested": requested, "used": args.peer_rows, "direct_mapped": direct is not None,
                     "direct_verified_rows": direct.verified_rows if direct is not None else 0,
                     "direct_error": direct_err[:400] if direct_err else None,
                     "what": "peer-row form of the reported passes after PeerDirect's all-or-nothing set-up "
                             "(direct_verified_rows: rows read through this rank's IPC mappings of the peers' "
                             "buffers and found bit-equal to the feature table before the first batch)"}
    stager = staging.Stager(store, exchange)
    torch.manual_seed(0)
    # dropout 0.1 as the reference (main.py:92-96); GNN_BENCH_DROPOUT only for cost measurements
    dropout = float(os.environ.get("GNN_BENCH_DROPOUT", "0.1"))
    model = build_model(args.model, store.F, args.nhid, [1, 1, 1], num_classes, dropout, fused=not args.unfused).to(dev)
    trainer = Trainer(model, args.lr, dev)
    if args.stage_gate is None:
        args.stage_gate = 1 if N < 1_000_000 else -1
    if args.stage_gate >= 0:
        gate = torch.cuda.Event()
        trainer.stage_gate = (gate, args.stage_gate)
        stager.gate = gate
    torch.cuda.synchronize()
    log(f"setup done ({time.time() - t0:.1f}s); params={trainer.num_params}")
    retire = staging.Retirement()

    # The step runs on a high-priority stream: the staging stream's gathers and operand builds
    # for the next batch (default priority) then fill the compute stream's gaps instead of
    # taking CU slots from the layer-0 aggregation they overlap (--compute-priority normal: off).
    lo_pri, hi_pri = torch.cuda.Stream.priority_range()
    compute_stream = torch.cuda.Stream(device=dev, priority=hi_pri) if args.compute_priority == "high" else None

    step_events = [] if os.environ.get("GNN_BENCH_STEP_EVENTS") == "1" else None
    host_trace = [] if os.environ.get("GNN_BENCH_HOST_TRACE") == "1" else None

    def pipeline(next_item, steps, carry=None):
        try:
            if compute_stream is None:
                return _pipeline(next_item, steps, carry)
            compute_stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(compute_stream):
                loss = _pipeline(next_item, steps, carry)
            torch.cuda.current_stream(dev).wait_stream(compute_stream)
            return loss
        finally:
            # N > 1: the last step of a pass may have prefetched the next batch's layer 0; the pass
            # that follows may use other batches (or none), so its workspace is not held across passes
            ex = getattr(trainer, "executor", None)
            if ex is not None:
                ex.drop_prefetch()

    def next_batch(ahead):
        """The batch after the current one, for the trainer's layer-0 prefetch during the gradient
        all-reduce (N > 1): already staged (its staging was issued a step or more ago)."""
        if not ahead:
            return None
        nb = ahead[0]
        x0n = nb.wait(retire)
        return x0n, nb.adjs, nb.batch.sampled_nodes, nb.batch.labels

    def _pipeline(next_item, steps, carry=None):
        """next_item() -> (StagePlan, batch_fn); batch_fn() makes the DeviceBatch (H2D when
        needed + the operand builds). The X0 staging and batch_fn of batches i+1 .. i+A (A =
        --stage-ahead) run on the side stream, issued before batch i's step, so they overlap
        that step's kernels; with A = 2 a batch's staging has two steps' worth of the compute
        stream's gaps to finish in (the compute kernels fill every CU, so staging kernels run
        only in their gaps), and the compute stream does not wait for it between steps.
        `carry` (a deque kept by the caller): the live stream's A staged-ahead batches persist
        from one call to the next, so a timed pass starts in the steady state the warm-up left
        (its first step's X0 already staged) and issues one staging per step like every other
        step, instead of refilling the pipeline inside the timed region (20-step windows read
        520-592 mini-batches/s that way against 600 over 300 steps)."""
        loss = None
        persistent = carry is not None
        ahead = carry if persistent else collections.deque()
        issued = 0
        if persistent:
            # one more in flight than --stage-ahead: the next staging is issued after the step
            # below, so batch i + A + 1's staging gets step i + 1's duration, as batch i + A's got
            # step i's when it was issued before the step
            while len(ahead) < max(1, args.stage_ahead) + 1:
                ahead.append(stager.issue(*next_item()))
        while not persistent and issued < min(max(1, args.stage_ahead) + 1, steps):
            ahead.append(stager.issue(*next_item()))
            issued += 1
        ph = host_phases
        for i in range(steps):
            t0_ = time.perf_counter()
            staged = ahead.popleft()
            x0 = staged.wait(retire)
            db = staged.batch
            t1_ = time.perf_counter()
            if step_events is not None:  # diagnostics (GNN_BENCH_STEP_EVENTS=1): per-step GPU spans
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                step_events.append(ev)
            loss = trainer.step(x0, staged.adjs, db.sampled_nodes, db.labels,
                                prefetch=(lambda: next_batch(ahead)) if world > 1 else None)
            t2_ = time.perf_counter()
            retire.retire(staged)  # held until the step has run (no per-tensor record_stream)
            t3_ = time.perf_counter()
            # the next batch's staging after this step's launches (its own stream: it still
            # overlaps this step, behind --stage-gate's event when set), so a timed pass's first
            # kernels start without waiting for it
            t4_ = t3_
            if persistent or issued < steps:
                item = next_item()  # the producer's next batch (blocks while it is still being sampled)
                t4_ = time.perf_counter()
                ahead.append(stager.issue(*item))
                issued += 1
            t5_ = time.perf_counter()
            ph[0] += t1_ - t0_
            ph[1] += t2_ - t1_
            ph[2] += t3_ - t2_
            ph[3] += t4_ - t3_
            ph[4] += t5_ - t4_
            if host_trace is not None:  # diagnostics (GNN_BENCH_HOST_TRACE=1): per-step phases, µs
                host_trace.append((round(1e6 * (t1_ - t0_)), round(1e6 * (t2_ - t1_)), round(1e6 * (t3_ - t2_)),
                                   round(1e6 * (t4_ - t3_)), round(1e6 * (t5_ - t4_))))
        return loss

    # 12 (was 3): interleaved on one box, the driver's 20-step form 605.8 / 604.4 with 12 against
    # 597.5 / 598.9 with 3 (profiles/round6/lead/); the total number of warm-up steps is unchanged
    lead_steps = int(os.environ.get("GNN_BENCH_LEAD", "12"))
    # host wall time per pipeline phase (staged-batch wait, step issue, retire, the producer's next
    # batch, next staging issue), accumulated by _pipeline and reset by timed(): where the issuing
    # thread's time goes
    host_phases = [0.0, 0.0, 0.0, 0.0, 0.0]

    def timed(fn_, lead=None):
        """barrier + sync on both sides, max over ranks; returns (seconds, host issue seconds).
        Python's cyclic GC is collected before and paused inside the timed region (a gen-2 pass
        over the process's objects would land in a 33 ms window as a multi-ms stall). `lead`: a
        few untimed steps run after the collection, right before the window's synchronize — the
        collection idles the GPU, and the steps after an idle gap run slow while the chip brings
        its clock back up (20-step window: 2.01, 1.93, 1.88, 1.82, 1.77 ms ... 1.65 ms from about
        the 12th step; profiles/round5/window/), so the window starts on a busy chip."""
        import gc

        gc.collect()
        gc.disable()
        try:
            if lead is not None and lead_steps > 0:
                lead()
            if world > 1:
                torch.distributed.barrier()
            torch.cuda.synchronize()
            retire.wait_s = 0.0
            host_phases[:] = [0.0, 0.0, 0.0, 0.0, 0.0]
            hc0 = host_counters()
            ts = time.perf_counter()
            cpu0 = time.thread_time()
            out = fn_()
            issued = time.perf_counter() - ts - retire.wait_s
            # the issuing thread's CPU time (HIP's blocking waits may spin: an upper bound)
            timed.cpu_s = time.thread_time() - cpu0
            timed.phases = list(host_phases)
            timed.host = host_delta(hc0, host_counters())
            torch.cuda.synchronize()
            if world > 1:
                torch.distributed.barrier()
            el = time.perf_counter() - ts
        finally:
            gc.enable()
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        return el, issued, out

    # ------------------------------------------------- headline: end to end, live sampling
    from gnn_amd.loader import BatchLoader, NativeBatch, NativeLoader, ToDevice

    workers = args.workers or default_workers(world)
    if args.sampler != "ladies" or args.host_extract or args.extract_layers == "none":
        dx = False
    elif args.extract_layers == "all":
        dx = True
    else:
        dx = [int(v) for v in args.extract_layers.split(",") if v]
    lkw = {}
    counts = args.column_counts
    if counts == "auto":
        counts = "mixed" if N >= 1_000_000 else "host"
    if counts in ("gpu", "mixed") and args.sampler == "ladies" and not args.python_loader:
        lkw["device_count"] = dev
        if counts == "mixed":
            lkw["device_count_workers"] = max(1, workers // 2)
    loader = (BatchLoader if args.python_loader else NativeLoader)(
        lap, labels, train, args.samp_num, args.batch_size, [1, 1, 1], pdev, pidx, rank=rank, world_size=world,
        store=store, workers=workers, seed=4242, kind=args.sampler, device_extract=dx,
        skewed_sampling_nodes=skewed, scale_factor=args.scale_factor, **lkw)
    if dx:  # the graph resident in HBM for the extraction (made once, outside every timed region)
        sampler.device_graph(loader.graph, dev)
        torch.cuda.synchronize()
    it = loader.forever()
    if exchange is not None and exchange.needs_negotiation:
        # each batch's peer negotiation off the training thread, 4 batches ahead
        it = staging.NegotiatedStream(it, exchange, depth=4)

    def nxt_live():
        lb = next(it)
        # ToDevice: Stager.issue stages a native-loader batch through one native call
        return lb.plan, (ToDevice(lb.host, dev) if isinstance(lb.host, NativeBatch)
                         else (lambda: lb.host.to_device(dev, with_coo=False)))

    # warm-up: at least the prefetch queue's depth, so the timed steps start in steady state
    # (the queue filled during setup holds pre-sampled batches that must not be timed)
    warm = max(args.warmup, loader.prefetch + 2)
    live_ahead = collections.deque()
    pipeline(nxt_live, warm - min(lead_steps, warm), live_ahead)
    # where the window's time goes: the compute stream's span (first step's first kernel to the last
    # step's last) beside the wall clock between the two device-wide synchronizations
    cs = compute_stream if compute_stream is not None else torch.cuda.current_stream(dev)
    w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def e2e_window():
        w0.record(cs)
        out = pipeline(nxt_live, args.steps, live_ahead)
        w1.record(cs)
        return out

    e2e_s, e2e_issue, loss = timed(e2e_window, lead=lambda: pipeline(nxt_live, min(lead_steps, warm), live_ahead))
    e2e_cpu, e2e_phases, e2e_host = timed.cpu_s, timed.phases, timed.host
    if step_events is not None:
        evs = step_events[-args.steps:] + [w1]
        log("e2e window step spans (ms): " + " ".join(f"{a.elapsed_time(b):.3f}" for a, b in zip(evs, evs[1:])))
    if host_trace is not None:
        log("e2e window host phases per step (us: batch_wait, step_issue, retire, producer_wait, staging_issue): "
            + " ".join("/".join(str(v) for v in t) for t in host_trace[-args.steps:]))
    window = {"wall_ms": round(1e3 * e2e_s, 3), "compute_stream_ms": round(w0.elapsed_time(w1), 3),
              "what": "the timed end-to-end window: wall clock between the barrier + synchronize pairs, and the "
                      "step stream's span over the same steps (the rest: the staging of the batches after the "
                      "window, which the closing synchronize waits for, and the first launch)"}
    # the batches staged for steps past the window: let their staging finish, then drop them
    torch.cuda.synchronize()
    live_ahead.clear()
    log(f"end to end: {world * args.steps / e2e_s:.1f} mini-batches/s ({time.time() - t0:.1f}s)")

    # ------------------------------------------------- GPU step over distinct pre-sampled batches
    gpu_step, roof, spmm_detail, staging_info, dp_ab, peer_ab, prefetch_ab = None, None, {}, None, None, None, None
    gemm_ab = None
    step_batches = []
    if not args.no_gpu_step:
        nwarm = max(2, min(args.warmup, 10))
        gsteps = max(1, min(args.steps, args.gpu_step_batches))
        pre = [next(it) for _ in range(nwarm + gsteps)]
        loader.close()
        if isinstance(it, staging.NegotiatedStream):
            # the look-ahead negotiations finish before the passes below re-negotiate these plans on
            # this thread (Stager.issue): never two threads' collectives on the metadata group
            it.close()
        native = not args.python_loader
        if native:
            # the batch blobs (CSR pieces or GPU-extraction inputs, labels, index arrays, host
            # rows) are uploaded in the timed region, one H2D each, as the live run does
            dbs = [None] * len(pre)
        else:
            # CSR pieces, labels and index arrays resident in HBM; the operand builder (the
            # create_coo_tensor kernel) runs for every step, on the staging stream ahead of it
            dbs = [lb.host.to_device(dev, build=False) for lb in pre]
        torch.cuda.synchronize()
        k_ = [0]

        def nxt_pre():
            j = k_[0]
            k_[0] += 1
            if native:
                return pre[j].plan, ToDevice(pre[j].host, dev, on_built=lambda db, j=j: dbs.__setitem__(j, db))
            db = dbs[j]
            return pre[j].plan, lambda: (db.build_operands(), db)[1]

        def negotiate_ahead():
            """A pass re-issues plans whose look-ahead negotiation was consumed: with a peer-row form
            that negotiates (all-to-all), negotiate them again here, outside the timed region, as the
            live run's NegotiatedStream does ahead of the step (collective: every rank, same order)."""
            ex = stager.exchange
            if ex is None or not ex.needs_negotiation:
                return
            from concurrent.futures import Future

            for lb in pre[nwarm:]:
                f = Future()
                f.set_result(ex.prepare(lb.plan))
                lb.plan.peer_meta = f

        pipeline(nxt_pre, nwarm)

        def pre_lead():
            """untimed steps on the warm-up batches right before a timed pass (timed's `lead`)"""
            was, tm = cso.timing_enabled(), stager.timing
            cso.enable_timing(False)
            stager.timing = None  # the lead's uploads are not the timed pass's staging
            k_[0] = 0
            pipeline(nxt_pre, min(lead_steps, nwarm))
            k_[0] = nwarm
            cso.enable_timing(was)
            stager.timing = tm

        recs = []
        if not args.no_roofline:
            # the aggregation launches timed with HIP events recorded on their stream, over a timed
            # pass of the distinct batches (the events cost ~3-5 % of the step, so the gpu_step
            # value comes from a second pass over the same batches without them)
            negotiate_ahead()
            cso.enable_timing(True)
            timed(lambda: pipeline(nxt_pre, gsteps), lead=pre_lead)
            cso.enable_timing(False)
            recs = cso.take_timing_records()
            k_[0] = nwarm
        if native:
            # every pass uploads each blob afresh: drop the device copies the warm-up / events pass
            # left on the batches (device_blob caches one), so the H2D is inside this timing too
            torch.cuda.synchronize()
            for j in range(len(dbs)):
                dbs[j] = None
                pre[j].host.drop_device()
        stager.timing = []
        negotiate_ahead()
        step_s, step_issue, _ = timed(lambda: pipeline(nxt_pre, gsteps), lead=pre_lead)
        step_cpu = timed.cpu_s
        h_bytes, h_sec = stager.take_timing()
        dp_ab = None
        if world > 1 and getattr(trainer, "bucketed", None) is not None and os.environ.get("GNN_BENCH_DP_AB", "1") == "1":
            # the other gradient exchange over the same batches (gnn_amd.dp vs one flat all-reduce),
            # after the reported passes (`value` and `gpu_step` keep the default exchange): RCCL over
            # xGMI cannot be measured on a one-GPU box, so every N > 1 run records both
            # (GNN_BENCH_DP_AB=0 skips it). Both exchanges are tested equal (tests/test_dist_gpu.py).
            first = "bucketed" if trainer.exchange is not None else "flat"
            trainer.exchange = None if first == "bucketed" else trainer.bucketed
            k_[0] = nwarm
            torch.cuda.synchronize()
            for j in range(len(dbs)):
                dbs[j] = None
                if native:
                    pre[j].host.drop_device()
            negotiate_ahead()
            alt_s, _, _ = timed(lambda: pipeline(nxt_pre, gsteps), lead=pre_lead)
            trainer.exchange = trainer.bucketed if first == "bucketed" else None
            dp_ab = {"default": first, first: round(world * gsteps / step_s, 3),
                     ("flat" if first == "bucketed" else "bucketed"): round(world * gsteps / alt_s, 3),
                     "what": "gpu_step mini-batches/s over the same pre-sampled batches with each gradient "
                             "exchange (bucketed: all-to-all per backward stage overlapped with the backward, "
                             "then the clip factors, shard sums and one gather; flat: clip + one all-reduce)"}
        prefetch_ab = None
        if world > 1 and trainer.exchange is None and os.environ.get("GNN_BENCH_PREFETCH_AB", "1") == "1":
            # the step without the next batch's layer-0 aggregation issued during the all-reduce
            # (GNN_PREFETCH_L0=0), over the same batches, after the reported passes
            k_[0] = nwarm
            torch.cuda.synchronize()
            for j in range(len(dbs)):
                dbs[j] = None
                if native:
                    pre[j].host.drop_device()
            negotiate_ahead()
            was = os.environ.get("GNN_PREFETCH_L0")
            os.environ["GNN_PREFETCH_L0"] = "0" if was != "0" else "1"
            try:
                alt_s, _, _ = timed(lambda: pipeline(nxt_pre, gsteps), lead=pre_lead)
            finally:
                if was is None:
                    os.environ.pop("GNN_PREFETCH_L0", None)
                else:
                    os.environ["GNN_PREFETCH_L0"] = was
            on = was != "0"
            prefetch_ab = {"default": "on" if on else "off", ("on" if on else "off"): round(world * gsteps / step_s, 3),
                           ("off" if on else "on"): round(world * gsteps / alt_s, 3),
                           "what": "gpu_step mini-batches/s over the same pre-sampled batches with and without the next "
                                   "batch's layer-0 aggregation issued while the gradient all-reduce runs "
                                   "(GNN_PREFETCH_L0; the flat exchange)"}
        gemm_ab = None
        if world == 1 and os.environ.get("GNN_BENCH_GEMM_AB", "1") == "1" and not args.unfused:
            # the layer GEMMs on the exact-f32 MFMA kernel (GNN_GEMM_ALGO=f32) instead of split3, over
            # the same batches, after the reported passes: how much of gpu_step the split3 route buys
            k_[0] = nwarm
            torch.cuda.synchronize()
            for j in range(len(dbs)):
                dbs[j] = None
                if native:
                    pre[j].host.drop_device()
            was = os.environ.get("GNN_GEMM_ALGO")
            os.environ["GNN_GEMM_ALGO"] = "f32"
            try:
                alt_s, _, _ = timed(lambda: pipeline(nxt_pre, gsteps), lead=pre_lead)
            finally:
                if was is None:
                    os.environ.pop("GNN_GEMM_ALGO", None)
                else:
                    os.environ["GNN_GEMM_ALGO"] = was
            gemm_ab = {"split3": round(world * gsteps / step_s, 3), "f32": round(world * gsteps / alt_s, 3),
                       "what": "gpu_step mini-batches/s over the same pre-sampled batches with the layer GEMMs on "
                               "split3 (bf16 matrix cores, exact three-way fp32 split; the default) and on the "
                               "f32-input MFMA kernel (bitwise fp32 products, GNN_GEMM_ALGO=f32)"}
        peer_ab = None
        if world > 1 and direct is not None and os.environ.get("GNN_BENCH_PEER_AB", "1") == "1":
            # the other peer-row form over the same batches (direct reads of the IPC-mapped peer
            # buffers vs the negotiated RCCL all-to-all), after the reported passes
            other = alltoall if exchange is direct else direct
            stager.exchange = other
            k_[0] = nwarm
            torch.cuda.synchronize()
            for j in range(len(dbs)):
                dbs[j] = None
                if native:
                    pre[j].host.drop_device()
            negotiate_ahead()
            alt_s, _, _ = timed(lambda: pipeline(nxt_pre, gsteps), lead=pre_lead)
            stager.exchange = exchange
            peer_ab = {"default": args.peer_rows, args.peer_rows: round(world * gsteps / step_s, 3),
                       ("alltoall" if exchange is direct else "direct"): round(world * gsteps / alt_s, 3),
                       "what": "gpu_step mini-batches/s over the same pre-sampled batches with each peer-row form "
                               "(direct: gather kernels reading the peers' IPC-mapped buffers over xGMI; alltoall: "
                               "host negotiation + gather + RCCL all_to_all_single + scatter)"}
        gpu_step = {"value": round(world * gsteps / step_s, 3), "unit": "mini-batches/s",
                    "ms_per_step": round(1e3 * step_s / gsteps, 3),
                    "host_issue_ms_per_step": round(1e3 * step_issue / gsteps, 3),
                    "host_cpu_ms_per_step": round(1e3 * step_cpu / gsteps, 3),
                    "what": f"{gsteps} distinct pre-sampled batches per rank (none cycled); "
                            + ("each batch's blob upload (one H2D), X0 staging, GPU layer extraction / operand builds "
                               "and the whole training step inside the timed region" if native else
                               "CSR pieces resident in HBM; X0 staging, operand builds and the whole training step "
                               "inside the timed region")}
        staging_info = {"mode": args.staging, "host_MB_per_batch": round(h_bytes / gsteps / 1e6, 2),
                        "h2d_GBps": round(h_bytes / h_sec / 1e9, 1) if h_sec > 0 else None,
                        "h2d_ms_per_batch": round(1e3 * h_sec / gsteps, 3),
                        "note": ("GPU gather of the host rows from the pinned, device-mapped feature table over "
                                 "PCIe" if args.staging == "zerocopy" else
                                 "host rows gathered into pinned memory by the sampler threads, one hipMemcpyAsync")
                                + " on the staging stream, overlapped with the previous step"}
        step_batches = [(lb.host, db) for lb, db in zip(pre[nwarm:], dbs[nwarm:])]
        if recs:
            roof, spmm_detail = roofline_from(recs, step_batches, args, traffic, gsteps, sites)
            try:  # the measured ceiling of the dominant kernel's own access shape (cache-resident)
                dom = roof["kernel"].split(" (")[0]
                ceil = gather_ceiling(step_batches[0][1].adjs[0], dom, dev)
                if ceil:
                    ceil["frac"] = round(roof["algorithmic"]["GBps"] / ceil["GBps"], 4)
                    roof["gather_ceiling"] = ceil
                if world == 1:  # the probe runs on device 0 as a child process
                    shape = access_shape_ceiling(step_batches[0][1].adjs[0].shape[1], dom)
                    if shape:
                        shape["frac_at_operand_K"] = round(
                            roof["algorithmic"]["GBps"] / shape["at_operand_K"]["GBps"], 4)
                        roof["access_shape"] = shape
                        roof["frac_access_shape"] = shape["frac_at_operand_K"]
            except Exception as e:  # a failed side measurement must not sink the benchmark
                log(f"gather ceiling skipped: {e!r}")
        if args.cprofile and rank == 0:
            import cProfile
            import pstats

            k_[0] = 0
            pr = cProfile.Profile()
            pr.enable()
            pipeline(nxt_pre, min(20, len(dbs)))
            torch.cuda.synchronize()
            pr.disable()
            with open(args.cprofile, "w") as fh:
                st = pstats.Stats(pr, stream=fh)
                st.sort_stats("tottime").print_stats(45)
                st.sort_stats("cumulative").print_stats(45)
    else:
        loader.close()
        if isinstance(it, staging.NegotiatedStream):
            it.close()
    final_loss = float(loss.item()) if loss is not None else float("nan")
    # every rank must end with bit-identical parameters (summed gradient + the same Adam update,
    # main.py:146-170): the N > 1 line carries its own consistency proof (collective)
    agree = trainer.check_ranks_agree()
    if not agree["identical"]:
        log(f"PARAMETERS DIFFER ACROSS RANKS: {agree['digests']}")
    if direct is not None:
        direct.close()  # every rank's staging is done before any buffer is unmapped / freed
        held["direct"] = None
    if dx:  # every GPU extraction of the run agreed with the host's counts (syncs; outside the timings)
        sampler.device_graph(loader.graph, dev).check()

    cpu = None
    sampler_cost = None
    dropin = None
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(args, probe_batch, feats, num_classes)
        if args.sampler == "ladies" and args.graph == "reddit" and not args.no_roofline:
            try:
                dropin = dropin_timing(probe_batch, feats, dev, 2 * args.nhid if args.model == "graphsage" else args.nhid)
            except Exception as e:  # a failed side measurement must not sink the benchmark
                log(f"drop-in timing skipped: {e!r}")
        chunks = sampler.rank_batches(train, args.batch_size, 0, 1, 99)[:4]
        t = time.perf_counter()
        for i, c in enumerate(chunks[:3]):
            fn(i, c, samp, N, lap, labels, [1, 1, 1], pdev, pidx, None, 1.0, [0])
        nat = (time.perf_counter() - t) / 3
        t = time.perf_counter()
        fn(3, chunks[3], samp, N, lap, labels, [1, 1, 1], pdev, pidx, None, 1.0, [0], native=False)
        sampler_cost = {"native_ms_per_batch_1thread": round(nat * 1e3, 1),
                        "numpy_ms_per_batch_1thread": round((time.perf_counter() - t) * 1e3, 1)}
        if dx:
            t = time.perf_counter()
            for i, c in enumerate(chunks[:3]):
                fn(i, c, samp, N, lap, labels, [1, 1, 1], pdev, pidx, None, 1.0, [0], device_extract=dx)
            sampler_cost["native_draw_only_ms_per_batch_1thread"] = round((time.perf_counter() - t) / 3 * 1e3, 1)
            sampler_cost["note"] = ("native: host extraction of every layer; draw_only: the layers below the top "
                                    "one left to the GPU extraction (what the end-to-end run uses)")

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(world * args.steps / e2e_s, 3),
            "unit": "mini-batches/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * e2e_s / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (Chung-Lu {spec.name}-shaped graph, N(0,1) features, random-init "
                    f"{'GraphSAGE' if args.model == 'graphsage' else 'GCN'}); end to end: live {args.sampler} "
                    f"sampling ({workers} sampler threads per rank) + host staging + H2D + the training step, "
                    f"warm-up of {warm} steps drains the prefetch queue first",
            "config": {"workload": workload_name(args, spec), "sampler": args.sampler, "model": args.model,
                       "global_batch": args.batch_size * world, "samp_num": args.samp_num, "nhid": args.nhid,
                       "feat_dim": int(store.F), "num_nodes": int(N), "graph_nnz": int(A.nnz),
                       "buffer_size": args.buffer_size, "parallelism": f"dp{world}",
                       "peer_rows": (args.peer_rows if world > 1 else None),
                       "nnz_per_batch": int(probe_batch.nnz()), "fused_epilogue": not args.unfused,
                       "stage_ahead": args.stage_ahead, "stage_gate": args.stage_gate, "dropout": dropout,
                       "locality_sampling": args.locality_sampling, "scale_factor": args.scale_factor,
                       "sampler_workers_per_rank": workers, "host_cpus": "gpu numa node" if len(numa_cpus) >= 4 else "all",
                       "batch_producer": "python threads" if args.python_loader else "native (C++ threads, one blob)",
                       "layer_extraction": ("gpu: layers " + args.extract_layers + "; host: the rest") if dx else "host",
                       "column_counts": (("gpu" if not getattr(loader, "device_count_workers", 0) else
                                          f"mixed ({loader.device_count_workers} of {workers} sampler threads on "
                                          "the GPU)") if getattr(loader, "device_count", False) else "host")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "gpu_step": gpu_step,
            "dp_exchange_ab": dp_ab,
            "prefetch_l0_ab": prefetch_ab,
            "gemm_ab": gemm_ab,
            "peer_rows_ab": peer_ab,
            "host_issue_ms_per_step_e2e": round(1e3 * e2e_issue / args.steps, 3),
            "host_cpu_ms_per_step_e2e": round(1e3 * e2e_cpu / args.steps, 3),
            "host_phases_ms_per_step_e2e": {k: round(1e3 * v / args.steps, 3) for k, v in
                                            zip(("batch_wait", "step_issue", "retire", "producer_wait",
                                                 "staging_issue"), e2e_phases)},
            "host_cpu_e2e": host_report(e2e_host, args.steps, workers),
            "e2e_window": window,
            "spmm_per_callsite": spmm_detail,
            "dropin": dropin,
            "sampler": sampler_cost,
            "feature_staging": staging_info,
            "final_loss": round(final_loss, 5),
            "ranks": {"params_identical_across_ranks": agree["identical"], "param_digests": agree["digests"],
                      "peer_rows": peer_info,
                      "what": "sha256 of every rank's parameters after all passes, all-gathered"},
            "peak_hbm_GB": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if not agree["identical"]:
        sys.exit(3)


if __name__ == "__main__":
    main()
