"""CPU: bench.py's per-call-site roofline bookkeeping (roofline_from) over timing records as the
native executor names them (fwd_L0, fwd_L1, fwd_L2, bwd_L1: the layer-2 backward folded into the
layer-1 tail leaves no record) and as the autograd path emits them (fwd / bwd, five per step in
call order): every record lands on its call site and its own step's batch."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from gnn_amd.sampler import HostLayer  # noqa: E402


class _HB:
    def __init__(self, seed):
        rng = np.random.default_rng(seed)
        self.layers = []
        for M, K in ((30, 40), (20, 30), (5, 20)):
            rowptr = np.concatenate([[0], np.cumsum(rng.integers(0, 4, M))]).astype(np.int32)
            colidx = np.sort(rng.integers(0, K, rowptr[-1])).astype(np.int32)
            self.layers.append(HostLayer(fullrowptr=rowptr, rowptr=rowptr, colidx=colidx,
                                         normfact=np.ones(K, np.float32), shape=(M, K)))


def _rec(tag, li, hb, F, kname):
    L = hb.layers[li]
    M, K = L.shape if tag.startswith("fwd") else L.shape[::-1]
    nnz = L.nnz
    return (tag, 0.01, nnz * F * 4 + nnz * 8 + (M + 1) * 4 + M * F * 4, kname,
            dict(M=M, K=K, nnz=nnz, F=F, res_rows=0))


def test_roofline_from_executor_tags_and_positional():
    hbs = [_HB(s) for s in range(3)]
    batches = [(hb, None) for hb in hbs]

    class A:
        pass

    # executor: four named records per step (the folded bwd_L2 has none)
    recs = []
    for hb in hbs:
        for tag, li in (("fwd_L0", 0), ("fwd_L1", 1), ("fwd_L2", 2), ("bwd_L1", 1)):
            recs.append(_rec(tag, li, hb, 8, "k_big" if li < 2 else "k_small"))
    roof, detail = bench.roofline_from(recs, batches, A(), None, len(hbs))
    assert sorted(detail) == ["bwd_L1", "bwd_L2", "fwd_L0", "fwd_L1", "fwd_L2"]
    assert "folded" in detail["bwd_L2"] and "avg_us" not in detail["bwd_L2"]  # listed, not timed
    assert all("dispatch" in detail[k]["timing"] for k in ("fwd_L0", "bwd_L1"))
    assert roof["kernel"].startswith("k_big") and "over 9 launches" in roof["kernel"]
    # autograd path: five unnamed records per step in call order
    recs = []
    for hb in hbs:
        for tag, li in (("fwd", 0), ("fwd", 1), ("fwd", 2), ("bwd", 2), ("bwd", 1)):
            recs.append(_rec(tag, li, hb, 8, "k_big" if li < 2 else "k_small"))
    roof, detail = bench.roofline_from(recs, batches, A(), None, len(hbs))
    assert sorted(detail) == ["bwd_L1", "bwd_L2", "fwd_L0", "fwd_L1", "fwd_L2"]
    assert "over 9 launches" in roof["kernel"]


def test_sites_from_trace():
    """The traced child run's dispatches -> per call site averages (bench.site_trace): steps cut at
    adam_kernel, aggregation main kernels named in call order, the warm-up steps dropped."""
    rows, ts = [], 0

    def disp(name, us):
        nonlocal ts
        rows.append({"Kernel_Name": f"void (anonymous namespace)::{name}(int const*, float*)",
                     "Start_Timestamp": str(ts), "End_Timestamp": str(ts + int(us * 1e3))})
        ts += int(us * 1e3) + 500

    for step in range(5):
        big = 300.0 if step < 2 else 240.0  # two slow warm-up steps, dropped below
        disp("spmm_unit_kernel<4, 16, 1, 4, false>", big)
        disp("spmm_combine_kernel<4, 4>", 10.0)
        disp("spmm_unit_kernel<4, 16, 1, 4, false>", 200.0)
        disp("spmm_unit_kernel<4, 64, 1, 16, false>", 16.0 + step)
        disp("sage_norm_bwd2_kernel<2, true>", 30.0)
        disp("spmm_unit_kernel<4, 32, 1, 4, true>", 201.0)
        disp("adam_kernel", 15.0)
    out = bench.sites_from_trace(rows, 3)
    assert sorted(out) == ["bwd_L1", "fwd_L0", "fwd_L1", "fwd_L2"]
    assert out["fwd_L0"] == {"rocprof_avg_us": 240.0, "launches": 3, "kernel": "spmm_unit_kernel<4, 16, 1, 4, false>"}
    assert out["fwd_L2"]["rocprof_avg_us"] == 19.0 and out["bwd_L1"]["kernel"].endswith("true>")


def test_host_report_reads_window_deltas():
    """bench.py's host diagnostics: per-step CPU time of the training thread and of
    the other threads, and the cgroup's busy CPUs and CFS throttling over the window."""
    a = {"wall": 10.0, "proc_cpu": 100.0, "thread_cpu": 20.0, "cg_usage_usec": 5_000_000, "cg_nr_periods": 100,
         "cg_nr_throttled": 3, "cg_throttled_usec": 1500}
    b = {"wall": 10.5, "proc_cpu": 106.0, "thread_cpu": 20.5, "cg_usage_usec": 11_000_000, "cg_nr_periods": 105,
         "cg_nr_throttled": 5, "cg_throttled_usec": 4500}
    d = bench.host_delta(a, b)
    r = bench.host_report(d, steps=100, workers=14)
    assert r["trainer_thread_cpu_ms_per_step"] == 5.0 and r["other_threads_cpu_ms_per_step"] == 55.0
    assert r["process_cpus_busy"] == 12.0 and r["sampler_workers"] == 14
    assert r["cgroup"] == {"cpus_busy": 12.0, "periods": 5, "throttled_periods": 2, "throttled_ms": 3.0}
    # no cgroup v2 counters (e.g. this container): the process part alone
    r = bench.host_report(bench.host_delta({"wall": 0.0, "proc_cpu": 0.0, "thread_cpu": 0.0},
                                           {"wall": 1.0, "proc_cpu": 2.0, "thread_cpu": 1.0}), steps=10, workers=2)
    assert "cgroup" not in r and r["process_cpus_busy"] == 2.0
    assert bench.host_report({}, steps=10, workers=2) is None
    c = bench.host_counters()
    assert {"wall", "proc_cpu", "thread_cpu"} <= set(c)
