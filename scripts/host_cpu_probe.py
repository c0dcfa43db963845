"""Host CPU probe: what the box grants this job and how loaded the machine is.

Prints the affinity set, the cgroup's CPU quota and throttling counters, the SMT layout, the
machine's load average, and two single-thread costs the batch producer pays per Reddit batch:
the host-row gather (13.8 k random 2,408-byte rows of a 561 MB table into one buffer) and a
sequential memcpy of the same bytes.

    python scripts/host_cpu_probe.py
"""
import json
import os
import time

import numpy as np


def read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def main():
    aff = sorted(os.sched_getaffinity(0))
    out = {"os_cpu_count": os.cpu_count(), "affinity": len(aff), "cpu.max": read("/sys/fs/cgroup/cpu.max"),
           "cpu.stat": read("/sys/fs/cgroup/cpu.stat"), "loadavg": read("/proc/loadavg")}
    sib = read(f"/sys/devices/system/cpu/cpu{aff[0]}/topology/thread_siblings_list") if aff else None
    out["smt_siblings_of_first_cpu"] = sib
    model = None
    for line in (read("/proc/cpuinfo") or "").splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    out["cpu_model"] = model
    rng = np.random.default_rng(0)
    table = rng.standard_normal((232_965, 602), dtype=np.float32)
    idx = np.sort(rng.choice(232_965, 13_800, replace=False))
    dst = np.empty((13_800, 608), np.float32)
    ts = []
    for _ in range(7):
        t = time.perf_counter()
        dst[:, :602] = table[idx]
        ts.append(time.perf_counter() - t)
    out["row_gather_ms"] = round(1e3 * float(np.median(ts)), 2)
    src = dst.copy()
    ts = []
    for _ in range(7):
        t = time.perf_counter()
        np.copyto(dst, src)
        ts.append(time.perf_counter() - t)
    out["memcpy_33MB_ms"] = round(1e3 * float(np.median(ts)), 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
