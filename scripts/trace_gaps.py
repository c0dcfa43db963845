"""Compute-stream gap analysis of a rocprofv3 kernel trace (scripts/gpu.sh ktrace step): per stream,
busy time (union of kernel intervals) vs wall time over the steady-state window, and the largest
idle gaps on the compute stream with the kernel that ended before / started after each gap.
Usage: python scripts/trace_gaps.py kernel_trace.csv[.gz]"""
import collections
import csv
import gzip
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:45]


def main(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        rows = list(csv.DictReader(f))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
    ks.sort()
    by = collections.defaultdict(list)
    for k in ks:
        by[k[2]].append(k)
    # the compute stream: the one running the layer-0 aggregation main kernel most often
    comp = max(by, key=lambda s: sum("spmm_unit_kernel<4, 16, 1, 4, false>" in k[3] for k in by[s]))
    ck = by[comp]
    # steady state: from the 20th step marker (adam_kernel ends a step) to the last
    ends = [k for k in ck if k[3].startswith("(anonymous namespace)::adam_kernel")]
    if len(ends) < 30:
        print("too few steps", len(ends))
        return
    t0, t1 = ends[19][1], ends[-1][1]
    nsteps = len(ends) - 20
    print(f"compute stream {comp}: {nsteps} steps, {(t1 - t0) / nsteps / 1e3:.1f} us per step")
    for s, lst in sorted(by.items()):
        busy, cur_s, cur_e = 0, None, None
        for a, b, _, _ in lst:
            a, b = max(a, t0), min(b, t1)
            if b <= a:
                continue
            if cur_e is None or a > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = a, b
            else:
                cur_e = max(cur_e, b)
        if cur_e is not None:
            busy += cur_e - cur_s
        n = sum(1 for k in lst if t0 <= k[0] < t1)
        print(f"  stream {s}: {n / nsteps:.1f} kernels/step, busy {busy / nsteps / 1e3:.1f} us/step")
    gaps = []
    prev = None
    for k in ck:
        if k[0] < t0 or k[1] > t1:
            prev = k
            continue
        if prev is not None and k[0] > prev[1]:
            gaps.append((k[0] - prev[1], prev[3], k[3]))
        prev = k
    tot = sum(g[0] for g in gaps)
    print(f"compute-stream idle: {tot / nsteps / 1e3:.1f} us/step over {len(gaps) / nsteps:.1f} gaps/step")
    agg = collections.defaultdict(lambda: [0, 0])
    for g, a, b in gaps:
        key = (short(a), short(b))
        agg[key][0] += g
        agg[key][1] += 1
    for (a, b), (g, n) in sorted(agg.items(), key=lambda x: -x[1][0])[:15]:
        print(f"  {g / nsteps / 1e3:6.1f} us/step  x{n / nsteps:.1f}  after {a}  before {b}")


if __name__ == "__main__":
    main(sys.argv[1])
