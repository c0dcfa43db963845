"""Join rocprofv3 counter passes with kernel statistics into a per-kernel HBM table (scripts/pmc_kernels.sh).

  python scripts/pmc_table.py reduce counter_collection.csv out.csv   # per kernel: dispatches, sum of the counter
  python scripts/pmc_table.py table fetch.csv write.csv kernel_stats.csv   # markdown table

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3's derived counters; bench.py reads them the same way). On gfx950 FETCH_SIZE reports
half the bytes of wide (16 B / lane) coalesced streaming reads (MI355X_MICROARCH.md §HBM): the table gives
the raw value and the 2× corrected one; a kernel's true read bytes lie between them when its reads mix
streaming and scattered lines. Durations are rocprofv3's kernel statistics of a run of the same command
(kernels beside other streams' kernels run longer than alone)."""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n).replace("void ", "")
    return re.sub(r"\(.*", "", n)[:60]


def reduce(src, dst):
    acc = collections.defaultdict(lambda: [0, 0.0, 0.0])  # dispatches, counter sum (KiB), duration sum (ns)
    seen = set()
    with open(src) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or ""
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), name)
            v = float(r.get("Counter_Value") or 0.0)
            a = acc[short(name)]
            if key not in seen:  # one row per (dispatch, counter); durations once per dispatch
                seen.add(key)
                a[0] += 1
                if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                    a[2] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            a[1] += v
    with open(dst, "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "sum_kib", "sum_ns"])
        for k, (n, s, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, n, f"{s:.1f}", f"{t:.0f}"])


def table(fetch, write, kstats):
    def load(p):
        with open(p) as f:
            return {r["kernel"]: (int(r["dispatches"]), float(r["sum_kib"]), float(r["sum_ns"])) for r in csv.DictReader(f)}

    F, W = load(fetch), load(write)
    ks = {}
    with open(kstats) as f:
        for r in csv.DictReader(f):
            k = short(r["Name"])
            c, t = ks.get(k, (0, 0.0))
            ks[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
    rows = []
    for k, (c, t) in ks.items():
        if k not in F or k not in W:
            continue
        nf, sf, tf = F[k]
        nw, sw, _ = W[k]
        rd, wr = sf / nf * 1024.0, sw / nw * 1024.0  # bytes per dispatch
        us = t / c / 1e3  # in the step (kernel statistics run)
        us_pmc = tf / nf / 1e3 if tf > 0 else float("nan")  # counter run: dispatches serialised
        rows.append((t, k, c, us, us_pmc, rd, wr))
    rows.sort(reverse=True)
    print("| kernel | calls | µs in step | µs alone (PMC run) | read MB (raw / 2×) | write MB | GB/s alone, raw read + write | same, 2× read | of 8 TB/s (2× read) |")
    print("|---|---|---|---|---|---|---|---|---|")
    for t, k, c, us, up, rd, wr in rows[:25]:
        g1 = (rd + wr) / (up * 1e3)
        g2 = (2 * rd + wr) / (up * 1e3)
        print(f"| {k} | {c} | {us:.1f} | {up:.1f} | {rd / 1e6:.1f} / {2 * rd / 1e6:.1f} | {wr / 1e6:.1f} | {g1:.0f} | {g2:.0f} | "
              f"{g2 / 8000:.2f} |")


if __name__ == "__main__":
    if sys.argv[1] == "reduce":
        reduce(sys.argv[2], sys.argv[3])
    else:
        table(*sys.argv[2:5])
