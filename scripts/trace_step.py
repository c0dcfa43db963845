"""Per-call breakdown of a rocprofv3 --kernel-trace CSV (scripts/gpu.sh ktrace step): the dispatches of
the k-th to last training step (adam_kernel closes a step), with start offset, duration, queue,
grid, and the compute queue's idle gaps. Usage: python scripts/trace_step.py TRACE.csv [k]"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"\(.*", "", n)[:56]


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    ad = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    i0, i1 = ad[-k - 1], ad[-k]  # k > 0: from the end; k < 0: from the start
    t0 = rows[i0]["e"]
    cq = rows[i1]["Queue_Id"]
    last_end, gaps = t0, 0.0
    for r in rows[i0 + 1:i1 + 1]:
        wg = max(1, int(r["Workgroup_Size_X"] or 1))
        gap = ""
        if r["Queue_Id"] == cq:
            g = (r["s"] - last_end) / 1e3
            if g > 1.0:
                gap = f"  <- gap {g:.1f}"
                gaps += g
            last_end = max(last_end, r["e"])
        print(f"{(r['s'] - t0) / 1e3:8.1f} {(r['e'] - r['s']) / 1e3:7.1f}us q{r['Queue_Id']} "
              f"grid={int(r['Grid_Size_X']) // wg}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} {short(r['Kernel_Name'])}{gap}")
    print(f"step {(rows[i1]['e'] - t0) / 1e3:.1f} us, compute-queue gaps {gaps:.1f} us")


if __name__ == "__main__":
    main()
