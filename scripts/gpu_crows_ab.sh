# Combine-kernel A/Bs under rocprofv3 kernel traces of the default bench (300 steps), the SpMM GPU
# tests first. Arguments: one env setting per run ("-" = defaults), e.g. "-" "GNN_SPMM_CROWS=16"
# (rows per combine workgroup) or "GNN_SPMM_CBATCH=4" (pieces per load round); none = the round-3
# rows-per-workgroup A/B/A/B.
set -o pipefail
TAG=${TAG:-cr}
mkdir -p gpurun_out/cr_$TAG
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/cr_$TAG/tests.log 2>&1 || { echo "tests failed"; exit 1; }
i=0
[ $# -eq 0 ] && set -- - GNN_SPMM_CROWS=16 - GNN_SPMM_CROWS=16
for E in "$@"; do
  i=$((i+1))
  v=${E#*=}; [ "$E" = "-" ] && { E=""; v=default; }
  (cd /tmp && env $E timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/cr_$i -o run -- \
      python -u $REPO/bench.py --steps 300 --no-cpu-baseline --no-traffic --no-roofline \
      > $REPO/gpurun_out/cr_$TAG/bench_${i}_$v.json 2> $REPO/gpurun_out/cr_$TAG/bench_${i}_$v.err) || exit 1
  python3 - "$i" "$v" <<'PY' >> gpurun_out/cr_$TAG/summary.txt
import csv, glob, sys, collections
i, v = sys.argv[1], sys.argv[2]
f = glob.glob(f"/tmp/cr_{i}/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
nadam = 0
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "adam_kernel" in n:
        nadam += 1
    if "spmm_combine" in n:
        d[int(r["Grid_Size_X"]) // 256].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(x) for x in d.values()) / max(nadam, 1)
print(i, v, "combine us/step", round(tot, 1), {g: (len(x), round(sum(x) / len(x), 1)) for g, x in sorted(d.items())})
PY
done
cat gpurun_out/cr_$TAG/summary.txt
echo "exit 0"
