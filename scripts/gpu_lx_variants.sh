# GPU box: per-kernel times (rocprofv3 --stats) of the extraction probe under env variants.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env $v REPS=10 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lxv$i -o x -- \
      python -u scripts/extract_probe.py > gpurun_out/lxv$i.log 2>&1 || { echo "variant $v failed"; exit 1; }
  f=$(find /tmp/lxv$i -name "*kernel_stats.csv")
  python - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
    if "lx_" in n:
        print(f'{sys.argv[2]:32s} {n:28s} {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:7.1f} min {float(r["MinNs"])/1e3:7.1f}')
PY
done
