# Column tiles as lane groups x chunks per lane on the step's real call shapes
# (scripts/spmm_ceiling.py QUICK=1). Arguments: "G:NJ" pairs ("-" = the default choice), each run twice
# in A B .. A B order.
set -o pipefail
TAG=${TAG:-nj}
mkdir -p gpurun_out/njsweep_$TAG
export TMPDIR=/tmp
[ $# -eq 0 ] && set -- - 16:2
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = "-" ]; then E=""; n=default; else E="GNN_SPMM_G=${v%%:*} GNN_SPMM_NJ=${v#*:}"; n="g${v%%:*}_nj${v#*:}"; fi
    env $E QUICK=1 timeout -k 10 240 python3 -u scripts/spmm_ceiling.py >> gpurun_out/njsweep_$TAG/$n.jsonl \
        2>> gpurun_out/njsweep_$TAG/$n.err || exit 1
  done
done
echo "exit 0"
