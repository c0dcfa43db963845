# The column-frequency relabel of the layer-0 operand (scripts/spmm_relabel.py): timings, then the
# L2 hit rate and L2 egress of the orig / freq cases, one rocprofv3 --pmc pass per counter set and
# case, each under its own kill timeout.
set -o pipefail
TAG=${1:-rl}
mkdir -p gpurun_out/relabel_$TAG
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 300 python3 -u scripts/spmm_relabel.py > gpurun_out/relabel_$TAG/timing.jsonl \
    2> gpurun_out/relabel_$TAG/timing.err || exit 1
cd /tmp
for CASE in orig freq; do
  i=0
  for C in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    CASE=$CASE REPS=10 WARM=5 timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d /tmp/rl_${CASE}_$i -o run -- \
        python3 $REPO/scripts/spmm_relabel.py > $REPO/gpurun_out/relabel_$TAG/pmc_${CASE}_$i.log 2>&1 || exit 1
    find /tmp/rl_${CASE}_$i -name "*counter_collection.csv" -exec cp {} $REPO/gpurun_out/relabel_$TAG/pmc_${CASE}_$i.csv \;
  done
done
echo "exit 0"
