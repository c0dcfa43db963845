# Round-4 GPU pass n: parameter-gradient epilogues on the aux stream (suite), EPI_AUX A/B/A/B under the bench, rocprofv3 stats.
set -o pipefail
TAG=${1:-r4n}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  GNN_STEP_EPI_AUX=$v timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_epi${v}_${TAG}_$i.json 2>> gpurun_out/bench_epi_$TAG.err || exit 1
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 200 --no-cpu-baseline --no-traffic > $REPO/gpurun_out/bench_prof_$TAG.json \
    2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/kstats_$TAG.csv \;
echo "exit $rc"
exit $rc
