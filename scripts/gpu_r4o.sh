# Round-4 GPU pass o: finalize kernel with 16 loads in flight, split-k reduce with 4 (same add order):
# the suite, two benches, rocprofv3 stats.
set -o pipefail
TAG=${1:-r4o}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 200 --no-cpu-baseline --no-traffic > $REPO/gpurun_out/bench_prof_$TAG.json \
    2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/kstats_$TAG.csv \;
echo "exit $rc"
exit $rc
