# The default bench under rocprofv3 kernel stats (no PMC), summary copied to gpurun_out/. Usage: TAG
set -o pipefail
TAG=${1:-rp}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --no-cpu-baseline --no-traffic > $REPO/gpurun_out/bench_prof_$TAG.json \
    2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
cd $REPO
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_$TAG.csv \; 2>/dev/null
echo "exit $rc"
exit $rc
