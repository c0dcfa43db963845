# Default bench (no PMC / CPU legs) + a rocprofv3 kernel-stats pass over a shorter bench. Usage: TAG [extra bench args]
set -o pipefail
TAG=${1:-b}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-traffic "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 200 --no-cpu-baseline --no-traffic --no-gpu-step "$@" \
    > $REPO/gpurun_out/bench_prof_$TAG.json 2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
cd $REPO
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_$TAG.csv \; 2>/dev/null
echo "exit $rc"
exit $rc
