# Round-4 GPU record on the final tree: the whole GPU suite, smoke, the default bench (PMC traffic +
# CPU baseline), config 1 on the CPU, the self-launched N = 2 / 4 rehearsals (gloo, ranks sharing
# the one GPU), rocprofv3 kernel stats of the default bench.
set -o pipefail
TAG=${1:-r4final}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 200 python -u bench.py --cpu --steps 30 --warmup 3 > gpurun_out/bench_cpu_cfg1_$TAG.json \
    2> gpurun_out/bench_cpu_cfg1_$TAG.err || exit 1
GNN_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 3 \
    > gpurun_out/bench_selflaunch2_$TAG.json 2> gpurun_out/bench_selflaunch2_$TAG.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 300 --no-cpu-baseline --no-traffic > $REPO/gpurun_out/bench_prof_$TAG.json \
    2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
cd $REPO
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_$TAG.csv \; 2>/dev/null
echo "exit $rc"
exit $rc
